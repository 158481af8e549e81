#!/bin/bash
# leaf-kernel wave priority A/B on the commit probe (4 GiB groups after 2 GiB ones) and the default
# line's copy-inclusive legs; commitment parity; per-call lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k "commit or stream or leaf or proof" > $O/pytest_commit.log 2>&1; rc=$?; tail -2 $O/pytest_commit.log; [ $rc -eq 0 ] || exit $rc
for v in base leaf0; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib TEC_DEBUG_KNOBS=1 TEC_COMMIT_TRACE=1 PRE="dev host" SEQ=auto:2,auto:4,auto:8,auto:4,device:4 timeout -k 10 400 python -u scripts/commit_windows_probe.py > $O/probe_$v.txt 2> $O/probe_$v.err || exit $?
  python3 -c "
import json
for l in open('$O/probe_$v.txt'):
    if l.startswith('{\"probe'): print('$v', [(r['hashing'], r['group_GiB'], r['GiBps']) for r in json.loads(l)['runs']])"
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --cpu-sample 0 > $O/default.json 2> $O/default.err && python3 -c "import json; d=json.load(open('$O/default.json')); print('default', d['roofline']['frac'], d['copy_inclusive']['value'], d['copy_inclusive_encode_commit']['by_window'], d['copy_inclusive_encode_commit']['stream_writer'], d['stream_sdk_shape']['value'], d['stream_sdk_shape']['chunk_latency_ms_p50_p90'])" || exit $?
timeout -k 10 300 python -u bench.py --mode percall --cpu-sample 0 > $O/percall.json 2> $O/percall.err && python3 -c "import json; d=json.load(open('$O/percall.json')); print({k: {c: v['ms_per_call'] for c, v in r.items()} for k, r in d['calls'].items()})"
