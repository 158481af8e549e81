#!/bin/bash
# parity after the level-2 DMA trim, pooled/polled piece events and the contended hashing-side
# choice; then the default line (copy-inclusive legs, SDK-shape leg) and the stream mode
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py tests/test_gpu_stream.py tests/test_golden.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/default.json 2> $O/default.err && python3 -c "import json; d=json.load(open('$O/default.json')); r=d['roofline']; print('default', r['avg_launch_ms'], r['frac'], r['box_ceiling_frac'], d['cpu_baseline']['gpu_matches_oracle_on_sample'], d['copy_inclusive']['value'], d['copy_inclusive_encode_commit']['by_window'], d['copy_inclusive_encode_commit']['stream_writer'], d['stream_sdk_shape']['value'], d['stream_sdk_shape']['chunk_latency_ms_p50_p90'])" || exit $?
timeout -k 10 400 python -u bench.py --mode stream --cpu-sample 0 > $O/stream.json 2> $O/stream.err && python3 -c "import json; d=json.load(open('$O/stream.json')); print('stream', {k: (v['GiBps'], v['chunk_latency_ms_p50_p90']) for k, v in d['legs'].items()})"
# store cache-policy variants of the encode (base = in-tree)
bash scripts/gpu_enc_var.sh r5j_st base e_st1 e_st3 e_st16 e_st18 e_st19 base
