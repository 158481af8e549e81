#!/bin/bash
# OuterCoder matrix kernel: parity (outer tests), encode/decode A/B against the register-transform
# kernel (TEC_RS16_NO_MATRIX) and the LDS-work kernel (rso); then the default line with the host
# cache released before the SDK-shape leg
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_outer.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
for v in base fftreg rso base fftreg; do
  lib=tape_amd/libtapeec.so; [ $v == rso ] && lib=varlib/lib_rso.so
  knob=""; [ $v == fftreg ] && knob="TEC_DEBUG_KNOBS=1 TEC_RS16_NO_MATRIX=1"
  env $knob TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode outer --steps 10 --warmup 3 > $O/o_${v}_$i.json 2> $O/o_${v}_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/o_${v}_$i.json')); r=d['roofline']; print('$v', r['avg_launch_ms'], r['frac'], d['outputs_verified'], d['decode']['roofline']['avg_launch_ms'], d['decode']['roofline']['frac'], d['decode']['outputs_verified'])"
  i=$((i+1))
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/default.json 2> $O/default.err && python3 -c "import json; d=json.load(open('$O/default.json')); r=d['roofline']; print('default', r['avg_launch_ms'], r['frac'], r['box_ceiling_frac'], d['copy_inclusive']['value'], d['copy_inclusive_encode_commit']['by_window'], d['stream_sdk_shape']['value'], d['stream_sdk_shape']['chunk_latency_ms_p50_p90'])"
