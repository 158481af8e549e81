#!/bin/bash
# OuterCoder encode: register-resident low-rate kernel (base) against the LDS-work kernel (rso)
# and a 2-waves/SIMD build (rsw2); parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/outer_ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_outer.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
for v in base rso rsw2 base rso; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode outer --steps 10 --warmup 3 > $O/o_${v}_$i.json 2> $O/o_${v}_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/o_${v}_$i.json')); r=d['roofline']; print('$v', r['avg_launch_ms'], r['frac'], d['outputs_verified'], d['decode']['roofline']['frac'])"
  i=$((i+1))
done
