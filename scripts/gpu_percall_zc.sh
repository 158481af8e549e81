#!/bin/bash
# per-call repair: zero-copy staging (the default: kernels on the pinned buffers) against H2D / D2H copies;
# the repair parity tests under the knob first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/percall_zc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_repair_sets.py tests/test_gpu_parity.py tests/test_gpu_engine.py -x -q -k "repair" --timeout 120 --timeout-method thread > $O/pytest_zc.log 2>&1; rc=$?; tail -2 $O/pytest_zc.log; [ $rc -eq 0 ] || exit $rc
for v in copy zc copy zc; do
  knob=""; [ $v == copy ] && knob="TEC_DEBUG_KNOBS=1 TEC_REPAIR_ZC=0"
  env $knob timeout -k 10 300 python bench.py --mode percall --cpu-sample 0 > $O/p_$v.json 2> $O/p_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/p_$v.json')); c=d['calls']; print('$v', {k: r['repair']['ms_per_call'] for k, r in c.items()}, d['outputs_verified'])"
done
