#!/bin/bash
# per-call encode: level-1 rows copied out while level 2 runs, against one D2H after both; parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/enc_overlap
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in ovl one ovl one; do
  knob=""; [ $v == one ] && knob="TEC_DEBUG_KNOBS=1 TEC_ENC_OVERLAP=0"
  env $knob timeout -k 10 300 python bench.py --mode percall --cpu-sample 0 > $O/p_$v.json 2> $O/p_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/p_$v.json')); c=d['calls']; print('$v', {k: r['encode']['ms_per_call'] for k, r in c.items()}, d['outputs_verified'])"
done
