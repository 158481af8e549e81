#!/bin/bash
# repair host path: repair tests, then the repair bench with every helper up and with one down
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/t9
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_repair_sets.py \
  -k "repair" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for u in 0 1; do
  timeout -k 10 300 python bench.py --mode repair --unavailable $u --steps 20 --warmup 3 --cpu-sample 0 --copy-objects 0 > $OUT/rep_u$u.json 2> $OUT/rep_u$u.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/rep_u$u.json')); print('repair u$u', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])"
done
