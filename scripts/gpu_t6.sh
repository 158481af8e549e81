#!/bin/bash
# repair fold staging fix: one-down tests on both register budgets, then the bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t6
for v in base wpe4; do
  TAPE_EC_LIB=varlib/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_repair_sets.py -m gpu -x -q --timeout 300 --timeout-method thread -k "repair" > gpurun_out/t6/pytest_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 gpurun_out/t6/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for u in 0 1; do
  for v in base wpe4 base wpe4; do
    TAPE_EC_LIB=varlib/lib_$v.so timeout -k 10 300 python bench.py --mode repair --unavailable $u --steps 20 --warmup 5 --cpu-sample 0 --copy-objects 0 > gpurun_out/t6/$v$u.json 2> gpurun_out/t6/$v$u.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/t6/$v$u.json')); print('$v u=$u', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])"
  done
done
