#!/bin/bash
# repair: folded-kernel tests + bench lines (all available / one peer down) + kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/t3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_repair_sets.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "repair" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for u in 0 1; do
  timeout -k 10 300 python bench.py --mode repair --unavailable $u --steps 20 --warmup 5 --cpu-sample 0 --copy-objects 0 > $OUT/bench_repair_u$u.json 2> $OUT/bench_repair_u$u.err || exit $?
  cat $OUT/bench_repair_u$u.json; echo
done
for u in 0 1; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_u$u -o run -- python3 bench.py --mode repair --unavailable $u --steps 5 --warmup 2 --cpu-sample 0 --copy-objects 0 > $OUT/prof_u$u.log 2>&1 || exit $?
grep -h "rep_fold\|rep_stage" $OUT/prof_u$u/run_kernel_stats.csv
done
find $OUT -name "*kernel_trace.csv" -delete
exit 0
