#!/bin/bash
# repair (folded, one launch) + fused recover: tests, bench lines, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/t4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_repair_sets.py tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -v --timeout 300 --timeout-method thread -k "repair or recover or reconstruct" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in "repair --unavailable 0" "repair --unavailable 1" "recover"; do
  f=$(echo $m | tr ' ' '_')
  timeout -k 10 300 python bench.py --mode $m --steps 20 --warmup 5 --cpu-sample 0 --copy-objects 0 > $OUT/bench_$f.json 2> $OUT/bench_$f.err || exit $?
  cat $OUT/bench_$f.json; echo
done
for m in "repair --unavailable 1" "recover"; do
  f=$(echo $m | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$f -o run -- python3 bench.py --mode $m --steps 5 --warmup 2 --cpu-sample 0 --copy-objects 0 > $OUT/prof_$f.log 2>&1 || exit $?
  grep -h "tec::" $OUT/prof_$f/run_kernel_stats.csv
done
find $OUT -name "*kernel_trace.csv" -delete
exit 0
