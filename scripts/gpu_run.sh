#!/bin/bash
# One gpurun call: optional GPU tests, bench lines, and a rocprofv3 kernel-stats pass.
#   TESTS="repair or recover"  pytest -m gpu -k expression ("all" = whole suite, empty = none)
#   MODES="repair decode"  bench.py --mode lines (env BENCH_ENV is prepended, e.g. TEC_DEBUG_KNOBS=1 TEC_REPAIR_KERNEL=stage)
#   PROF="repair"          bench modes to run under rocprofv3 --kernel-trace --stats
# Every GPU step has its own time limit and the script stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/run
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  sel="$TESTS"; [ "$TESTS" == "all" ] && sel=""
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$sel" > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for m in $MODES; do
  timeout -k 10 300 env $BENCH_ENV python bench.py --mode $m --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 $BENCH_ARGS > $OUT/bench_$m.json 2> $OUT/bench_$m.err || exit $?
  cat $OUT/bench_$m.json
done
for m in $PROF; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$m -o run -- python3 bench.py --mode $m --steps 5 --warmup 2 --cpu-sample 0 --copy-objects 0 $BENCH_ARGS > $OUT/prof_$m.log 2>&1 || exit $?
  find $OUT/prof_$m -name "*kernel_stats.csv" -exec cat {} \;
  find $OUT/prof_$m -name "*kernel_trace.csv" -delete
done
exit 0
