#!/bin/bash
# round-3 check: repair helper sets + stream writer GPU tests, repair bench lines, encode bench
# with the copy-inclusive legs (stream writer), rocprof stats of the one-down repair line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/t2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_repair_sets.py tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_engine.py -m gpu -x -v --timeout 300 --timeout-method thread -k "repair or two_devices or multi or stream or commit" > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for u in 0 1; do
  timeout -k 10 300 python bench.py --mode repair --unavailable $u --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 > $OUT/bench_repair_u$u.json 2> $OUT/bench_repair_u$u.err || exit $?
  cat $OUT/bench_repair_u$u.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_u1 -o run -- python3 bench.py --mode repair --unavailable 1 --steps 5 --warmup 2 --cpu-sample 0 --copy-objects 0 > $OUT/prof_u1.log 2>&1 || exit $?
find $OUT/prof_u1 -name "*kernel_stats.csv" -exec cat {} \;
find $OUT -name "*kernel_trace.csv" -delete
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > $OUT/bench_encode.json 2> $OUT/bench_encode.err || exit $?
cat $OUT/bench_encode.json
exit 0
