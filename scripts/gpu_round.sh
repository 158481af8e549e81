#!/bin/bash
# Round GPU pass 1: parity tests, headline bench (encode, incl. copy-inclusive and CPU baseline),
# rocprofv3 kernel-trace stats of the same bench command.  Outputs under gpurun_out/round/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $OUT/bench_encode.json 2> $OUT/bench_encode.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_encode -o run -- \
    python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --copy-objects 0 > $OUT/trace_encode.log 2>&1 || exit $?
find $OUT -name "*kernel_trace.csv" -size +2M -delete
exit $rc
