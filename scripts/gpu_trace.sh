#!/bin/bash
# rocprofv3 kernel-trace stats of one bench mode: scripts/gpu_trace.sh <mode> [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
m=$1; shift
OUT=gpurun_out/trace_$m
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --mode $m --steps 5 --warmup 2 --cpu-sample 0 --copy-objects 0 "$@" > $OUT/bench.log 2>&1 || exit $?
find $OUT -name "*kernel_trace.csv" -delete
