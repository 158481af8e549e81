#!/bin/bash
# per-call line + its kernel trace (which kernels a 4 MiB / 64 MiB call runs, and for how long)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/percall_prof
mkdir -p $O
export TMPDIR=/tmp
true
true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --mode percall --cpu-sample 0 > $O/prof.log 2>&1 || exit $?
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv && cp $(find $O/prof -name "*kernel_trace.csv" | head -1) $O/kernel_trace.csv
cut -c1-160 $O/kernel_stats.csv | head -14
