#!/bin/bash
# PMC passes over the encode microbench (one counter group per pass, each under its own limit).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmck
mkdir -p $OUT
KB=${KB:-./scripts/kbench}
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $KB 1024 r q > $OUT/p$i.log 2>&1 || exit $?
done
python3 scripts/pmc_sum.py $OUT > $OUT/summary.txt 2>&1
find $OUT -name "*.csv" -size +4M -delete
