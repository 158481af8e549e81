#!/bin/bash
# PMC comparison of the DMA and stage encode kernels (kbench quick mode), one counter group per pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmccmp
mkdir -p $OUT
i=0
for grp in "$@"; do
  i=$((i+1))
  for k in dma stage; do
    arg=""; [ $k == stage ] && arg=s
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/$k$i -o run -- ./scripts/kbench 1024 r q $arg > $OUT/$k$i.log 2>&1 || exit $?
  done
done
for k in dma stage; do echo "== $k"; python3 scripts/pmc_sum.py $OUT "" | grep -i "$([ $k == dma ] && echo enc_dma || echo enc_stage)"; done > $OUT/summary.txt 2>&1
find $OUT -name "*.csv" -size +4M -delete
