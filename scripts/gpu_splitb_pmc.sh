#!/bin/bash
# HBM traffic of the batch encode split (level-1 rows on 7 workgroups per stripe + level 2): does
# the L2 serve the second read of a row when the seven level-1 workgroups run side by side?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/splitb_pmc
mkdir -p $O
B="python3 bench.py --mode encode --steps 3 --warmup 1 --cpu-sample 0 --copy-objects 0 --sdk-chunks 0"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum"; do
  i=$((i+1))
  TEC_DEBUG_KNOBS=1 TEC_ENC_SPLIT_BATCH=1 timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- $B > $O/p$i.log 2>&1 || exit $?
done
python3 scripts/pmc_sum.py $O enc_dma > $O/summary.txt 2>&1; cat $O/summary.txt
find $O -name "*.csv" -size +4M -delete
