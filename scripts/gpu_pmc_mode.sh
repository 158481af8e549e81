#!/bin/bash
# PMC passes over one bench mode (one counter group per pass, each a separate run under its own
# limit: pool rules, no trace domain with --pmc).  Summary -> gpurun_out/pmcm/<mode>/summary.txt.
#   MODE=decode PAT=tec_dec_fixed BENCH_ARGS="--objects 1024" bash scripts/gpu_pmc_mode.sh [groups...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
M=${MODE:-encode}
OUT=gpurun_out/pmcm/$M
mkdir -p $OUT
B="python3 bench.py --mode $M --steps 3 --warmup 1 --cpu-sample 0 --copy-objects 0 $BENCH_ARGS"
if [ $# -eq 0 ]; then
  set -- "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
    "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL"
fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $B > $OUT/p$i.log 2>&1 || exit $?
done
python3 scripts/pmc_sum.py $OUT ${PAT:-tec} > $OUT/summary.txt 2>&1
find $OUT -name "*.csv" -size +4M -delete
find $OUT -name "*.db" -delete
cat $OUT/summary.txt
exit 0
