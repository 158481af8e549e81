#!/bin/bash
# PMC passes over one bench mode; per-kernel averages for kernels matching <filter>.
#   scripts/gpu_pmc.sh <mode> <kernel-name-filter>   -> gpurun_out/pmc_<mode>/summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
m=$1; f=$2
OUT=gpurun_out/pmc_$m
rm -rf $OUT; mkdir -p $OUT
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT" \
         "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --mode $m --steps 2 --warmup 1 --cpu-sample 0 --copy-objects 0 > $OUT/p$i.log 2>&1 || exit $?
done
python3 - "$OUT" "$f" <<'PY' > $OUT/summary.txt
import csv, glob, sys
out, f = sys.argv[1], sys.argv[2]
agg = {}
for cf in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(cf)):
        if f not in r.get("Kernel_Name", ""): continue
        a = agg.setdefault(r["Counter_Name"], [0.0, 0]); a[0] += float(r["Counter_Value"]); a[1] += 1
for c, (v, n) in sorted(agg.items()):
    print(f"{c:32s} {v / n:18.1f}   (n={n})")
PY
find $OUT -name "*.csv" -size +1M -delete
