#!/bin/bash
# PMC-only passes (8 SQ counters each) for the encode bench; summaries in gpurun_out/prof2.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof2
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 ${BENCH_ARGS}"
i=0
for C in "SQ_LEVEL_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" \
         "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/p$i -o run -- $B > $OUT/p$i.log 2>&1 || exit $?
done
python3 - <<'PY' > $OUT/summary.txt
import csv, glob, os
agg = {}
for cf in glob.glob("gpurun_out/prof2/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(cf)):
        k = r.get("Kernel_Name", "")
        if "tec::" not in k or "meta" in k: continue
        key = (k.split("(")[0][-40:], r["Counter_Name"])
        a = agg.setdefault(key, [0.0, 0]); a[0] += float(r["Counter_Value"]); a[1] += 1
for (k, c), (v, n) in sorted(agg.items()):
    print(f"{k:40s} {c:32s} {v / n:16.1f}")
PY
find $OUT -name "*.csv" -delete
