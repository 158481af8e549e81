#!/bin/bash
# Round GPU pass 2: repair / decode benches (configs 3, 4) with their kernel-trace stats, and the
# FETCH_SIZE / WRITE_SIZE passes (separate runs, per the pool rules) for roofline.traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
for m in repair decode commit recover; do
  timeout -k 10 400 python bench.py --mode $m > $OUT/bench_$m.json 2> $OUT/bench_$m.err || exit $?
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$m -o run -- \
      python3 bench.py --mode $m --steps 5 --warmup 2 > $OUT/trace_$m.log 2>&1 || exit $?
done
B="python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 --copy-objects 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1 || exit $?
# FETCH_SIZE / WRITE_SIZE calibration on kernels of known byte counts (MI355X_MICROARCH.md: only
# 16-B streaming reads are calibrated; ours are 4-B loads and 16-B unaligned stores):
# vmem_bench4 "ld W4 unaligned" reads 1024 x 4 MiB with the encode's dword loads; vmem_bench7
# writes 1024 x 20 x 715,048 B with the encode's row stores.
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o run -- ./scripts/vmem_bench4 1024 > $OUT/cal_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o run -- ./scripts/vmem_bench7 > $OUT/cal_write.log 2>&1 || exit $?
python3 scripts/round_summary.py $OUT > $OUT/summary.log 2>&1
find $OUT -name "*kernel_trace.csv" -size +2M -delete
find $OUT -name "*counter_collection.csv" -size +4M -delete
find $OUT -name "*.db" -delete
