#!/bin/bash
# rocprofv3 kernel trace + PMC passes for the encode bench (separate passes per the pool rules).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 ${BENCH_ARGS}"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq -o run -- $B > $OUT/pmc_sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq2 -o run -- $B > $OUT/pmc_sq2.log 2>&1 || exit $?

python3 scripts/prof_summary.py $OUT > $OUT/summary.txt 2>&1
find $OUT -name "*.csv" -size +2M -delete
find $OUT -name "*.db" -delete
