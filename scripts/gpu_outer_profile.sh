#!/bin/bash
# OuterCoder kernels -- bench line, kernel stats, SQ instruction / wait counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/outer_profile
mkdir -p $O
B="python3 bench.py --mode outer --steps 3 --warmup 1 --cpu-sample 0"
timeout -k 10 300 python3 -u bench.py --mode outer --cpu-sample 0 > $O/outer.json 2> $O/outer.err && cat $O/outer.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/sq -o run -- $B > $O/sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/sq2 -o run -- $B > $O/sq2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1
python3 scripts/pmc_sum.py $O/sq rs16 > $O/pmc_summary.txt 2>&1; python3 scripts/pmc_sum.py $O/sq2 rs16 >> $O/pmc_summary.txt 2>&1; python3 scripts/pmc_sum.py $O/fetch rs16 >> $O/pmc_summary.txt 2>&1
find $O -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O -name "*.csv" -size +2M -delete; find $O -name "*.db" -delete
cat $O/pmc_summary.txt; cat $O/kernel_stats.csv | cut -c1-200
