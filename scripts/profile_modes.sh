#!/bin/bash
# Per bench mode: rocprofv3 kernel-trace stats, then PMC passes (FETCH_SIZE; WRITE_SIZE; the L2's
# memory-side request counters), each a separate run under its own limit (pool rules: never
# --pmc with a trace domain; at most 4 TCC counters per pass).  Summaries -> gpurun_out/prof/.
#   MODES="encode repair decode decode:random recover"  BENCH_ARGS="--objects 1024"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
rocprofv3 -L 2>/dev/null | grep -o "TCC_EA0_[A-Z0-9_]*" | sort -u > $OUT/tcc_ea_counters.txt || true
for m in ${MODES:-encode}; do
  mode=${m%%:*}; pat=""; [ "$m" != "$mode" ] && pat="--pattern ${m#*:}"
  B="python3 bench.py --mode $mode $pat --steps 3 --warmup 1 --cpu-sample 0 --copy-objects 0 $BENCH_ARGS"
  D=$OUT/${m/:/_}
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $B > $D/trace.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- $B > $D/fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- $B > $D/write.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $D/req -o run -- $B > $D/req.log 2>&1 || exit $?
  python3 scripts/pmc_sum.py $D tec:: > $D/pmc_summary.txt 2>&1
  find $D -name "*kernel_stats.csv" -exec cp {} $D/kernel_stats.csv \;
  find $D -name "*.csv" -size +2M -delete
  find $D -name "*.db" -delete
  cat $D/pmc_summary.txt
done
exit 0
