#!/bin/bash
# Per bench mode: a kernel-trace --stats run, then PMC passes (FETCH_SIZE; WRITE_SIZE; the L2's
# memory-side read requests by size), each pass a separate run under its own limit (pool rules: no
# trace domain with --pmc; at most 4 TCC counters per pass).  scripts/traffic.py turns the counter
# CSVs into profiles/traffic.json.
#   bash scripts/profile_modes.sh encode decode:random recover repair
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_modes
for spec in "$@"; do
  m=${spec%%:*}; pat=${spec#*:}; [ "$pat" == "$spec" ] && pat=worst
  d=$OUT/${spec/:/_}
  mkdir -p $d
  B="python3 bench.py --mode $m --pattern $pat --steps 3 --warmup 1 --cpu-sample 0 --copy-objects 0 --sdk-chunks 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/stats -o run -- $B > $d/stats.log 2>&1 || exit $?
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $d/p$i -o run -- $B > $d/p$i.log 2>&1 || exit $?
  done
  find $d -name "*.db" -delete
  echo "profiled $spec"
done
