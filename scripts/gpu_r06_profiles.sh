#!/bin/bash
# Round-6 profiles: rocprofv3 --kernel-trace --stats of the bench lines' own commands (encode
# default, random-pattern decode, recover, repair); for the class-kernel lines, whose kernels run
# side by side on forked streams, the per-call span (first class-kernel start to last end) from the
# kernel trace (scripts/class_span.py) is what must agree with the line's in-run device time; then
# the PMC traffic passes of decode:random and recover (scripts/profile_modes.sh).
#   usage: scripts/gpu_r06_profiles.sh <outdir-name>   (PMC=0 skips the counter passes; SPECS="mode[:pattern] ...")
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06_prof}
mkdir -p $O
for spec in ${SPECS:-encode decode:random recover repair}; do
  m=${spec%%:*}; pat=${spec#*:}; [ "$pat" == "$spec" ] && pat=worst
  d=$O/${spec/:/_}
  B="python3 bench.py --mode $m --pattern $pat --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 --sdk-chunks 0"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- $B > $d.json 2> $d.log || exit $?
  cp $(find $d -name "*kernel_stats.csv" | head -1) $d.kernel_stats.csv
  python3 scripts/class_span.py $(find $d -name "*kernel_trace.csv" | head -1) $d.json > $d.span.txt || exit $?
  find $d -name "*kernel_trace.csv" -delete
  cat $d.span.txt
done
if [ "${PMC:-1}" == "1" ]; then
  bash scripts/profile_modes.sh decode:random recover || exit $?
fi
