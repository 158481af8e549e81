#!/bin/bash
# rocprofv3 --kernel-trace --stats of the bench modes' own commands (the roofline's kernel average
# must agree with the line's in-run HIP-event figure): decode random / worst, recover, repair
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/mode_stats
mkdir -p $O
for spec in decode:random decode:worst recover repair; do
  m=${spec%%:*}; pat=${spec#*:}; [ "$pat" == "$spec" ] && pat=worst
  d=$O/${spec/:/_}
  B="python3 bench.py --mode $m --pattern $pat --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 --sdk-chunks 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- $B > $d.json 2> $d.log || exit $?
  cp $(find $d -name "*kernel_stats.csv" | head -1) $d.kernel_stats.csv
  python3 - "$d.kernel_stats.csv" "$d.json" "$spec" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
print(sys.argv[3], 'line avg_launch_ms', d['roofline'].get('avg_launch_ms'), '| rocprof top:',
      [(r['Name'][:50], r['Calls'], round(float(r['AverageNs']) / 1e6, 4)) for r in rows[:2]])
PY
done
