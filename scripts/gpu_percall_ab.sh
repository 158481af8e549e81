#!/bin/bash
# per-call entry points: spin-wait on an event (default) against hipStreamSynchronize
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/percall_ab
mkdir -p $O
for v in spin sync spin sync; do
  knob=""; [ $v == sync ] && knob="TEC_DEBUG_KNOBS=1 TEC_PERCALL_SPIN=0"
  env $knob timeout -k 10 300 python bench.py --mode percall --cpu-sample 0 > $O/p_$v.json 2> $O/p_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/p_$v.json')); c=d['calls']; print('$v', {k: {n: v2['ms_per_call'] for n, v2 in r.items()} for k, r in c.items() if k.startswith('4MiB')}, d['outputs_verified'])"
done
