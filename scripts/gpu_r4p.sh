#!/bin/bash
# round-4 GPU call: OuterCoder decode step time vs steps (host enqueue rate)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4p
mkdir -p $O
for st in 3 10 20; do
  timeout -k 10 300 python3 -u bench.py --mode outer --cpu-sample 0 --steps $st > $O/outer_s$st.json 2> $O/outer_s$st.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/outer_s$st.json')); x=d['decode']; print('steps $st', x['ms_per_step'], x['roofline']['avg_launch_ms'], d['ms_per_step'])"
done
