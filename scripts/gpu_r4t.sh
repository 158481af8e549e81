#!/bin/bash
# round-4 GPU call: the default line with the one-shot commit's per-group hashing choice traced
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4t
mkdir -p $O
TEC_DEBUG_KNOBS=1 TEC_COMMIT_TRACE=1 timeout -k 10 400 python3 -u bench.py --cpu-sample 0 > $O/nocpu.json 2> $O/nocpu.err || exit 1
grep -c "commit group" $O/nocpu.err; grep "commit group" $O/nocpu.err | sort | uniq -c | sort -rn | head -20
python3 -c "
import json; d=json.load(open('$O/nocpu.json')); print(d['copy_inclusive_encode_commit']['by_window'])"
