#!/bin/bash
# round-4 GPU call: the default line's 4 GiB commit window with and without the CPU baseline leg
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 400 python3 -u bench.py --cpu-sample 0 > $O/nocpu.json 2> $O/nocpu.err || exit 1
timeout -k 10 600 python3 -u bench.py > $O/default.json 2> $O/default.err || exit 1
python3 -c "
import json
for f in ('nocpu','default'):
    d=json.load(open('$O/'+f+'.json')); x=d['copy_inclusive_encode_commit']; print(f, x['by_window'], d['value'])"
