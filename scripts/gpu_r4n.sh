#!/bin/bash
# round-4 GPU call: OuterCoder decode, two elements per thread -- outer tests, bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_outer.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --mode outer --cpu-sample 0 > $O/outer.json 2> $O/outer.err && python3 -c "
import json; d=json.load(open('$O/outer.json')); print('enc', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac']); x=d['decode']; print('dec', x['value'], x['roofline']['avg_launch_ms'], x['roofline']['frac'], x['outputs_verified'])"
