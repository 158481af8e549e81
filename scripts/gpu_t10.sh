#!/bin/bash
# stream writer / encode+commit: their GPU tests, then the default bench line's copy-inclusive legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/t10
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_engine.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['frac']); print(json.dumps(d.get('copy_inclusive_encode_commit'))); print(json.dumps(d.get('copy_inclusive', {}).get('value')))"
