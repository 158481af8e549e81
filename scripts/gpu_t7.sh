#!/bin/bash
# full GPU suite after the decode host rework, then decode (random / worst) and recover lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/t7
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in "decode --pattern random --decode-jit off" "decode --pattern worst --decode-jit off" "recover"; do
  f=$(echo $m | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --mode $m --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 > $OUT/bench_$f.json 2> $OUT/bench_$f.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/bench_$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])"
done
exit 0
