#!/bin/bash
# decode random (host path after the store), then traffic profiles of repair (one down) and recover
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/t8
mkdir -p $OUT
for m in "decode --pattern random --decode-jit off"; do
  timeout -k 10 300 python bench.py --mode $m --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 > $OUT/dec_random.json 2> $OUT/dec_random.err || exit $?
  python3 -c "import json; d=json.load(open('$OUT/dec_random.json')); print('random', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])"
done
MODES="repair recover" bash scripts/profile_modes.sh > $OUT/prof.log 2>&1 || exit $?
BENCH_ARGS="--unavailable 1" MODES="repair" bash -c 'OUT=1; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/prof_u1; cp -r gpurun_out/prof/repair gpurun_out/prof_u1/repair0 2>/dev/null; true'
tail -40 $OUT/prof.log
exit 0
