#!/bin/bash
# repair folded-kernel register budget A/B + one-down line after the host-side pattern cache
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t5
for u in 0 1; do
  for v in base wpe4 base wpe4; do
    TAPE_EC_LIB=varlib/lib_$v.so timeout -k 10 300 python bench.py --mode repair --unavailable $u --steps 20 --warmup 5 --cpu-sample 0 --copy-objects 0 > gpurun_out/t5/$v$u.json 2> gpurun_out/t5/$v$u.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/t5/$v$u.json')); print('$v u=$u', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])"
  done
done
