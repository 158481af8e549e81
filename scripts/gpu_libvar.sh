#!/bin/bash
# Bench one mode against alternate builds of the library (varlib/lib_<name>.so, TAPE_EC_LIB).
#   MODE=decode bash scripts/gpu_libvar.sh a b c
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/libvar
for v in "$@"; do
  TAPE_EC_LIB=varlib/lib_$v.so timeout -k 10 300 python bench.py --mode ${MODE:-decode} --steps 5 --warmup 2 --cpu-sample 0 --copy-objects 0 > gpurun_out/libvar/$v.json 2> gpurun_out/libvar/$v.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/libvar/$v.json')); print('$v', d['value'], d['roofline']['avg_launch_ms'], d['outputs_verified'])"
done
