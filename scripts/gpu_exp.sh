#!/bin/bash
# decode bench under environment variants: scripts/gpu_exp.sh "VAR=1 VAR2=3" "VAR=2" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/exp.txt
for v in "" "$@"; do
  env $v timeout -k 10 200 python bench.py --mode ${MODE:-decode} --steps 5 --warmup 2 --cpu-sample 0 --copy-objects 0 > gpurun_out/exp_one.json 2> gpurun_out/exp_one.err || exit $?
  echo "[$v] $(python3 -c "import json;d=json.load(open('gpurun_out/exp_one.json'));print(d['value'], d['roofline']['avg_launch_ms'])")" >> gpurun_out/exp.txt
done
