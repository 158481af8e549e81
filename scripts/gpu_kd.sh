#!/bin/bash
# encode kernel variants: scripts/gpu_kd.sh <binary suffix>...  -> gpurun_out/kd.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kd.txt
for v in "$@"; do
  echo "== $v" >> gpurun_out/kd.txt
  timeout -k 10 120 ./scripts/kbench_$v 1024 r q >> gpurun_out/kd.txt 2>&1 || exit $?
done
