#!/bin/bash
# Ablation timings of the DMA encode kernel (timing builds; outputs not checked).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
for a in "$@"; do
  echo -n "ablate $a: " >> gpurun_out/abl/abl.log
  timeout -k 10 60 ./scripts/kbench_a$a 1024 r q >> gpurun_out/abl/abl.log 2>&1 || exit $?
done
cat gpurun_out/abl/abl.log
