#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/vmem_bench7 > gpurun_out/vb7.log 2>&1 || exit $?

