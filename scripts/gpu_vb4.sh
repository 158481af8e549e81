#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/vmem_bench5 1024 > gpurun_out/vb5.log 2>&1 || exit $?

