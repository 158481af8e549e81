#!/bin/bash
# full GPU suite on the current build, then the per-call spin/sync A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_percall_ab.sh
