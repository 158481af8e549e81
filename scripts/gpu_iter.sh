#!/bin/bash
# Quick kernel iteration: DMA-vs-stage output check, encode microbench, then the GPU parity suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/iter
timeout -k 10 120 ./scripts/kbench 64 r c > gpurun_out/iter/check.log 2>&1; rc=$?; cat gpurun_out/iter/check.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 ./scripts/kbench 1024 r q > gpurun_out/iter/kbench.log 2>&1 || exit $?
timeout -k 10 120 ./scripts/kbench 1024 r q s >> gpurun_out/iter/kbench.log 2>&1 || exit $?
cat gpurun_out/iter/kbench.log
[ "$1" == "notest" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/iter/pytest_gpu.log; exit $rc
