#!/bin/bash
# Quick GPU pass: kernel microbench (quick), parity tests, short bench.  Outputs in gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/kbench 1024 r q > gpurun_out/kbench.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-sample 16 --copy-objects 64 > gpurun_out/bench1.log 2>&1 || exit $?
exit $rc
