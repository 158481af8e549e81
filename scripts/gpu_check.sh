#!/bin/bash
# GPU parity suite (verbose, per-test timeout), then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/check/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/check/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/check/bench.json 2> gpurun_out/check/bench.err || exit $?
cat gpurun_out/check/bench.json
