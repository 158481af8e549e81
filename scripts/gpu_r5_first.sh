#!/bin/bash
# round-5 first GPU pass: the decode store tests (per-stream reader events), then the bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5a
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode_store.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5a/pytest_store.log 2>&1; rc=$?
tail -3 gpurun_out/r5a/pytest_store.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_lines.sh r5a
