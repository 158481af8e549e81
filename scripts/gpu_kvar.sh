#!/bin/bash
# Encode-kernel variant sweep (kbench builds with different -D knobs) + GPU parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > gpurun_out/kvar.log
for b in scripts/kbench_*; do
  echo "== $b" >> gpurun_out/kvar.log
  timeout -k 10 120 ./$b 1024 >> gpurun_out/kvar.log 2>&1 || exit $?
done
exit $rc
