#!/bin/bash
# GPU parity tests, then the repair (and optionally decode) bench lines.  Outputs in gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in "$@"; do
  timeout -k 10 300 python bench.py --mode $m --steps 5 --warmup 2 > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err || exit $?
done
