#!/bin/bash
# outer-coder register kernel A/B (parity first), then the SDK-leg slow-state probe
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_outer_ab.sh || exit $?
mkdir -p gpurun_out/r5k
timeout -k 10 600 python -u scripts/sdk_state_probe.py > gpurun_out/r5k/sdk_probe.log 2>&1; rc=$?; cat gpurun_out/r5k/sdk_probe.log | grep -v Warning; exit $rc
