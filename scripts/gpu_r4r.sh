#!/bin/bash
# round-4 GPU call: one-shot encode + commit per group size and hashing side, in several orders
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 400 python3 -u scripts/commit_windows_probe.py > $O/probe.log 2>&1; rc=$?; cat $O/probe.log | grep -v amdgpu.ids; exit $rc
