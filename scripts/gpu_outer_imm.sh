#!/bin/bash
# OuterCoder matrix kernel: immediate-offset table reads (base) against the SGPR-base addressing
# (old: TEC_RS16_MAT_IMM=0) -- parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/outer_imm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_outer.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_outer_var.sh outer_imm base old base old base old
