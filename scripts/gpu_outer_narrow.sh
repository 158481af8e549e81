#!/bin/bash
# OuterCoder matrix kernel: narrow tail-group entries (base: 2 B for one row, 4 B for two) against
# the 8-byte entries throughout (wide: TEC_RS16_MAT_NARROW=0) -- parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/outer_narrow
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_outer.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_outer_var.sh outer_narrow base wide base wide base wide
