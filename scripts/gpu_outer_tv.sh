#!/bin/bash
# OuterCoder matrix kernel: VALU tail row (rows = 8 h + 1) -- parity, then encode / decode kernel
# time against the table-only build (notv) and the interleaved-tail build (tv0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/outer_tv
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_outer.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
TAPE_EC_LIB=varlib/lib_tv0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_outer.py -x -q --timeout 120 --timeout-method thread > $O/pytest_tv0.log 2>&1; rc=$?; tail -1 $O/pytest_tv0.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_outer_var.sh outer_tv base notv tv0 base notv tv0
