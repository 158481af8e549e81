#!/bin/bash
# decode table kernel: MDS loop with known inputs outside (j4), the same at 5 waves per SIMD with
# its spills (j5), the shipped loop at 5 waves (w5) -- parity of j5 first, then random / recover
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/dec_jouter
mkdir -p $O
TAPE_EC_LIB=varlib/lib_j5.so timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_store.py tests/test_gpu_parity.py tests/test_gpu_repair_sets.py -x -q --timeout 120 --timeout-method thread -k "decode or recover" > $O/pytest_j5.log 2>&1; rc=$?; tail -1 $O/pytest_j5.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_dec_var.sh dec_jouter base j5 j4 w5 base j5
