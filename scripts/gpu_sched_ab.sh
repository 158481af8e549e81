#!/bin/bash
# backend scheduler strategies (-mllvm -amdgpu-sched-strategy=...) for the encode and decode
# kernels: parity of each build first, then interleaved timings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sched_ab
mkdir -p $O
for v in e_ilp e_mem; do
  TAPE_EC_LIB=varlib/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "encode or slicer" > $O/pytest_$v.log 2>&1; rc=$?; echo "$v $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in d_ilp d_mem d_iilp; do
  TAPE_EC_LIB=varlib/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_store.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "decode" > $O/pytest_$v.log 2>&1; rc=$?; echo "$v $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_enc_var.sh sched_ab/enc base e_ilp e_mem base e_ilp e_mem && bash scripts/gpu_dec_var.sh sched_ab/dec base d_ilp d_mem d_iilp base d_ilp d_mem d_iilp
