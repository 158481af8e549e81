#!/bin/bash
# OuterCoder matrix kernel under the max-memory-clause and iterative-ILP scheduling strategies
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sched_ab3
mkdir -p $O
for v in o_mem o_iilp; do
  TAPE_EC_LIB=varlib/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_outer.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?; echo "$v $(tail -1 $O/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_outer_var.sh sched_ab3/outer base o_mem o_iilp base o_mem o_iilp
