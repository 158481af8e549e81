#!/bin/bash
# line-exact systematic stores (TEC_DMA_SYSLX): parity suites, then interleaved A/B against the
# r05 kernel without them (e_nolx)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py tests/test_golden.py tests/test_gpu_extremes.py tests/test_gpu_repair_sets.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_enc_var.sh r5i base e_nolx base e_nolx base e_nolx
