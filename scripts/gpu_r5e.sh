#!/bin/bash
# encode parity with the per-row DMA policy default; DMA / store policy variants; the commit
# slow-state probe with CPU accounting; per-call lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $O/pytest_enc.log 2>&1; rc=$?; tail -2 $O/pytest_enc.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_enc_var.sh r5e base e_rp0 e_st0 e_l2d e_sc0nt e_sc1nt e_sc01nt base e_rp0 e_st0 e_l2d e_sc0nt e_sc1nt e_sc01nt || exit $?
PRE="dev host" timeout -k 10 400 python -u scripts/commit_windows_probe.py > $O/commit_probe.txt 2>&1; rc=$?; grep -v "^{\"probe" $O/commit_probe.txt | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode percall --cpu-sample 0 > $O/percall.json 2> $O/percall.err && python3 -c "import json; d=json.load(open('$O/percall.json')); print({k: {c: v['ms_per_call'] for c, v in r.items()} for k, r in d['calls'].items()})"
