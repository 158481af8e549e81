#!/bin/bash
# encode DMA-policy / store-policy variants A/B, then the per-call path traced (kernels + copies)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_enc_var.sh r5d base e_rp1 e_rp2 e_st0 base e_rp1 e_rp2 e_st0 || exit $?
O=gpurun_out/r5d
timeout -k 10 300 python -u bench.py --mode percall --cpu-sample 0 > $O/percall.json 2> $O/percall.err && cat $O/percall.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_percall -o percall -- python3 -u bench.py --mode percall --cpu-sample 0 > $O/percall_traced.json 2> $O/percall_traced.err
