#!/bin/bash
# round-4 first GPU call: skeleton4, row-piece encode parity, smoke, encode bench (row-piece vs LDS-DMA kernel)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 120 ./scripts/enc_skeleton4 > $O/sk4.txt 2>&1 && cat $O/sk4.txt &&
TEC_DEBUG_KNOBS=1 TEC_ENCODE_KERNEL=r10 timeout -k 10 400 python -u -m pytest tests/test_gpu_encode_r10.py -x -v --timeout 300 --timeout-method thread > $O/pytest_r10.log 2>&1; rc=$?; tail -15 $O/pytest_r10.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" &&
TEC_DEBUG_KNOBS=1 TEC_ENCODE_KERNEL=r10 timeout -k 10 300 python bench.py --cpu-sample 0 --copy-objects 0 > $O/bench_r10.json 2> $O/bench_r10.err && cat $O/bench_r10.json &&
TEC_DEBUG_KNOBS=1 TEC_ENCODE_KERNEL=dma timeout -k 10 300 python bench.py --cpu-sample 0 --copy-objects 0 > $O/bench_dma.json 2> $O/bench_dma.err && cat $O/bench_dma.json
