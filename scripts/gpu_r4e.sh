#!/bin/bash
# round-4 GPU call: interleaved host leaf hashing (te_host_hash_lanes) -- stream tests, the SDK
# stream shape at the calibrated lane count and at 1 lane (A/B), with the CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -8 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --mode stream --stream-chunks 64 > $O/stream.json 2> $O/stream.err && cat $O/stream.json &&
TEC_DEBUG_KNOBS=1 TEC_HOST_HASH_LANES=1 timeout -k 10 400 python -u bench.py --mode stream --stream-chunks 64 --cpu-sample 0 > $O/stream_l1.json 2> $O/stream_l1.err && cat $O/stream_l1.json &&
TEC_DEBUG_KNOBS=1 TEC_HOST_HASH_LANES=4 timeout -k 10 400 python -u bench.py --mode stream --stream-chunks 64 --cpu-sample 0 > $O/stream_l4.json 2> $O/stream_l4.err && cat $O/stream_l4.json
