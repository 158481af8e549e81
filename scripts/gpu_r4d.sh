#!/bin/bash
# round-4 GPU call: decode-store tests at the new cap, 2,048-object random decode, stream shape with
# per-chunk latency, and a rocprofv3 kernel + memory-copy trace of the stream shape
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode_store.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -8 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 --mode decode --pattern random --objects 2048 > $O/decode_random_2048.json 2> $O/decode_random_2048.err && cat $O/decode_random_2048.json &&
timeout -k 10 400 python -u bench.py --mode stream --stream-chunks 64 --cpu-sample 0 > $O/stream.json 2> $O/stream.err && cat $O/stream.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --mode stream --stream-chunks 24 --cpu-sample 0 > $O/trace.log 2>&1 &&
find $O/trace -name "*.csv" | head -20
