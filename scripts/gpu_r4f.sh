#!/bin/bash
# round-4 GPU call: row-piece D2H with hashing as the pieces land -- stream tests, then the SDK
# stream shape with pieces (default), 2-D vs per-row piece copies, and pieces off (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -8 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --mode stream --stream-chunks 64 --cpu-sample 0 > $O/stream.json 2> $O/stream.err && cat $O/stream.json &&
TEC_DEBUG_KNOBS=1 TEC_D2H_ROWS=1 timeout -k 10 400 python -u bench.py --mode stream --stream-chunks 64 --cpu-sample 0 > $O/stream_rows.json 2> $O/stream_rows.err && cat $O/stream_rows.json &&
TEC_DEBUG_KNOBS=1 TEC_D2H_PIECE=0 timeout -k 10 400 python -u bench.py --mode stream --stream-chunks 64 --cpu-sample 0 > $O/stream_nopiece.json 2> $O/stream_nopiece.err && cat $O/stream_nopiece.json &&
TEC_DEBUG_KNOBS=1 TEC_D2H_PIECE=4194304 timeout -k 10 400 python -u bench.py --mode stream --stream-chunks 64 --cpu-sample 0 > $O/stream_p4m.json 2> $O/stream_p4m.err && cat $O/stream_p4m.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 bench.py --mode stream --stream-chunks 24 --cpu-sample 0 > $O/trace.log 2>&1
