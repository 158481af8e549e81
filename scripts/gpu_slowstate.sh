#!/bin/bash
# The copy-inclusive "slow state" (VERDICT r04 weak #5): the SDK-shape stream in a fresh process,
# the default line with more hardware queues per process, and a kernel trace of the default line
# (are the slow windows' D2H copies blit kernels?).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --mode stream --stream-chunks 16 --cpu-sample 0 > $O/stream16.json 2> $O/stream16.err && python3 -c "import json; d=json.load(open('$O/stream16.json')); print('fresh stream16', d['legs']['auto_pinned'])" &&
GPU_MAX_HW_QUEUES=16 timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > $O/default_hwq16.json 2> $O/default_hwq16.err && python3 -c "import json; d=json.load(open('$O/default_hwq16.json')); print('hwq16', d['copy_inclusive_encode_commit']['by_window'], d['stream_sdk_shape']['value'], d['stream_sdk_shape']['chunk_latency_ms_p50_p90'])" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o trace -- python3 -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > $O/default_traced.json 2> $O/default_traced.err && python3 -c "import json; d=json.load(open('$O/default_traced.json')); print('traced', d['copy_inclusive_encode_commit']['by_window'], d['stream_sdk_shape']['value'])"
