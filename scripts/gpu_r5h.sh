#!/bin/bash
# (1) the default line's SDK-shape leg with whole-object D2H (no row pieces) in the slow state;
# (2) decode load-policy variants
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5h
mkdir -p $O
TEC_DEBUG_KNOBS=1 TEC_D2H_PIECE=0 timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > $O/default_nopiece.json 2> $O/default_nopiece.err && python3 -c "import json; d=json.load(open('$O/default_nopiece.json')); print('nopiece', d['copy_inclusive_encode_commit']['by_window'], d['stream_sdk_shape']['value'], d['stream_sdk_shape']['chunk_latency_ms_p50_p90'])" || exit $?
timeout -k 10 300 python -u bench.py --mode stream --stream-chunks 16 --cpu-sample 0 > $O/stream16.json 2> $O/stream16.err && python3 -c "import json; d=json.load(open('$O/stream16.json')); print('fresh stream16', d['legs'])" || exit $?
bash scripts/gpu_dec_var.sh r5h base dpnt donnt dboth base dpnt donnt dboth
