#!/bin/bash
# stream-shape latency probes -- submit-call time, the pool's aggregate hash rate,
# row-piece size and lane count A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/stream_probe
mkdir -p $O
S="python -u bench.py --mode stream --stream-chunks 64 --cpu-sample 0"
timeout -k 10 300 $S > $O/stream.json 2> $O/stream.err && cat $O/stream.json &&
TEC_DEBUG_KNOBS=1 TEC_D2H_PIECE=4194304 timeout -k 10 300 $S > $O/p4m.json 2> $O/p4m.err &&
TEC_DEBUG_KNOBS=1 TEC_D2H_PIECE=4194304 TEC_HOST_HASH_LANES=2 timeout -k 10 300 $S > $O/p4m_l2.json 2> $O/p4m_l2.err &&
TEC_DEBUG_KNOBS=1 TEC_D2H_PIECE=4194304 TEC_HOST_HASH_LANES=1 timeout -k 10 300 $S > $O/p4m_l1.json 2> $O/p4m_l1.err &&
TEC_DEBUG_KNOBS=1 TEC_D2H_PIECE=4194304 timeout -k 10 300 $S --hash-threads 32 > $O/p4m_t32.json 2> $O/p4m_t32.err &&
TEC_DEBUG_KNOBS=1 TEC_D2H_PIECE=0 timeout -k 10 300 $S > $O/nopiece.json 2> $O/nopiece.err
