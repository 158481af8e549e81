#!/bin/bash
# round-4 GPU call: per-call, random-pattern decode (1024 / 2048 objects), recover, repair, stream with
# 32 hash threads, then the encode kernel's rocprof stats + PMC traffic (profile_modes.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4c
mkdir -p $O
B="python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0"
timeout -k 10 400 python -u bench.py --mode percall > $O/percall.json 2> $O/percall.err && cat $O/percall.json &&
timeout -k 10 300 $B --mode decode --pattern random > $O/decode_random.json 2> $O/decode_random.err && cat $O/decode_random.json &&
timeout -k 10 400 $B --mode decode --pattern random --objects 2048 > $O/decode_random_2048.json 2> $O/decode_random_2048.err && cat $O/decode_random_2048.json &&
timeout -k 10 300 $B --mode recover > $O/recover.json 2> $O/recover.err && cat $O/recover.json &&
timeout -k 10 300 $B --mode repair > $O/repair.json 2> $O/repair.err && cat $O/repair.json &&
timeout -k 10 400 python -u bench.py --mode stream --hash-threads 32 > $O/stream_t32.json 2> $O/stream_t32.err && cat $O/stream_t32.json &&
MODES="encode" bash scripts/profile_modes.sh > $O/prof.log 2>&1 && tail -20 $O/prof.log
