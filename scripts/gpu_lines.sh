#!/bin/bash
# The bench lines with their CPU baselines: default encode (box ceiling, copy-inclusive, SDK-shape
# stream leg), repair, worst and random decode, recover.  Usage: scripts/gpu_lines.sh <outdir-name>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-lines}
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err && cat $O/bench_default.json &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --mode repair > $O/bench_repair.json 2> $O/bench_repair.err && cat $O/bench_repair.json &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --mode decode --pattern random > $O/bench_decode_random.json 2> $O/bench_decode_random.err && cat $O/bench_decode_random.json &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --mode decode > $O/bench_decode_worst.json 2> $O/bench_decode_worst.err && cat $O/bench_decode_worst.json &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --mode recover > $O/bench_recover.json 2> $O/bench_recover.err && cat $O/bench_recover.json
