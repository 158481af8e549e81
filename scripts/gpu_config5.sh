#!/bin/bash
# BASELINE config 5 at N = 1 on one box: the 64 GiB stream (16,384 x 4 MiB) resident in HBM,
# encoded in device batches of 2,048, plus the copy-inclusive leg (every rank's share from a pinned
# host ring); the 8-GPU line is the driver's (python bench.py --gpus 8 --workload config5)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/config5
mkdir -p $O
timeout -k 10 900 python -u bench.py --workload config5 --steps 3 --warmup 1 > $O/config5_n1.json 2> $O/config5_n1.err && cat $O/config5_n1.json
