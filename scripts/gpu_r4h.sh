#!/bin/bash
# round-4 box call (host CPU only): leaf-hash throughput vs thread placement and lane count
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4h
mkdir -p $O
lscpu > $O/lscpu.txt 2>&1; numactl -H > $O/numa.txt 2>&1; cat /sys/fs/cgroup/cpu.max > $O/cpu_max.txt 2>&1
timeout -k 10 200 python -u scripts/hash_placement.py > $O/place16.json 2>&1 && cat $O/place16.json &&
TEC_DEBUG_KNOBS=1 TEC_HOST_HASH_LANES=1 timeout -k 10 200 python -u scripts/hash_placement.py > $O/place16_l1.json 2>&1 && cat $O/place16_l1.json &&
THREADS=8 timeout -k 10 200 python -u scripts/hash_placement.py > $O/place8.json 2>&1 && cat $O/place8.json
bash scripts/gpu_r4i.sh
