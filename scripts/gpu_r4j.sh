#!/bin/bash
# round-4 GPU call: hash placement vs buffer kind (pageable / te_host_alloc pinned) and the NUMA
# node the buffers land on; stream shape with blocking ticket waits
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4j
mkdir -p $O
cat /sys/devices/system/node/node*/cpulist > $O/node_cpus.txt 2>&1
for d in /sys/class/drm/card*/device; do echo "$d $(cat $d/numa_node 2>/dev/null)"; done > $O/gpu_numa.txt 2>&1
timeout -k 10 200 python -u scripts/hash_placement.py > $O/place_pageable.json 2>&1 && cat $O/place_pageable.json &&
BUF=pinned timeout -k 10 200 python -u scripts/hash_placement.py > $O/place_pinned.json 2>&1 && cat $O/place_pinned.json &&
timeout -k 10 300 python -u bench.py --mode stream --stream-chunks 64 --cpu-sample 0 > $O/stream.json 2> $O/stream.err && python3 -c "
import json; d=json.load(open('$O/stream.json')); c=d['config']
print(c['host_hash_GBps_all_threads'], {k:(v['GiBps'],v['chunk_latency_ms_p50_p90']) for k,v in d['legs'].items()})"
