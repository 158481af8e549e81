#!/bin/bash
# round-4 GPU call: commit window slowdown with VMM-backed (TEC_VMM_BUFS=1) vs hipMalloc buffers
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4aa
mkdir -p $O
for vm in 0 1; do
  TEC_DEBUG_KNOBS=1 TEC_VMM_BUFS=$vm PRE=host SEQ=auto:3,auto:4,auto:4 timeout -k 10 400 python3 -u scripts/commit_windows_probe.py > $O/p$vm.log 2>&1 || exit 1
  echo "== vmm $vm"; grep "^{'hashing'" $O/p$vm.log
done
TEC_DEBUG_KNOBS=1 TEC_VMM_BUFS=1 timeout -k 10 400 python3 -u bench.py --cpu-sample 0 > $O/nocpu_vmm.json 2> $O/nocpu_vmm.err || exit 1
python3 -c "
import json; d=json.load(open('$O/nocpu_vmm.json')); x=d['copy_inclusive_encode_commit']; print('bench vmm', x['by_window'], d['copy_inclusive']['value'], d['value'], d['outputs_verified'], x['matches_device_resident'])"
