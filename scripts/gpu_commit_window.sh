#!/bin/bash
# The one-shot commit's 4 GiB-group slowdown (open): group sizes in sequences after a
# copy-inclusive encode, with hipMalloc and with VMM-backed buffers (TEC_VMM_BUFS), host time per
# group traced (TEC_COMMIT_TRACE)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/commit_window
mkdir -p $O
for q in "device:2,auto:4,auto:4" "host:2,auto:4,auto:4" "auto:3,auto:4,auto:4" "host:8,auto:4"; do
  PRE=host SEQ=$q timeout -k 10 400 python3 -u scripts/commit_windows_probe.py > $O/p.log 2>&1 || exit 1
  echo "== $q"; grep "^{'hashing'" $O/p.log
done
for vm in 0 1; do
  TEC_DEBUG_KNOBS=1 TEC_VMM_BUFS=$vm TEC_COMMIT_TRACE=1 PRE=host SEQ=auto:3,auto:4,auto:4 \
    timeout -k 10 400 python3 -u scripts/commit_windows_probe.py > $O/vmm$vm.log 2>&1 || exit 1
  echo "== vmm $vm"; grep -E "^\{'hashing'|host ms" $O/vmm$vm.log | tail -12
done
