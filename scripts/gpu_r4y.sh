#!/bin/bash
# round-4 GPU call: host-side time per commit group in the slow 4 GiB case (TEC_COMMIT_TRACE)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4y
mkdir -p $O
for q in "auto:3,auto:4,auto:4" "auto:4,auto:4"; do
  TEC_DEBUG_KNOBS=1 TEC_COMMIT_TRACE=1 PRE=host SEQ=$q timeout -k 10 400 python3 -u scripts/commit_windows_probe.py > $O/p.log 2>&1 || exit 1
  echo "== $q"; grep "^{'hashing'" $O/p.log
  grep -E "commit group|host ms" $O/p.log | tail -24
done
