#!/bin/bash
# round-4 GPU call: does the 4 GiB commit window's slowdown follow host-hashed runs or growth?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4w
mkdir -p $O
for q in "device:2,auto:4,auto:4" "host:2,auto:4,auto:4" "auto:3,auto:4,auto:4" "host:8,auto:4"; do
  PRE=host SEQ=$q timeout -k 10 400 python3 -u scripts/commit_windows_probe.py > $O/p.log 2>&1 || exit 1
  echo "== $q"; grep "^{'hashing'" $O/p.log
done
