#!/bin/bash
# round-4 GPU call: which earlier phase slows the 4 GiB commit window (bench.py context)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4v
mkdir -p $O
for pre in host dev devhost; do
  PRE=$pre timeout -k 10 400 python3 -u scripts/commit_windows_probe.py > $O/probe_$pre.log 2>&1 || exit 1
  echo "== $pre"; grep "^{'hashing'" $O/probe_$pre.log
done
