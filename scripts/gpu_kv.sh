#!/bin/bash
# Encode-kernel variants: scripts/kbench* binaries given as arguments, quick mode, one line each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kv.log
for b in "$@"; do
  echo "== $b" >> gpurun_out/kv.log
  timeout -k 10 120 ./$b 1024 r q >> gpurun_out/kv.log 2>&1 || exit $?
done
