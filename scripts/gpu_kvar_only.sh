#!/bin/bash
# Encode-kernel variant sweep (kbench builds with different -D knobs), random input, each
# variant run twice in alternating order (box-to-box HBM speed differs by ~20%: compare
# variants only within one call).  KB_ARGS="r q" for quick mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/kvar.log
# warm-up (clocks / HBM training): one untimed pass of the first variant
first=$(ls scripts/kbench_* | head -1)
timeout -k 10 120 ./$first 1024 r q > /dev/null 2>&1 || exit $?
for pass in 1 2; do
  for b in scripts/kbench_*; do
    echo "== $b (pass $pass)" >> gpurun_out/kvar.log
    timeout -k 10 120 ./$b 1024 ${KB_ARGS:-r} >> gpurun_out/kvar.log 2>&1 || exit $?
  done
done
