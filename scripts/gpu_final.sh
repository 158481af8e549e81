#!/bin/bash
# Closing check on one box: whole GPU suite, smoke, the default line, BASELINE config 5 at N = 1,
# and the repair / random-decode / recover / outer / per-call lines.
#   usage: scripts/gpu_final.sh <outdir-name>   (GPU_SUITE=0 skips the test suite)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-final}
mkdir -p $O
if [ "${GPU_SUITE:-1}" == "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit $?
fi
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err && echo default ok &&
timeout -k 10 900 python -u bench.py --workload config5 --steps 3 --warmup 1 > $O/bench_config5_n1.json 2> $O/bench_config5_n1.err && echo config5 ok &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --copy-objects 0 --mode repair > $O/bench_repair.json 2> $O/bench_repair.err && echo repair ok &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --copy-objects 0 --mode decode --pattern random > $O/bench_decode_random.json 2> $O/bench_decode_random.err && echo random ok &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --copy-objects 0 --mode decode > $O/bench_decode_worst.json 2> $O/bench_decode_worst.err && echo worst ok &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --copy-objects 0 --mode recover > $O/bench_recover.json 2> $O/bench_recover.err && echo recover ok &&
timeout -k 10 300 python3 -u bench.py --mode outer > $O/bench_outer.json 2> $O/bench_outer.err && echo outer ok &&
timeout -k 10 300 python3 -u bench.py --mode percall > $O/bench_percall.json 2> $O/bench_percall.err && echo percall ok
