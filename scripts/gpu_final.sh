#!/bin/bash
# whole GPU suite (verbose, per-test limit), smoke, and the bench lines: default, stream shape, random decode, recover, outer
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && cat $O/smoke.log &&
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err && cat $O/bench_default.json &&
timeout -k 10 400 python -u bench.py --mode stream > $O/bench_stream.json 2> $O/bench_stream.err && cat $O/bench_stream.json &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 --mode decode --pattern random > $O/bench_decode_random.json 2> $O/bench_decode_random.err && cat $O/bench_decode_random.json &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 --mode recover > $O/bench_recover.json 2> $O/bench_recover.err && cat $O/bench_recover.json &&
timeout -k 10 300 python3 -u bench.py --mode outer --cpu-sample 0 > $O/bench_outer.json 2> $O/bench_outer.err && cat $O/bench_outer.json
