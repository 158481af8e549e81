#!/bin/bash
# interleaved encode A/B: every library's bench line, R rounds (box-to-box spread is ~10 %, so
# only same-call, interleaved numbers are compared).   R=2 bash scripts/gpu_enc_ab2.sh main orig
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/encab2
mkdir -p $OUT
for r in $(seq ${R:-2}); do
for v in "$@"; do
  lib=tape_amd/libtapeec.so; [ $v != main ] && lib=varlib/lib_$v.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --steps 30 --warmup 3 --cpu-sample 0 --copy-objects 0 ${BENCH_ARGS:-} > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('r$r $v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
done
