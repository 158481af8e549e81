#!/bin/bash
# encode parity (main library) then the encode bench line for the main library and each variant
#   bash scripts/gpu_enc_ab.sh slp3 orig
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/encab
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_golden.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in main "$@"; do
  lib=tape_amd/libtapeec.so; [ $v != main ] && lib=varlib/lib_$v.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 --copy-objects 0 > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
