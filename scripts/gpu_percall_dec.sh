#!/bin/bash
# per-call decode: pageable slices gathered into pinned staging (base) -- parity first -- and the
# decode kernel with loads issued at the step's start (early) instead of late, for small calls
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/percall_dec
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -k "decode or Decode" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
for v in base early base early; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode percall --cpu-sample 0 > $O/p_${v}_$i.json 2> $O/p_${v}_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/p_${v}_$i.json')); c=d['calls']; print('$v', {k: {n: v2['ms_per_call'] for n, v2 in r.items()} for k, r in c.items()}, d['outputs_verified'])"
  i=$((i+1))
done
