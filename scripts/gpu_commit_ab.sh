#!/bin/bash
# SHA-256 leaf kernel: Ch / Maj as 2-cycle v_bitop3 (base) against the backend's v_bfi_b32 (old);
# commitment parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/commit_ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread -k "commit or leaf or root or proof or merkle or stream" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
i=0
for v in base old base old; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode commit --steps 5 --warmup 2 --cpu-sample 0 > $O/c_${v}_$i.json 2> $O/c_${v}_$i.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/c_${v}_$i.json') if l.startswith('{')][-1]); print('$v', d['value'], d['unit'], d['ms_per_step'], d.get('outputs_verified'))"
  i=$((i+1))
done
