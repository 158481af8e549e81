#!/bin/bash
# per-call decode with one-wave workgroups (small calls) against the batch geometry; parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/dec_small
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_store.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in small batch small batch; do
  knob=""; [ $v == batch ] && knob="TEC_DEBUG_KNOBS=1 TEC_DEC_SMALL=0"
  env $knob timeout -k 10 300 python bench.py --mode percall --cpu-sample 0 > $O/p_$v.json 2> $O/p_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/p_$v.json')); c=d['calls']; print('$v', {k: {n: v2['ms_per_call'] for n, v2 in r.items()} for k, r in c.items() if k.startswith('4')}, d['outputs_verified'])"
done
bash scripts/gpu_enc_splitb.sh
