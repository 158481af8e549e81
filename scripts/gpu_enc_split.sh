#!/bin/bash
# per-call encode split into level-1 rows on seven workgroups + the level-2 chain: parity first
# (Slicer.encode is the per-call entry point), then per-call times split vs unsplit
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/enc_split
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in split nosplit split nosplit; do
  knob=""; [ $v == nosplit ] && knob="TEC_DEBUG_KNOBS=1 TEC_ENC_SPLIT=0"
  env $knob timeout -k 10 300 python bench.py --mode percall --cpu-sample 0 > $O/p_$v.json 2> $O/p_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/p_$v.json')); c=d['calls']; print('$v', {k: {n: v2['ms_per_call'] for n, v2 in r.items()} for k, r in c.items()}, d['outputs_verified'])"
done
