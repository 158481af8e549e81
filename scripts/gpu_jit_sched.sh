#!/bin/bash
# worst-case decode (13 erasures, hipRTC pattern kernels): default scheduling vs the backend's
# max-ILP strategy for the run-time compiled kernels (TEC_DEC_JIT_SCHED, measurement knob)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/jit_sched
mkdir -p $O
TEC_DEBUG_KNOBS=1 TEC_DEC_JIT_SCHED=max-ilp timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_jit.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "ilp $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
i=0
for v in base ilp base ilp base ilp; do
  knob=""; [ $v == ilp ] && knob="TEC_DEBUG_KNOBS=1 TEC_DEC_JIT_SCHED=max-ilp"
  env $knob timeout -k 10 400 python bench.py --mode decode --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 > $O/d_${v}_$i.json 2> $O/d_${v}_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/d_${v}_$i.json')); r=d['roofline']; print('$v worst', r['avg_launch_ms'], r['frac'], d['outputs_verified'])"
  i=$((i+1))
done
