#!/bin/bash
# Decode class kernels (decode_class.hip) against the table-driven kernel: the decode GPU tests,
# then random-pattern and worst-case (hipRTC kernels off) decode lines per variant, interleaved.
#   usage: scripts/gpu_dec_class.sh <outdir-name>
#   TESTS=0 skips the tests; ROUNDS (default 2); OBJECTS (default 1024); PERCALL=1 adds --mode percall
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dec_class}
mkdir -p $O
if [ "${TESTS:-1}" == "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "decode or parity or golden or extremes or percall or recover" > $O/pytest.log 2>&1; rc=$?
  tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
B="python -u bench.py --steps 10 --warmup 3 --copy-objects 0 --cpu-sample 0 --objects ${OBJECTS:-1024}"
declare -A V=( [class4]="TEC_DEBUG_KNOBS=1" [class1]="TEC_DEBUG_KNOBS=1 TEC_DEC_CLASS_STREAMS=1" [table]="TEC_DEBUG_KNOBS=1 TEC_DEC_CLASS=0" )
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in class4 class1 table; do
    timeout -k 10 300 env ${V[$v]} $B --mode decode --pattern random > $O/random_${v}_$r.json 2> $O/random_${v}_$r.err || exit $?
  done
done
for v in class4 table; do
  timeout -k 10 300 env ${V[$v]} $B --mode decode --decode-jit off > $O/worst_$v.json 2> $O/worst_$v.err || exit $?
  if [ "${PERCALL:-0}" == "1" ]; then
    timeout -k 10 300 env ${V[$v]} python -u bench.py --mode percall --cpu-sample 0 > $O/percall_$v.json 2> $O/percall_$v.err || exit $?
  fi
done
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + '/*.json')):
    d = json.loads([l for l in open(f) if l.startswith('{')][-1])
    if 'calls' in d:
        print(os.path.basename(f), {k: (v['decode']['ms_per_call'], v['encode']['ms_per_call']) for k, v in d['calls'].items()})
    else:
        print(os.path.basename(f), d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])
PY
