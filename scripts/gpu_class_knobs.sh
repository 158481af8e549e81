#!/bin/bash
# Decode class kernels under measurement knobs (TEC_DEBUG_KNOBS=1): random-pattern decode, worst
# case (hipRTC off) and recover lines per knob setting, interleaved.
#   usage: scripts/gpu_class_knobs.sh <outdir-name>   (KNOBS: space-separated name=ENV,ENV settings)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-class_knobs}
mkdir -p $O
B="python -u bench.py --steps 10 --warmup 3 --copy-objects 0 --cpu-sample 0"
for r in $(seq 1 ${ROUNDS:-2}); do
  for kv in ${KNOBS:-base=TEC_DEBUG_KNOBS=0}; do
    n=${kv%%=*}; E=${kv#*=}; E=${E//,/ }
    timeout -k 10 300 env TEC_DEBUG_KNOBS=1 $E $B --mode decode --pattern random > $O/random_${n}_$r.json 2> $O/random_${n}_$r.err || exit $?
    [ "${WORST:-1}" == "1" ] && { timeout -k 10 300 env TEC_DEBUG_KNOBS=1 $E $B --mode decode --decode-jit off > $O/worst_${n}_$r.json 2> $O/worst_${n}_$r.err || exit $?; }
    [ "${RECOVER:-1}" == "1" ] && { timeout -k 10 300 env TEC_DEBUG_KNOBS=1 $E $B --mode recover > $O/recover_${n}_$r.json 2> $O/recover_${n}_$r.err || exit $?; }
  done
done
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + '/*.json')):
    d = json.loads([l for l in open(f) if l.startswith('{')][-1])
    print(os.path.basename(f), d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])
PY
