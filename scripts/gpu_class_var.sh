#!/bin/bash
# Decode class-kernel library variants (scripts/build_class_var.sh -> varlib/lib_<name>.so) against
# the shipped library and the table-driven kernel: random-pattern and worst-case (hipRTC off)
# decode lines, interleaved.   usage: VARS="late wpe6" scripts/gpu_class_var.sh <outdir-name>
# TESTS=1: the decode / recover GPU tests first; JIT=1: the hipRTC worst case, base and with the
# knobs in JIT_ALT (default TEC_DEC_JIT_FUSE=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-class_var}
mkdir -p $O
if [ "${TESTS:-0}" == "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "decode or parity or golden or extremes or percall or recover or repair" > $O/pytest.log 2>&1; rc=$?
  tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
B="python -u bench.py --steps 10 --warmup 3 --copy-objects 0 --cpu-sample 0 --mode decode"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in base table $VARS; do
    case $v in
      base) E="TEC_DEBUG_KNOBS=0";;
      table) E="TEC_DEBUG_KNOBS=1 TEC_DEC_CLASS=0";;
      *) E="TAPE_EC_LIB=$GRAFT_REPO_ROOT/varlib/lib_$v.so";;
    esac
    timeout -k 10 300 env $E $B --pattern random > $O/random_${v}_$r.json 2> $O/random_${v}_$r.err || exit $?
    timeout -k 10 300 env $E $B --decode-jit off > $O/worst_${v}_$r.json 2> $O/worst_${v}_$r.err || exit $?
    timeout -k 10 300 env $E ${B/--mode decode/--mode recover} > $O/recover_${v}_$r.json 2> $O/recover_${v}_$r.err || exit $?
  done
done
if [ "${JIT:-0}" == "1" ]; then  # worst case on the hipRTC pattern kernels (after their compile), fused vs not
  for r in 1 2; do
    timeout -k 10 300 env TEC_DEBUG_KNOBS=0 $B > $O/jit_base_$r.json 2> $O/jit_base_$r.err || exit $?
    timeout -k 10 300 env TEC_DEBUG_KNOBS=1 ${JIT_ALT:-TEC_DEC_JIT_FUSE=0} $B > $O/jit_alt_$r.json 2> $O/jit_alt_$r.err || exit $?
  done
fi
python3 - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + '/*.json')):
    d = json.loads([l for l in open(f) if l.startswith('{')][-1])
    print(os.path.basename(f), d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])
PY
