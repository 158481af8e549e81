#!/bin/bash
# Per-call decode (the one-wave class kernels with a loader wave, zero-copy staging): the decode
# GPU tests, then --mode percall with the shipped library, with the knobs in ALT (default the
# copies instead of zero-copy, TEC_DECODE_ZC=0) and with the table-driven kernel (TEC_DEC_CLASS=0); random decode and recover
# lines as a regression check of the batch kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-percall_class}; mkdir -p $O
if [ "${TESTS:-1}" == "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "decode or parity or golden or extremes or percall or recover or repair or class" > $O/pytest.log 2>&1; rc=$?
  tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --mode percall --cpu-sample 0 > $O/pc_class.json 2> $O/pc.err || exit $?
env TEC_DEBUG_KNOBS=1 ${ALT:-TEC_DECODE_ZC=0} timeout -k 10 300 python -u bench.py --mode percall --cpu-sample 0 > $O/pc_alt.json 2>> $O/pc.err || exit $?
TEC_DEBUG_KNOBS=1 TEC_DEC_CLASS=0 timeout -k 10 300 python -u bench.py --mode percall --cpu-sample 0 > $O/pc_table.json 2>> $O/pc.err || exit $?
B="python -u bench.py --steps 10 --warmup 3 --copy-objects 0 --cpu-sample 0"
timeout -k 10 300 $B --mode decode --pattern random > $O/random.json 2> $O/random.err || exit $?
timeout -k 10 300 $B --mode recover > $O/recover.json 2> $O/recover.err || exit $?
for f in $O/pc_class.json $O/pc_alt.json $O/pc_table.json; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1])
for k,v in d['calls'].items(): print('$f'.split('/')[-1], k, {n:(x['ms_per_call'],x.get('kernel_ms_per_call')) for n,x in v.items()})
print('verified', d['outputs_verified'])"; done
for f in $O/random.json $O/recover.json; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])"; done
