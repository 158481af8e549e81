#!/bin/bash
# round-4 GPU call: decode table kernel, next-step loads issued late (fewer live registers):
# random decode + recover with the shipped build and varlib/lib_dec_late{4,5}.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
B="python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0"
for v in base late4 late5 base2; do
  L=""; [ "${v#late}" != "$v" ] && L=$GRAFT_REPO_ROOT/varlib/lib_dec_$v.so
  TAPE_EC_LIB=$L timeout -k 10 300 $B --mode decode --pattern random > $O/dr_$v.json 2> $O/dr_$v.err || exit 1
  TAPE_EC_LIB=$L timeout -k 10 300 $B --mode recover > $O/rc_$v.json 2> $O/rc_$v.err || exit 1
  python3 -c "
import json
for f in ('dr','rc'):
    d=json.load(open('$O/'+f+'_$v.json')); r=d['roofline']; print('$v', f, r['avg_launch_ms'], r['frac'], d['outputs_verified'])"
done
for v in base rs_persist; do
  L=""; [ $v != base ] && L=$GRAFT_REPO_ROOT/varlib/lib_$v.so
  TAPE_EC_LIB=$L timeout -k 10 300 python3 -u bench.py --mode outer --cpu-sample 0 > $O/outer_$v.json 2> $O/outer_$v.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/outer_$v.json')); print('$v enc', d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'] if 'outputs_verified' in d else '')"
done
