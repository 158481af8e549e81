#!/bin/bash
# repair folded-kernel register budget A/B + one-down line after the host-side pattern cache
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t5
for u in 0 1; do
  for v in base wpe4 base wpe4; do
    TAPE_EC_LIB=varlib/lib_$v.so timeout -k 10 300 python bench.py --mode repair --unavailable $u --steps 20 --warmup 5 --cpu-sample 0 --copy-objects 0 > gpurun_out/t5/$v$u.json 2> gpurun_out/t5/$v$u.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/t5/$v$u.json')); print('$v u=$u', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])"
  done
done
for p in random worst; do
  timeout -k 10 300 python bench.py --mode decode --pattern $p --decode-jit off --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 > gpurun_out/t5/dec_$p.json 2> gpurun_out/t5/dec_$p.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/t5/dec_$p.json')); print('decode $p', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])"
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/t5/enc.json 2> gpurun_out/t5/enc.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/t5/enc.json')); print('encode', d['value'], d['roofline']['frac'], json.dumps(d['copy_inclusive_encode_commit']))"
