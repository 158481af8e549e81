#!/bin/bash
# Decode / recover variants (varlib/lib_<name>.so; "base" = in-tree), interleaved.
#   bash scripts/gpu_dec_var.sh OUTDIR base v1 base v1 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
i=0
for v in "$@"; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode decode --pattern random --steps 10 --warmup 3 --cpu-sample 0 > $O/dec_${v}_$i.json 2> $O/dec_${v}_$i.err || exit $?
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode recover --steps 10 --warmup 3 --cpu-sample 0 > $O/rec_${v}_$i.json 2> $O/rec_${v}_$i.err || exit $?
  python3 -c "import json; a=json.load(open('$O/dec_${v}_$i.json')); b=json.load(open('$O/rec_${v}_$i.json')); print('$v random', a['roofline']['avg_launch_ms'], a['roofline']['frac'], a['outputs_verified'], 'recover', b['roofline']['avg_launch_ms'], b['roofline']['frac'], b['outputs_verified'])"
  i=$((i+1))
done
