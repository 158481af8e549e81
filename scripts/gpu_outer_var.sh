#!/bin/bash
# OuterCoder matrix-kernel variants (varlib/lib_<name>.so; base = in-tree): encode / decode kernel
# ms, HBM fraction, outputs verified.   bash scripts/gpu_outer_var.sh OUTDIR base m_x ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
i=0
for v in "$@"; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode outer --steps 10 --warmup 3 --cpu-sample 0 > $O/o_${v}_$i.json 2> $O/o_${v}_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/o_${v}_$i.json')); r=d['roofline']; print('$v', r['avg_launch_ms'], r['frac'], d['outputs_verified'], d['decode']['roofline']['avg_launch_ms'], d['decode']['roofline']['frac'], d['decode']['outputs_verified'])"
  i=$((i+1))
done
