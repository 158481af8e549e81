#!/bin/bash
# Encode kernel variants (varlib/lib_<name>.so; "base" = the in-tree library), interleaved:
# kernel ms, HBM fraction, the box ceiling of each run, and a 32-object oracle byte check.
#   bash scripts/gpu_enc_var.sh OUTDIR base e_rp1 base e_rp1 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
i=0
for v in "$@"; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-sample 32 --copy-objects 0 --sdk-chunks 0 > $O/enc_${v}_$i.json 2> $O/enc_${v}_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/enc_${v}_$i.json')); r=d['roofline']; print('$v', r['avg_launch_ms'], r['frac'], r['box_ceiling_frac'], r['box_ceiling']['blocks_ms'], d['cpu_baseline']['gpu_matches_oracle_on_sample'])"
  i=$((i+1))
done
