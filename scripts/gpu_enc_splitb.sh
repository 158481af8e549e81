#!/bin/bash
# batch encode split into level-1 parts (TEC_ENC_SPLIT_BATCH = rows per workgroup: 1 -> 7 parts,
# 2 -> 4, 4 -> 2, 7 -> 1) + the level-2 launch, against the one-launch kernel; the bench's oracle
# byte-compare of 32 objects in each line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/enc_splitb
mkdir -p $O
for v in ${VARIANTS:-0 1 0 1}; do
  knob=""; [ $v != 0 ] && knob="TEC_DEBUG_KNOBS=1 TEC_ENC_SPLIT_BATCH=$v"
  env $knob timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-sample 32 --copy-objects 0 --sdk-chunks 0 > $O/e_$v.json 2> $O/e_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/e_$v.json')); r=d['roofline']; print('split $v', r['avg_launch_ms'], r['frac'], r['box_ceiling_frac'], d['ms_per_step'], d['cpu_baseline']['gpu_matches_oracle_on_sample'])"
done
