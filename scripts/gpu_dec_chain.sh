#!/bin/bash
# per-call decode chain: dec_stage_kernel time per 4 MiB call (G = 1) and per 64 MiB call (G = 2)
# for the shipped build and the scratch-early measurement builds (se0: all next-step loads at the
# step's start; se1: scratch only) -- outputs of se* are wrong where a step reads what the
# previous one wrote
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/dec_chain
mkdir -p $O
export TMPDIR=/tmp
for v in base se0 se1; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 bench.py --mode percall --cpu-sample 0 > $O/$v.json 2> $O/$v.err || exit $?
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" "$O/$v.json" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.loads([l for l in open(sys.argv[3]) if l.startswith('{')][-1])
print(sys.argv[2], {r['Name'][:48]: round(float(r['AverageNs']) / 1e3, 1) for r in rows if 'dec_stage' in r['Name']}, 'verified', d['outputs_verified'])
PY
done
