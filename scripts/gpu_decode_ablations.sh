#!/bin/bash
# what bounds the table-driven decode kernel -- random-pattern decode with the
# shipped build and with ablation builds (varlib/lib_dec_abl*.so, built first with scripts/build_var.sh
# dec_ablN "-DTEC_DEC_ABLATE=N" decode_stage.hip: 1 no scratch loads, 2 no MDS
# products, 8 no input loads, 9 = 1+8, 11 = 1+2+8); outputs of ablations are wrong by design
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/decode_ablations
mkdir -p $O
B="python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0 --mode decode --pattern random"
timeout -k 10 300 $B > $O/base.json 2> $O/base.err || exit 1
for v in abl1 abl2 abl8 abl9 abl11 cond; do
  TAPE_EC_LIB=$GRAFT_REPO_ROOT/varlib/lib_dec_$v.so timeout -k 10 300 $B > $O/$v.json 2> $O/$v.err || exit 1
done
timeout -k 10 300 $B > $O/base2.json 2> $O/base2.err || exit 1
python3 - <<'PY'
import json
for f in ("base","abl1","abl2","abl8","abl9","abl11","cond","base2"):
    d=json.load(open(f"gpurun_out/r4k/{f}.json")); r=d["roofline"]
    print(f, r["avg_launch_ms"], r["frac"], d["outputs_verified"])
PY
