#!/bin/bash
# round-4 GPU call: decode tables in LDS (TEC_DEC_TAB_LDS=1, the default build) against the
# scalar-loaded tables (varlib/lib_dec_sgpr.so): decode / recover / store tests, then random decode,
# recover and table-driven worst-case decode with each library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_decode_jit.py tests/test_gpu_repair_sets.py tests/test_gpu_decode_store.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --copy-objects 0"
for v in lds sgpr; do
  if [ $v = sgpr ]; then export TAPE_EC_LIB=$GRAFT_REPO_ROOT/varlib/lib_dec_sgpr.so; fi
  timeout -k 10 300 $B --mode decode --pattern random > $O/decode_random_$v.json 2> $O/decode_random_$v.err || exit 1
  timeout -k 10 300 $B --mode recover > $O/recover_$v.json 2> $O/recover_$v.err || exit 1
  timeout -k 10 300 $B --mode decode --decode-jit off > $O/decode_worst_table_$v.json 2> $O/decode_worst_table_$v.err || exit 1
done
unset TAPE_EC_LIB
timeout -k 10 300 $B --mode decode --pattern random > $O/decode_random_lds2.json 2> $O/decode_random_lds2.err
python3 - <<'PY'
import json
for f in ("decode_random_lds","decode_random_sgpr","decode_random_lds2","recover_lds","recover_sgpr","decode_worst_table_lds","decode_worst_table_sgpr"):
    d=json.load(open(f"gpurun_out/r4i/{f}.json")); r=d["roofline"]
    print(f, d["ms_per_step"], r["avg_launch_ms"], r["frac"], d["outputs_verified"])
PY
