#!/bin/bash
# (1) the slow copy state with SDMA off (copies as blit kernels); (2) decode WPL=2 variants:
# parity (decode tests through the variant library), then A/B timing of random decode and recover
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5c
mkdir -p $O
HSA_ENABLE_SDMA=0 timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > $O/default_nosdma.json 2> $O/default_nosdma.err && python3 -c "import json; d=json.load(open('$O/default_nosdma.json')); print('nosdma', d['copy_inclusive']['value'], d['copy_inclusive_encode_commit']['by_window'], d['copy_inclusive_encode_commit']['stream_writer'], d['stream_sdk_shape']['value'], d['stream_sdk_shape']['chunk_latency_ms_p50_p90'])" &&
TAPE_EC_LIB=varlib/lib_dw2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_store.py tests/test_gpu_repair_sets.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest_dw2.log 2>&1; rc=$?; tail -3 $O/pytest_dw2.log; [ $rc -eq 0 ] || exit $rc
for v in base dw2 dw2w3 base dw2; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode decode --pattern random --steps 10 --warmup 3 --cpu-sample 0 > $O/dec_$v.json 2> $O/dec_$v.err || exit $?
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode recover --steps 10 --warmup 3 --cpu-sample 0 > $O/rec_$v.json 2> $O/rec_$v.err || exit $?
  python3 -c "import json; a=json.load(open('$O/dec_$v.json')); b=json.load(open('$O/rec_$v.json')); print('$v random', a['roofline']['avg_launch_ms'], a['roofline']['frac'], a['outputs_verified'], 'recover', b['roofline']['avg_launch_ms'], b['roofline']['frac'], b['outputs_verified'])"
done
bash scripts/gpu_r5d.sh
