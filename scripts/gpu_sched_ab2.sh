#!/bin/bash
# max-ilp backend scheduling for the repair (fold), OuterCoder and commitment kernels, and a
# confirmation round of the decode one: parity first, then interleaved timings
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sched_ab2
mkdir -p $O
TAPE_EC_LIB=varlib/lib_r_ilp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_repair_sets.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "repair" > $O/pytest_r.log 2>&1; rc=$?; echo "r_ilp $(tail -1 $O/pytest_r.log)"; [ $rc -eq 0 ] || exit $rc
TAPE_EC_LIB=varlib/lib_o_ilp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_outer.py -x -q --timeout 120 --timeout-method thread > $O/pytest_o.log 2>&1; rc=$?; echo "o_ilp $(tail -1 $O/pytest_o.log)"; [ $rc -eq 0 ] || exit $rc
TAPE_EC_LIB=varlib/lib_c_ilp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread -k "commit or leaf or root or proof or merkle or stream" > $O/pytest_c.log 2>&1; rc=$?; echo "c_ilp $(tail -1 $O/pytest_c.log)"; [ $rc -eq 0 ] || exit $rc
i=0
for v in base r_ilp base r_ilp base r_ilp; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode repair --steps 20 --warmup 5 --cpu-sample 0 --copy-objects 0 > $O/rep_${v}_$i.json 2> $O/rep_${v}_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/rep_${v}_$i.json')); print('$v repair', d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['outputs_verified'])"
  i=$((i+1))
done
bash scripts/gpu_outer_var.sh sched_ab2/outer base o_ilp base o_ilp || exit $?
i=0
for v in base c_ilp base c_ilp; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode commit --steps 5 --warmup 2 --cpu-sample 0 > $O/c_${v}_$i.json 2> $O/c_${v}_$i.err || exit $?
  python3 -c "import json; d=json.loads([l for l in open('$O/c_${v}_$i.json') if l.startswith('{')][-1]); print('$v commit', d['value'], d['ms_per_step'], d.get('outputs_verified'))"
  i=$((i+1))
done
bash scripts/gpu_dec_var.sh sched_ab2/dec base d_ilp base d_ilp base d_ilp
