#!/bin/bash
# traffic + kernel stats per mode (r05 binaries); commit probe with clocks and group trace;
# per-call lines; decode put_out variant A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f
mkdir -p $O
bash scripts/profile_modes.sh encode decode:random recover repair || exit $?
TEC_DEBUG_KNOBS=1 TEC_COMMIT_TRACE=1 PRE="dev host" SEQ=auto:2,auto:4,auto:8,auto:4 timeout -k 10 400 python -u scripts/commit_windows_probe.py > $O/commit_probe.txt 2> $O/commit_probe.err; rc=$?; grep "GiBps" $O/commit_probe.txt | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode percall --cpu-sample 0 > $O/percall.json 2> $O/percall.err && python3 -c "import json; d=json.load(open('$O/percall.json')); print({k: {c: v['ms_per_call'] for c, v in r.items()} for k, r in d['calls'].items()})" || exit $?
for v in base d_put1 base d_put1; do
  lib=varlib/lib_$v.so; [ $v == base ] && lib=tape_amd/libtapeec.so
  TAPE_EC_LIB=$lib timeout -k 10 300 python bench.py --mode decode --pattern random --steps 10 --warmup 3 --cpu-sample 0 > $O/dec_$v.json 2> $O/dec_$v.err || exit $?
  python3 -c "import json; a=json.load(open('$O/dec_$v.json')); print('$v random', a['roofline']['avg_launch_ms'], a['roofline']['frac'], a['outputs_verified'])"
done
