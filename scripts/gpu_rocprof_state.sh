set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/rp_state; mkdir -p $O
timeout -k 10 120 python -u scripts/hbm_state_probe.py --samples 2 --load-s 1 > $O/plain1.jsonl 2> $O/err1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o run -- python3 -u scripts/hbm_state_probe.py --samples 2 --load-s 1 > $O/rocprof.jsonl 2> $O/err2 || exit $?
timeout -k 10 120 python -u scripts/hbm_state_probe.py --samples 2 --load-s 1 > $O/plain2.jsonl 2> $O/err3 || exit $?
timeout -k 10 200 rocprofv3 --stats --kernel-trace --output-format csv -d $O/rp2 -o run -- python3 -u scripts/hbm_state_probe.py --samples 2 --load-s 1 > $O/rocprof2.jsonl 2> $O/err4 || exit $?
find $O -name "*.csv" -delete
env | grep -i "^HSA\|^HIP\|^ROC\|^GPU\|^AMD" > $O/env_plain.txt
for f in plain1 rocprof plain2 rocprof2; do echo $f; cat $O/$f.jsonl | cut -c1-120; done
