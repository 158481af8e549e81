set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/jitab; mkdir -p $O
B="python3 bench.py --steps 10 --warmup 3 --copy-objects 0 --cpu-sample 0 --mode decode"
for r in 1 2; do
timeout -k 10 400 $B > $O/worst_jit_$r.json 2> $O/worst_jit_$r.err || exit $?
timeout -k 10 300 $B --decode-jit off > $O/worst_off_$r.json 2> $O/worst_off_$r.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_random -o run -- python3 bench.py --mode decode --pattern random --steps 3 --warmup 1 --cpu-sample 0 --copy-objects 0 > $O/prof_random.log 2>&1 || exit $?
find $O -name "*kernel_trace.csv" -delete; find $O -name "*.db" -delete
for f in $O/*.json; do echo $f $(python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print(d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('decode_jit'))"); done
cat $(find $O/prof_random -name "*kernel_stats.csv") | cut -c1-150 | head -20
