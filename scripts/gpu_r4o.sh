#!/bin/bash
# round-4 GPU call: OuterCoder decode, enqueue-only calls -- kernel trace (durations and gaps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --mode outer --steps 3 --warmup 1 --cpu-sample 0 > $O/trace.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r4o/trace/**/*kernel_trace.csv", recursive=True)[0]
ks = [r for r in csv.DictReader(open(f)) if "rs16_decode" in r["Kernel_Name"]]
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks]
g = [(int(ks[i + 1]["Start_Timestamp"]) - int(ks[i]["End_Timestamp"])) / 1e3 for i in range(len(ks) - 1)]
print("decode kernels", len(d), "mean us", sum(d) / len(d), "min", min(d), "max", max(d))
print("gaps us mean", sum(g) / len(g), "median", sorted(g)[len(g) // 2], "max", max(g))
PY
find $O -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O -name "*.csv" -size +2M -delete; find $O -name "*.db" -delete
