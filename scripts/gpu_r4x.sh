#!/bin/bash
# round-4 GPU call: kernel + copy trace of the slow 4 GiB commit window (after 3 GiB runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
PRE=host SEQ=auto:3,auto:4 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 scripts/commit_windows_probe.py > $O/p.log 2>&1 || exit 1
grep "^{'hashing'" $O/p.log
python3 - <<'PY'
import csv, glob
d = "gpurun_out/r4x/trace"
ks = list(csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0])))
leaf = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks if "leaf_kernel" in r["Kernel_Name"]]
leaf.sort()
print("leaf launches", len(leaf), "ms:", [round((b - a) / 1e6, 1) for a, b in leaf])
enc = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks if "enc_dma" in r["Kernel_Name"]]
print("encode launches", len(enc), "mean ms", round(sum(b - a for a, b in enc) / len(enc) / 1e6, 3))
cp = list(csv.DictReader(open(glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)[0])))
d2h = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in cp if "DEVICE_TO_HOST" in r["Direction"])
# per-second busy fraction of D2H over the last ~2.5 s (the 4 GiB runs)
t_end = max(b for a, b in d2h)
for w in range(6):
    lo, hi = t_end - (w + 1) * 500_000_000, t_end - w * 500_000_000
    busy = sum(max(0, min(b, hi) - max(a, lo)) for a, b in d2h)
    nl = [x for x in leaf if lo <= x[0] < hi]
    print(f"window -{(w+1)*0.5:.1f}s..-{w*0.5:.1f}s: D2H busy {busy / 5e8:.2f}, leaf launches {len(nl)} ms {[round((b-a)/1e6,1) for a,b in nl]}")
PY
find $O -name "*.csv" -size +20M -delete
