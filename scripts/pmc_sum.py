"""Summarise rocprofv3 --pmc passes: per counter, the per-dispatch mean over kernels matching a
pattern.  usage: pmc_sum.py DIR [kernel-substring]"""
import csv
import glob
import os
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "stage"
agg = {}
for cf in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(cf)):
        k = r.get("Kernel_Name", "")
        if pat not in k:
            continue
        key = (k.split("(")[0][-48:], r["Counter_Name"])
        disp = r.get("Dispatch_Id", "")
        a = agg.setdefault(key, {})
        a[disp] = a.get(disp, 0.0) + float(r["Counter_Value"])
for (k, c), d in sorted(agg.items()):
    v = list(d.values())
    print(f"{k:48s} {c:36s} {sum(v) / len(v):18.1f}  (n={len(v)})")
