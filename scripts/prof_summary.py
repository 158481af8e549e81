"""Condense rocprofv3 CSV output into small summaries (run on the GPU box after profile.sh)."""
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
out = {}
for st in glob.glob(os.path.join(root, "trace", "**", "*kernel_stats.csv"), recursive=True):
    with open(st) as f:
        out["kernel_stats"] = list(csv.DictReader(f))[:15]
for kt in glob.glob(os.path.join(root, "trace", "**", "*kernel_trace.csv"), recursive=True):
    rows = list(csv.DictReader(open(kt)))
    byk = {}
    for r in rows:
        name = r.get("Kernel_Name", "")
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        e = byk.setdefault(name, {"n": 0, "total_ns": 0, "vgpr": r.get("VGPR_Count"), "sgpr": r.get("SGPR_Count"),
                                  "lds": r.get("LDS_Block_Size"), "grid": r.get("Grid_Size"), "wg": r.get("Workgroup_Size")})
        e["n"] += 1
        e["total_ns"] += d
    for v in byk.values():
        v["avg_us"] = round(v["total_ns"] / v["n"] / 1e3, 2)
    out["kernels"] = dict(sorted(byk.items(), key=lambda kv: -kv[1]["total_ns"])[:8])
for name in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2"):
    for cf in glob.glob(os.path.join(root, name, "**", "*counter_collection.csv"), recursive=True):
        agg = {}
        for r in csv.DictReader(open(cf)):
            k = r.get("Kernel_Name", "")
            if "enc_stage" not in k and "gpe_kernel" not in k and "repair_kernel" not in k:
                continue
            key = (k[:60], r["Counter_Name"])
            a = agg.setdefault(key, [0.0, 0])
            a[0] += float(r["Counter_Value"])
            a[1] += 1
        out[name] = {f"{k[0]} | {k[1]}": {"sum": v[0], "dispatches": v[1], "per_dispatch": v[0] / max(1, v[1])}
                     for k, v in agg.items()}
json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)
print(json.dumps(out.get("kernels", {}), indent=1)[:3000])
