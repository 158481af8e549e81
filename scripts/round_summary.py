"""Condense gpurun_out/round (gpu_round*.sh) rocprofv3 output into small committed summaries.

Writes <out>/summary.json (per-kernel launch stats per bench mode, PMC per dispatch) and, when
the FETCH_SIZE/WRITE_SIZE passes exist, <out>/traffic.json in the form bench.py reads for
roofline.traffic.  HBM-byte correction per MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts 128-B fabric reads at 64 B, so it is doubled.
"""
import csv
import glob
import json
import os
import sys

OURS = ("enc_stage", "dec_stage", "rep_stage", "leaf_kernel", "tree_kernel", "gpe_kernel", "repair_kernel", "meta_kernel")


def kernel_stats(d):
    res = {}
    for kt in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(kt)):
            name = r.get("Kernel_Name", "")
            dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            e = res.setdefault(name[:90], {"n": 0, "total_ns": 0, "vgpr": r.get("VGPR_Count"),
                                           "lds": r.get("LDS_Block_Size"), "grid": r.get("Grid_Size"),
                                           "wg": r.get("Workgroup_Size")})
            e["n"] += 1
            e["total_ns"] += dur
    for v in res.values():
        v["avg_us"] = round(v["total_ns"] / v["n"] / 1e3, 2)
    if not res:  # trace csv deleted for size: fall back to the stats csv
        for st in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(st)):
                res[r["Name"][:90]] = {"n": int(r["Calls"]), "total_ns": int(r["TotalDurationNs"]),
                                       "avg_us": round(float(r["AverageNs"]) / 1e3, 2)}
    return dict(sorted(res.items(), key=lambda kv: -kv[1]["total_ns"])[:8])


def pmc(d):
    agg = {}
    for cf in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(cf)):
            k = r.get("Kernel_Name", "")
            if not any(o in k for o in OURS):
                continue
            a = agg.setdefault((k[:70], r["Counter_Name"]), [0.0, 0])
            a[0] += float(r["Counter_Value"])
            a[1] += 1
    return {f"{k} | {c}": {"per_dispatch": v[0] / max(1, v[1]), "dispatches": v[1]} for (k, c), v in agg.items()}


def pmc_all(d):
    agg = {}
    for cf in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(cf)):
            a = agg.setdefault((r.get("Kernel_Name", "")[:70], r["Counter_Name"]), [0.0, 0])
            a[0] += float(r["Counter_Value"])
            a[1] += 1
    return {f"{k} | {c}": v[0] / max(1, v[1]) for (k, c), v in agg.items()}


def calibration(root):
    """bytes counted / bytes moved for the encode's own access shapes (known byte counts)."""
    cal = {}
    f = pmc_all(os.path.join(root, "cal_fetch"))
    for k, v in f.items():
        if "rows<4, false, 1, 0>" in k:  # 1024 x 4 MiB read with dword loads at 2-aligned rows
            cal["fetch_kib_per_byte_dword_loads"] = v * 1024 / (1024 * 4 * 1024 * 1024)
    w = pmc_all(os.path.join(root, "cal_write"))
    for k, v in w.items():
        if "enc1<1, false, 1>" in k:  # 1024 x 20 x 715,048 B of whole-row 16-B stores
            cal["write_kib_per_byte_row_stores"] = v * 1024 / (1024 * 20 * 715048)
    return cal


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/round"
    out = {}
    for d in sorted(glob.glob(os.path.join(root, "trace_*"))):
        out[os.path.basename(d)] = kernel_stats(d)
    for d in sorted(glob.glob(os.path.join(root, "pmc_*"))):
        out[os.path.basename(d)] = pmc(d)
    json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)
    f = out.get("pmc_fetch", {})
    w = out.get("pmc_write", {})
    fk = [v["per_dispatch"] for k, v in f.items() if "enc_stage" in k and "FETCH_SIZE" in k]
    wk = [v["per_dispatch"] for k, v in w.items() if "enc_stage" in k and "WRITE_SIZE" in k]
    cal = calibration(root)
    out["calibration"] = cal
    json.dump(out, open(os.path.join(root, "summary.json"), "w"), indent=1)
    if fk and wk:
        # counted bytes -> bytes, with this pattern's own calibration when present (else the
        # guide's x2 for FETCH_SIZE on gfx950)
        fr = cal.get("fetch_kib_per_byte_dword_loads") or 0.5
        wr = cal.get("write_kib_per_byte_row_stores") or 1.0
        fetch_b = fk[0] * 1024 / fr
        write_b = wk[0] * 1024 / wr
        t = {"mode": "encode", "objects": 1024, "kernel": "enc_stage_kernel<7,6,false>",
             "fetch_size_kib": fk[0], "write_size_kib": wk[0],
             "fetch_counted_per_byte": fr, "write_counted_per_byte": wr,
             "hbm_bytes_per_launch": int(fetch_b + write_b),
             "correction": "FETCH_SIZE/WRITE_SIZE KiB -> bytes, divided by the counted/true ratio measured on "
                           "vmem_bench4 (dword loads) and vmem_bench7 (row stores) in the same run"}
        json.dump(t, open(os.path.join(root, "traffic.json"), "w"), indent=1)
        print(json.dumps(t))
    print(json.dumps({k: v for k, v in out.items() if k.startswith("trace")}, indent=1)[:4000])


if __name__ == "__main__":
    main()
