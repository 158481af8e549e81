"""HBM traffic per bench step from scripts/profile_modes.sh output -> profiles/traffic.json.

usage: traffic.py PROF_DIR OBJECTS [MODE ...]

Per mode, the counters of the kernels bench.KERNELS names are averaged over their dispatches and
summed over the kernels of one step.  Corrections (MI355X_MICROARCH.md, HBM section):
  * reads: the L2's memory-side read requests by size, 32 B / 64 B / 128 B (FETCH_SIZE tallies a
    128-B request at 64 B, i.e. reports half of a wide streaming read); without the 64 B / 128 B
    split, every request that is not a 32-B one counts 128 B (an upper bound);
  * writes: WRITE_SIZE, exact for 16-B-per-lane stores (every row store here is one).
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def names_of(m):
    """kernel names of a traffic.json key: a bench mode, or mode:pattern (decode:random)."""
    mode, _, pat = m.partition(":")
    return bench.kernel_names(mode, "async", pat or "worst")


def per_step(d, m):
    names = names_of(m)
    tot = {}
    for cf in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = {}
        for r in csv.DictReader(open(cf)):
            k = r.get("Kernel_Name", "")
            kn = next((n for n in names if k.startswith(n) or ("void " + n) in k), None)
            if kn is None:
                continue
            # per distinct kernel (each decode / recover class kernel is launched once per step)
            key = (k, r["Counter_Name"])
            disp = per.setdefault(key, {})
            disp[r.get("Dispatch_Id", "")] = disp.get(r.get("Dispatch_Id", ""), 0.0) + float(r["Counter_Value"])
        for (kn, c), disp in per.items():
            tot[c] = tot.get(c, 0.0) + sum(disp.values()) / len(disp) * bench.LAUNCHES_PER_STEP.get(m, 1)
    return tot


def main():
    root, objects = sys.argv[1], int(sys.argv[2])
    modes = sys.argv[3:] or ["encode"]
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    if "mode" in out:  # the round-1 single-mode layout
        out = {}
    for m in modes:
        c = per_step(os.path.join(root, (m if m != "outer_decode" else "outer").replace(":", "_")), m)
        if not c:
            print(m, "no counters")
            continue
        r, r32 = c.get("TCC_EA0_RDREQ_sum", 0.0), c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        r64 = c.get("TCC_EA0_RDREQ_64B_sum", 0.0)
        read_b = 32.0 * r32 + 64.0 * r64 + 128.0 * (r - r32 - r64)
        write_b = c.get("WRITE_SIZE", 0.0) * 1024.0
        out[m] = {
            "objects": objects,
            "kernels": names_of(m),
            "hbm_bytes_per_step": int(read_b + write_b),
            "read_bytes": int(read_b),
            "write_bytes": int(write_b),
            "counters_per_step": {k: round(v, 1) for k, v in sorted(c.items())},
            "fetch_size_x2_bytes": int(c.get("FETCH_SIZE", 0.0) * 1024.0 * 2),
            "correction": "read = 32 B x RDREQ_32B + 64 B x RDREQ_64B + 128 B x other RDREQ (FETCH_SIZE x 2 for "
                          "wide reads, shown for comparison); write = WRITE_SIZE KiB x 1024",
        }
        print(m, json.dumps(out[m], indent=1))
    json.dump(out, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
