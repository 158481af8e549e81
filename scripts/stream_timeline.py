#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel + memory-copy trace of `bench.py --mode stream`.

Usage: stream_timeline.py TRACE_DIR [first last]
Prints the copies longer than 0.5 ms and the encode / leaf kernels in time order, then per
direction the mean copy time, so the per-chunk pipeline (H2D, encode, D2H, host hashing gaps)
can be read off.
"""
import csv
import os
import sys


def main():
    d = sys.argv[1]
    lo, hi = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (40, 90)
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r["Direction"].replace("MEMORY_COPY_", ""), r["Stream_Id"]))
    for k in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        n = k["Kernel_Name"]
        if "enc_dma" in n or "leaf" in n:
            ev.append((int(k["Start_Timestamp"]), int(k["End_Timestamp"]),
                       "K:" + n.split("(")[0][-22:], k["Stream_Id"]))
    ev.sort()
    big = [e for e in ev if (e[1] - e[0]) > 500_000 or e[2].startswith("K")]
    t0 = big[0][0]
    for e in big[lo:hi]:
        print(f"{(e[0]-t0)/1e6:9.3f} -> {(e[1]-t0)/1e6:9.3f} ({(e[1]-e[0])/1e6:6.3f} ms) {e[2]:28s} s={e[3]}")
    per = {}
    for e in big:
        per.setdefault(e[2], []).append((e[1] - e[0]) / 1e6)
    for k, v in sorted(per.items()):
        print(f"{k:28s} n={len(v):4d} mean={sum(v)/len(v):7.3f} ms")


if __name__ == "__main__":
    main()
