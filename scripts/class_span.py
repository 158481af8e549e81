"""Device time per bench call from a rocprofv3 kernel trace, for lines whose kernels overlap (the
decode / recover class kernels run side by side on forked streams, so their summed durations
overstate the call): the calls are the groups of tape_amd kernels separated by idle gaps, and
each call's span is its first kernel start to its last kernel end.  Prints the spans of the timed
calls next to the line's in-run `roofline.avg_launch_ms` (HIP events on the launch stream).

usage: class_span.py KERNEL_TRACE_CSV BENCH_LINE_JSON
"""
import csv
import json
import sys


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1]))
            if ("tec::" in r["Kernel_Name"] or "tec_dec_fixed" in r["Kernel_Name"]) and "meta_kernel" not in r["Kernel_Name"]]
    line = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
    # submission order; a call's kernels have distinct names (one launch per class, or the one
    # encode / repair kernel), so a name seen again starts the next call
    ev = sorted((int(r.get("Dispatch_Id", 0) or 0), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in rows)
    calls, cur = [], None
    for _, s, e, name in ev:
        if cur is None or name in cur[3]:
            cur = [s, e, 0, set()]
            calls.append(cur)
        cur[0], cur[1] = min(cur[0], s), max(cur[1], e)
        cur[2] += 1
        cur[3].add(name)
    steps = line.get("steps") or 0
    timed = calls[-steps:] if steps else calls
    spans = [(c[1] - c[0]) / 1e6 for c in timed]
    kinds = sorted({n.split("(")[0].replace("void ", "") for _, _, _, n in ev})
    print(json.dumps({"line": line.get("metric"), "line_avg_launch_ms": line["roofline"].get("avg_launch_ms"),
                      "trace_calls": len(calls), "timed_calls": len(timed),
                      "span_ms_mean": round(sum(spans) / max(1, len(spans)), 4) if spans else None,
                      "span_ms_min": round(min(spans), 4) if spans else None,
                      "kernels_per_call": [c[2] for c in timed][:3], "kernel_kinds": kinds[:12]}))


if __name__ == "__main__":
    main()
