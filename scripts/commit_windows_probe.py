#!/usr/bin/env python3
"""te_encode_commit_batch_host on 1024 x 4 MiB pinned objects: GiB/s per hashing group size and
hashing side (auto / device / host), each size run in several orders, to separate an ordering
effect from the group size itself (bench.py's copy_inclusive_commit runs 2, 4, 8 GiB in order).
Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import tape_amd as T  # noqa: E402
from tape_amd import batch  # noqa: E402


def threads_cpu():
    """Per-thread CPU ticks (utime + stime) of this process, from /proc."""
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            f = open(f"/proc/self/task/{tid}/stat").read().rsplit(")", 1)[1].split()
            out[tid] = (int(f[11]) + int(f[12]), open(f"/proc/self/task/{tid}/comm").read().strip())
        except OSError:
            pass
    return out


class ClockSampler:
    """Samples the GPU's current sclk / mclk DPM level (sysfs pp_dpm_*) every 5 ms while active."""

    def __init__(self):
        import threading
        p = torch.cuda.get_device_properties(0)
        self.base = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        self.samples = []
        self.on = False
        self.th = threading.Thread(target=self.loop, daemon=True)
        self.th.start()

    def cur(self, fn):
        try:
            for l in open(os.path.join(self.base, fn)):
                if l.strip().endswith("*"):
                    return l.split(":")[1].strip().rstrip("*").strip()
        except OSError:
            return None

    def loop(self):
        while True:
            if self.on:
                self.samples.append((self.cur("pp_dpm_sclk"), self.cur("pp_dpm_mclk"), self.cur("pp_dpm_fclk")))
            time.sleep(0.005)

    def start(self):
        self.samples = []
        self.on = True

    def stop(self):
        self.on = False
        import collections
        return dict(collections.Counter(self.samples).most_common(4))


def idle_cpu(sec=0.5):
    """CPU the process burns while the caller sleeps (a spinning thread shows here): ticks per
    second of wall time, and the busiest threads."""
    a = threads_cpu()
    time.sleep(sec)
    b = threads_cpu()
    hz = os.sysconf("SC_CLK_TCK")
    d = sorted(((b[t][0] - a.get(t, (0,))[0]) / hz / sec, b[t][1], t) for t in b)
    busy = [(round(x, 2), n, t) for x, n, t in d[::-1][:4] if x > 0.02]
    return round(sum(x for x, _, _ in d), 2), busy


def main():
    m, L = 1024, 4 << 20
    s = T.Slicer.clay_default()
    per = 20 * s.geometry(L).slice_len
    h_in = torch.randint(0, 256, (m * L,), dtype=torch.uint8).pin_memory()
    h_out = torch.empty(m * per, dtype=torch.uint8).pin_memory()
    leaf = torch.empty(m * 20 * 32, dtype=torch.uint8).pin_memory()
    root = torch.empty(m * 32, dtype=torch.uint8).pin_memory()
    proof = torch.empty(m * 20 * 5 * 32, dtype=torch.uint8).pin_memory()
    objs = batch.encode_descs([(i * L, L, i * per, 0) for i in range(m)])
    res = []
    pre = os.environ.get("PRE", "")
    if "dev" in pre:  # bench.py's device-resident encode first (torch buffers, the caller's stream)
        d_in = h_in.cuda()
        d_out = torch.empty(m * per, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            batch.encode_batch(s, d_in, [(i * L, L, i * per, 0) for i in range(m)], d_out)
        torch.cuda.synchronize()
    if "host" in pre:  # bench.py's copy-inclusive encode first (te_encode_batch_host)
        for _ in range(3):
            batch.encode_batch_host(s, h_in, objs, h_out)
    seq = (("auto", 2), ("auto", 4), ("auto", 8), ("auto", 4)) if pre else \
        (("auto", 4), ("auto", 2), ("auto", 4), ("auto", 8), ("auto", 4), ("device", 4),
         ("device", 2), ("device", 8), ("host", 4), ("device", 4), ("auto", 4))
    if os.environ.get("SEQ"):  # e.g. SEQ=device:2,auto:4
        seq = tuple((h, int(g)) for h, g in (x.split(":") for x in os.environ["SEQ"].split(",")))
    d_probe = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")

    def d2h_rate(dst):
        """plain D2H of 1 GiB into the front of a pinned host buffer (GB/s)"""
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst[:1 << 30].copy_(d_probe, non_blocking=True)
        torch.cuda.synchronize()
        return round((1 << 30) / (time.perf_counter() - t0) / 1e9, 1)

    fresh = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    clk = ClockSampler()
    print({"d2h_GBps_h_out": d2h_rate(h_out), "d2h_GBps_fresh": d2h_rate(fresh)}, flush=True)
    for hashing, gib in seq:
        batch.set_commit_hashing(hashing)
        batch.encode_commit_batch_host(s, h_in, objs, h_out, leaf, root, proof, window_bytes=gib << 30)
        t = time.perf_counter()
        c0 = time.process_time()
        clk.start()
        for _ in range(2):
            batch.encode_commit_batch_host(s, h_in, objs, h_out, leaf, root, proof, window_bytes=gib << 30)
        el = time.perf_counter() - t
        clocks = clk.stop()
        cpu = time.process_time() - c0
        idle, busy = idle_cpu()
        res.append({"hashing": hashing, "group_GiB": gib, "GiBps": round(2 * m * L / el / 2**30, 3),
                    "cpu_cores_during": round(cpu / el, 2), "cpu_cores_idle_after": idle, "busy_threads_idle": busy,
                    "d2h_GBps_h_out_after": d2h_rate(h_out), "d2h_GBps_fresh_after": d2h_rate(fresh),
                    "clocks_sclk_mclk_fclk": {" / ".join(map(str, k)): v for k, v in clocks.items()}})
        print(res[-1], flush=True)
    batch.set_commit_hashing("auto")
    print(json.dumps({"probe": "encode_commit_batch_host group size / hashing", "runs": res}), flush=True)


if __name__ == "__main__":
    main()
