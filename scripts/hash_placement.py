#!/usr/bin/env python3
"""Host leaf-hash throughput vs thread placement (CPU only; run on the GPU box's host).

16 threads (the pool's default) each hash te_host_hash_lanes slices of 9.7 MB at a time with
te_hash_leaves (ctypes drops the GIL), pinned per policy: unpinned, one thread per physical core
spread over the machine, one per core within each NUMA node, and SMT siblings packed.  Prints one
JSON line: aggregate GB/s per policy."""
import ctypes as C
import json
import os
import threading
import time

import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tape_amd import _lib

lib = _lib.lib
SL, N, NT = 9_724_048, 20, int(os.environ.get("THREADS", "16"))


def topo():
    cpus = sorted(os.sched_getaffinity(0))
    info = {}
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            core = int(open(base + "core_id").read())
            pkg = int(open(base + "physical_package_id").read())
        except OSError:
            core, pkg = c, 0
        node = 0
        for d in os.listdir(f"/sys/devices/system/cpu/cpu{c}"):
            if d.startswith("node"):
                node = int(d[4:])
        info[c] = (pkg, core, node)
    return info


def policies(info):
    first_of_core, sib = {}, {}
    for c, (pkg, core, node) in sorted(info.items()):
        first_of_core.setdefault((pkg, core), c)
        sib.setdefault((pkg, core), []).append(c)
    cores = sorted(first_of_core.values())
    nodes = sorted({v[2] for v in info.values()})
    pol = {"unpinned": None, "spread_cores": [cores[i * len(cores) // NT] for i in range(NT)] if len(cores) >= NT else None}
    for nd in nodes:
        cs = [c for c in cores if info[c][2] == nd]
        if len(cs) >= NT:
            pol[f"node{nd}_cores"] = cs[:NT]
    pairs = [s for s in sib.values() if len(s) >= 2]
    if len(pairs) * 2 >= NT:
        pol["smt_packed"] = [c for s in pairs[:NT // 2] for c in s[:2]]
    return pol


def run(cpus, bufs, lanes):
    outs = [(C.c_uint8 * (32 * N))() for _ in range(NT)]
    done = [0] * NT

    def worker(w):
        if cpus is not None:
            os.sched_setaffinity(0, {cpus[w]})
        b = bufs[w]
        p = C.cast(b.ctypes.data, C.POINTER(C.c_uint8))
        for _ in range(3):
            for i0 in range(0, N, lanes):
                L = min(lanes, N - i0)
                lib.te_hash_leaves(C.cast(b.ctypes.data + i0 * SL, C.POINTER(C.c_uint8)), SL, L, lanes, outs[w])
                done[w] += L * SL
        del p

    ths = [threading.Thread(target=worker, args=(w,)) for w in range(NT)]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return sum(done) / (time.perf_counter() - t) / 1e9


def page_node(addr):
    """NUMA node of the page at addr (get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR)), or -1."""
    libc = C.CDLL(None, use_errno=True)
    mode = C.c_int(-1)
    r = libc.syscall(239, C.byref(mode), None, C.c_ulong(0), C.c_void_p(addr), C.c_ulong(3))  # SYS_get_mempolicy
    return mode.value if r == 0 else -1


def main():
    info = topo()
    lanes = lib.te_host_hash_lanes()
    rng = np.random.default_rng(1)
    kind = os.environ.get("BUF", "pageable")
    if kind == "pinned":  # te_host_alloc (hipHostMalloc, portable), as the stream writer's buffers
        from tape_amd import batch
        bufs = []
        for _ in range(NT):
            b = batch.host_empty(N * SL)
            b[:] = rng.integers(0, 256, N * SL, dtype=np.uint8)
            bufs.append(b)
    else:
        bufs = [rng.integers(0, 256, N * SL, dtype=np.uint8) for _ in range(NT)]
    res = {"threads": NT, "lanes": lanes, "buffers": kind, "affinity_cpus": len(info),
           "numa_nodes": sorted({v[2] for v in info.values()}),
           "buffer_nodes": sorted({page_node(b.ctypes.data + i * (1 << 21)) for b in bufs for i in range(0, 90, 30)}),
           "one_thread_GBps": None, "GBps": {}}
    res["one_thread_GBps"] = round(run_one(bufs[0], lanes), 3)
    for name, cpus in policies(info).items():
        if name != "unpinned" and cpus is None:
            continue
        res["GBps"][name] = round(run(cpus, bufs, lanes), 2)
    print(json.dumps(res), flush=True)


def run_one(b, lanes):
    out = (C.c_uint8 * (32 * N))()
    t = time.perf_counter()
    for i0 in range(0, N, lanes):
        lib.te_hash_leaves(C.cast(b.ctypes.data + i0 * SL, C.POINTER(C.c_uint8)), SL, min(lanes, N - i0), lanes, out)
    return N * SL / (time.perf_counter() - t) / 1e9


if __name__ == "__main__":
    main()
