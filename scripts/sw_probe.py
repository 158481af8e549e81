"""Stream-writer probe (not product code): te_stream_writer over 1024 x 4 MiB pinned objects in
windows of W objects, <= 4 in flight (bench.py's protocol), each size timed R times; and the
one-shot te_encode_commit_batch_host.   python scripts/sw_probe.py [group_GiB]"""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tape_amd as T
from tape_amd import batch

m, L, N, H = 1024, 4 << 20, 20, 5
gb = int(float(sys.argv[1]) * (1 << 30)) if len(sys.argv) > 1 else 4 << 30
only = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [32, 64, 128, 256]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
s = T.Slicer.clay_default()
per = s.geometry(L).slice_len * N
h_in = torch.randint(0, 256, (m * L,), dtype=torch.uint8).pin_memory()
h_out = torch.empty(m * per, dtype=torch.uint8).pin_memory()
leaf = torch.empty(m * N * 32, dtype=torch.uint8).pin_memory()
root = torch.empty(m * 32, dtype=torch.uint8).pin_memory()
proof = torch.empty(m * N * H * 32, dtype=torch.uint8).pin_memory()
objs = batch.encode_descs([(i * L, L, i * per, 0) for i in range(m)])
batch.encode_commit_batch_host(s, h_in, objs, h_out, leaf, root, proof, window_bytes=4 << 30)
t = time.perf_counter()
batch.encode_commit_batch_host(s, h_in, objs, h_out, leaf, root, proof, window_bytes=4 << 30)
print("one-shot 4GiB groups", round(m * L / (time.perf_counter() - t) / 2**30, 2), "GiB/s", flush=True)
sw = batch.StreamWriter([s], height=H, group_bytes=gb)


def run(wobj):
    t = 0
    for a in range(0, m, wobj):
        b = min(m, a + wobj)
        o = batch.encode_descs([(i * L, L, i * per, 0) for i in range(a, b)])
        t = sw.submit(h_in, o, h_out, leaf[a * N * 32:], root[a * 32:], proof[a * N * H * 32:])
        if t > 4:
            sw.wait(t - 4)
    sw.wait(t)


for wobj in only:
    run(wobj)
    r = []
    for _ in range(reps):
        t0 = time.perf_counter()
        run(wobj)
        r.append(round(m * L / (time.perf_counter() - t0) / 2**30, 2))
    print(f"group {gb >> 20} MiB window {wobj}: {r} GiB/s", flush=True)
sw.close()
