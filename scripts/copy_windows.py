"""Probe (not a test): copy-inclusive encode rate of te_encode_batch_host vs window size, 1024 x
4 MiB pinned objects (bench.py's copy_inclusive leg uses the library default, 1 GiB)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tape_amd as T  # noqa: E402
from tape_amd import batch  # noqa: E402

L, m = 4 << 20, 1024
s = T.Slicer.clay_default()
per = 20 * s.geometry(L).slice_len if hasattr(s, "geometry") else 20 * 715_048
h_in = torch.randint(0, 256, (m * L,), dtype=torch.uint8).pin_memory()
h_out = torch.empty(m * per, dtype=torch.uint8).pin_memory()
objs = batch.encode_descs([(i * L, L, i * per, 0) for i in range(m)])
for w in [int(x) << 20 for x in (sys.argv[1:] or ["256", "512", "1024", "2048"])]:
    batch.encode_batch_host(s, h_in, objs, h_out, w)
    t = time.perf_counter()
    for _ in range(2):
        batch.encode_batch_host(s, h_in, objs, h_out, w)
    el = (time.perf_counter() - t) / 2
    print(f"window {w >> 20:5d} MiB: {m * L / el / 2**30:6.2f} GiB/s ({el * 1e3:.1f} ms per batch)", flush=True)
