"""Probe (not a test): one te_encode_commit_batch_host call over 1024 x 4 MiB pinned objects, for a
rocprofv3 --kernel-trace --memory-copy-trace timeline of the host pipeline."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import tape_amd as T  # noqa: E402
from tape_amd import batch  # noqa: E402

L, m = 4 << 20, 1024
s = T.Slicer.clay_default()
per = 20 * 715_048
h_in = torch.randint(0, 256, (m * L,), dtype=torch.uint8).pin_memory()
h_out = torch.empty(m * per, dtype=torch.uint8).pin_memory()
objs = [(i * L, L, i * per, 0) for i in range(m)]
leaf = torch.empty(m * 20 * 32, dtype=torch.uint8).pin_memory()
roots = torch.empty(m * 32, dtype=torch.uint8).pin_memory()
proofs = torch.empty(m * 20 * 5 * 32, dtype=torch.uint8).pin_memory()
w = int(sys.argv[1]) << 20 if len(sys.argv) > 1 else 1 << 30
if "null" in sys.argv[2:]:  # device work on torch's stream first, as bench.py does
    d = torch.ones(1 << 20, device="cuda")
    torch.cuda.synchronize()
    print("device work on the current stream first:", float(d.sum()))
if "resident" in sys.argv[2:]:  # bench.py's device-resident buffers
    d_in = torch.empty(m * L, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(m * per, dtype=torch.uint8, device="cuda")
    batch.encode_batch(s, d_in, batch.encode_descs([(i * L, L, i * per, 0) for i in range(m)]), d_out,
                       torch.cuda.current_stream())
    torch.cuda.synchronize()
    print("device-resident encode first")
for rep in range(2):
    t = time.perf_counter()
    batch.encode_commit_batch_host(s, h_in, objs, h_out, leaf, roots, proofs, window_bytes=w)
    print(f"window {w >> 20} MiB: {m * L / (time.perf_counter() - t) / 2**30:.2f} GiB/s", flush=True)
