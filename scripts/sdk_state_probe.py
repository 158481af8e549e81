"""Which earlier leg of the default bench line leaves the SDK-shape stream leg slow (r05: 7.2 GiB/s
and 33.7 ms chunk latency inside the default line; 15.5 GiB/s and 15-20 ms in a fresh --mode
stream process).  One process: the SDK leg fresh, then after each earlier leg in turn.
  python scripts/sdk_state_probe.py [steps...]   steps: sdk copy commit_win trim"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import tape_amd as T  # noqa: E402
from tape_amd import batch  # noqa: E402

seq = sys.argv[1:] or ["sdk", "copy", "sdk", "commit_win", "sdk", "trim", "sdk"]
args = argparse.Namespace(sdk_chunks=16, cpu_sample=0, copy_objects=-1, copy_steps=2, objects=1024)
dev = torch.device("cuda:0")
s = T.Slicer.clay_default()
L = 4 << 20
g = s.geometry(L)
per = 20 * g.slice_len
n = args.objects
d_in = torch.empty(n * L, dtype=torch.uint8, device=dev)
bench.splitmix_fill(torch, d_in, 0, n, L)
d_out = torch.empty(n * per, dtype=torch.uint8, device=dev)
batch.encode_batch(s, d_in, [(i * L, L, i * per, 0) for i in range(n)], d_out)
torch.cuda.synchronize()




for st in seq:
    t = time.perf_counter()
    if st == "sdk":
        r = bench.stream_sdk_short(args, torch, None, 1, 0, dev, T, batch)
        out = {"GiBps": r["value"], "lat": r["chunk_latency_ms_p50_p90"], "ok": r["outputs_verified"]}
    elif st == "copy":
        r = bench.copy_inclusive(args, torch, None, 1, s, batch, d_in, d_out, per, L, dev)
        out = {"GiBps": r["value"]}
    elif st == "commit_win":
        r = bench.copy_inclusive_commit(args, torch, None, 1, s, batch, d_in, d_out, per, L, dev)
        out = {"by_window": r["by_window"], "stream": r["stream_writer"]}
    elif st == "trim":  # hand the caching host allocator's pinned blocks back
        torch._C._host_emptyCache() if hasattr(torch._C, "_host_emptyCache") else None
        out = {}
    else:
        continue
    print(st, round(time.perf_counter() - t, 1), "s", json.dumps(out), flush=True)
