import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch, numpy as np
import tape_amd as T
from tape_amd import batch
from oracle import oracle as O
N, MiB = 20, 1024 * 1024
o = O.OracleClay(20, 7, 16)
def run(sizes, mode):
    s0, s1 = T.Slicer.clay_default(), T.Slicer.clay_default()
    geo = [s0.geometry(L) for L in sizes]
    in_off, out_off = [], []; a = b = 0
    for L, g in zip(sizes, geo):
        in_off.append(a); out_off.append(b); a += L; b += N * g.slice_len
    h_in = torch.empty(max(1, a), dtype=torch.uint8).pin_memory()
    datas = [O.splitmix64_bytes(i + 31, L) for i, L in enumerate(sizes)]
    for i, d in enumerate(datas): h_in[in_off[i]:in_off[i] + sizes[i]] = torch.from_numpy(d)
    objs = [(in_off[i], sizes[i], out_off[i], i) for i in range(len(sizes))]
    h_out = torch.zeros(b, dtype=torch.uint8).pin_memory()
    if mode == "multi": batch.encode_batch_host_multi([s0, s1], h_in, objs, h_out, window_bytes=16 * MiB)
    elif mode == "single": batch.encode_batch_host(s0, h_in, objs, h_out, window_bytes=16 * MiB)
    else:
        d_in = h_in.cuda(); d_out = torch.zeros(b, dtype=torch.uint8, device="cuda")
        batch.encode_batch(s0, d_in, objs, d_out); torch.cuda.synchronize(); h_out = d_out.cpu()
    got = h_out.numpy()
    for i, L in enumerate(sizes):
        exp = np.frombuffer(b"".join(O.slicer_encode(o, datas[i].tobytes(), chunk_index=i)), np.uint8)
        g = got[out_off[i]:out_off[i] + N * geo[i].slice_len]
        bad = np.nonzero(g != exp)[0]
        if len(bad): print(mode, "obj", i, "size", L, "in_off%4", in_off[i] % 4, "nbad", len(bad), "first", bad[:8].tolist())
    print(mode, "done")
sizes = [4 * MiB, 1_000_003, 77, 2 * MiB + 5, 4 * MiB, 0, 3_333_333]
for m in ("device", "single", "multi"): run(sizes, m)
run([3, 77, 5, 1001, 77], "device")
