"""GPU checks of the engine around the kernels: device binding, concurrency, windowed recover,
multi-handle host pipelines and the bench's per-rank object partition.

Every output is compared byte for byte with the oracle restatement or with the original slices.
"""
import os
import random
import threading

import numpy as np
import pytest

import tape_amd as T
from tape_amd import batch

pytestmark = pytest.mark.gpu
N = 20
MiB = 1024 * 1024


def test_handle_from_a_thread_that_never_set_a_device(oracle):
    """te_clay binds to its creating thread's device; calls from another thread (which never
    called te_set_device / hipSetDevice) run there and leave that thread's device alone."""
    s = T.Slicer.clay_default()
    assert s.coder.device() == 0
    data = oracle.splitmix64_bytes(0xB1D, 2_345_679).tobytes()
    exp = oracle.slicer_encode(oracle.OracleClay(20, 7, 16), data)
    got = {}

    def worker():
        got["sl"] = s.encode(data)
        got["dec"] = s.decode([(i, got["sl"][i]) for i in range(13, 20)])

    th = threading.Thread(target=worker)
    th.start()
    th.join()
    assert got["sl"] == exp
    assert got["dec"] == data
    s.coder.bind_device(0)  # re-binding drains and frees the device state; the handle still works
    assert s.coder.device() == 0
    assert s.encode(data) == exp


def test_recover_two_threads_two_streams(oracle):
    """Two recover batches on one handle from two threads on two streams: the shared workspaces
    are ordered by the handle's event (no silent cross-stream reuse)."""
    import torch
    s = T.Slicer.clay_default()
    L = 1_500_001
    g = s.geometry(L)
    per = N * g.slice_len
    nobj = 8
    host = bytearray()
    sl_all = []
    for o in range(nobj):
        sl = s.encode(oracle.splitmix64_bytes(o + 100, L).tobytes())
        sl_all.append(sl)
        host += b"".join(sl)
    metas = b"".join(sl[0][-48:] for sl in sl_all)
    dev = torch.frombuffer(host, dtype=torch.uint8).cuda()
    outs, streams, jobs = [], [], []
    for t in range(2):
        rnd = random.Random(t)
        objs, exp = [], []
        for o in range(nobj):
            lost = rnd.randrange(N)
            avail = rnd.sample([i for i in range(N) if i != lost], 7)
            objs.append((o * per, g.slice_len, sum(1 << i for i in avail), lost, o * g.slice_len))
            exp.append(sl_all[o][lost])
        outs.append(torch.empty(nobj * g.slice_len, dtype=torch.uint8, device="cuda"))
        streams.append(torch.cuda.Stream())
        jobs.append((objs, b"".join(exp)))
    errs = []

    def run(t):
        try:
            for _ in range(3):
                batch.recover_batch(s, dev, jobs[t][0], metas, outs[t], streams[t])
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    ths = [threading.Thread(target=run, args=(t,)) for t in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    torch.cuda.synchronize()
    assert not errs, errs
    for t in range(2):
        assert outs[t].cpu().numpy().tobytes() == jobs[t][1], t


@pytest.mark.parametrize("window", ["1", str(3 * MiB)])
def test_recover_in_windows(oracle, window):
    """te_recover_batch_device in bounded windows (TEC_RECOVER_WINDOW_BYTES forces one object per
    window, or a few), data-lost and parity-lost stripes, an empty blob and a ragged tail."""
    import torch
    s = T.Slicer.clay_default()
    sizes = [4 * MiB, 0, 1_000_001, 999, 3 * MiB + 7]
    objs, exp, host, metas = [], [], bytearray(), b""
    off = out_off = 0
    for o, L in enumerate(sizes):
        sl = s.encode(oracle.splitmix64_bytes(o * 7 + 1, L).tobytes())
        slen = len(sl[0])
        host += b"".join(sl)
        for lost in (o % N, (o * 7 + 13) % N):
            avail = [(lost + 1 + j) % N for j in range(7)]
            objs.append((off, slen, sum(1 << i for i in avail), lost, out_off))
            exp.append(sl[lost])
            metas += sl[0][-48:]
            out_off += slen
        off += N * slen
    dev = torch.frombuffer(host, dtype=torch.uint8).cuda()
    out = torch.zeros(out_off, dtype=torch.uint8, device="cuda")
    os.environ["TEC_DEBUG_KNOBS"] = "1"  # measurement knobs are read only with this set
    os.environ["TEC_RECOVER_WINDOW_BYTES"] = window
    try:
        batch.recover_batch(s, dev, objs, metas, out)
        torch.cuda.synchronize()
    finally:
        del os.environ["TEC_RECOVER_WINDOW_BYTES"]
        del os.environ["TEC_DEBUG_KNOBS"]
    assert out.cpu().numpy().tobytes() == b"".join(exp)


def test_recover_rejects_inconsistent_peers(oracle):
    s = T.Slicer.clay_default()
    sl = s.encode(oracle.splitmix64_bytes(3, 200_000).tobytes())
    with pytest.raises(T.DecodeError):
        batch.reconstruct(s, 0, [(i, sl[i]) for i in range(1, 8)] + [(9, sl[9][:-1])])
    with pytest.raises(T.DecodeError):
        batch.reconstruct(s, 0, [(i, sl[i]) for i in range(1, 8)] + [(1, sl[1])])


def test_encode_batch_host_multi(oracle):
    """te_encode_batch_host_multi over two handles (here both on device 0): same bytes as one
    host pipeline, objects split into contiguous ranges."""
    import torch
    s0, s1 = T.Slicer.clay_default(), T.Slicer.clay_default()
    sizes = [4 * MiB, 1_000_003, 77, 2 * MiB + 5, 4 * MiB, 0, 3_333_333]
    geo = [s0.geometry(L) for L in sizes]
    in_off, out_off = [], []
    a = b = 0
    for L, g in zip(sizes, geo):
        in_off.append(a)
        out_off.append(b)
        a += L
        b += N * g.slice_len
    h_in = torch.empty(max(1, a), dtype=torch.uint8).pin_memory()
    datas = [oracle.splitmix64_bytes(i + 31, L) for i, L in enumerate(sizes)]
    for i, d in enumerate(datas):
        h_in[in_off[i]:in_off[i] + sizes[i]] = torch.from_numpy(d)
    objs = [(in_off[i], sizes[i], out_off[i], i) for i in range(len(sizes))]
    h_out = torch.zeros(b, dtype=torch.uint8).pin_memory()
    batch.encode_batch_host_multi([s0, s1], h_in, objs, h_out, window_bytes=16 * MiB)
    o = oracle.OracleClay(20, 7, 16)
    got = h_out.numpy()
    for i, L in enumerate(sizes):
        exp = b"".join(oracle.slicer_encode(o, datas[i].tobytes(), chunk_index=i))
        assert got[out_off[i]:out_off[i] + N * geo[i].slice_len].tobytes() == exp, i


@pytest.mark.skipif(T.device_count() < 2, reason="needs two HIP devices")
def test_encode_batch_host_multi_two_devices(oracle):
    """The SDK shape of DESIGN §6: one process, one handle per GPU (devices 0 and 1), launched
    from two host threads at once -- each thread's first launch raises the kernels' LDS limit on
    its own device (ensure_dyn_lds); bytes equal the oracle's."""
    import torch
    s0, s1 = T.Slicer.clay_default(), T.Slicer.clay_default()
    s1.coder.bind_device(1)
    assert (s0.coder.device(), s1.coder.device()) == (0, 1)
    sizes = [4 * MiB, 1_000_003, 4 * MiB, 3_333_333, 2 * MiB + 5, 4 * MiB]
    geo = [s0.geometry(L) for L in sizes]
    in_off, out_off, a, b = [], [], 0, 0
    for L, g in zip(sizes, geo):
        in_off.append(a)
        out_off.append(b)
        a += L
        b += N * g.slice_len
    datas = [oracle.splitmix64_bytes(i + 91, L) for i, L in enumerate(sizes)]
    h_in = torch.from_numpy(np.concatenate(datas)).pin_memory()
    h_out = torch.zeros(b, dtype=torch.uint8).pin_memory()
    objs = [(in_off[i], sizes[i], out_off[i], 0) for i in range(len(sizes))]
    batch.encode_batch_host_multi([s0, s1], h_in, objs, h_out, window_bytes=8 * MiB)
    o = oracle.OracleClay(20, 7, 16)
    got = h_out.numpy()
    for i, L in enumerate(sizes):
        exp = b"".join(oracle.slicer_encode(o, datas[i].tobytes()))
        assert got[out_off[i]:out_off[i] + N * geo[i].slice_len].tobytes() == exp, i


def test_rank_partition_matches_oracle(oracle):
    """bench.py's multi-GPU partition: rank 3 of 8 owns global objects
    6144.. of the 16,384-object stream; its device-generated SplitMix64 objects and their HIP
    encodes equal the oracle's for that global id range (sampled)."""
    import torch
    import bench
    rank, per_rank = 3, 2048
    first, last = bench.rank_objects(rank, per_rank)
    assert (first, last) == (6144, 8192)
    sample = [0, 1, 1023, 2047]  # local indices
    L = 4 * MiB
    d_in = torch.empty(len(sample) * L, dtype=torch.uint8, device="cuda")
    for j, i in enumerate(sample):
        bench.splitmix_fill(torch, d_in[j * L:(j + 1) * L], first + i, 1, L)
    s = T.Slicer.clay_default()
    g = s.geometry(L)
    per = N * g.slice_len
    d_out = torch.empty(len(sample) * per, dtype=torch.uint8, device="cuda")
    batch.encode_batch(s, d_in, [(j * L, L, j * per, 0) for j in range(len(sample))], d_out)
    torch.cuda.synchronize()
    o = oracle.OracleClay(20, 7, 16)
    for j, i in enumerate(sample):
        data = oracle.splitmix64_bytes(0x7A9E5EED ^ (first + i), L)
        assert np.array_equal(d_in[j * L:(j + 1) * L].cpu().numpy(), data), i
        exp = b"".join(oracle.slicer_encode(o, data.tobytes()))
        assert d_out[j * per:(j + 1) * per].cpu().numpy().tobytes() == exp, i


@pytest.mark.parametrize("sizes", [[3, 77, 5, 1001, 77, 100_003], [4 * MiB + 1, 1_000_003, 2_345_679]])
def test_odd_offsets_encode_decode(oracle, sizes):
    """Objects packed back to back at odd device offsets (every alignment mod 4): encode equals
    the oracle, and decode into odd output offsets returns the objects."""
    import torch
    s = T.Slicer.clay_default()
    o = oracle.OracleClay(20, 7, 16)
    geo = [s.geometry(L) for L in sizes]
    in_off, out_off, a, b = [], [], 1, 0  # start at an odd offset
    for L, g in zip(sizes, geo):
        in_off.append(a)
        out_off.append(b)
        a += L
        b += N * g.slice_len
    datas = [oracle.splitmix64_bytes(i * 13 + 5, L) for i, L in enumerate(sizes)]
    h_in = np.zeros(a + 16, np.uint8)
    for i, d in enumerate(datas):
        h_in[in_off[i]:in_off[i] + sizes[i]] = d
    d_in = torch.from_numpy(h_in).cuda()
    d_out = torch.zeros(b, dtype=torch.uint8, device="cuda")
    batch.encode_batch(s, d_in, [(in_off[i], sizes[i], out_off[i], 0) for i in range(len(sizes))], d_out)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    for i in range(len(sizes)):
        exp = b"".join(oracle.slicer_encode(o, datas[i].tobytes()))
        assert got[out_off[i]:out_off[i] + N * geo[i].slice_len].tobytes() == exp, i
    # decode (slices 0..12 erased) into odd output offsets
    metas = b"".join(got[out_off[i] + geo[i].slice_len - 48:out_off[i] + geo[i].slice_len].tobytes()
                     for i in range(len(sizes)))
    dec_off, c = [], 3
    for L in sizes:
        dec_off.append(c)
        c += L
    d_dec = torch.zeros(c + 16, dtype=torch.uint8, device="cuda")
    mask = sum(1 << j for j in range(13, 20))
    batch.decode_batch(s, d_out, [(out_off[i], geo[i].slice_len, mask, dec_off[i]) for i in range(len(sizes))],
                       metas, d_dec)
    torch.cuda.synchronize()
    dec = d_dec.cpu().numpy()
    for i, L in enumerate(sizes):
        assert np.array_equal(dec[dec_off[i]:dec_off[i] + L], datas[i]), i
    assert not dec[:3].any() and not dec[c:].any()  # nothing written outside the objects


@pytest.mark.parametrize("window", [0, 24 * MiB, 64 * MiB])
def test_encode_commit_batch_host(oracle, window):
    """te_encode_commit_batch_host = BlobEncoder::encode_with_proofs per object (encoder.rs:220-260)
    over a host -> host pipeline: slices equal the oracle's, leaf hashes / roots / proofs equal the
    merkle oracle's; mixed sizes (runs of equal slice length), an empty blob, several windows."""
    import torch
    from oracle import merkle_oracle as O
    s = T.Slicer.clay_default()
    sizes = [4 * MiB, 4 * MiB, 4 * MiB, 1_000_003, 0, 77, 3 * MiB + 5, 3 * MiB + 5]
    geo = [s.geometry(L) for L in sizes]
    in_off, out_off, a, b = [], [], 0, 0
    for L, g in zip(sizes, geo):
        in_off.append(a)
        out_off.append(b)
        a += L
        b += N * g.slice_len
    datas = [oracle.splitmix64_bytes(i + 71, L) for i, L in enumerate(sizes)]
    h_in = torch.empty(max(1, a), dtype=torch.uint8).pin_memory()
    for i, d in enumerate(datas):
        h_in[in_off[i]:in_off[i] + sizes[i]] = torch.from_numpy(d)
    h_out = torch.zeros(b, dtype=torch.uint8).pin_memory()
    nobj, H = len(sizes), T.SLICE_TREE_HEIGHT
    leaf = torch.zeros(nobj * N * 32, dtype=torch.uint8).pin_memory()
    root = torch.zeros(nobj * 32, dtype=torch.uint8).pin_memory()
    proof = torch.zeros(nobj * N * H * 32, dtype=torch.uint8).pin_memory()
    objs = [(in_off[i], sizes[i], out_off[i], i) for i in range(nobj)]
    batch.encode_commit_batch_host(s, h_in, objs, h_out, leaf, root, proof, window_bytes=window)
    o = oracle.OracleClay(20, 7, 16)
    got, lb, rb, pb = (t.numpy().tobytes() for t in (h_out, leaf, root, proof))
    for i, L in enumerate(sizes):
        sl_len = geo[i].slice_len
        exp = oracle.slicer_encode(o, datas[i].tobytes(), chunk_index=i)
        assert got[out_off[i]:out_off[i] + N * sl_len] == b"".join(exp), i
        leaves, r, proofs = O.commit_slices(exp, H)
        assert lb[i * N * 32:(i + 1) * N * 32] == b"".join(leaves), i
        assert rb[i * 32:(i + 1) * 32] == r, i
        gp = [[pb[((i * N + j) * H + l) * 32:((i * N + j) * H + l + 1) * 32] for l in range(H)] for j in range(N)]
        assert gp == proofs, i


def test_node_repair_over_the_wire(oracle):
    """The node's repair_track flow (network/node/src/features/spool/repair.rs:271-350, test
    clay_repair): plan, one RepairRequest per helper, each helper serves it from its stored slice,
    Slicer::repair on the GPU rebuilds the lost slice."""
    s = T.Slicer.clay_default()
    data = oracle.splitmix64_bytes(0xC1A7, 3_000_001).tobytes()
    sl = s.encode(data)
    for lost in (2, 17):
        avail = [i for i in range(N) if i != lost]
        plan = s.repair_plan(lost, avail, sl[avail[0]])
        served = {h: T.serve_repair_request(s.coder, sl[h], T.repair_request(plan, h)) for h in avail}
        served = {h: v for h, v in served.items() if v}
        assert s.repair(plan, served, sl[avail[0]][-48:]) == sl[lost], lost
