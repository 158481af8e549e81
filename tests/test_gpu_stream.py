"""GPU checks of te_stream_writer: the stream writer's ordered encode stage (sdk/src/stream/
write.rs:332-362 -- up to min(cores, 4) chunk encodes in flight, handed on in order through
FuturesOrdered), each window = BlobEncoder::encode_with_proofs of its objects (encoder.rs:220-260).

Several windows are submitted before the first wait; every window's slices equal the oracle's and
its leaf hashes / roots / proofs the merkle oracle's, and waits complete windows in order.
"""
import numpy as np
import pytest

import tape_amd as T
from tape_amd import batch

pytestmark = pytest.mark.gpu
N = 20
MiB = 1024 * 1024
H = T.SLICE_TREE_HEIGHT


def _window(oracle, s, sizes, seed):
    import torch
    geo = [s.geometry(L) for L in sizes]
    in_off, out_off, a, b = [], [], 0, 0
    for L, g in zip(sizes, geo):
        in_off.append(a)
        out_off.append(b)
        a += L
        b += N * g.slice_len
    datas = [oracle.splitmix64_bytes(seed + i, L) for i, L in enumerate(sizes)]
    h_in = torch.empty(max(1, a), dtype=torch.uint8).pin_memory()
    for i, d in enumerate(datas):
        h_in[in_off[i]:in_off[i] + sizes[i]] = torch.from_numpy(d)
    nobj = len(sizes)
    w = {"sizes": sizes, "geo": geo, "datas": datas, "out_off": out_off, "in": h_in,
         "objs": [(in_off[i], sizes[i], out_off[i], 0) for i in range(nobj)],
         "out": torch.zeros(max(1, b), dtype=torch.uint8).pin_memory(),
         "leaf": torch.zeros(nobj * N * 32, dtype=torch.uint8).pin_memory(),
         "root": torch.zeros(nobj * 32, dtype=torch.uint8).pin_memory(),
         "proof": torch.zeros(nobj * N * H * 32, dtype=torch.uint8).pin_memory()}
    return w


def _check(oracle, w):
    from oracle import merkle_oracle as O
    o = oracle.OracleClay(20, 7, 16)
    got, lb, rb, pb = (t.numpy().tobytes() for t in (w["out"], w["leaf"], w["root"], w["proof"]))
    for i, L in enumerate(w["sizes"]):
        sl_len = w["geo"][i].slice_len
        exp = oracle.slicer_encode(o, w["datas"][i].tobytes())
        assert got[w["out_off"][i]:w["out_off"][i] + N * sl_len] == b"".join(exp), i
        leaves, r, proofs = O.commit_slices(exp, H)
        assert lb[i * N * 32:(i + 1) * N * 32] == b"".join(leaves), i
        assert rb[i * 32:(i + 1) * 32] == r, i
        gp = [[pb[((i * N + j) * H + l) * 32:((i * N + j) * H + l + 1) * 32] for l in range(H)] for j in range(N)]
        assert gp == proofs, i


@pytest.mark.parametrize("hashing", ["device", "host"])
@pytest.mark.parametrize("handles,group", [(1, 0), (1, 20 * MiB), (2, 0)])
def test_stream_writer_windows_in_order(oracle, handles, group, hashing):
    """Four windows submitted before the first wait (one or two handles on device 0; small groups
    split a window into several hashing groups); waiting on ticket 3 completes 1..3 in order.
    Leaves hashed by the device's leaf kernel or by the host pool (host_hash.hpp)."""
    slicers = [T.Slicer.clay_default() for _ in range(handles)]
    sw = batch.StreamWriter(slicers, group_bytes=group, hashing=hashing)
    wins = [_window(oracle, slicers[0], sizes, 1000 * k) for k, sizes in enumerate(
        [[4 * MiB] * 3, [1_000_003, 0, 4 * MiB, 77], [3 * MiB + 5] * 4, [2 * MiB, 4 * MiB + 9]])]
    tickets = [sw.submit(w["in"], w["objs"], w["out"], w["leaf"], w["root"], w["proof"]) for w in wins]
    assert tickets == [1, 2, 3, 4]
    sw.wait(3)
    for w in wins[:3]:
        _check(oracle, w)
    sw.wait(4)
    _check(oracle, wins[3])
    # the pipeline persists across waits: more windows on the same writer
    more = [_window(oracle, slicers[0], [4 * MiB, 999], 7000 + k) for k in range(3)]
    t = [sw.submit(w["in"], w["objs"], w["out"], w["leaf"], w["root"], w["proof"]) for w in more]
    assert t == [5, 6, 7]
    sw.wait(7)
    for w in more:
        _check(oracle, w)
    sw.close()


def test_stream_writer_without_proofs(oracle):
    s = T.Slicer.clay_default()
    sw = batch.StreamWriter([s])
    w = _window(oracle, s, [4 * MiB, 2 * MiB], 55)
    t = sw.submit(w["in"], w["objs"], w["out"], w["leaf"], w["root"])
    sw.wait(t)
    from oracle import merkle_oracle as O
    exp = oracle.slicer_encode(oracle.OracleClay(20, 7, 16), w["datas"][0].tobytes())
    leaves, r, _ = O.commit_slices(exp, H)
    assert w["leaf"].numpy().tobytes()[:N * 32] == b"".join(leaves)
    assert w["root"].numpy().tobytes()[:32] == r
    assert not w["proof"].numpy().any()  # no proofs requested, none written
    sw.close()


@pytest.mark.skipif(T.device_count() < 2, reason="needs two HIP devices")
def test_stream_writer_two_devices(oracle):
    s0, s1 = T.Slicer.clay_default(), T.Slicer.clay_default()
    s1.coder.bind_device(1)
    sw = batch.StreamWriter([s0, s1])
    wins = [_window(oracle, s0, [4 * MiB, 3 * MiB], 300 * k) for k in range(4)]
    for w in wins:
        sw.submit(w["in"], w["objs"], w["out"], w["leaf"], w["root"], w["proof"])
    sw.wait(4)
    for w in wins:
        _check(oracle, w)
    sw.close()


def test_stream_writer_errors():
    s = T.Slicer.clay_default()
    sw = batch.StreamWriter([s])
    with pytest.raises(T.EngineError):
        sw.wait(1)  # never submitted
    sw.close()


def test_stream_writer_shared_group_waits(oracle):
    """Windows share a hashing group (default group size): a wait on the first window hashes the
    open group that also holds the second; windows with and without proofs share it; later
    windows open a new group on the same writer."""
    s = T.Slicer.clay_default()
    sw = batch.StreamWriter([s])
    w1 = _window(oracle, s, [4 * MiB, 5000], 4242)
    w2 = _window(oracle, s, [2 * MiB + 3], 4343)
    t1 = sw.submit(w1["in"], w1["objs"], w1["out"], w1["leaf"], w1["root"], w1["proof"])
    t2 = sw.submit(w2["in"], w2["objs"], w2["out"], w2["leaf"], w2["root"])  # no proofs
    sw.wait(t1)
    _check(oracle, w1)
    sw.wait(t2)
    from oracle import merkle_oracle as O
    exp = oracle.slicer_encode(oracle.OracleClay(20, 7, 16), w2["datas"][0].tobytes())
    leaves, r, _ = O.commit_slices(exp, H)
    assert w2["out"].numpy().tobytes()[:N * len(exp[0])] == b"".join(exp)
    assert w2["leaf"].numpy().tobytes()[:N * 32] == b"".join(leaves)
    assert w2["root"].numpy().tobytes()[:32] == r
    assert not w2["proof"].numpy().any()
    w3 = _window(oracle, s, [4 * MiB] * 2, 4444)
    t3 = sw.submit(w3["in"], w3["objs"], w3["out"], w3["leaf"], w3["root"], w3["proof"])
    assert t3 == 3
    sw.close()  # waits for the open group
    _check(oracle, w3)


@pytest.mark.parametrize("hashing", ["auto", "device"])
def test_stream_writer_sdk_chunk_shape(oracle, hashing):
    """The SDK's stream shape (sdk/src/stream/write.rs:54-57, 219, 332-362; manifest.rs:22): a
    stream cut into MAX_TRACK_SIZE = 64 MiB chunks (the last one short), one encode_with_proofs
    window per chunk, at most MAX_ENCODE_WORKERS = 4 in flight -- the 5th chunk is submitted only
    after the oldest has been waited for.  "auto" hashes these 9.7 MB slices on the host pool; the
    device leaf kernel must give the same bytes."""
    import collections
    s = T.Slicer.clay_default()
    sw = batch.StreamWriter([s], hashing=hashing)
    sizes = [64 * MiB] * 5 + [13 * MiB + 5] if hashing == "auto" else [64 * MiB, 64 * MiB + 0, 5 * MiB + 3]
    wins, inflight = [], collections.deque()
    for k, L in enumerate(sizes):
        if len(inflight) >= 4:
            sw.wait(inflight.popleft())
        w = _window(oracle, s, [L], 90_000 + 17 * k)
        wins.append(w)
        inflight.append(sw.submit(w["in"], w["objs"], w["out"], w["leaf"], w["root"], w["proof"]))
    sw.wait(inflight[-1])
    for w in wins:
        _check(oracle, w)
    sw.close()


def test_stream_writer_row_pieces_mixed(oracle):
    """Host-hashed windows into pinned output: objects with slices >= 2 MiB are copied out in 1 MiB
    row pieces and hashed as the pieces land (the last piece short), smaller ones in one copy hashed
    after the window's copies -- both kinds in one window, and windows of each kind back to back."""
    s = T.Slicer.clay_default()
    sw = batch.StreamWriter([s], hashing="host")
    wins = [_window(oracle, s, sizes, 60_000 + 11 * k) for k, sizes in enumerate(
        [[20 * MiB + 7, 4 * MiB, 1000], [15 * MiB], [3 * MiB, 14 * MiB + 1], [0, 1]])]
    tickets = [sw.submit(w["in"], w["objs"], w["out"], w["leaf"], w["root"], w["proof"]) for w in wins]
    sw.wait(tickets[-1])
    for w in wins:
        _check(oracle, w)
    sw.close()


def test_stream_writer_failed_window_is_isolated(oracle):
    """A window that fails its checks (an object too large for 32-bit slices: TooMuchData) fails
    alone: the windows before it, sharing its device's open hashing group, and after it complete
    with the right bytes (one bad window used to fail every window of the group)."""
    s = T.Slicer.clay_default()
    sw = batch.StreamWriter([s], hashing="device")
    w1 = _window(oracle, s, [4 * MiB, 3 * MiB], 31)
    w3 = _window(oracle, s, [2 * MiB + 1], 33)
    t1 = sw.submit(w1["in"], w1["objs"], w1["out"], w1["leaf"], w1["root"], w1["proof"])
    bad = _window(oracle, s, [16], 32)
    with pytest.raises(T.EncodeError):
        sw.submit(bad["in"], [(0, 1 << 40, 0, 0)], bad["out"], bad["leaf"], bad["root"])
    t3 = sw.submit(w3["in"], w3["objs"], w3["out"], w3["leaf"], w3["root"], w3["proof"])
    assert (t1, t3) == (1, 3)
    sw.wait(t1)
    _check(oracle, w1)
    with pytest.raises(T.EncodeError):
        sw.wait(t3)  # completes ticket 2 (failed) and 3
    _check(oracle, w3)
    sw.close()


def test_host_hashing_one_shot(oracle):
    """te_encode_commit_batch_host with the host pool forced (te_set_commit_hashing): same slices,
    leaves, roots and proofs as the oracle; back to auto afterwards."""
    s = T.Slicer.clay_default()
    w = _window(oracle, s, [4 * MiB, 1_000_001, 4 * MiB + 8, 18 * MiB + 3], 4711)  # the last in row pieces
    batch.set_commit_hashing("host")
    try:
        batch.encode_commit_batch_host(s, w["in"], w["objs"], w["out"], w["leaf"], w["root"], w["proof"])
    finally:
        batch.set_commit_hashing("auto")
    _check(oracle, w)


def test_pinned_host_buffers(oracle):
    """te_host_alloc / te_host_register: encode_batch_host from and into pinned
    buffers the library allocated, and from a pageable array pinned in place, equal the oracle."""
    s = T.Slicer.clay_default()
    sizes = [4 * MiB, 1_234_567]
    geo = [s.geometry(L) for L in sizes]
    datas = [oracle.splitmix64_bytes(77 + i, L) for i, L in enumerate(sizes)]
    per = [N * g.slice_len for g in geo]
    objs = [(0, sizes[0], 0, 0), (sizes[0], sizes[1], per[0], 0)]
    exp = b"".join(b"".join(oracle.slicer_encode(oracle.OracleClay(20, 7, 16), d.tobytes())) for d in datas)
    h_in = batch.host_empty(sum(sizes))
    h_in[:] = np.concatenate(datas)
    h_out = batch.host_empty(sum(per))
    batch.encode_batch_host(s, h_in, objs, h_out)
    assert h_out.tobytes() == exp
    del h_in, h_out  # freed by their finalizers
    p_in = np.concatenate(datas)
    p_out = np.zeros(sum(per), np.uint8)
    batch.host_register(p_in)
    batch.host_register(p_out)
    try:
        batch.encode_batch_host(s, p_in, objs, p_out)
    finally:
        batch.host_unregister(p_in)
        batch.host_unregister(p_out)
    assert p_out.tobytes() == exp
