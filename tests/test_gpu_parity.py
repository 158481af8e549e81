"""GPU parity: libtapeec (gfx950 kernels) vs the CPU oracle, bit-exact, through the C ABI.

Bar: integer/byte work -> every output byte identical to the oracle restatement on the same seeded
inputs (encode: all 20 slices incl. metadata; decode: the blob; repair: the slice).  Full-size
(BASELINE) batches are checked through size-independent properties (decode(encode) round trip,
repair == encode) plus oracle hash comparison on a sample.
"""
import hashlib
import random

import numpy as np
import pytest

import tape_amd as T

pytestmark = pytest.mark.gpu
N = 20
MiB = 1024 * 1024


def _sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.fixture(scope="module")
def o716(oracle):
    return oracle.OracleClay(20, 7, 16)


@pytest.fixture(scope="module")
def o1019(oracle):
    return oracle.OracleClay(20, 10, 19)


# ---------------------------------------------------------------- raw ClayCoder ----------
@pytest.mark.parametrize("params", [(20, 7, 16), (20, 10, 19), (20, 5, 14), (12, 8, 11), (20, 7, 19), (6, 3, 5)])
@pytest.mark.parametrize("ln", [1, 100, 1400, 10_000, 123_457])
def test_clay_encode_matches_oracle(oracle, params, ln):
    c = T.ClayCoder(*params)
    o = oracle.OracleClay(*params)
    data = oracle.splitmix64_bytes(ln * 31 + params[1], ln).tobytes()
    assert c.encode(data) == o.encode(data)


@pytest.mark.parametrize("params", [(20, 7, 16), (20, 8, 17), (20, 9, 18), (20, 10, 19), (20, 5, 14), (12, 8, 11),
                                    (20, 7, 19)])
def test_clay_decode_any_k(oracle, params):
    c = T.ClayCoder(*params)
    n, k, _ = params
    data = oracle.splitmix64_bytes(77, 50_000).tobytes()
    ch = c.encode(data)
    rnd = random.Random(params[1])
    patterns = [list(range(k)), list(range(n - k, n)), list(range(n))]
    patterns += [sorted(rnd.sample(range(n), rnd.randint(k, n))) for _ in range(25)]
    for keep in patterns:
        rec = c.decode([(i, ch[i]) for i in keep])
        assert rec[:len(data)] == data, keep


@pytest.mark.parametrize("params", [(20, 7, 16), (20, 10, 19), (20, 5, 14), (12, 8, 11), (20, 7, 19)])
def test_clay_repair_every_lost(oracle, params):
    c = T.ClayCoder(*params)
    n = params[0]
    data = oracle.splitmix64_bytes(5, 40_000).tobytes()
    ch = c.encode(data)
    cs = len(ch[0])
    sc = cs // c.alpha()
    for lost in range(n):
        plan = c.plan_repair(lost, [i for i in range(n) if i != lost])
        helpers = {h: b"".join(ch[h][z * sc:(z + 1) * sc] for z in pl) for h, pl in plan}
        assert c.repair(lost, helpers, cs) == ch[lost], lost


# ---------------------------------------------------------------- Slicer --------------------
@pytest.mark.parametrize("rotated", [True, False])
@pytest.mark.parametrize("ln", [0, 1, 500, 1000, 10_000, 100_000, 250_000, 1_000_001, MiB, 4 * MiB])
def test_slicer_encode_matches_oracle(oracle, o716, rotated, ln):
    data = oracle.splitmix64_bytes(0x7A9E5EED ^ ln, ln).tobytes()
    s = T.Slicer.clay_default() if rotated else T.Slicer.new(T.ClayCoder(20, 7, 16))
    got = s.encode(data)
    exp = oracle.slicer_encode(o716, data, rotated=rotated)
    assert len(got) == N
    for i in range(N):
        assert got[i] == exp[i], f"slice {i}"


def test_slicer_encode_reference_pattern(oracle, o716):  # (i % 251) payloads, slicer.rs:397-399
    s = T.Slicer.clay_default()
    for ln in (1000, 1_048_576):
        p = oracle.test_pattern(ln)
        assert s.encode(p) == oracle.slicer_encode(o716, p)


def test_slicer_chunk_index(oracle, o716):
    s = T.Slicer.clay_default()
    s.set_chunk_index(9)
    data = bytes(1000)
    assert s.encode(data) == oracle.slicer_encode(o716, data, chunk_index=9)


@pytest.mark.parametrize("params", [(20, 10, 19)])
@pytest.mark.parametrize("ln", [500, 3000, 5000, 250_000])
def test_slicer_1019_roundtrip(oracle, params, ln):  # slicer.rs:472-566 on the GPU path
    for rotated in (False, True):
        s = T.Slicer.with_profile(T.ClayCoder(*params), 1024, rotated, T.EncodingProfile.clay_default())
        payload = oracle.test_pattern(ln)
        sl = s.encode(payload)
        o = oracle.OracleClay(*params)
        assert sl == oracle.slicer_encode(o, payload, rotated=rotated)
        assert s.decode(list(enumerate(sl))) == payload
        assert s.decode([(i, sl[i]) for i in range(10)]) == payload
        with pytest.raises(T.DecodeError) as e:
            s.decode([(i, sl[i]) for i in range(9)])
        assert e.value.variant == "NotEnoughSlices"


def test_slicer_empty_roundtrip():
    s = T.Slicer.clay_default()
    sl = s.encode(b"")
    assert len(sl) == N and len(sl[0]) == 14_448
    assert s.decode(list(enumerate(sl))) == b""


def test_slicer_decode_patterns_4mib(oracle):
    s = T.Slicer.clay_default()
    data = oracle.splitmix64_bytes(21, 4 * MiB).tobytes()
    sl = s.encode(data)
    rnd = random.Random(3)
    pats = [list(range(13, 20)), list(range(7)), list(range(0, 20, 3))]
    pats += [sorted(rnd.sample(range(N), rnd.randint(7, 19))) for _ in range(6)]
    for keep in pats:
        assert s.decode([(i, sl[i]) for i in keep]) == data, keep


@pytest.mark.parametrize("ln", [1, 999, 14_001, 100_003, 1_000_001])
def test_slicer_decode_ragged_patterns(oracle, ln):
    # staged decode: output shares ending inside a data row (ragged blobs, stripe < k * cs), every
    # erasure count from 0 to n - k, both slice layouts
    data = oracle.splitmix64_bytes(ln ^ 0x5EED, ln).tobytes()
    rnd = random.Random(ln)
    for rotated in (True, False):
        s = T.Slicer.clay_default() if rotated else T.Slicer.new(T.ClayCoder(20, 7, 16))
        sl = s.encode(data)
        for ne in range(0, 14):
            keep = sorted(rnd.sample(range(N), N - ne))
            assert s.decode([(i, sl[i]) for i in keep]) == data, (rotated, keep)


def test_slicer_layout_errors(oracle):
    s = T.Slicer.clay_default()
    sl = s.encode(oracle.test_pattern(2000))
    bad = [(i, x) for i, x in enumerate(sl)]
    bad[1] = (1, sl[1][:-1])
    with pytest.raises(T.DecodeError):
        s.decode(bad)


@pytest.mark.parametrize("ln", [10_000, 300_000, 4 * MiB])
def test_slicer_repair_every_lost(oracle, o716, ln):
    s = T.Slicer.clay_default()
    data = oracle.splitmix64_bytes(ln, ln).tobytes()
    sl = s.encode(data)
    for lost in range(N):
        helpers = [(i, sl[i]) for i in range(N) if i != lost]
        assert s.repair_full(lost, helpers) == sl[lost], lost


def test_slicer_repair_exactly_d_and_insufficient(oracle):  # repair.rs:531-549, 615-633
    s = T.Slicer.with_stripe_size(T.ClayCoder(20, 10, 19), 100_000)
    sl = s.encode(oracle.test_pattern(10_000))
    d = s.coder.d()
    assert s.repair_full(0, [(i, sl[i]) for i in range(1, 1 + d)]) == sl[0]
    with pytest.raises(T.RepairError):
        s.repair_full(0, [(i, sl[i]) for i in range(1, d)])


def test_slicer_repair_missing_helper(oracle):
    s = T.Slicer.clay_default()
    sl = s.encode(oracle.test_pattern(50_000))
    avail = list(range(1, N))
    plan = s.repair_plan(0, avail, sl[1])
    partial = {i: T.extract_repair_data(sl[i], plan, i) for i in avail}
    del partial[avail[0]]
    with pytest.raises(T.RepairError) as e:
        s.repair(plan, partial, sl[1][-48:])
    assert e.value.variant == "MissingHelper"


# ---------------------------------------------------------------- device batch API ----------
torch = pytest.importorskip("torch")


def test_batch_encode_decode_repair_device(oracle, o716):
    from tape_amd import batch
    nobj, L = 12, 4 * MiB
    dev = torch.device("cuda:0")
    host = np.concatenate([oracle.splitmix64_bytes(0x7A9E5EED ^ i, L) for i in range(nobj)])
    d_in = torch.from_numpy(host).to(dev)
    s = T.Slicer.clay_default()
    g = s.geometry(L)
    per = N * g.slice_len
    d_out = torch.zeros(nobj * per, dtype=torch.uint8, device=dev)
    batch.encode_batch(s, d_in, [(i * L, L, i * per, i) for i in range(nobj)], d_out)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for i in (0, 5, nobj - 1):
        exp = oracle.slicer_encode_np(o716, host[i * L:(i + 1) * L], chunk_index=i)
        assert np.array_equal(out[i * per:(i + 1) * per].reshape(N, -1), exp), i
    # worst-case decode: slices 0..12 erased
    d_dec = torch.zeros(nobj * L, dtype=torch.uint8, device=dev)
    metas = b"".join(out[i * per + g.slice_len - 48:i * per + g.slice_len].tobytes() for i in range(nobj))
    mask = sum(1 << j for j in range(13, 20))
    batch.decode_batch(s, d_out, [(i * per, g.slice_len, mask, i * L) for i in range(nobj)], metas, d_dec)
    torch.cuda.synchronize()
    assert np.array_equal(d_dec.cpu().numpy(), host)
    # repair slice (i mod 20) of every object from pre-extracted helper buffers
    plans, offs, blobs = [], [], []
    cur = 0
    for i in range(nobj):
        lost = i % N
        avail = [j for j in range(N) if j != lost]
        p = s.repair_plan_from_params(lost, avail, L, g.stripe_size)
        o = {}
        for h in avail:
            b = T.extract_repair_data(out[i * per + h * g.slice_len:i * per + (h + 1) * g.slice_len].tobytes(), p, h)
            if b:
                o[h] = cur
                blobs.append(b)
                cur += len(b)
        plans.append(p)
        offs.append(o)
    d_help = torch.from_numpy(np.frombuffer(b"".join(blobs), np.uint8).copy()).to(dev)
    d_rep = torch.zeros(nobj * g.slice_len, dtype=torch.uint8, device=dev)
    objs = [(plans[i], offs[i], i * g.slice_len, out[i * per + g.slice_len - 48:i * per + g.slice_len].tobytes())
            for i in range(nobj)]
    batch.repair_batch(s.coder, d_help, objs, d_rep)
    torch.cuda.synchronize()
    rep = d_rep.cpu().numpy()
    for i in range(nobj):
        lost = i % N
        assert np.array_equal(rep[i * g.slice_len:(i + 1) * g.slice_len],
                              out[i * per + lost * g.slice_len:i * per + (lost + 1) * g.slice_len]), i


def test_batch_mixed_sizes(oracle, o716):
    from tape_amd import batch
    dev = torch.device("cuda:0")
    sizes = [0, 1, 1000, 99_999, 1_000_000, 1_000_001, 3 * MiB + 7]
    s = T.Slicer.clay_default()
    offs, cur, outs, ocur = [], 0, [], 0
    for ln in sizes:
        offs.append(cur)
        cur += ln + 13  # deliberately odd offsets: the kernels must not assume alignment
        g = s.geometry(ln)
        outs.append(ocur)
        ocur += N * g.slice_len
    host = np.zeros(cur, np.uint8)
    for ln, o in zip(sizes, offs):
        host[o:o + ln] = oracle.splitmix64_bytes(ln + 1, ln)
    d_in = torch.from_numpy(host).to(dev)
    d_out = torch.zeros(ocur, dtype=torch.uint8, device=dev)
    batch.encode_batch(s, d_in, [(offs[i], sizes[i], outs[i], 0) for i in range(len(sizes))], d_out)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    for i, ln in enumerate(sizes):
        g = s.geometry(ln)
        exp = oracle.slicer_encode_np(o716, host[offs[i]:offs[i] + ln])
        assert np.array_equal(out[outs[i]:outs[i] + N * g.slice_len].reshape(N, -1), exp), ln


@pytest.mark.parametrize("pinned", [False, True])
def test_batch_encode_host_pipeline(oracle, o716, pinned):
    """te_encode_batch_host: host -> host, windows small enough to force many pipeline slots."""
    from tape_amd import batch
    sizes = [4 * MiB] * 6 + [1, 0, 777_777, 2 * MiB + 3]
    s = T.Slicer.clay_default()
    offs, cur, outs, ocur = [], 0, [], 0
    for ln in sizes:
        offs.append(cur)
        cur += ln + (5 if ln % 2 else 0)  # contiguous runs and gaps
        outs.append(ocur)
        ocur += N * s.geometry(ln).slice_len
    h_in = torch.zeros(cur, dtype=torch.uint8)
    h_out = torch.zeros(ocur, dtype=torch.uint8)
    if pinned:
        h_in, h_out = h_in.pin_memory(), h_out.pin_memory()
    npin = h_in.numpy()
    for i, ln in enumerate(sizes):
        npin[offs[i]:offs[i] + ln] = oracle.splitmix64_bytes(1000 + i, ln)
    objs = [(offs[i], sizes[i], outs[i], i) for i in range(len(sizes))]
    batch.encode_batch_host(s, h_in, objs, h_out, window_bytes=40 * MiB)
    out = h_out.numpy()
    for i, ln in enumerate(sizes):
        g = s.geometry(ln)
        if i in (0, 5) or ln < 4 * MiB:  # oracle on a sample, SHA of device path on the rest
            o = oracle.slicer_encode_np(o716, npin[offs[i]:offs[i] + ln], chunk_index=i)
            assert np.array_equal(out[outs[i]:outs[i] + N * g.slice_len].reshape(N, -1), o), (i, ln)
    # identical to the device-resident batch path for every object
    d_out = torch.zeros(ocur, dtype=torch.uint8, device="cuda:0")
    batch.encode_batch(s, h_in.to("cuda:0"), objs, d_out)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy(), out)


# ---------------------------------------------------------------- commitments (§8f-1) -------
@pytest.mark.parametrize("slen", [4, 8, 52, 56, 60, 64, 116, 120, 124, 1000, 14_448, 286_048, 715_048])
def test_commit_batch_matches_oracle(slen):
    import torch
    from oracle import merkle_oracle as O
    from tape_amd import merkle
    n, nobj, H = 20, 3, 5
    host = torch.from_numpy(np.frombuffer(np.random.default_rng(slen).bytes(nobj * n * slen), dtype=np.uint8).copy())
    dev = host.cuda()
    leaf = torch.empty(nobj * n * 32, dtype=torch.uint8, device="cuda")
    root = torch.empty(nobj * 32, dtype=torch.uint8, device="cuda")
    proof = torch.empty(nobj * n * H * 32, dtype=torch.uint8, device="cuda")
    merkle.commit_batch(dev, n * slen, slen, n, nobj, leaf, root, proof, H)
    torch.cuda.synchronize()
    lb, rb, pb = (t.cpu().numpy().tobytes() for t in (leaf, root, proof))
    raw = host.numpy().tobytes()
    for o in range(nobj):
        sl = [raw[(o * n + i) * slen:(o * n + i + 1) * slen] for i in range(n)]
        leaves, r, proofs = O.commit_slices(sl, H)
        assert lb[o * n * 32:(o + 1) * n * 32] == b"".join(leaves), (slen, o)
        assert rb[o * 32:(o + 1) * 32] == r, (slen, o)
        got = [[pb[((o * n + i) * H + l) * 32:((o * n + i) * H + l + 1) * 32] for l in range(H)] for i in range(n)]
        assert got == proofs, (slen, o)


def test_encode_with_proofs_4mib(oracle):  # BlobEncoder::encode_with_proofs, encoder.rs:220-234
    from oracle import merkle_oracle as O
    from tape_amd import merkle
    data = oracle.splitmix64_bytes(99, 4 * MiB).tobytes()
    sl = T.Slicer.clay_default().encode(data)
    leaves, root, proofs = merkle.commit_slices(sl)
    exp = O.commit_slices(sl)
    assert (leaves, root, proofs) == exp
    for i in range(N):
        assert merkle.verify_proof(sl[i], root, proofs[i], i)


def test_commit_leaves_only_and_partial_wave():
    import torch
    from oracle import merkle_oracle as O
    from tape_amd import merkle
    n, nobj, slen = 7, 5, 1_000  # 35 streams: a partial wave
    host = torch.from_numpy(np.frombuffer(np.random.default_rng(1).bytes(nobj * n * slen + 64), dtype=np.uint8).copy())
    dev = host.cuda()
    leaf = torch.empty(nobj * n * 32, dtype=torch.uint8, device="cuda")
    merkle.commit_batch(dev, n * slen + 8, slen, n, nobj, leaf)  # obj_stride != n * slice_len
    torch.cuda.synchronize()
    raw, lb = host.numpy().tobytes(), leaf.cpu().numpy().tobytes()
    for o in range(nobj):
        for i in range(n):
            off = o * (n * slen + 8) + i * slen
            assert lb[(o * n + i) * 32:(o * n + i + 1) * 32] == O.hash_leaf(raw[off:off + slen])


@pytest.mark.parametrize("params", [(20, 7, 16), (20, 8, 17), (20, 9, 18), (20, 10, 19)])
def test_clay_decode_many_patterns_vs_oracle(oracle, params):
    # staged decode (one plane program per erasure pattern, kernels for k = 7..10) against the
    # oracle's own decode on 60 random survivor sets of exactly k .. n-1 chunks
    c = T.ClayCoder(*params)
    o = oracle.OracleClay(*params)
    n, k, _ = params
    data = oracle.splitmix64_bytes(k * 1000 + 7, 30_000).tobytes()
    ch = c.encode(data)
    assert ch == o.encode(data)
    rnd = random.Random(k)
    for _ in range(60):
        keep = sorted(rnd.sample(range(n), rnd.choice([k, k, k + 1, rnd.randint(k, n - 1)])))
        got = c.decode([(i, ch[i]) for i in keep])
        assert got[:len(data)] == data, keep


# ---------------------------------------------------------------- node recover (§8f-2) ------
@pytest.mark.parametrize("ln", [1, 999, 100_003, 1_000_001, 4 * MiB])
def test_reconstruct_matches_original_slice(oracle, ln):  # recover.rs:411-442
    from tape_amd import batch
    data = oracle.splitmix64_bytes(ln ^ 0xC0FFEE, ln).tobytes()
    s = T.Slicer.clay_default()
    s.set_chunk_index(3)
    sl = s.encode(data)
    rnd = random.Random(ln)
    for lost in (0, 6, 7, 19, rnd.randrange(N)):
        avail = sorted(rnd.sample([i for i in range(N) if i != lost], rnd.choice([7, 10, 19])))
        got = batch.reconstruct(T.Slicer.clay_default(), lost, [(i, sl[i]) for i in avail])
        assert got == sl[lost], (lost, avail)


def test_recover_batch_device(oracle):
    from tape_amd import batch
    nobj, L = 6, 300_000
    s = T.Slicer.clay_default()
    g = s.geometry(L)
    per = N * g.slice_len
    host = bytearray()
    metas = b""
    objs, exp = [], []
    rnd = random.Random(11)
    for o in range(nobj):
        sl = s.encode(oracle.splitmix64_bytes(o + 1, L).tobytes())
        host += b"".join(sl)
        lost = rnd.randrange(N)
        avail = rnd.sample([i for i in range(N) if i != lost], 7 + o)
        mask = sum(1 << i for i in avail)
        objs.append((o * per, g.slice_len, mask, lost, o * g.slice_len))
        exp.append(sl[lost])
        metas += sl[0][-48:]
    dev = torch.frombuffer(host, dtype=torch.uint8).cuda()
    out = torch.empty(nobj * g.slice_len, dtype=torch.uint8, device="cuda")
    batch.recover_batch(s, dev, objs, metas, out)
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == b"".join(exp)
