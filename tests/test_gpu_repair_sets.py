"""GPU parity of Clay(20,7,16) repair when the helper set is not the all-available one.

A node repairs its slice from whichever peers answer (network/node/src/features/spool/repair.rs:
228-267, 351-371): with a peer down, ClayCoder::plan_repair (repair.rs:53-70 -> minimum_to_repair)
still takes the lost node's 9 column-mates but the first 7 *available* nodes of the other column,
so the aloof set -- and the decoding matrix -- changes.  With one of the other column's first 7
down the engine runs the folded kernel instantiated for that known set (repair_fold.hip); with two
down, the table-driven one (repair_stage.hip).  Bar: the repaired slice equals the encoded one,
byte for byte, and the raw ClayCoder output equals the oracle's chunk.
"""
import random

import numpy as np
import pytest

import tape_amd as T

pytestmark = pytest.mark.gpu
N = 20
MiB = 1024 * 1024


@pytest.fixture(scope="module")
def encoded_4mib(oracle):
    s = T.Slicer.clay_default()
    data = oracle.splitmix64_bytes(0xD0E5, 4 * MiB).tobytes()
    return s, s.encode(data)


def test_repair_one_peer_down_rotated(encoded_4mib):
    """Lost slice L, slice L+10 down: under rotation the down shard sits in the other column at the
    lost shard's position x_l, which moves with the stripe -- every stripe of every L takes either
    a one-down folded set (x_l < 7) or the all-available one (x_l >= 7)."""
    s, sl = encoded_4mib
    for lost in range(N):
        down = (lost + 10) % N
        helpers = [(i, sl[i]) for i in range(N) if i not in (lost, down)]
        assert s.repair_full(lost, helpers) == sl[lost], (lost, down)


@pytest.mark.parametrize("lost", [0, 4, 9, 10, 16, 19])
def test_repair_every_single_down_identity(oracle, lost):
    """Identity layout (shard = slice): the down node at each position of the other column."""
    s = T.Slicer.new(T.ClayCoder(20, 7, 16))
    data = oracle.splitmix64_bytes(0xBEEF ^ lost, 2 * MiB + 333).tobytes()
    sl = s.encode(data)
    other = 10 if lost < 10 else 0
    for p in range(10):
        down = other + p
        helpers = [(i, sl[i]) for i in range(N) if i not in (lost, down)]
        assert s.repair_full(lost, helpers) == sl[lost], (lost, down)


def test_repair_two_down_identity(oracle):
    """Two of the other column down: no folded set, the table-driven kernel; and a column-mate down
    is minimum_to_repair's error (RepairError::Clay)."""
    s = T.Slicer.new(T.ClayCoder(20, 7, 16))
    data = oracle.splitmix64_bytes(77, 3 * MiB).tobytes()
    sl = s.encode(data)
    rnd = random.Random(5)
    for lost in (2, 13):
        other = 10 if lost < 10 else 0
        for _ in range(4):
            downs = rnd.sample(range(other, other + 10), 2)
            helpers = [(i, sl[i]) for i in range(N) if i != lost and i not in downs]
            assert s.repair_full(lost, helpers) == sl[lost], (lost, downs)
        mate = (lost // 10) * 10 + (lost % 10 + 1) % 10
        with pytest.raises(T.RepairError) as e:
            s.repair_full(lost, [(i, sl[i]) for i in range(N) if i not in (lost, mate)])
        assert e.value.variant == "Clay"


def test_clay_repair_sets_match_oracle(oracle):
    """Raw ClayCoder::repair (clay.rs:75-88) for every lost chunk with each single other-column
    node down: the plan equals the oracle's minimum_to_repair and the chunk equals the encode."""
    c = T.ClayCoder(20, 7, 16)
    o = oracle.OracleClay(20, 7, 16)
    data = oracle.splitmix64_bytes(9, 1_000_000).tobytes()
    ch = c.encode(data)
    cs = len(ch[0])
    sc = cs // c.alpha()
    for lost in range(N):
        other = 10 if lost < 10 else 0
        for p in (0, 3, 6, 8):
            avail = [i for i in range(N) if i not in (lost, other + p)]
            plan = c.plan_repair(lost, avail)
            assert plan == o.minimum_to_repair(lost, avail), (lost, p)
            helpers = {h: b"".join(ch[h][z * sc:(z + 1) * sc] for z in pl) for h, pl in plan}
            assert c.repair(lost, helpers, cs) == ch[lost], (lost, p)


def test_repair_batch_peer_down(oracle):
    """te_repair_batch_device over 12 x 4 MiB objects, object i losing slice i mod 20 with slice
    (i + 10) mod 20 down: one batch mixing the folded kernels of several known sets."""
    import torch
    from tape_amd import batch
    nobj, L = 12, 4 * MiB
    dev = torch.device("cuda:0")
    host = np.concatenate([oracle.splitmix64_bytes(0x5EED ^ i, L) for i in range(nobj)])
    s = T.Slicer.clay_default()
    g = s.geometry(L)
    per = N * g.slice_len
    d_out = torch.zeros(nobj * per, dtype=torch.uint8, device=dev)
    batch.encode_batch(s, torch.from_numpy(host).to(dev), [(i * L, L, i * per, 0) for i in range(nobj)], d_out)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    plans, offs, blobs, cur, objs = [], [], [], 0, []
    for i in range(nobj):
        lost, down = i % N, (i + 10) % N
        avail = [j for j in range(N) if j not in (lost, down)]
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
        objs.append((p, o, i * g.slice_len, out[i * per + g.slice_len - 48:i * per + g.slice_len].tobytes()))
    d_help = torch.from_numpy(np.frombuffer(b"".join(blobs), np.uint8).copy()).to(dev)
    d_rep = torch.zeros(nobj * g.slice_len, dtype=torch.uint8, device=dev)
    batch.repair_batch(s.coder, d_help, objs, d_rep)
    torch.cuda.synchronize()
    rep = d_rep.cpu().numpy()
    for i in range(nobj):
        lost = i % N
        assert np.array_equal(rep[i * g.slice_len:(i + 1) * g.slice_len],
                              out[i * per + lost * g.slice_len:i * per + (lost + 1) * g.slice_len]), i


# ---------------------------------------------------------------- node recover ----------------
@pytest.mark.parametrize("params", [(20, 7, 16), (20, 10, 19), (20, 8, 17), (12, 8, 11)])
def test_recover_every_lost_node(oracle, params):
    """te_recover_batch_device = recover.rs:411-442 `reconstruct` for every lost slice: q = 10,
    t = 2 profiles run the fused decode whose program outputs the lost node's chunk directly (data
    or parity); (12,8,11) has no plane program and takes the decode + re-encode path.  Peers are
    exactly k random slices, or all others."""
    from tape_amd import batch
    n, k, _ = params
    s = T.Slicer.with_profile(T.ClayCoder(*params), 1_000_000, True, T.EncodingProfile.clay(T.ClayParams.new(*params)))
    data = oracle.splitmix64_bytes(sum(params), 2_345_678).tobytes()
    sl = s.encode(data)
    rnd = random.Random(n * k)
    for lost in range(n):
        for nav in (k, n - 1):
            avail = sorted(rnd.sample([i for i in range(n) if i != lost], nav))
            s2 = T.Slicer.with_profile(T.ClayCoder(*params), 1_000_000, True, T.EncodingProfile.clay(T.ClayParams.new(*params)))
            assert batch.reconstruct(s2, lost, [(i, sl[i]) for i in avail]) == sl[lost], (lost, avail)


def test_recover_batch_4mib_random_peers(oracle):
    """12 x 4 MiB objects, each losing a random slice and keeping 7 random peers (the node's
    fetch_slices shape, recover.rs:279-408), in one fused launch."""
    import torch
    from tape_amd import batch
    nobj, L = 12, 4 * MiB
    s = T.Slicer.clay_default()
    g = s.geometry(L)
    per = N * g.slice_len
    host = np.concatenate([oracle.splitmix64_bytes(0xAB ^ i, L) for i in range(nobj)])
    d_in = torch.from_numpy(host).cuda()
    d_sl = torch.zeros(nobj * per, dtype=torch.uint8, device="cuda")
    batch.encode_batch(s, d_in, [(i * L, L, i * per, 0) for i in range(nobj)], d_sl)
    torch.cuda.synchronize()
    out = d_sl.cpu().numpy()
    rnd = random.Random(77)
    objs, metas, exp = [], b"", []
    for i in range(nobj):
        lost = rnd.randrange(N)
        avail = rnd.sample([j for j in range(N) if j != lost], 7)
        objs.append((i * per, g.slice_len, sum(1 << j for j in avail), lost, i * g.slice_len))
        metas += out[i * per + g.slice_len - 48:i * per + g.slice_len].tobytes()
        exp.append(out[i * per + lost * g.slice_len:i * per + (lost + 1) * g.slice_len])
    d_rec = torch.zeros(nobj * g.slice_len, dtype=torch.uint8, device="cuda")
    batch.recover_batch(s, d_sl, objs, metas, d_rec)
    torch.cuda.synchronize()
    got = d_rec.cpu().numpy()
    for i in range(nobj):
        assert np.array_equal(got[i * g.slice_len:(i + 1) * g.slice_len], exp[i]), i


@pytest.mark.parametrize("small_only", [False, True])
def test_recover_mixed_batch_split(oracle, small_only):
    """A batch mixing 4 MiB objects (fused decode: 7 slices in, the lost one out) with tiny objects
    whose sub-chunks are below the staged kernel's 8 bytes (windowed decode + re-encode) recovers
    every object: the batch is split by path (one small object used to send the whole
    batch to the windowed path).  small_only: the windowed path on its own."""
    import torch
    from tape_amd import batch
    sizes = [1000, 3000] if small_only else [4 * MiB, 1000, 4 * MiB + 8, 3000, 2 * MiB]
    s = T.Slicer.clay_default()
    geo = [s.geometry(L) for L in sizes]
    datas = [oracle.splitmix64_bytes(0x51 + i, L).tobytes() for i, L in enumerate(sizes)]
    enc = [T.Slicer.clay_default().encode(d) for d in datas]
    for e, d in zip(enc, datas):
        assert e == oracle.slicer_encode(oracle.OracleClay(20, 7, 16), d)
    host, offs, a = bytearray(), [], 0
    for e in enc:
        offs.append(len(host))
        host += b"".join(e)
    d_sl = torch.frombuffer(bytes(host), dtype=torch.uint8).cuda()
    rnd = random.Random(len(sizes))
    objs, metas, exp, out_off = [], b"", [], 0
    for i, (g, e) in enumerate(zip(geo, enc)):
        lost = rnd.randrange(N)
        avail = rnd.sample([j for j in range(N) if j != lost], 7)
        objs.append((offs[i], g.slice_len, sum(1 << j for j in avail), lost, out_off))
        metas += e[0][-48:]
        exp.append((out_off, e[lost]))
        out_off += g.slice_len
    d_rec = torch.zeros(out_off, dtype=torch.uint8, device="cuda")
    batch.recover_batch(s, d_sl, objs, metas, d_rec)
    torch.cuda.synchronize()
    got = d_rec.cpu().numpy().tobytes()
    for i, (o, sl) in enumerate(exp):
        assert got[o:o + len(sl)] == sl, i
