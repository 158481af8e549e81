"""The reference's own lib/slicer unit tests, ported against the CPU oracle (oracle/).

These pin the oracle to everything the reference tests pin (sizes, layouts, maps, round trips,
repair == encode, helper counts, bandwidth).  Encoded parity BYTES are not pinned by any
reference test or fixture (parity unpinned -- DESIGN.md).  Each test names the Rust test it ports.
"""
import itertools
import random

import pytest

N = 20


@pytest.fixture(scope="module")
def c1019(oracle):
    return oracle.OracleClay(20, 10, 19)


@pytest.fixture(scope="module")
def c716(oracle):
    return oracle.OracleClay(20, 7, 16)


# ---------------- clay.rs tests (lib/slicer/src/clay.rs:125-292) ----------------
def test_params(c1019):  # clay.rs:137-144
    assert (c1019.k, c1019.m, c1019.n, c1019.d) == (10, 10, 20, 19)


def test_default_layout(c716):  # encoding.rs:236-239 + SURVEY Appendix A
    assert (c716.q, c716.t, c716.nu, c716.alpha, c716.beta) == (10, 2, 0, 100, 10)


def test_chunk_count_uniform(oracle, c1019):  # clay.rs:155-170
    ch = c1019.encode(oracle.test_pattern(10_000))
    assert len(ch) == 20 and all(len(c) == len(ch[0]) for c in ch)


@pytest.mark.parametrize("keep", ["all", "data", "parity", "mixed"])
def test_roundtrip(oracle, c1019, keep):  # clay.rs:172-238
    original = oracle.test_pattern(10_000)
    ch = c1019.encode(original)
    idx = {"all": range(20), "data": range(10), "parity": range(10, 20), "mixed": range(0, 20, 2)}[keep]
    rec = c1019.decode({i: ch[i] for i in idx})
    assert rec[:len(original)] == original
    assert rec[len(original):] == bytes(len(rec) - len(original))


def test_insufficient(oracle, c1019):  # clay.rs:240-255
    ch = c1019.encode(oracle.test_pattern(10_000))
    with pytest.raises(ValueError, match="NotEnoughSlices"):
        c1019.decode({i: ch[i] for i in range(9)})


def test_empty_fails(c1019):  # clay.rs:257-262
    with pytest.raises(ValueError, match="EmptyInput"):
        c1019.encode(b"")


def test_chunk_size_for(oracle, c1019):  # clay.rs:264-282
    for ln in [100, 1000, 2000, 10_000, 100_000, 1_000_000]:
        ch = c1019.encode(oracle.test_pattern(ln))
        assert c1019.chunk_size_for(ln) == len(ch[0])


def test_chunk_size_for_min(c1019):  # clay.rs:284-290
    assert c1019.chunk_size_for(1) >= c1019.alpha * 2


def test_any_k_decodes_716(oracle, c716):  # SURVEY Appendix A invariant: any 7 of 20 decode
    data = oracle.splitmix64_bytes(7, 30_000).tobytes()
    ch = c716.encode(data)
    rnd = random.Random(1)
    combos = [rnd.sample(range(20), 7) for _ in range(40)] + [list(range(7)), list(range(13, 20))]
    for keep in combos:
        assert c716.decode({i: ch[i] for i in keep})[:len(data)] == data, keep


# ---------------- slicer.rs tests (lib/slicer/src/slicer.rs:389-728) ----------------
def test_identity_and_rotated_inverse(oracle):  # slicer.rs:413-435
    for stripe in range(10):
        for shard in range(N):
            assert oracle.shard_to_slice(False, N, stripe, shard) == shard
            s = oracle.shard_to_slice(True, N, stripe, shard)
            assert oracle.slice_to_shard(True, N, stripe, s) == shard


def test_distribution(oracle):  # slicer.rs:445-461
    hits = [0] * N
    for stripe in range(100):
        for shard in range(N):
            hits[oracle.shard_to_slice(True, N, stripe, shard)] += 1
    assert hits == [100] * N


def test_stripe_size(oracle):  # slicer.rs:463-470 + adaptive.rs:55-88
    S = oracle.STRIPE_SIZES
    assert oracle.pick_stripe_size(100) == S[0]
    assert oracle.pick_stripe_size(500_000) == S[0]
    assert oracle.pick_stripe_size(1_000_000) == S[0]
    assert oracle.pick_stripe_size(1_000_001) == S[1]
    assert oracle.pick_stripe_size(50_000_000) == S[1]
    assert oracle.pick_stripe_size(100_000_000) == S[1]
    assert oracle.pick_stripe_size(100_000_001) == S[2]
    assert oracle.num_stripes(0, 100_000) == 1
    assert oracle.num_stripes(1, 100_000) == 1
    assert oracle.num_stripes(100_000, 100_000) == 1
    assert oracle.num_stripes(100_001, 100_000) == 2
    assert oracle.num_stripes(250_000, 100_000) == 3
    assert all(s % 2000 == 0 for s in S)


@pytest.mark.parametrize("rotated", [False, True])
@pytest.mark.parametrize("ln", [0, 500, 1000, 3000, 5000, 250_000])
def test_slicer_roundtrip_1019(oracle, c1019, rotated, ln):  # slicer.rs:472-566
    payload = oracle.test_pattern(ln)
    sl = oracle.slicer_encode(c1019, payload, rotated=rotated)
    assert len(sl) == N and all(len(s) == len(sl[0]) for s in sl)
    assert oracle.slicer_decode(c1019, dict(enumerate(sl)), rotated) == payload
    if ln:
        assert oracle.slicer_decode(c1019, {i: sl[i] for i in range(10)}, rotated) == payload
        with pytest.raises(ValueError, match="NotEnoughSlices"):
            oracle.slicer_decode(c1019, {i: sl[i] for i in range(9)}, rotated)


def test_clay_default_roundtrip(oracle, c716):  # slicer.rs:579-591
    payload = oracle.test_pattern(1000)
    sl = oracle.slicer_encode(c716, payload)
    assert oracle.slicer_decode(c716, dict(enumerate(sl))) == payload


def test_metadata_suffix(oracle, c1019):  # slicer.rs:601-611, metadata.rs:115-151
    sl = oracle.slicer_encode(c1019, oracle.test_pattern(2000), rotated=False)
    meta = sl[0][-48:]
    assert int.from_bytes(meta[0:8], "little") == 0
    assert int.from_bytes(meta[8:16], "little") == 2000
    assert int.from_bytes(meta[16:24], "little") in oracle.STRIPE_SIZES
    assert int.from_bytes(meta[24:32], "little") == 2
    assert int.from_bytes(meta[32:40], "little") == 0x100714


def test_layout_mismatch(oracle, c1019):  # slicer.rs:689-702
    sl = oracle.slicer_encode(c1019, oracle.test_pattern(2000), rotated=False)
    d = dict(enumerate(sl))
    d[1] = d[1][:-1]
    with pytest.raises(ValueError, match="InvalidLayout"):
        oracle.slicer_decode(c1019, d, False)


def test_layout_valid_250k(oracle, c1019):  # slicer.rs:673-687
    sl = oracle.slicer_encode(c1019, oracle.test_pattern(250_000), rotated=False)
    S, ns, cs, slen = oracle.geometry(c1019, 250_000)
    assert ns == 3 and cs > 0 and len(sl[0]) == slen == 3 * cs + 48


def test_chunk_index_differentiates(oracle, c716):  # slicer.rs:704-727
    z = bytes(1000)
    a = oracle.slicer_encode(c716, z, rotated=False, chunk_index=0)
    b = oracle.slicer_encode(c716, z, rotated=False, chunk_index=1)
    assert a != b
    assert [s[:-48] for s in a] == [s[:-48] for s in b]


def test_geometry_4mib(oracle, c716):
    S, ns, cs, slen = oracle.geometry(c716, 4 * 1024 * 1024)
    assert (S, ns, cs, slen) == (1_000_000, 5, 143_000, 715_048)
    S, ns, cs, slen = oracle.geometry(c716, 1024 * 1024)
    assert (S, ns, cs, slen) == (1_000_000, 2, 143_000, 286_048)
    S, ns, cs, slen = oracle.geometry(c716, 0)
    assert (S, ns, cs, slen) == (100_000, 1, 14_400, 14_448)


# ---------------- repair.rs tests (lib/slicer/src/repair.rs:369-634) ----------------
def _helpers_for(chunks, cs, alpha, plan):
    sc = cs // alpha
    return {h: b"".join(chunks[h][z * sc:(z + 1) * sc] for z in pl) for h, pl in plan}


@pytest.mark.parametrize("lost", [0, 5, 19])
def test_repair_coder_direct(oracle, c1019, lost):  # repair.rs:397-430
    ch = c1019.encode(oracle.test_pattern(10_000))
    cs = len(ch[0])
    plan = c1019.minimum_to_repair(lost, [i for i in range(20) if i != lost])
    assert len(plan) == c1019.d
    assert c1019.repair(lost, _helpers_for(ch, cs, c1019.alpha, plan), cs) == ch[lost]


def test_repair_all_lost_716(oracle, c716):  # repair == encode for all 20 (Appendix A)
    ch = c716.encode(oracle.splitmix64_bytes(3, 50_000).tobytes())
    cs = len(ch[0])
    for lost in range(20):
        plan = c716.minimum_to_repair(lost, [i for i in range(20) if i != lost])
        assert len(plan) == 16 and all(len(p) == c716.beta for _, p in plan)
        assert c716.repair(lost, _helpers_for(ch, cs, c716.alpha, plan), cs) == ch[lost]


@pytest.mark.parametrize("rotated,stripe_hint", [(False, 100_000), (True, 2000)])
def test_repair_full(oracle, c1019, rotated, stripe_hint):  # repair.rs:432-461
    payload = oracle.test_pattern(10_000)
    sl = oracle.slicer_encode(c1019, payload, rotated=rotated)
    for lost in range(N):
        avail = [i for i in range(N) if i != lost]
        meta = sl[avail[0]][-48:]
        blob_len = int.from_bytes(meta[8:16], "little")
        stripe = int.from_bytes(meta[16:24], "little")
        cs, stripes = oracle.repair_plan(c1019, lost, avail, blob_len, stripe, rotated)
        hd = {h: oracle.extract_repair_data(sl[h], cs, c1019.alpha, stripes, h) for h in avail}
        assert oracle.slicer_repair(c1019, cs, stripes, hd, meta) == sl[lost]


def test_repair_plan_helpers_and_bandwidth(oracle, c1019):  # repair.rs:463-504
    sl = oracle.slicer_encode(c1019, oracle.test_pattern(50_000), rotated=False)
    avail = list(range(1, N))
    cs, stripes = oracle.repair_plan(c1019, 0, avail, 50_000, 100_000, False)
    assert all(len(h) == 19 for (_, _, h) in stripes)
    sc = cs // c1019.alpha
    repair_bytes = sum(len(pl) * sc for (_, _, hs) in stripes for (_, _, pl) in hs)
    assert repair_bytes < c1019.k * len(sl[0]) // 5


def test_repair_plan_rotation(oracle, c1019):  # repair.rs:506-529
    cs, stripes = oracle.repair_plan(c1019, 0, list(range(1, N)), 300_000, 100_000, True)
    assert len(stripes) > 1
    assert len({ls for (_, ls, _) in stripes}) > 1


def test_repair_exactly_d_and_insufficient(oracle, c1019):  # repair.rs:531-549, 615-633
    sl = oracle.slicer_encode(c1019, oracle.test_pattern(10_000), rotated=False)
    avail = list(range(1, 1 + c1019.d))
    cs, stripes = oracle.repair_plan(c1019, 0, avail, 10_000, 100_000, False)
    hd = {h: oracle.extract_repair_data(sl[h], cs, c1019.alpha, stripes, h) for h in avail}
    assert oracle.slicer_repair(c1019, cs, stripes, hd, sl[1][-48:]) == sl[0]
    with pytest.raises(ValueError):
        oracle.repair_plan(c1019, 0, list(range(1, c1019.d)), 10_000, 100_000, False)


def test_repair_716_rotated_4mib(oracle, c716):  # BASELINE config 3 shape, one object
    data = oracle.splitmix64_bytes(0x7A9E5EED, 4 * 1024 * 1024).tobytes()
    sl = oracle.slicer_encode(c716, data)
    lost = 11
    avail = [i for i in range(N) if i != lost]
    cs, stripes = oracle.repair_plan(c716, lost, avail, len(data), 1_000_000, True)
    hd = {h: oracle.extract_repair_data(sl[h], cs, c716.alpha, stripes, h) for h in avail}
    assert sum(len(v) for v in hd.values()) == 16 * 71_500
    assert oracle.slicer_repair(c716, cs, stripes, hd, sl[0][-48:]) == sl[lost]


def test_worst_case_decode_716(oracle, c716):  # BASELINE config 4 shape: slices 0..12 erased
    data = oracle.splitmix64_bytes(11, 1024 * 1024).tobytes()
    sl = oracle.slicer_encode(c716, data)
    assert oracle.slicer_decode(c716, {i: sl[i] for i in range(13, 20)}) == data
