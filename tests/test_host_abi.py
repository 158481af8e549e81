"""CPU-side checks of the product library (no GPU compute here):

* libtapeec.so loads and exports every symbol include/tape_ec.h declares;
* compute entry points fail loudly (NoDeviceError) without a device -- no CPU fallback;
* host-only bookkeeping (geometry, rotation maps, metadata, repair plans, helper gather)
  matches the oracle restatement of lib/slicer.
"""
import ctypes as C
import random

import pytest

import tape_amd as T
from tape_amd import _lib

N = 20


def test_exports_every_declared_symbol():
    names = _lib.declared_symbols()
    assert len(names) >= 30
    so = C.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing


def test_no_cpu_fallback():
    if T.device_count() > 0:
        pytest.skip("device present")
    s = T.Slicer.clay_default()
    with pytest.raises(T.NoDeviceError):
        s.encode(b"hello world")
    c = T.ClayCoder(20, 7, 16)
    with pytest.raises(T.NoDeviceError):
        c.encode(b"x" * 100)


def test_invalid_params_assert():  # clay.rs:24-34 asserts
    for n, k, d in [(7, 7, 6), (20, 0, 5), (20, 7, 7), (20, 7, 20)]:
        with pytest.raises(AssertionError):
            T.ClayCoder(n, k, d)


def test_info_and_chunk_size(oracle):
    for (n, k, d) in [(20, 7, 16), (20, 10, 19), (20, 5, 14), (12, 8, 11), (20, 7, 19)]:
        c = T.ClayCoder(n, k, d)
        o = oracle.OracleClay(n, k, d)
        assert (c.k(), c.m(), c.n(), c.d(), c.alpha(), c.beta()) == (o.k, o.m, o.n, o.d, o.alpha, o.beta)
        for ln in [0, 1, 999, 1400, 1401, 100_000, 194_304, 1_000_000, 10_000_000]:
            assert c.chunk_size_for(ln) == o.chunk_size_for(ln)


def test_geometry_matches_oracle(oracle):
    s = T.Slicer.clay_default()
    o = oracle.OracleClay(20, 7, 16)
    for ln in [0, 1, 5000, 100_000, 1_000_000, 1_000_001, 1024 * 1024, 4 * 1024 * 1024, 64 * 1024 * 1024,
               100_000_001]:
        g = s.geometry(ln)
        assert (g.stripe_size, g.num_stripes, g.chunk_size, g.slice_len) == oracle.geometry(o, ln)


def test_rotation_maps_match_oracle(oracle):
    for stripe in range(45):
        for x in range(N):
            for rot in (T.MappingStrategy.Identity, T.MappingStrategy.Rotated):
                r = rot == T.MappingStrategy.Rotated
                assert T.shard_to_slice(rot, N, stripe, x) == oracle.shard_to_slice(r, N, stripe, x)
                assert T.slice_to_shard(rot, N, stripe, x) == oracle.slice_to_shard(r, N, stripe, x)


def test_metadata_roundtrip():  # metadata.rs:115-151
    m = T.SliceMetadata.new(12345, T.STRIPE_SIZES[0])
    m.chunk_index = 42
    b = m.to_bytes()
    assert len(b) == 48 == T.SliceMetadata.SIZE
    p = T.SliceMetadata.from_slice(bytes(100) + b)
    assert (p.blob_len, p.stripe_size, p.version, p.chunk_index) == (12345, 100_000, 0, 42)
    assert p.profile == T.EncodingProfile.clay_default()
    with pytest.raises(T.DecodeError):
        T.SliceMetadata.from_slice(bytes(47))
    bad = T.SliceMetadata.new(1000, 999)
    with pytest.raises(T.DecodeError):
        T.SliceMetadata.from_slice(bad.to_bytes())


@pytest.mark.parametrize("params", [(20, 7, 16), (20, 10, 19)])
def test_repair_plans_match_oracle(oracle, params):
    c = T.ClayCoder(*params)
    o = oracle.OracleClay(*params)
    rnd = random.Random(5)
    for rotated in (False, True):
        sl = T.Slicer(c, strategy=T.MappingStrategy.Rotated if rotated else T.MappingStrategy.Identity)
        for trial in range(12):
            lost = rnd.randrange(N)
            others = [i for i in range(N) if i != lost]
            navail = rnd.choice([c.d(), N - 1])
            avail = sorted(rnd.sample(others, navail))
            blob_len = rnd.choice([0, 1, 10_000, 300_000, 4 * 1024 * 1024])
            stripe = T.pick_stripe_size(blob_len)
            try:
                cs, stripes = oracle.repair_plan(o, lost, avail, blob_len, stripe, rotated)
            except ValueError:
                with pytest.raises(T.RepairError):
                    sl.repair_plan_from_params(lost, avail, blob_len, stripe)
                continue
            p = sl.repair_plan_from_params(lost, avail, blob_len, stripe)
            assert p.chunk_size == cs and p.num_stripes == len(stripes)
            assert p.sub_chunk_size == cs // o.alpha
            for st, (s, ls, hs) in zip(p.stripes, stripes):
                assert st.lost_shard == ls
                assert [(h.slice, h.shard, h.sub_chunks) for h in st.helpers] == [tuple(x) for x in hs]


def test_plan_repair_clay_level(oracle):
    c = T.ClayCoder(20, 7, 16)
    o = oracle.OracleClay(20, 7, 16)
    for lost in range(N):
        avail = [i for i in range(N) if i != lost]
        assert c.plan_repair(lost, avail) == o.minimum_to_repair(lost, avail)
    with pytest.raises(T.RepairError):
        c.plan_repair(0, list(range(1, 16)))  # d-1 available


def test_plan_failures_are_clay_errors():
    """ClayCoder::plan_repair maps every minimum_to_repair failure to RepairError::Clay(String)
    (repair.rs:59-62); repair_plan_from_params propagates it (repair.rs:170)."""
    c = T.ClayCoder(20, 7, 16)
    with pytest.raises(T.RepairError) as e:
        c.plan_repair(0, list(range(1, 16)))  # d - 1 available
    assert e.value.variant == "Clay" and "need 16 helpers" in str(e.value)
    with pytest.raises(T.RepairError) as e:
        c.plan_repair(0, [i for i in range(1, N) if i != 3])  # a column-mate of node 0 missing
    assert e.value.variant == "Clay" and "column-mate" in str(e.value)
    s = T.Slicer.clay_default()
    with pytest.raises(T.RepairError) as e:
        s.repair_plan_from_params(5, list(range(6, 20)), 4 * 1024 * 1024, 1_000_000)
    assert e.value.variant == "Clay"
    # repair_full with no helpers stays NotEnoughHelpers (repair.rs:293-296)
    with pytest.raises(T.RepairError) as e:
        s.repair_full(0, [])
    assert e.value.variant == "NotEnoughHelpers"


def test_device_binding_without_device():
    if T.device_count() > 0:
        pytest.skip("device present")
    c = T.ClayCoder(20, 7, 16)
    from tape_amd._lib import lib
    assert lib.te_clay_device(c.handle) == 0
    assert lib.te_clay_bind_device(c.handle, 0) == _lib.TE_ERR_NO_DEVICE
    assert lib.te_clay_bind_device(None, 0) == _lib.TE_ERR_INVALID_ARG


def test_extract_repair_data_matches_oracle(oracle):
    o = oracle.OracleClay(20, 7, 16)
    data = oracle.splitmix64_bytes(9, 300_000).tobytes()
    sl = oracle.slicer_encode(o, data)
    s = T.Slicer.clay_default()
    for lost in (0, 7, 19):
        avail = [i for i in range(N) if i != lost]
        p = s.repair_plan(lost, avail, sl[avail[0]])
        cs, stripes = oracle.repair_plan(o, lost, avail, len(data), T.pick_stripe_size(len(data)), True)
        for h in avail:
            assert T.extract_repair_data(sl[h], p, h) == oracle.extract_repair_data(sl[h], cs, o.alpha, stripes, h)
        with pytest.raises(T.RepairError):
            T.extract_repair_data(sl[avail[0]][:100], p, avail[0])


def test_kernel_timing_api_without_device():
    """te_kernel_timing / te_kernel_time_ms are host bookkeeping: usable with no GPU, no events."""
    import ctypes as C
    from tape_amd._lib import lib
    assert lib.te_kernel_timing(1) == 0
    ms, n = C.c_double(-1), C.c_uint32(7)
    assert lib.te_kernel_time_ms(C.byref(ms), C.byref(n)) == 0
    assert ms.value == 0.0 and n.value == 0
    assert lib.te_kernel_timing(0) == 0


def test_recover_needs_device():
    import ctypes as C
    from tape_amd import _lib
    if _lib.device_count() > 0:
        pytest.skip("device present")
    c = C.c_void_p()
    assert _lib.lib.te_clay_new(20, 7, 16, C.byref(c)) == 0
    cfg = _lib.te_slicer_cfg()
    obj = _lib.te_recover_object(0, 715_048, 0xFFFFE, 0, 0)
    meta = (C.c_uint8 * 48)()
    r = _lib.lib.te_recover_batch_device(c, C.byref(cfg), C.c_void_p(16), C.byref(obj), meta, 1, C.c_void_p(16), None)
    assert r == _lib.TE_ERR_NO_DEVICE
    _lib.lib.te_clay_free(c)


def test_encode_commit_argument_checks():
    """te_encode_commit_batch_host validates the tree before touching a device: height 0 or > 32
    is an invalid argument, n = 20 leaves in a height-4 tree is TREE_FULL (tree.rs:344-350)."""
    import ctypes as C
    from tape_amd import _lib
    c = C.c_void_p()
    assert _lib.lib.te_clay_new(20, 7, 16, C.byref(c)) == 0
    cfg = _lib.te_slicer_cfg()
    obj = _lib.te_object(0, 1000, 0, 0)
    buf = C.c_void_p(16)

    def call(height):
        return _lib.lib.te_encode_commit_batch_host(c, C.byref(cfg), buf, C.byref(obj), 1, buf, height, buf, buf,
                                                    None, 0)
    assert call(0) == _lib.TE_ERR_INVALID_ARG
    assert call(33) == _lib.TE_ERR_INVALID_ARG
    assert call(4) == _lib.TE_ERR_MERKLE_TREE_FULL
    if _lib.device_count() == 0:
        assert call(5) == _lib.TE_ERR_NO_DEVICE
    _lib.lib.te_clay_free(c)


def test_repair_request_round_trip(oracle):
    """The node repair wire: per_helper_reqs (node repair.rs:468-491) inverts the
    plan into one RepairRequest per helper (protocol types.rs:75-85); the helper serves it from its
    stored slice alone (node repair.rs:496-553).  Served bytes equal the plan-side
    extract_repair_data (slicer repair.rs:97-130) and the oracle's, for every helper."""
    o = oracle.OracleClay(20, 7, 16)
    s = T.Slicer.clay_default()
    for L in (1, 300_000, 2_500_001):
        data = oracle.splitmix64_bytes(L, L).tobytes()
        sl = oracle.slicer_encode(o, data)
        for lost in (0, 12):
            avail = [i for i in range(N) if i != lost]
            p = s.repair_plan(lost, avail, sl[avail[0]])
            cs, stripes = oracle.repair_plan(o, lost, avail, L, T.pick_stripe_size(L), True)
            served_from = set()
            for h in avail:
                req = T.repair_request(p, h)
                exp_req = [(st, planes) for (st, _ls, helpers) in stripes for (slc, _sh, planes) in helpers if slc == h]
                assert req == exp_req, (L, lost, h)
                got = T.serve_repair_request(s.coder, sl[h], req)
                assert got == T.extract_repair_data(sl[h], p, h) == oracle.extract_repair_data(sl[h], cs, o.alpha,
                                                                                               stripes, h)
                if req:
                    served_from.add(h)
            assert len(served_from) >= s.coder.d()


def test_serve_repair_request_errors(oracle):
    """extract_repair_data's error strings (node repair.rs:507-546) via te_last_error_detail."""
    o = oracle.OracleClay(20, 7, 16)
    s = T.Slicer.clay_default()
    sl = oracle.slicer_encode(o, oracle.splitmix64_bytes(5, 2_500_000).tobytes())[3]
    cases = [
        (sl[:40], [(0, [0])], "slice too short for metadata"),
        (sl[:1000] + sl[-48:], [(0, [0])], "slice layout is inconsistent"),
        (sl, [(3, [0])], "slice too short for requested stripe"),
        (sl, [(0, [100])], "sub-chunk out of bounds"),
    ]
    for blob, req, msg in cases:
        with pytest.raises(T.RepairError) as e:
            T.serve_repair_request(s.coder, blob, req)
        assert msg in str(e.value), (msg, str(e.value))
    assert T.serve_repair_request(s.coder, sl, []) == b""


def test_outer_decode_batch_argument_checks():
    """te_outer_decode_device_batch validates every segment before enqueueing anything or touching a
    device: chunk_bytes not a multiple of 64 is INVALID_LAYOUT, overlapping segment outputs are an
    invalid argument, a segment with fewer than k chunks is NOT_ENOUGH_SLICES (outer.rs:127-129)
    even when the segments before it are complete, and a valid call without a device is NO_DEVICE."""
    k, n, cb = 4, 6, 128
    fake = 1 << 20  # never dereferenced: every path below returns before device work

    def call(segs, chunk_bytes=cb, seg_out=k * cb):
        flat = [None if x is None else fake + 4096 * i for i, x in enumerate(c for s in segs for c in s)]
        ptrs = (C.c_void_p * len(flat))(*flat)
        return _lib.lib.te_outer_decode_device_batch(k, n, C.cast(ptrs, C.POINTER(C.c_void_p)), len(segs),
                                                     chunk_bytes, C.c_void_p(fake), seg_out, None)
    full = [1] * n
    two_missing = [None, 1, None, 1, 1, 1]
    three_missing = [None, None, None, 1, 1, 1]
    assert call([full], chunk_bytes=100) == _lib.TE_ERR_INVALID_LAYOUT
    assert call([full, full], seg_out=k * cb - 64) == _lib.TE_ERR_INVALID_ARG
    assert call([full, two_missing, three_missing]) == _lib.TE_ERR_NOT_ENOUGH_SLICES
    if _lib.device_count() == 0:
        assert call([full, two_missing, two_missing]) == _lib.TE_ERR_NO_DEVICE
        assert call([full], seg_out=0) == _lib.TE_ERR_NO_DEVICE  # one segment: seg_out unused


def _ranges(lens, nparts):
    objs = (_lib.te_object * max(1, len(lens)))()
    for i, l in enumerate(lens):
        objs[i].blob_len = l
    cuts = (C.c_size_t * (nparts + 1))()
    assert _lib.lib.te_balance_object_ranges(objs, len(lens), nparts, cuts) == 0
    return list(cuts)


def test_balance_object_ranges():
    """te_encode_batch_host_multi's split (pure host code): contiguous ranges that
    cover every object once, in order, each part's bytes within one object of total / nparts."""
    rnd = random.Random(7)
    for trial in range(200):
        nobj = rnd.choice([0, 1, 2, 3, 7, 64, 1000])
        nparts = rnd.choice([1, 2, 3, 4, 8])
        lens = [rnd.choice([0, 1, 4 << 20, rnd.randrange(1, 8 << 20)]) for _ in range(nobj)]
        cuts = _ranges(lens, nparts)
        assert cuts[0] == 0 and cuts[-1] == nobj and cuts == sorted(cuts)
        w = [l + 1 for l in lens]
        total, biggest = sum(w), max(w, default=0)
        for p in range(nparts):
            part = sum(w[cuts[p]:cuts[p + 1]])
            assert abs(part - total / nparts) <= biggest, (trial, p, part, total / nparts)
    assert _ranges([4 << 20] * 8, 8) == list(range(9))      # equal objects: one each
    assert _ranges([4 << 20] * 16, 4) == [0, 4, 8, 12, 16]
    assert _ranges([100], 4)[-1] == 1


def test_encode_batch_host_multi_joins_without_device():
    """The per-handle threads of te_encode_batch_host_multi start, fail (no device) and are all
    joined; the first handle's status comes back on the calling thread, with its detail text."""
    if T.device_count() > 0:
        pytest.skip("device present")
    from tape_amd import batch
    slicers = [T.Slicer.clay_default() for _ in range(4)]
    L = 1000
    buf_in = bytearray(8 * L)
    buf_out = bytearray(8 * 20 * 4000)
    import numpy as np
    a_in = np.frombuffer(buf_in, np.uint8)
    a_out = np.frombuffer(buf_out, np.uint8)
    for _ in range(20):  # repeated: every thread is joined each time (no leak, no hang)
        with pytest.raises(T.NoDeviceError):
            batch.encode_batch_host_multi(slicers, a_in, [(i * L, L, i * 20 * 4000, 0) for i in range(8)], a_out)
