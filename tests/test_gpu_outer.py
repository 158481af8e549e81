"""GPU parity of the OuterCoder (lib/slicer/src/outer.rs:19-197) against the GF(2^16)
Leopard RS oracle (oracle/rs16_oracle.c; parity unpinned vs reed-solomon-simd 3.1.0, which is not
in the container): encoded chunks byte for byte, decodes against the original data, and the
reference's own OuterCoder tests (outer.rs:206-391) on the GPU path."""
import random

import numpy as np
import pytest

from oracle import rs16
from tape_amd.outer import OuterCoder
import tape_amd as T

pytestmark = pytest.mark.gpu
SPOOL_GROUP_COUNT, TEST_K = 50, 17


def make_data(n):  # outer.rs:206-208
    return bytes(i % 251 for i in range(n))


# matrix kernel shapes (rs16_matrix_kernel, image <= 80 KB, k <= 32): 4-row groups G odd / even,
# input slots KB = 16 / 32, G at its cap of 16 (5, 69), a high-rate shape (20, 40); transform
# kernels for the rest: (32, 64) and (40, 49) exceed the image budget
@pytest.mark.parametrize("k,n", [(17, 50), (7, 50), (4, 6), (10, 14), (32, 64), (40, 49), (3, 8), (1, 2),
                                 (16, 48), (20, 40), (5, 69), (31, 40)])
@pytest.mark.parametrize("size", [1, 1000, 100_003])
def test_encode_matches_oracle(k, n, size):
    data = np.random.default_rng(k * 1000 + n + size).bytes(size)
    got = OuterCoder(k, n).encode(data)
    exp = rs16.OracleOuter(k, n).encode(data)
    assert len(got) == n and got == exp


def test_encode_max_chunk_matches_oracle():
    k, n = TEST_K, SPOOL_GROUP_COUNT
    data = np.random.default_rng(7).bytes(k * (4 * 1024 * 1024) - 100)  # chunk = MAX_CHUNK_BYTES
    got = OuterCoder(k, n).encode(data)
    assert len(got[0]) == 4 * 1024 * 1024
    exp = rs16.OracleOuter(k, n).encode(data)
    assert got == exp
    with pytest.raises(T.EncodeError):
        OuterCoder(k, n).encode(bytes(k * 4 * 1024 * 1024 + 1))  # outer.rs:82-84 TooMuchData


@pytest.mark.parametrize("k,n", [(17, 50), (7, 50), (10, 14), (32, 64), (16, 48), (5, 69), (31, 40)])
def test_decode_patterns(k, n):
    rnd = random.Random(k + n)
    c = OuterCoder(k, n)
    data = make_data(123_457)
    ch = list(enumerate(c.encode(data)))
    sets = [ch[:k], ch[n - k:], [x for x in ch if x[0] % 3 == 0][:k]] + \
           [[ch[i] for i in sorted(rnd.sample(range(n), k))] for _ in range(6)]
    for avail in sets:
        if len(avail) < k:
            continue
        assert c.decode(avail)[:len(data)] == data, [i for i, _ in avail]


def test_reference_outer_tests_on_gpu():  # outer.rs:210-390
    c = OuterCoder(TEST_K, SPOOL_GROUP_COUNT)
    ch = list(enumerate(c.encode(make_data(100_000))))
    assert len(ch) == SPOOL_GROUP_COUNT and len({len(x) for _, x in ch}) == 1
    with pytest.raises(T.DecodeError):
        c.decode(ch[:TEST_K - 1])
    e = list(enumerate(c.encode(b"")))
    assert len(e[0][1]) == 64 and not any(c.decode(e[TEST_K:2 * TEST_K]))
    for sz in (1, 13, TEST_K, 1000, 50_000, 200_000):
        d = make_data(sz)
        ch = list(enumerate(c.encode(d)))
        assert c.decode(ch[:TEST_K])[:sz] == d and c.decode(ch[-TEST_K:])[:sz] == d
    one = OuterCoder(1, 1)
    d = make_data(10_000)
    assert one.decode(list(enumerate(one.encode(d))))[:len(d)] == d


def test_encode_device_segments():
    import torch
    from tape_amd import outer
    k, m, cb, segs = TEST_K, SPOOL_GROUP_COUNT - TEST_K, 64 * 1024, 5
    host = np.random.default_rng(3).integers(0, 256, segs * k * cb, dtype=np.uint8)
    d_in = torch.from_numpy(host).cuda()
    d_out = torch.zeros(segs * m * cb, dtype=torch.uint8, device="cuda")
    outer.encode_device(k, m, d_in, cb, segs, k * cb, d_out, m * cb)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    for g in (0, segs - 1):
        shards = [host[(g * k + j) * cb:(g * k + j + 1) * cb].tobytes() for j in range(k)]
        exp = b"".join(rs16.encode(k, m, shards))
        assert got[g * m * cb:(g + 1) * m * cb].tobytes() == exp, g


# ---- ReedSolomonCoder (lib/slicer/src/reed_solomon.rs:182-351, k = 10, m = 10) ----
def _rs():
    from tape_amd.outer import ReedSolomonCoder
    return ReedSolomonCoder(10, 10)


def test_rs_coder_reference_tests():
    c = _rs()
    o = rs16.OracleOuter(10, 20)
    for sz in (1, 9, 10, 11, 20, 5_000, 20_000, 30_000):  # test_many_sizes
        d = make_data(sz)
        ch = c.encode(d)
        assert ch == o.encode(d) and len(ch) == 20 and len({len(x) for x in ch}) == 1
        assert c.decode(list(enumerate(ch))[:10])[:sz] == d
    ch = list(enumerate(c.encode(make_data(20_000))))
    assert c.decode(ch)[:20_000] == make_data(20_000)                        # test_roundtrip_all
    assert c.decode([x for x in ch if x[0] % 2 == 0])[:20_000] == make_data(20_000)  # mixed
    assert c.decode(ch[10:])[:20_000] == make_data(20_000)                   # parity only
    with pytest.raises(T.DecodeError):
        c.decode(ch[:9])                                                     # test_insufficient
    bad = [(i, x[:-1] if i == 0 else x) for i, x in ch]
    with pytest.raises(T.DecodeError):
        c.decode(bad)                                                        # test_size_mismatch
    e = list(enumerate(c.encode(b"")))                                       # test_empty
    assert len(e) == 20 and not any(c.decode(e[10:]))
    with pytest.raises(T.EncodeError):
        c.encode(bytes(10 * 4096 + 1))                                       # past MAX_SLICE_BYTES


@pytest.mark.parametrize("k,n", [(17, 50), (40, 49), (4, 6)])
@pytest.mark.parametrize("present", ["parity_only", "mixed", "data_only"])
def test_decode_device_matches_original(k, n, present):
    """te_outer_decode_device (snapshot reads on device buffers) restores the data chunks from
    device chunks: parity-only, mixed and data-only sets, against the original bytes."""
    import torch
    from tape_amd import outer
    data = np.random.default_rng(k * 100 + n).bytes(k * 64 * 1000 - 7)
    chunks = OuterCoder(k, n).encode(data)
    cb = len(chunks[0])
    m = n - k
    if present == "parity_only":
        keep = list(range(k, k + min(k, m)))
        keep += [i for i in range(k) if len(keep) < k][: k - len(keep)]
    elif present == "mixed":
        keep = sorted(random.Random(k + n).sample(range(n), k))
    else:
        keep = list(range(k))
    dev = [torch.tensor(np.frombuffer(c, np.uint8), device="cuda") if i in keep else None for i, c in enumerate(chunks)]
    d_out = torch.empty(k * cb, dtype=torch.uint8, device="cuda")
    outer.decode_device(k, n, dev, cb, d_out)
    assert d_out.cpu().numpy().tobytes() == b"".join(chunks[:k])


def test_decode_device_batch_mixed_patterns():
    """te_outer_decode_device_batch: 12 segments of OuterCoder(17, 50) in one call, with three
    erasure patterns among them (parity only, mixed, data only) and more segments per pattern than
    one launch's shard pointers hold -- every segment's data chunks equal its original bytes, and
    the per-segment entry point gives the same bytes."""
    import torch
    from tape_amd import outer
    k, n = 17, 50
    rng = np.random.default_rng(99)
    segs, keeps, datas = [], [], []
    for g in range(12):
        data = rng.bytes(k * 64 * 300 - 5 * g)
        datas.append(data)
        chunks = OuterCoder(k, n).encode(data)
        cb = len(chunks[0])
        if g % 3 == 0:
            keep = list(range(k, 2 * k))
        elif g % 3 == 1:
            keep = sorted(random.Random(7).sample(range(n), k))
        else:
            keep = list(range(k))
        keeps.append(keep)
        segs.append([torch.tensor(np.frombuffer(c, np.uint8), device="cuda") if i in keep else None
                     for i, c in enumerate(chunks)])
    cb = segs[0][keeps[0][0]].numel()
    assert all(s[kp[0]].numel() == cb for s, kp in zip(segs, keeps))
    d_out = torch.zeros(12 * k * cb, dtype=torch.uint8, device="cuda")
    outer.decode_device_batch(k, n, segs, cb, d_out, k * cb)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().tobytes()
    for g in range(12):
        want = b"".join(OuterCoder(k, n).encode(datas[g])[:k])
        assert got[g * k * cb:(g + 1) * k * cb] == want, g
        one = torch.zeros(k * cb, dtype=torch.uint8, device="cuda")
        outer.decode_device(k, n, segs[g], cb, one)
        torch.cuda.synchronize()
        assert one.cpu().numpy().tobytes() == want, g
