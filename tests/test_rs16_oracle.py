"""CPU checks of the GF(2^16) Leopard RS oracle (oracle/rs16_oracle.c) -- parity
unpinned: no reference file holds reed-solomon-simd 3.1.0 output bytes.  What the reference's own
tests pin is restated here: lib/slicer/src/outer.rs:206-391 (OuterCoder chunk counts and sizes,
systematic data chunks, decode from data-only / parity-only / mixed chunk sets, k-1 chunks ->
NotEnoughSlices, empty data, sizes 1 .. 200,000, custom k), plus the field and code structure
the algorithm implies (log/exp inverse tables, MDS: any k shards decode)."""
import random

import pytest

from oracle import rs16

SPOOL_GROUP_COUNT, TEST_K = 50, 17  # outer.rs:203-204


def make_data(n):  # outer.rs:206-208
    return bytes(i % 251 for i in range(n))


def test_field_tables():
    L = rs16._lib()
    # exp/log are inverse on the non-zero elements; log(0) is the "zero" mark 65535
    for x in (1, 2, 3, 0x1234, 0xFFFF, 0x8000):
        assert L.rs16_exp(L.rs16_log(x)) == x
    assert L.rs16_log(0) == 65535
    assert len({L.rs16_log(x) for x in range(1, 4096)}) == 4095


@pytest.mark.parametrize("k,m", [(17, 33), (7, 43), (4, 2), (10, 4), (5, 3), (3, 5), (32, 32), (1, 1), (2, 7)])
def test_mds_any_k_shards(k, m):
    rng = random.Random(k * 100 + m)
    shards = [bytes(rng.randrange(256) for _ in range(128)) for _ in range(k)]
    rec = rs16.encode(k, m, shards)
    assert len(rec) == m and all(len(r) == 128 for r in rec)
    allsh = shards + rec
    for _ in range(6):
        keep = rng.sample(range(k + m), k)
        assert rs16.decode(k, m, {i: allsh[i] for i in keep}) == shards, keep


def test_linear_and_zero():
    k, m = 6, 5
    rng = random.Random(3)
    a = [bytes(rng.randrange(256) for _ in range(64)) for _ in range(k)]
    b = [bytes(rng.randrange(256) for _ in range(64)) for _ in range(k)]
    x = [bytes(p ^ q for p, q in zip(u, v)) for u, v in zip(a, b)]
    ra, rb, rx = rs16.encode(k, m, a), rs16.encode(k, m, b), rs16.encode(k, m, x)
    assert rx == [bytes(p ^ q for p, q in zip(u, v)) for u, v in zip(ra, rb)]
    assert rs16.encode(k, m, [bytes(64)] * k) == [bytes(64)] * m


def test_rate_choice():
    assert rs16.use_high_rate(17, 33) == 0 and rs16.use_high_rate(7, 43) == 0  # OuterCoder shapes: low rate
    assert rs16.use_high_rate(10, 4) == 1 and rs16.use_high_rate(32, 32) == 1
    assert rs16.use_high_rate(0, 4) == -1


def test_chunk_count():  # outer.rs:210-224
    c = rs16.OracleOuter(TEST_K, SPOOL_GROUP_COUNT)
    chunks = c.encode(make_data(100_000))
    assert len(chunks) == SPOOL_GROUP_COUNT and c.m == SPOOL_GROUP_COUNT - TEST_K
    assert len({len(x) for x in chunks}) == 1 and len(chunks[0]) % 64 == 0


def test_single_group_no_parity():  # outer.rs:226-240
    c = rs16.OracleOuter(1, 1)
    data = make_data(10_000)
    ch = c.encode(data)
    assert len(ch) == 1
    assert c.decode([(0, ch[0])])[:len(data)] == data


@pytest.mark.parametrize("pick", ["all", "data", "parity", "mixed"])
def test_roundtrips(pick):  # outer.rs:242-313
    c = rs16.OracleOuter(TEST_K, SPOOL_GROUP_COUNT)
    data = make_data(100_000)
    ch = list(enumerate(c.encode(data)))
    avail = {"all": ch, "data": ch[:TEST_K], "parity": ch[TEST_K:2 * TEST_K],
             "mixed": [x for x in ch if x[0] % 3 == 0][:TEST_K]}[pick]
    assert c.decode(avail)[:len(data)] == data
    assert ch[0][1] == data[:len(ch[0][1])]  # systematic


def test_insufficient_and_empty():  # outer.rs:315-346
    c = rs16.OracleOuter(TEST_K, SPOOL_GROUP_COUNT)
    ch = list(enumerate(c.encode(make_data(10_000))))
    with pytest.raises(ValueError, match="NotEnoughSlices"):
        c.decode(ch[:TEST_K - 1])
    e = list(enumerate(c.encode(b"")))
    assert len(e) == SPOOL_GROUP_COUNT and len(e[0][1]) == 64
    assert not any(c.decode(e))


@pytest.mark.parametrize("size", [1, 13, TEST_K, 1000, 50_000, 200_000])
def test_various_sizes(size):  # outer.rs:348-371
    c = rs16.OracleOuter(TEST_K, SPOOL_GROUP_COUNT)
    data = make_data(size)
    ch = list(enumerate(c.encode(data)))
    assert c.decode(ch[:TEST_K])[:size] == data
    assert c.decode(ch[-TEST_K:])[:size] == data


def test_custom_k():  # outer.rs:373-390
    c = rs16.OracleOuter(7, SPOOL_GROUP_COUNT)
    data = make_data(50_000)
    ch = list(enumerate(c.encode(data)))
    assert len(ch) == SPOOL_GROUP_COUNT
    assert c.decode(ch[:7])[:len(data)] == data
    assert c.decode(ch[20:27])[:len(data)] == data
