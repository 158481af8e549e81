"""GPU checks of the decode pattern store's overflow paths.

Slicer::decode from any k slices (lib/slicer/src/slicer.rs:298-364; the SDK's downloader takes
whichever k arrive, sdk/src/transfer/downloader.rs:79-109), so a batch of reads has one erasure
pattern per stripe.  The engine keeps compiled patterns in a device-resident store that grows by
doubling up to its cap (16,384 by default; these tests set 8,192 with te_clay_set_decode_store_cap
to keep them small):
  * one call with more distinct stripe patterns than the store holds uploads its patterns with
    the call (the arena path);
  * calls whose union overflows the store empty it once its last reader is done (the clear path).
Every decoded object must equal the original bytes.  Objects of 20,000 B have one stripe of
sub-chunk 30 (staged kernel), so ~9,000 distinct patterns cost ~0.5 GB of slices.
"""
import random

import pytest

import tape_amd as T
from tape_amd import batch

pytestmark = pytest.mark.gpu
N = 20
L = 20_000


def _masks(rnd, count, exclude=frozenset()):
    seen = set()
    while len(seen) < count:
        m = sum(1 << j for j in rnd.sample(range(N), 7))
        if m not in exclude:
            seen.add(m)
    return sorted(seen)


def _encoded(torch, s, nobj, seed):
    g = s.geometry(L)
    per = N * g.slice_len
    gen = torch.Generator(device="cuda")
    gen.manual_seed(seed)
    d_in = torch.randint(0, 256, (nobj * L,), dtype=torch.uint8, device="cuda", generator=gen)
    d_out = torch.empty(nobj * per, dtype=torch.uint8, device="cuda")
    batch.encode_batch(s, d_in, [(i * L, L, i * per, 0) for i in range(nobj)], d_out)
    torch.cuda.synchronize()
    meta = d_out[g.slice_len - 48:g.slice_len].cpu().numpy().tobytes()  # same geometry for all
    return d_in, d_out, g, per, meta


def _decode(torch, s, d_out, g, per, meta, masks, first=0):
    nobj = len(masks)
    d_dec = torch.zeros(nobj * L, dtype=torch.uint8, device="cuda")
    objs = [((first + i) * per, g.slice_len, masks[i], i * L) for i in range(nobj)]
    batch.decode_batch(s, d_out, objs, meta * nobj, d_dec)
    torch.cuda.synchronize()
    return d_dec


def test_decode_store_arena_path():
    """One call, 9,000 objects, 9,000 distinct 7-of-20 survivor sets (> the 8,192-slot store)."""
    import torch
    s = T.Slicer.clay_default()
    s.coder.set_decode_jit("off")
    s.coder.set_decode_store_cap(8192)
    nobj = 9000
    d_in, d_out, g, per, meta = _encoded(torch, s, nobj, 11)
    masks = _masks(random.Random(5), nobj)
    random.Random(6).shuffle(masks)
    d_dec = _decode(torch, s, d_out, g, per, meta, masks)
    assert torch.equal(d_dec, d_in)
    st = s.coder.decode_store_stats()
    assert st["arena_calls"] >= 1, st
    # the store still serves a normal call afterwards
    d_dec2 = _decode(torch, s, d_out, g, per, meta, masks[:100])
    assert torch.equal(d_dec2, d_in[:100 * L])


def test_decode_store_clear_path():
    """Back-to-back calls of 5,000 fresh patterns each: the first grows the store to 8,192 slots,
    the second overflows it (emptied after the first call's launches, on the device), a third
    call reuses the second call's slots in place."""
    import torch
    s = T.Slicer.clay_default()
    s.coder.set_decode_jit("off")
    s.coder.set_decode_store_cap(8192)
    nobj = 5000
    d_in, d_out, g, per, meta = _encoded(torch, s, nobj, 12)
    m1 = _masks(random.Random(7), nobj)
    m2 = _masks(random.Random(8), nobj, exclude=frozenset(m1))
    st0 = s.coder.decode_store_stats()
    a = _decode(torch, s, d_out, g, per, meta, m1)
    st1 = s.coder.decode_store_stats()
    b = _decode(torch, s, d_out, g, per, meta, m2)
    st2 = s.coder.decode_store_stats()
    c = _decode(torch, s, d_out, g, per, meta, m2[::-1])
    st3 = s.coder.decode_store_stats()
    assert torch.equal(a, d_in) and torch.equal(b, d_in)
    assert torch.equal(c.view(nobj, L), d_in.view(nobj, L))  # masks reversed, same objects
    assert st1["grows"] > st0["grows"] and st1["capacity"] == 8192, st1
    assert st2["clears"] == st1["clears"] + 1 and st2["used"] == nobj, st2
    assert st3["clears"] == st2["clears"] and st3["used"] == nobj, st3  # all hits


def test_decode_store_two_streams():
    """Patterns filled by a call on one stream are read by a call on another stream right after
    (the fill is stream-ordered; the second call waits for it on the device)."""
    import torch
    s = T.Slicer.clay_default()
    s.coder.set_decode_jit("off")
    nobj = 600
    d_in, d_out, g, per, meta = _encoded(torch, s, nobj, 13)
    masks = _masks(random.Random(9), nobj)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    o1 = torch.zeros(nobj * L, dtype=torch.uint8, device="cuda")
    o2 = torch.zeros(nobj * L, dtype=torch.uint8, device="cuda")
    objs = [(i * per, g.slice_len, masks[i], i * L) for i in range(nobj)]
    torch.cuda.synchronize()  # the zero fills above ran on the default stream
    batch.decode_batch(s, d_out, objs, meta * nobj, o1, s1)  # fills the store on s1
    batch.decode_batch(s, d_out, objs, meta * nobj, o2, s2)  # same patterns, read on s2
    torch.cuda.synchronize()
    assert torch.equal(o1, d_in) and torch.equal(o2, d_in)


def test_decode_store_default_cap_holds_2048_random_objects():
    """The default cap holds the ~10,000 stripe patterns of 2,048 random-survivor reads in place:
    a second call over the same patterns compiles and uploads nothing (no arena call, no clear)."""
    import torch
    s = T.Slicer.clay_default()
    s.coder.set_decode_jit("off")
    nobj = 10_000  # one stripe each: ~2,048 x 4 MiB objects' worth of distinct patterns
    d_in, d_out, g, per, meta = _encoded(torch, s, nobj, 14)
    masks = _masks(random.Random(10), nobj)
    a = _decode(torch, s, d_out, g, per, meta, masks)
    st1 = s.coder.decode_store_stats()
    b = _decode(torch, s, d_out, g, per, meta, masks)
    st2 = s.coder.decode_store_stats()
    assert torch.equal(a, d_in) and torch.equal(b, d_in)
    assert st1["arena_calls"] == 0 and st1["capacity"] == 16384 and st1["used"] == nobj, st1
    assert st2 == st1, (st1, st2)


def test_decode_store_clear_after_readers_on_two_streams():
    """the store is emptied and refilled by a call on a third stream while calls on two
    other streams may still be reading it.  The refill must wait for the last reader on EVERY
    stream (per-stream reader events), not only the most recent one: call A (3,000 objects over 300
    patterns) on s1, call B (200 other patterns) on s2, then call C (300 fresh patterns, overflowing
    a 512-slot store) on s3, with no host wait between them -- all three outputs exact."""
    import torch
    s = T.Slicer.clay_default()
    s.coder.set_decode_jit("off")
    s.coder.set_decode_store_cap(512)
    nobj = 3000
    d_in, d_out, g, per, meta = _encoded(torch, s, nobj, 15)
    rnd = random.Random(16)
    pa = _masks(rnd, 300)
    pb = _masks(rnd, 200, exclude=frozenset(pa))
    pc = _masks(rnd, 300, exclude=frozenset(pa) | frozenset(pb))
    ma = [pa[i % 300] for i in range(nobj)]
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    oa = torch.zeros(nobj * L, dtype=torch.uint8, device="cuda")
    ob = torch.zeros(200 * L, dtype=torch.uint8, device="cuda")
    oc = torch.zeros(300 * L, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    batch.decode_batch(s, d_out, [(i * per, g.slice_len, ma[i], i * L) for i in range(nobj)], meta * nobj, oa, s1)
    batch.decode_batch(s, d_out, [(i * per, g.slice_len, pb[i], i * L) for i in range(200)], meta * 200, ob, s2)
    st1 = s.coder.decode_store_stats()
    batch.decode_batch(s, d_out, [(i * per, g.slice_len, pc[i], i * L) for i in range(300)], meta * 300, oc, s3)
    st2 = s.coder.decode_store_stats()
    torch.cuda.synchronize()
    assert st2["clears"] == st1["clears"] + 1, (st1, st2)  # C emptied the store
    assert torch.equal(oa, d_in)
    assert torch.equal(ob, d_in[:200 * L])
    assert torch.equal(oc, d_in[:300 * L])
