"""GPU parity of the row-piece encode kernel (encode_r10.hip) against the oracle, and of its
fallbacks.

Slicer::encode (lib/slicer/src/slicer.rs:237-296) of objects whose stripes the row-piece kernel
takes -- 1 MB stripes, object and slices 4-aligned, data ending on a dword -- and of objects next to
them that it must leave to encode_dma.hip (data end inside a dword, 2-mod-4 offsets) or the generic
kernel (odd offsets), in one batch.  Every slice byte (and the metadata suffix) equals the oracle's.
"""
import numpy as np
import pytest

import tape_amd as T
from tape_amd import batch

pytestmark = pytest.mark.gpu
N = 20
MiB = 1024 * 1024


@pytest.mark.parametrize("ln", [1_000_000, 1_048_576, 2_000_000, 3 * MiB + 4, 4 * MiB, 7_000_000 + 8, 64 * MiB])
@pytest.mark.parametrize("rotated", [True, False])
def test_r10_slicer_encode_matches_oracle(oracle, ln, rotated):
    s = T.Slicer.clay_default() if rotated else T.Slicer.new(T.ClayCoder(20, 7, 16))
    data = oracle.splitmix64_bytes(ln + 3, ln).tobytes()
    got = s.encode(data)
    exp = oracle.slicer_encode(oracle.OracleClay(20, 7, 16), data, rotated=rotated)
    assert got == exp


def test_r10_batch_mixed_alignment(oracle):
    """One batch: 16-aligned objects (row-piece kernel), a 2-mod-4 offset and a data end inside a
    dword (encode_dma.hip), an odd offset (generic kernel); chunk indices differ per object."""
    import torch
    sizes = [4 * MiB, 1_000_003, 2 * MiB + 2, 4 * MiB, 1_500_000, 3 * MiB]
    offs, a = [], 0
    skew = [0, 0, 2, 0, 1, 0]  # extra bytes before the object
    for L, k in zip(sizes, skew):
        a = (a + 15) & ~15
        a += k
        offs.append(a)
        a += L
    s = T.Slicer.clay_default()
    geo = [s.geometry(L) for L in sizes]
    outs, b = [], 0
    for g in geo:
        outs.append(b)
        b += N * g.slice_len
    datas = [oracle.splitmix64_bytes(900 + i, L) for i, L in enumerate(sizes)]
    h = np.zeros(a + 16, np.uint8)
    for o, d in zip(offs, datas):
        h[o:o + d.size] = d
    d_in = torch.from_numpy(h).cuda()
    d_out = torch.zeros(b, dtype=torch.uint8, device="cuda")
    batch.encode_batch(s, d_in, [(offs[i], sizes[i], outs[i], 10 + i) for i in range(len(sizes))], d_out)
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().tobytes()
    o = oracle.OracleClay(20, 7, 16)
    for i, d in enumerate(datas):
        exp = b"".join(oracle.slicer_encode(o, d.tobytes(), chunk_index=10 + i))
        assert got[outs[i]:outs[i] + len(exp)] == exp, i


def test_r10_large_batch_roundtrip(oracle):
    """128 x 4 MiB in one launch: a sample of objects against the oracle, every object through a
    worst-case decode (slices 0..12 erased) back to its bytes."""
    import torch
    s = T.Slicer.clay_default()
    L, nobj = 4 * MiB, 128
    g = s.geometry(L)
    per = N * g.slice_len
    gen = torch.Generator(device="cuda")
    gen.manual_seed(4)
    d_in = torch.randint(0, 256, (nobj * L,), dtype=torch.uint8, device="cuda", generator=gen)
    d_out = torch.empty(nobj * per, dtype=torch.uint8, device="cuda")
    batch.encode_batch(s, d_in, [(i * L, L, i * per, 0) for i in range(nobj)], d_out)
    torch.cuda.synchronize()
    o = oracle.OracleClay(20, 7, 16)
    for i in (0, 1, 77, nobj - 1):
        exp = b"".join(oracle.slicer_encode(o, d_in[i * L:(i + 1) * L].cpu().numpy().tobytes()))
        assert d_out[i * per:(i + 1) * per].cpu().numpy().tobytes() == exp, i
    metas = b"".join(d_out[i * per + g.slice_len - 48:i * per + g.slice_len].cpu().numpy().tobytes()
                     for i in range(nobj))
    d_dec = torch.zeros(nobj * L, dtype=torch.uint8, device="cuda")
    batch.decode_batch(s, d_out, [(i * per, g.slice_len, sum(1 << j for j in range(13, 20)), i * L)
                                  for i in range(nobj)], metas, d_dec)
    torch.cuda.synchronize()
    assert torch.equal(d_dec, d_in)
