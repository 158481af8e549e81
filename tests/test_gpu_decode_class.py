"""Decode class kernels (tape_amd/csrc/decode_class.hip, dec_class.hpp): every class of 7-of-20
survivor sets of Clay(20,7,16), for Slicer::decode (slicer.rs:298-364; classes by the number a0
of known column-0 nodes) and for node recover (recover.rs:411-442; classes by a0 and the lost
node's column), against the original bytes.  Single-stripe calls run one class kernel with one
wave per workgroup; the batches of >= 1024 stripes run every class of the call side by side on
forked streams (their own scratch ranges), the production shape of random reads.
"""
import random

import numpy as np
import pytest

import tape_amd as T

pytestmark = pytest.mark.gpu
N = 20


def _survivors(rnd, a0):
    return sorted(rnd.sample(range(10), a0) + rnd.sample(range(10, 20), 7 - a0))


@pytest.mark.parametrize("a0", range(8))
def test_class_decode_raw_every_class(oracle, a0):
    c = T.ClayCoder(20, 7, 16)
    data = oracle.splitmix64_bytes(0xD0 + a0, 31_000).tobytes()
    ch = c.encode(data)
    rnd = random.Random(a0)
    for _ in range(6):
        keep = _survivors(rnd, a0)
        assert c.decode([(i, ch[i]) for i in keep])[:len(data)] == data, keep


def _encoded_batch(oracle, nobj, L):
    import torch
    from tape_amd import batch
    s = T.Slicer.clay_default()
    g = s.geometry(L)
    per = N * g.slice_len
    host = np.concatenate([oracle.splitmix64_bytes(0x5EED ^ i, L) for i in range(nobj)])
    d_in = torch.from_numpy(host).cuda()
    d_sl = torch.zeros(nobj * per, dtype=torch.uint8, device="cuda")
    batch.encode_batch(s, d_in, [(i * L, L, i * per, 0) for i in range(nobj)], d_sl)
    torch.cuda.synchronize()
    return s, g, per, d_in, d_sl


def test_class_decode_batch_all_classes(oracle):
    """1,200 one-stripe objects, survivor sets cycling through the 8 classes, one call."""
    import torch
    from tape_amd import batch
    nobj, L = 1200, 20_000
    s, g, per, d_in, d_sl = _encoded_batch(oracle, nobj, L)
    host = d_sl.cpu().numpy()
    rnd = random.Random(1200)
    objs, metas = [], b""
    for i in range(nobj):
        keep = _survivors(rnd, i % 8)
        objs.append((i * per, g.slice_len, sum(1 << j for j in keep), i * L))
        metas += host[i * per + g.slice_len - 48:i * per + g.slice_len].tobytes()
    d_dec = torch.zeros(nobj * L, dtype=torch.uint8, device="cuda")
    batch.decode_batch(s, d_sl, objs, metas, d_dec)
    torch.cuda.synchronize()
    assert torch.equal(d_dec, d_in)


def test_class_recover_batch_all_classes(oracle):
    """1,056 one-stripe objects: 66 per recover class (a0 known column-0 nodes, lost node's
    column), the lost node a random erased node of that column, one call."""
    import torch
    from tape_amd import batch
    nobj, L = 1056, 20_000
    s, g, per, d_in, d_sl = _encoded_batch(oracle, nobj, L)
    host = d_sl.cpu().numpy()
    rnd = random.Random(1056)
    objs, metas, exp = [], b"", []
    for i in range(nobj):
        cls = i % 16
        a0, yl = cls // 2, cls % 2
        keep = _survivors(rnd, a0)
        lost = rnd.choice([j for j in range(10 * yl, 10 * yl + 10) if j not in keep])
        objs.append((i * per, g.slice_len, sum(1 << j for j in keep), lost, i * g.slice_len))
        metas += host[i * per + g.slice_len - 48:i * per + g.slice_len].tobytes()
        exp.append(host[i * per + lost * g.slice_len:i * per + (lost + 1) * g.slice_len])
    d_rec = torch.zeros(nobj * g.slice_len, dtype=torch.uint8, device="cuda")
    batch.recover_batch(s, d_sl, objs, metas, d_rec)
    torch.cuda.synchronize()
    got = d_rec.cpu().numpy()
    for i in range(nobj):
        assert np.array_equal(got[i * g.slice_len:(i + 1) * g.slice_len], exp[i]), (i, objs[i])


@pytest.mark.parametrize("a0", [0, 3, 7])
def test_class_recover_small_calls(oracle, a0):
    """Per-call recover of one object (one stripe, one class: the class kernel with one wave per
    workgroup), every lost node of both columns."""
    from tape_amd import batch
    data = oracle.splitmix64_bytes(0x7C + a0, 50_000).tobytes()
    s = T.Slicer.clay_default()
    sl = s.encode(data)
    rnd = random.Random(a0 + 40)
    keep = _survivors(rnd, a0)
    for lost in [j for j in range(N) if j not in keep]:
        assert batch.reconstruct(T.Slicer.clay_default(), lost, [(i, sl[i]) for i in keep]) == sl[lost], lost
