"""Per-call decode (te_slicer_decode / te_clay_decode) through each host-buffer path of
upload_slices (engine.cpp): pageable slices gathered into pinned staging (slices <= 2 MiB),
page-locked slices copied directly (te_host_alloc), a mix of the two (gathered), and long
pageable slices handed to the driver.  Every decoded blob must equal the original bytes
(Slicer::decode's contract, slicer.rs:298-364); the survivor sets include the worst case (13..19)
and random ones.  The encode under them is checked against the oracle in test_gpu_parity.py."""
import ctypes as C
import random

import numpy as np
import pytest

import tape_amd as T
from tape_amd import batch
from tape_amd._lib import lib

pytestmark = pytest.mark.gpu
N = 20
MiB = 1024 * 1024


def _encode(s, data):
    cfg, hdl = s._cfg(), s.coder.handle
    g = s.geometry(len(data))
    out = np.empty(N * g.slice_len, np.uint8)
    src = np.frombuffer(data, np.uint8)
    assert lib.te_slicer_encode(hdl, C.byref(cfg), C.c_void_p(src.ctypes.data), len(data),
                                C.c_void_p(out.ctypes.data), out.size) == 0
    return out, g.slice_len


def _decode(s, slices, sl, n):
    cfg, hdl = s._cfg(), s.coder.handle
    ptrs = (C.c_void_p * N)()
    for i, a in slices.items():
        ptrs[i] = a.ctypes.data
    dec = np.empty(max(1, n), np.uint8)
    got = C.c_size_t()
    assert lib.te_slicer_decode(hdl, C.byref(cfg), ptrs, sl, C.c_void_p(dec.ctypes.data), dec.size, C.byref(got)) == 0
    assert got.value == n
    return dec[:n].tobytes()


@pytest.mark.parametrize("ln", [1, 4096, 1_000_000, 4 * MiB, 16 * MiB + 77])
@pytest.mark.parametrize("kind", ["pageable", "pinned", "mixed"])
def test_slicer_decode_host_paths(ln, kind):
    rng = random.Random(ln * 7 + len(kind))
    data = bytes(rng.getrandbits(8) for _ in range(min(ln, 4096))) * (ln // 4096 + 1)
    data = data[:ln]
    s = T.Slicer.clay_default()
    out, sl = _encode(s, data)
    for survivors in (list(range(13, 20)), sorted(rng.sample(range(N), 7)), sorted(rng.sample(range(N), 11))):
        slices = {}
        for j, i in enumerate(survivors):
            pin = kind == "pinned" or (kind == "mixed" and j % 2 == 0)
            a = batch.host_empty(sl) if pin else np.empty(sl, np.uint8)
            a[:] = out[i * sl:(i + 1) * sl]
            slices[i] = a
        assert _decode(s, slices, sl, ln) == data, (kind, survivors)


@pytest.mark.parametrize("kind", ["pageable", "pinned"])
def test_clay_decode_host_paths(kind):
    c = T.ClayCoder(20, 7, 16)
    data = bytes(random.Random(5).getrandbits(8) for _ in range(300_001))
    chunks = c.encode(data)
    cs = len(chunks[0])
    ptrs = (C.c_void_p * N)()
    keep = []
    for i in range(6, 13):
        a = batch.host_empty(cs) if kind == "pinned" else np.empty(cs, np.uint8)
        a[:] = np.frombuffer(chunks[i], np.uint8)
        keep.append(a)
        ptrs[i] = a.ctypes.data
    out = np.empty(7 * cs, np.uint8)
    assert lib.te_clay_decode(c.handle, ptrs, cs, C.c_void_p(out.ctypes.data), out.size) == 0
    assert out.tobytes()[:len(data)] == data
