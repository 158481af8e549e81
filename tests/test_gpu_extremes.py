"""GPU parity at the production extremes (SURVEY 8a at its size limits):

* a 64 MiB track -- the SDK's stream chunk (sdk/src/stream/manifest.rs:22): 68 stripes of 1 MB;
* an object over 100 MB, so pick_stripe_size (adaptive.rs:15-49) picks 10 MB stripes
  (sub-chunk 14,286 B, ten workgroups per stripe row);
* an object whose n * slice_len reaches 2^31, past the 32-bit buffer ranges of the fast kernels:
  encode and decode run on the generic layered kernel (gpe.hip), repair on its own kernels.

Encodes are compared byte for byte with the oracle restatement; decodes with the original object;
repairs and reconstructs with the encoded slice.
"""
import numpy as np
import pytest

import tape_amd as T
from tape_amd import batch

pytestmark = pytest.mark.gpu
N = 20
MiB = 1024 * 1024


def _roundtrip(oracle, L, seed, losts, decode_sets):
    s = T.Slicer.clay_default()
    data = oracle.splitmix64_bytes(seed, L)
    sl = s.encode(data.tobytes())
    exp = oracle.slicer_encode_np(oracle.OracleClay(20, 7, 16), data)
    assert len(sl) == N and len(sl[0]) == exp.shape[1]
    for i in range(N):
        assert np.array_equal(np.frombuffer(sl[i], np.uint8), exp[i]), i
    del exp
    for keep in decode_sets:
        dec = s.decode([(i, sl[i]) for i in keep])
        assert len(dec) == L and np.array_equal(np.frombuffer(dec, np.uint8), data), keep
    for lost in losts:
        assert s.repair_full(lost, [(i, sl[i]) for i in range(N) if i != lost]) == sl[lost], lost
    return s, sl


def test_track_64mib(oracle):
    L = 64 * MiB
    s, sl = _roundtrip(oracle, L, 0x64, losts=(0, 7, 13, 19),
                       decode_sets=[range(13, 20), (0, 2, 4, 9, 11, 17, 19)])
    g = s.geometry(L)
    assert (g.stripe_size, g.num_stripes) == (1_000_000, 68)
    # node recover of one slice from 7 peers (recover.rs:411-442)
    assert batch.reconstruct(s, 5, [(i, sl[i]) for i in range(8, 15)]) == sl[5]


def test_object_over_100mb_uses_10mb_stripes(oracle):
    L = 120_000_007
    s, _ = _roundtrip(oracle, L, 0x100, losts=(3, 16), decode_sets=[range(13, 20)])
    g = s.geometry(L)
    assert g.stripe_size == 10_000_000 and g.chunk_size == 1_428_600  # sub-chunk 14,286 B


def test_generic_kernel_past_2gib_of_slices(oracle):
    L = 760_000_000
    s = T.Slicer.clay_default()
    g = s.geometry(L)
    assert N * g.slice_len >= 2**31  # the fast kernels' buffer ranges would overflow
    _roundtrip(oracle, L, 0x2EB, losts=(11,), decode_sets=[range(13, 20), (1, 3, 5, 7, 9, 12, 18)])
