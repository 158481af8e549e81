"""The oracle's threaded decode / repair / recover helper (bench.py's CPU baselines of the decode,
repair and recover lines) against the oracle's own single-object entry points."""
import numpy as np


def test_slicer_many_matches_single_object_paths(oracle):
    O = oracle
    c = O.OracleClay(20, 7, 16)
    L, n = 1_048_576 + 777, 4
    objs = [O.splitmix64_bytes(11 + i, L) for i in range(n)]
    sl = [O.slicer_encode_np(c, o, chunk_index=i) for i, o in enumerate(objs)]
    slen = sl[0].shape[1]
    per = 20 * slen
    buf = np.concatenate([s.reshape(-1) for s in sl])
    masks = [sum(1 << j for j in range(13, 20)), sum(1 << j for j in (0, 3, 5, 9, 11, 15, 19)), 0x7F, 0xFE000]
    out = np.zeros(n * L, np.uint8)
    assert O.slicer_many(c, "decode", buf, per, slen, n, out, L, 3, masks=masks) == 0
    for i in range(n):
        assert (out[i * L:(i + 1) * L] == objs[i]).all()
    lost, down = [0, 7, 19, 12], [10, -1, 9, 2]
    rep = np.zeros(n * slen, np.uint8)
    assert O.slicer_many(c, "repair", buf, per, slen, n, rep, slen, 3, lost=lost, down=down) == 0
    for i, l in enumerate(lost):
        assert (rep[i * slen:(i + 1) * slen] == sl[i][l]).all()
    rec = np.zeros(n * slen, np.uint8)
    assert O.slicer_many(c, "recover", buf, per, slen, n, rec, slen, 2, masks=masks, lost=[0, 7, 19, 1]) == 0
    for i, l in enumerate([0, 7, 19, 1]):
        assert (rec[i * slen:(i + 1) * slen] == sl[i][l]).all()
    # six slices: NotEnoughSlices reported per object, not a crash
    bad = np.zeros(L, np.uint8)
    assert O.slicer_many(c, "decode", buf, per, slen, 1, bad, L, 1, masks=[0x3F]) == 1
