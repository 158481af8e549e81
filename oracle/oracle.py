"""ctypes front-end for the TEST-ONLY oracle (oracle/clay_oracle.c).

This module is the parity checker and the CPU-baseline restatement of the reference hot path
(lib/slicer/src/{clay,slicer,repair,metadata,adaptive}.rs over the absent `clay-codes` 0.1.1 /
`reed-solomon-erasure` 6.0.0 crates).  Only tests/, __graft_entry__.smoke() and bench.py's
`cpu_baseline` leg may import it.  Parity of encoded *parity* bytes with the real crate is
UNPINNED (no reference fixture pins them).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "libclay_oracle.so")
META = 48
STRIPE_SIZES = (100_000, 1_000_000, 10_000_000)
CLAY_DEFAULT_PARAMS = 20 | (7 << 8) | (16 << 16)  # lib/core/src/encoding.rs:236-239
ENCODING_CLAY = 2                                   # lib/core/src/encoding.rs:25


def build() -> str:
    """Compile the oracle with gcc (make)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def _lib():
    global _L
    try:
        return _L
    except NameError:
        pass
    if not os.path.exists(_SO) or os.path.getmtime(_SO) < os.path.getmtime(os.path.join(_HERE, "clay_oracle.c")):
        build()
    L = C.CDLL(_SO)
    vp, i, sz, u64 = C.c_void_p, C.c_int, C.c_size_t, C.c_uint64
    ip = C.POINTER(C.c_int)
    L.oc_clay_sizeof.restype = i
    L.oc_clay_init.argtypes = [vp, i, i, i]
    L.oc_clay_param.argtypes = [vp, i]
    L.oc_chunk_size_for.argtypes = [vp, sz]
    L.oc_chunk_size_for.restype = sz
    L.oc_clay_encode.argtypes = [vp, vp, sz, vp]
    L.oc_clay_decode.argtypes = [vp, vp, ip, sz, vp]
    L.oc_repair_subchunks.argtypes = [vp, i, ip]
    L.oc_minimum_to_repair.argtypes = [vp, i, ip, i, ip]
    L.oc_clay_repair.argtypes = [vp, i, ip, i, vp, sz, vp]
    L.oc_pick_stripe_size.argtypes = [sz]
    L.oc_pick_stripe_size.restype = sz
    L.oc_num_stripes.argtypes = [sz, sz]
    L.oc_num_stripes.restype = sz
    L.oc_shard_to_slice.argtypes = [i, i, i, i]
    L.oc_slice_to_shard.argtypes = [i, i, i, i]
    L.oc_slicer_geometry.argtypes = [vp, sz, C.POINTER(sz), C.POINTER(sz), C.POINTER(sz)]
    L.oc_slicer_geometry.restype = sz
    L.oc_slicer_encode.argtypes = [vp, i, u64, u64, u64, vp, sz, vp]
    L.oc_slicer_decode.argtypes = [vp, i, vp, ip, sz, vp]
    L.oc_slicer_decode.restype = C.c_long
    L.oc_repair_plan.argtypes = [vp, i, i, ip, i, sz, sz, ip, ip, ip, ip]
    L.oc_repair_plan.restype = C.c_long
    L.oc_slicer_encode_many.argtypes = [vp, vp, sz, i, vp, sz, i]
    L.oc_slicer_many.argtypes = [vp, i, vp, sz, sz, vp, vp, vp, i, vp, sz, i, vp]
    L.oc_generator.argtypes = [vp, vp]
    L.oc_gf_mul.argtypes = [C.c_uint8, C.c_uint8]
    L.oc_gf_mul.restype = C.c_uint8
    _L = L
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _ip(lst):
    arr = (C.c_int * max(1, len(lst)))(*lst)
    return arr


def gf_mul(a: int, b: int) -> int:
    return int(_lib().oc_gf_mul(a, b))


class OracleClay:
    """Restatement of ClayCoder over clay_codes::ClayCode (lib/slicer/src/clay.rs:13-122)."""

    def __init__(self, n: int, k: int, d: int):
        L = _lib()
        self._buf = C.create_string_buffer(L.oc_clay_sizeof())
        r = L.oc_clay_init(self._buf, n, k, d)
        if r:
            raise ValueError(f"invalid clay params ({n},{k},{d}): {r}")
        p = [L.oc_clay_param(self._buf, j) for j in range(9)]
        self.n, self.k, self.m, self.d, self.q, self.t, self.nu, self.alpha, self.beta = p

    @property
    def h(self):
        return self._buf

    def generator(self) -> np.ndarray:
        qt = self.q * self.t
        out = np.zeros((qt, self.k + self.nu), np.uint8)
        _lib().oc_generator(self._buf, _ptr(out))
        return out

    def chunk_size_for(self, n: int) -> int:
        return int(_lib().oc_chunk_size_for(self._buf, n))

    def encode(self, data: bytes) -> list[bytes]:
        if len(data) == 0:
            raise ValueError("EmptyInput")
        cs = self.chunk_size_for(len(data))
        src = np.frombuffer(bytes(data), np.uint8)
        out = np.zeros(self.n * cs, np.uint8)
        r = _lib().oc_clay_encode(self._buf, _ptr(src), len(data), _ptr(out))
        assert r == 0, r
        return [out[i * cs:(i + 1) * cs].tobytes() for i in range(self.n)]

    def decode(self, chunks: dict[int, bytes]) -> bytes:
        if len(chunks) < self.k:
            raise ValueError("NotEnoughSlices")
        cs = len(next(iter(chunks.values())))
        buf = np.zeros(self.n * cs, np.uint8)
        avail = [0] * self.n
        for i, c in chunks.items():
            buf[i * cs:(i + 1) * cs] = np.frombuffer(c, np.uint8)
            avail[i] = 1
        out = np.zeros(self.k * cs, np.uint8)
        r = _lib().oc_clay_decode(self._buf, _ptr(buf), _ip(avail), cs, _ptr(out))
        if r:
            raise ValueError(f"BadEncoding ({r})")
        return out.tobytes()

    def repair_subchunks(self, lost: int) -> list[int]:
        pl = (C.c_int * self.alpha)()
        nb = _lib().oc_repair_subchunks(self._buf, lost, pl)
        return list(pl[:nb])

    def minimum_to_repair(self, lost: int, available: list[int]) -> list[tuple[int, list[int]]]:
        hs = (C.c_int * 64)()
        h = _lib().oc_minimum_to_repair(self._buf, lost, _ip(available), len(available), hs)
        if h < 0:
            raise ValueError(f"clay: cannot repair ({h})")
        planes = self.repair_subchunks(lost)
        return [(hs[j], list(planes)) for j in range(h)]

    def repair(self, lost: int, helpers: dict[int, bytes], chunk_size: int) -> bytes:
        ids = sorted(helpers)
        rb = len(helpers[ids[0]])
        buf = np.zeros(len(ids) * rb, np.uint8)
        for j, i in enumerate(ids):
            buf[j * rb:(j + 1) * rb] = np.frombuffer(helpers[i], np.uint8)
        out = np.zeros(chunk_size, np.uint8)
        r = _lib().oc_clay_repair(self._buf, lost, _ip(ids), len(ids), _ptr(buf), chunk_size, _ptr(out))
        if r:
            raise ValueError(f"clay repair failed ({r})")
        return out.tobytes()


def pick_stripe_size(n: int) -> int:
    return int(_lib().oc_pick_stripe_size(n))


def num_stripes(n: int, s: int) -> int:
    return int(_lib().oc_num_stripes(n, s))


def shard_to_slice(rotated: bool, n: int, stripe: int, shard: int) -> int:
    return _lib().oc_shard_to_slice(int(rotated), n, stripe, shard)


def slice_to_shard(rotated: bool, n: int, stripe: int, sl: int) -> int:
    return _lib().oc_slice_to_shard(int(rotated), n, stripe, sl)


def geometry(clay: OracleClay, blob_len: int) -> tuple[int, int, int, int]:
    S, ns, cs = C.c_size_t(), C.c_size_t(), C.c_size_t()
    sl = _lib().oc_slicer_geometry(clay.h, blob_len, C.byref(S), C.byref(ns), C.byref(cs))
    return int(S.value), int(ns.value), int(cs.value), int(sl)


def slicer_encode(clay: OracleClay, data: bytes, rotated: bool = True, chunk_index: int = 0,
                  params: int | None = None, encoding: int = ENCODING_CLAY) -> list[bytes]:
    """Slicer<ClayCoder>::encode (lib/slicer/src/slicer.rs:237-296)."""
    if params is None:
        params = CLAY_DEFAULT_PARAMS
    S, ns, cs, sl = geometry(clay, len(data))
    src = np.frombuffer(bytes(data), np.uint8) if len(data) else np.zeros(1, np.uint8)
    out = np.zeros(clay.n * sl, np.uint8)
    r = _lib().oc_slicer_encode(clay.h, int(rotated), encoding, params, chunk_index, _ptr(src), len(data), _ptr(out))
    assert r == 0
    return [out[i * sl:(i + 1) * sl].tobytes() for i in range(clay.n)]


def slicer_encode_np(clay: OracleClay, data: np.ndarray, rotated: bool = True, chunk_index: int = 0) -> np.ndarray:
    """Same as slicer_encode but numpy in/out: returns (n, slice_len) uint8."""
    S, ns, cs, sl = geometry(clay, data.size)
    out = np.zeros((clay.n, sl), np.uint8)
    src = np.ascontiguousarray(data) if data.size else np.zeros(1, np.uint8)
    r = _lib().oc_slicer_encode(clay.h, int(rotated), ENCODING_CLAY, CLAY_DEFAULT_PARAMS, chunk_index,
                                _ptr(src), data.size, _ptr(out))
    assert r == 0
    return out


def slicer_decode(clay: OracleClay, slices: dict[int, bytes], rotated: bool = True) -> bytes:
    """Slicer::decode (lib/slicer/src/slicer.rs:298-364)."""
    if not slices:
        raise ValueError("NotEnoughSlices")
    sl = len(next(iter(slices.values())))
    if any(len(v) != sl for v in slices.values()):
        raise ValueError("InvalidLayout")
    buf = np.zeros(clay.n * sl, np.uint8)
    avail = [0] * clay.n
    for i, s in slices.items():
        buf[i * sl:(i + 1) * sl] = np.frombuffer(s, np.uint8)
        avail[i] = 1
    meta = next(iter(slices.values()))[-META:]
    blob_len = int.from_bytes(meta[8:16], "little")
    out = np.zeros(max(1, blob_len), np.uint8)
    r = _lib().oc_slicer_decode(clay.h, int(rotated), _ptr(buf), _ip(avail), sl, _ptr(out))
    if r == -1:
        raise ValueError("NotEnoughSlices")
    if r == -2:
        raise ValueError("InvalidLayout")
    if r < 0:
        raise ValueError("BadEncoding")
    return out[:r].tobytes()


def repair_plan(clay: OracleClay, lost: int, available: list[int], blob_len: int, stripe: int,
                rotated: bool = True):
    """repair_plan_from_params (lib/slicer/src/repair.rs:137-201).
    Returns (chunk_size, [(stripe, lost_shard, [(slice, shard, [planes])...])...])."""
    ns = num_stripes(blob_len, stripe)
    d, b = clay.d, clay.beta
    ls = (C.c_int * ns)()
    hsl = (C.c_int * (ns * d))()
    hsh = (C.c_int * (ns * d))()
    pl = (C.c_int * (ns * d * b))()
    cs = _lib().oc_repair_plan(clay.h, int(rotated), lost, _ip(available), len(available), blob_len, stripe,
                               ls, hsl, hsh, pl)
    if cs < 0:
        raise ValueError(f"repair plan failed ({cs})")
    stripes = []
    for s in range(ns):
        helpers = [(hsl[s * d + j], hsh[s * d + j], list(pl[(s * d + j) * b:(s * d + j + 1) * b])) for j in range(d)]
        stripes.append((s, ls[s], helpers))
    return int(cs), stripes


def extract_repair_data(slice_bytes: bytes, cs: int, alpha: int, stripes, helper: int) -> bytes:
    """extract_repair_data (lib/slicer/src/repair.rs:97-130)."""
    sc = cs // alpha
    out = bytearray()
    for (s, _lost, helpers) in stripes:
        for (slc, _sh, planes) in helpers:
            if slc != helper:
                continue
            chunk = slice_bytes[s * cs:(s + 1) * cs]
            for z in planes:
                out += chunk[z * sc:(z + 1) * sc]
    return bytes(out)


def slicer_repair(clay: OracleClay, cs: int, stripes, helper_data: dict[int, bytes], metadata: bytes) -> bytes:
    """Slicer::repair (lib/slicer/src/repair.rs:324-367)."""
    sc = cs // clay.alpha
    offsets = {}
    out = bytearray()
    for (s, lost_shard, helpers) in stripes:
        per = {}
        for (slc, sh, planes) in helpers:
            buf = helper_data[slc]
            off = offsets.get(slc, 0)
            nbytes = len(planes) * sc
            per[sh] = buf[off:off + nbytes]
            offsets[slc] = off + nbytes
        out += clay.repair(lost_shard, per, cs)
    out += metadata
    return bytes(out)


def encode_many(clay: OracleClay, data: np.ndarray, obj_len: int, nobj: int, out: np.ndarray,
                out_stride: int, threads: int) -> None:
    """CPU-baseline helper: Slicer::clay_default().encode over nobj objects on `threads` threads."""
    _lib().oc_slicer_encode_many(clay.h, _ptr(data), obj_len, nobj, _ptr(out), out_stride, threads)


MANY_KIND = {"decode": 0, "repair": 1, "recover": 2}


def slicer_many(clay: OracleClay, kind: str, slices: np.ndarray, obj_stride: int, slice_len: int, nobj: int,
                out: np.ndarray, out_stride: int, threads: int, masks=None, lost=None, down=None) -> int:
    """CPU-baseline helper (bench.py decode / repair / recover lines): one object per task on
    `threads` threads, object o's 20 slices at slices[o * obj_stride:].
      decode : Slicer::decode from the slices in masks[o] (slicer.rs:298-364) -> out (blob_len bytes);
      repair : Slicer::repair of slice lost[o] from the plan over every slice but lost[o] and down[o]
               (repair.rs:137-201, 97-130, 324-367) -> out (one slice);
      recover: decode from masks[o], re-encode, keep slice lost[o] (recover.rs:411-442) -> out.
    Returns the number of objects that failed."""
    def arr(v, ct):
        if v is None:
            return None
        a = (ct * max(1, nobj))(*[int(x) for x in v])
        return a
    st = (C.c_int * max(1, nobj))()
    m, l, d = arr(masks, C.c_uint32), arr(lost, C.c_int), arr(down, C.c_int)
    return int(_lib().oc_slicer_many(clay.h, MANY_KIND[kind], _ptr(slices), obj_stride, slice_len, m, l, d, nobj,
                                     _ptr(out), out_stride, threads, st))


def splitmix64_bytes(seed: int, nbytes: int) -> np.ndarray:
    """byte j = SplitMix64(seed) stream word floor(j/8), little-endian."""
    nw = (nbytes + 7) // 8
    idx = np.arange(1, nw + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()


def test_pattern(n: int) -> bytes:
    """(i % 251) as u8 -- lib/slicer/src/slicer.rs:397-399, clay.rs:133-135."""
    return (np.arange(n, dtype=np.int64) % 251).astype(np.uint8).tobytes()
