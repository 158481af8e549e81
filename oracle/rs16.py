"""TEST INFRASTRUCTURE ONLY: ctypes front of oracle/rs16_oracle.c (GF(2^16) Leopard RS, the
algorithm of reed-solomon-simd 3.1.0 -- parity unpinned, see the C file's header) and a
restatement of lib/slicer/src/outer.rs OuterCoder on top of it.  Never imported by tape_amd."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "librs16_oracle.so")
MAX_CHUNK_BYTES = 4 * 1024 * 1024  # outer.rs:12
_L = None


def _lib():
    global _L
    if _L is None:
        if not os.path.exists(_SO):
            subprocess.run(["make", "-s", "-C", _HERE, "librs16_oracle.so"], check=True)
        L = C.CDLL(_SO)
        sz, vp = C.c_size_t, C.c_void_p
        L.rs16_use_high_rate.argtypes = [sz, sz]
        L.rs16_encode.argtypes = [sz, sz, sz, C.POINTER(vp), C.POINTER(vp)]
        L.rs16_decode.argtypes = [sz, sz, sz, C.POINTER(vp), C.POINTER(vp)]
        for f in ("rs16_exp", "rs16_log", "rs16_skew"):
            getattr(L, f).argtypes = [C.c_uint32]
            getattr(L, f).restype = C.c_uint16
        _L = L
    return _L


def use_high_rate(k: int, m: int) -> int:
    return _lib().rs16_use_high_rate(k, m)


def encode(k: int, m: int, shards: list[bytes]) -> list[bytes]:
    """ReedSolomonEncoder: k equal original shards (len % 64 == 0) -> m recovery shards."""
    n = len(shards[0])
    bufs = [C.create_string_buffer(bytes(s), n) for s in shards]
    outs = [C.create_string_buffer(n) for _ in range(m)]
    ip = (C.c_void_p * k)(*[C.cast(b, C.c_void_p) for b in bufs])
    op = (C.c_void_p * m)(*[C.cast(b, C.c_void_p) for b in outs])
    r = _lib().rs16_encode(k, m, n, ip, op)
    if r:
        raise ValueError(f"unsupported shape k={k} m={m} bytes={n}")
    return [o.raw for o in outs]


def decode(k: int, m: int, present: dict[int, bytes]) -> list[bytes]:
    """ReedSolomonDecoder: shards by index (originals 0..k, recovery k..k+m) -> the k originals."""
    n = len(next(iter(present.values())))
    bufs = {i: C.create_string_buffer(bytes(s), n) for i, s in present.items()}
    outs = [C.create_string_buffer(n) for _ in range(k)]
    ip = (C.c_void_p * (k + m))(*[C.cast(bufs[i], C.c_void_p) if i in bufs else None for i in range(k + m)])
    op = (C.c_void_p * k)(*[C.cast(b, C.c_void_p) for b in outs])
    r = _lib().rs16_decode(k, m, n, ip, op)
    if r == -2:
        raise ValueError("NotEnoughSlices")
    if r:
        raise ValueError("InvalidLayout")
    return [o.raw for o in outs]


class OracleOuter:
    """lib/slicer/src/outer.rs:19-197 over the oracle codec."""

    def __init__(self, k: int, n: int):
        assert k > 0 and k <= n  # outer.rs:30-31
        self.k, self.n, self.m = k, n, n - k

    @staticmethod
    def chunk_bytes(k: int, data_len: int) -> int:  # outer.rs:74-80
        if data_len == 0:
            return 64
        raw = (data_len + k - 1) // k
        return (raw + 63) // 64 * 64

    def encode(self, data: bytes) -> list[bytes]:  # outer.rs:70-118
        cb = self.chunk_bytes(self.k, len(data))
        if cb > MAX_CHUNK_BYTES:
            raise ValueError("TooMuchData")
        padded = bytes(data) + bytes(self.k * cb - len(data))
        chunks = [padded[i * cb:(i + 1) * cb] for i in range(self.k)]
        if self.m == 0:
            return chunks
        return chunks + encode(self.k, self.m, chunks)

    def decode(self, chunks: list[tuple[int, bytes]]) -> bytes:  # outer.rs:126-197
        if len(chunks) < self.k:
            raise ValueError("NotEnoughSlices")
        cb = len(chunks[0][1])
        if any(len(d) != cb for _, d in chunks):
            raise ValueError("InvalidLayout")
        have = {}
        for i, d in chunks:
            if i >= self.n:
                raise ValueError("InvalidLayout")
            have[i] = d
        if self.m == 0:
            if any(i not in have for i in range(self.k)):
                raise ValueError("InvalidLayout")
            return b"".join(have[i] for i in range(self.k))
        return b"".join(decode(self.k, self.m, have))
