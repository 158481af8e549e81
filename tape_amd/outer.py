"""OuterCoder (lib/slicer/src/outer.rs:19-197): single-level Reed-Solomon over GF(2^16)
distributing data over n chunks such that any k reconstruct it -- the snapshot coder
(lib/snapshot/src/encode.rs:66-76).  The codec is the Leopard construction of reed-solomon-simd
3.1.0, run on the GPU by libtapeec (te_outer_*); parity unpinned against the absent crate."""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import lib
from .slicer import DecodeError, EncodeError, _buf, _check

MAX_CHUNK_BYTES = 4 * 1024 * 1024  # outer.rs:12


class OuterCoder:
    def __init__(self, k: int, n: int):
        assert k > 0, "k must be > 0"      # outer.rs:30
        assert k <= n, "k must be <= n"    # outer.rs:31
        self._k, self._n = k, n

    def k(self) -> int:
        return self._k

    def n(self) -> int:
        return self._n

    def m(self) -> int:
        return self._n - self._k

    def encode(self, data: bytes) -> list[bytes]:
        """OuterCoder::encode (outer.rs:70-118): n chunks, the first k the zero-padded data."""
        cb = int(lib.te_outer_chunk_bytes(self._k, len(data)))
        out = (C.c_uint8 * (self._n * cb))()
        got = C.c_size_t()
        r = lib.te_outer_encode(self._k, self._n, _buf(data), len(data), out, len(out), C.byref(got))
        _check(r, "encode")
        raw = bytes(out)
        return [raw[i * cb:(i + 1) * cb] for i in range(self._n)]

    def decode(self, chunks: list[tuple[int, bytes]]) -> bytes:
        """OuterCoder::decode (outer.rs:126-197): the k data chunks (with their padding)."""
        if len(chunks) < self._k:
            raise DecodeError("NotEnoughSlices")
        cb = len(chunks[0][1])
        if any(len(d) != cb for _, d in chunks) or any(i >= self._n or i < 0 for i, _ in chunks):
            raise DecodeError("InvalidLayout")
        ptrs = (C.c_void_p * self._n)()
        keep = {}
        for i, d in chunks:
            keep[i] = C.create_string_buffer(bytes(d), cb)
            ptrs[i] = C.cast(keep[i], C.c_void_p)
        out = (C.c_uint8 * max(1, self._k * cb))()
        r = lib.te_outer_decode(self._k, self._n, ptrs, cb, out, len(out))
        _check(r, "decode")
        return bytes(out)[:self._k * cb]


class ReedSolomonCoder(OuterCoder):
    """ReedSolomonCoder (lib/slicer/src/reed_solomon.rs:17-181): the Basic profile's coder
    ("testing/debugging only", reed_solomon.rs:10-13) -- the same GF(2^16) codec with
    (k data, m parity) and a slice-size ceiling (MAX_SLICE_BYTES = 4 KiB by default)."""

    MAX_SLICE_BYTES = 1 << 12  # reed_solomon.rs:13

    def __init__(self, k: int, m: int, max_slice_bytes: int = MAX_SLICE_BYTES):
        assert k > 0, "k must be > 0"                      # reed_solomon.rs:38-40
        assert m > 0, "m must be > 0"
        assert max_slice_bytes > 0, "max_slice_bytes must be > 0"
        assert k + m <= 65536, "too many total slices for RS field"
        super().__init__(k, k + m)
        self.max_slice_bytes = max_slice_bytes

    def encode(self, data: bytes) -> list[bytes]:
        if int(lib.te_outer_chunk_bytes(self._k, len(data))) > self.max_slice_bytes:
            raise EncodeError("TooMuchData")               # reed_solomon.rs:85-87
        return super().encode(data)


def encode_device(k: int, m: int, d_in, chunk_bytes: int, segments: int, seg_in: int, d_out, seg_out: int,
                  stream=None) -> None:
    """te_outer_encode_device: `segments` OuterCoder encodes on device buffers (torch tensors)."""
    sp = stream.cuda_stream if stream is not None else None
    r = lib.te_outer_encode_device(k, m, C.c_void_p(d_in.data_ptr()), chunk_bytes, segments, seg_in,
                                   C.c_void_p(d_out.data_ptr()), seg_out, C.c_void_p(sp) if sp else None)
    _check(r, "encode")


def decode_device(k: int, n: int, chunks: list, chunk_bytes: int, d_out, stream=None) -> None:
    """te_outer_decode_device: the k data chunks into d_out (a torch tensor of k * chunk_bytes)
    from device chunks (`chunks[i]`: a device address, a torch tensor, or None when missing)."""
    ptrs = (C.c_void_p * n)(*[None if c is None else (c.data_ptr() if hasattr(c, "data_ptr") else int(c))
                              for c in chunks])
    sp = stream.cuda_stream if stream is not None else None
    r = lib.te_outer_decode_device(k, n, C.cast(ptrs, C.POINTER(C.c_void_p)), chunk_bytes,
                                   C.c_void_p(d_out.data_ptr()), C.c_void_p(sp) if sp else None)
    _check(r, "decode")


def decode_device_batch(k: int, n: int, chunks: list, chunk_bytes: int, d_out, seg_out: int, stream=None) -> None:
    """te_outer_decode_device_batch: `len(chunks)` segments in one call; chunks[g] is segment g's
    list of n device chunks (address, tensor or None), its k data chunks go to d_out + g * seg_out.
    Enqueued on the stream (segments sharing an erasure pattern share launches)."""
    segs = len(chunks)
    flat = [None if c is None else (c.data_ptr() if hasattr(c, "data_ptr") else int(c)) for seg in chunks for c in seg]
    if any(len(seg) != n for seg in chunks):
        raise ValueError("every segment needs n chunk entries")
    ptrs = (C.c_void_p * max(1, len(flat)))(*flat)
    sp = stream.cuda_stream if stream is not None else None
    r = lib.te_outer_decode_device_batch(k, n, C.cast(ptrs, C.POINTER(C.c_void_p)), segs, chunk_bytes,
                                         C.c_void_p(d_out.data_ptr()), seg_out, C.c_void_p(sp) if sp else None)
    _check(r, "decode")


__all__ = ["OuterCoder", "ReedSolomonCoder", "encode_device", "decode_device", "decode_device_batch", "MAX_CHUNK_BYTES", "EncodeError",
           "DecodeError", "_lib"]
