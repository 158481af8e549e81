"""Device-resident batch entry points over torch tensors (the stream-encode / repair-worker seam).

torch is plumbing here: it owns device memory and the HIP stream; the work is enqueued by
libtapeec.so's te_*_batch_device on that stream.
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import lib
from .slicer import SLICE_TREE_HEIGHT, ClayCoder, DecodeError, RepairPlan, Slicer, _check


def _stream_ptr(stream) -> C.c_void_p:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _is_desc(objs) -> bool:
    return hasattr(objs, "_length_")  # a prepared ctypes descriptor array


def encode_descs(objs: list[tuple[int, int, int, int]]):
    """Prepared te_object array for encode_batch / encode_batch_host (build once, reuse)."""
    return (_lib.te_object * len(objs))(*[_lib.te_object(*o) for o in objs])


def encode_batch(slicer: Slicer, data, objs, out, stream=None) -> None:
    """objs: (data_off, blob_len, out_off, chunk_index) per object, or encode_descs(...) of them;
    data/out are uint8 cuda tensors."""
    arr = objs if _is_desc(objs) else encode_descs(objs)
    cfg = slicer._cfg()
    r = lib.te_encode_batch_device(slicer.coder.handle, C.byref(cfg), C.c_void_p(data.data_ptr()), arr, len(arr),
                                   C.c_void_p(out.data_ptr()), _stream_ptr(stream))
    _check(r, "encode")


def encode_batch_host(slicer: Slicer, data, objs: list[tuple[int, int, int, int]], out, window_bytes: int = 0) -> None:
    """Host -> host batched encode (te_encode_batch_host): data/out are host buffers (numpy arrays
    or CPU tensors, pinned for full PCIe rate); objs as for encode_batch, offsets into data/out."""
    arr = objs if _is_desc(objs) else encode_descs(objs)
    cfg = slicer._cfg()
    r = lib.te_encode_batch_host(slicer.coder.handle, C.byref(cfg), C.c_void_p(_host_ptr(data)), arr, len(arr),
                                 C.c_void_p(_host_ptr(out)), window_bytes)
    _check(r, "encode")


def encode_batch_host_multi(slicers: list[Slicer], data, objs: list[tuple[int, int, int, int]], out,
                            window_bytes: int = 0) -> None:
    """te_encode_batch_host_multi: one host -> host pipeline per handle (typically one handle per
    device, ClayCoder.bind_device), objects split into contiguous ranges; same profile/config."""
    arr = objs if _is_desc(objs) else encode_descs(objs)
    cfg = slicers[0]._cfg()
    hs = (C.c_void_p * len(slicers))(*[s.coder.handle.value for s in slicers])
    r = lib.te_encode_batch_host_multi(hs, len(slicers), C.byref(cfg), C.c_void_p(_host_ptr(data)), arr, len(arr),
                                       C.c_void_p(_host_ptr(out)), window_bytes)
    _check(r, "encode")


def encode_commit_batch_host(slicer: Slicer, data, objs: list[tuple[int, int, int, int]], out, leaf_hashes, roots,
                             proofs=None, height: int = SLICE_TREE_HEIGHT, window_bytes: int = 0) -> None:
    """te_encode_commit_batch_host: BlobEncoder::encode_with_proofs (sdk/src/codec/encoder.rs:220-260)
    over a batch, host -> host: slices to `out` as encode_batch_host, plus per object n leaf hashes
    (`leaf_hashes`, nobj*n*32 bytes), the root (`roots`, nobj*32) and, if `proofs` is given, the n
    proofs of `height` hashes each (nobj*n*height*32).  Host buffers (pinned for PCIe rate)."""
    arr = objs if _is_desc(objs) else encode_descs(objs)
    cfg = slicer._cfg()
    pp = C.c_void_p(_host_ptr(proofs)) if proofs is not None else None
    r = lib.te_encode_commit_batch_host(slicer.coder.handle, C.byref(cfg), C.c_void_p(_host_ptr(data)), arr, len(arr),
                                        C.c_void_p(_host_ptr(out)), height, C.c_void_p(_host_ptr(leaf_hashes)),
                                        C.c_void_p(_host_ptr(roots)), pp, window_bytes)
    _check(r, "encode")


class StreamWriter:
    """te_stream_writer: the stream writer's ordered encode stage (sdk/src/stream/write.rs:332-362,
    FuturesOrdered over chunk encodes) as one GPU pipeline per handle.  submit() enqueues a window --
    te_encode_commit_batch_host's outputs for its objects -- and returns its ticket at once; wait()
    completes every window up to a ticket in submission order.  The window's host buffers (pinned
    for full overlap) are kept referenced here until its ticket has been waited for."""

    def __init__(self, slicers: list[Slicer], height: int = SLICE_TREE_HEIGHT, group_bytes: int = 0,
                 hashing: str = "auto"):
        self._cfg = slicers[0]._cfg()
        self._coders = [s.coder for s in slicers]  # the handles outlive the writer
        hs = (C.c_void_p * len(slicers))(*[s.coder.handle.value for s in slicers])
        h = C.c_void_p()
        _check(lib.te_stream_writer_new(hs, len(slicers), C.byref(self._cfg), height, group_bytes, C.byref(h)),
               "encode")
        self._h = h
        self._keep = {}
        self.set_hashing(hashing)

    def set_hashing(self, mode: str) -> None:
        """Who hashes the leaves (te_stream_writer_set_hashing): "auto" (per window, from its slice
        count and length), "device" (leaf kernel over groups of windows) or "host" (worker pool
        over the host slices as their D2H copies land -- the SDK's 64 MiB chunk shape)."""
        _check(lib.te_stream_writer_set_hashing(self._h, HASHING[mode]), "encode")

    def submit(self, data, objs, out, leaf_hashes, roots, proofs=None) -> int:
        arr = objs if _is_desc(objs) else encode_descs(objs)
        t = C.c_uint64()
        pp = C.c_void_p(_host_ptr(proofs)) if proofs is not None else None
        r = lib.te_stream_submit(self._h, C.c_void_p(_host_ptr(data)), arr, len(arr), C.c_void_p(_host_ptr(out)),
                                 C.c_void_p(_host_ptr(leaf_hashes)), C.c_void_p(_host_ptr(roots)), pp, C.byref(t))
        self._keep[t.value] = (data, arr, out, leaf_hashes, roots, proofs)
        _check(r, "encode")
        return t.value

    def wait(self, ticket: int) -> None:
        r = lib.te_stream_wait(self._h, ticket)
        for t in [t for t in self._keep if t <= ticket]:
            del self._keep[t]
        _check(r, "encode")

    def close(self) -> None:
        if self._h:
            lib.te_stream_writer_free(self._h)
            self._h = None
            self._keep.clear()

    def __del__(self):
        self.close()


HASHING = {"auto": 0, "device": 1, "host": 2}  # TE_HASH_AUTO / _DEVICE / _HOST


def set_commit_hashing(mode: str) -> None:
    """Process default for te_encode_commit_batch_host and new stream writers (te_set_commit_hashing)."""
    _check(lib.te_set_commit_hashing(HASHING[mode]), "encode")


def set_host_hash_threads(threads: int) -> None:
    """Host hashing pool size (te_set_host_hash_threads; 0 = min(16, affinity CPUs))."""
    _check(lib.te_set_host_hash_threads(threads), "encode")


def host_hash_threads() -> int:
    return lib.te_host_hash_threads()


def kernel_timing(enable: bool) -> None:
    """te_kernel_timing: record HIP events around every batch call's kernel launches."""
    _check(lib.te_kernel_timing(1 if enable else 0), "kernel timing")


def kernel_time_ms() -> tuple[float, int]:
    """(summed kernel ms, calls) since the last read (te_kernel_time_ms; synchronises)."""
    ms, n = C.c_double(0), C.c_uint32(0)
    _check(lib.te_kernel_time_ms(C.byref(ms), C.byref(n)), "kernel timing")
    return ms.value, n.value


def host_empty(nbytes: int):
    """A numpy uint8 array in page-locked host memory (te_host_alloc), freed with the array: the
    host buffers of encode_batch_host / StreamWriter.submit copy at full PCIe rate from it."""
    import weakref
    import numpy as np
    p = C.c_void_p()
    _check(lib.te_host_alloc(nbytes, C.byref(p)), "encode")
    raw = (C.c_uint8 * max(1, nbytes)).from_address(p.value)
    weakref.finalize(raw, lib.te_host_free, C.c_void_p(p.value))
    return np.frombuffer(raw, dtype=np.uint8)[:nbytes]


def host_register(arr) -> None:
    """Pin an existing host array in place (te_host_register); undo with host_unregister."""
    _check(lib.te_host_register(C.c_void_p(_host_ptr(arr)), arr.nbytes), "encode")


def host_unregister(arr) -> None:
    _check(lib.te_host_unregister(C.c_void_p(_host_ptr(arr))), "encode")


def _host_ptr(buf) -> int:
    if hasattr(buf, "data_ptr"):
        assert not buf.is_cuda, "host buffer expected"
        return buf.data_ptr()
    return buf.ctypes.data


def decode_descs(objs: list[tuple[int, int, int, int]]):
    """Prepared te_decode_object array for decode_batch (build once, reuse)."""
    return (_lib.te_decode_object * len(objs))(*[_lib.te_decode_object(o[0], o[1], o[2], 0, o[3]) for o in objs])


def decode_batch(slicer: Slicer, slices, objs, metas: bytes, out, stream=None) -> None:
    """objs: (slices_off, slice_len, avail_mask, out_off), or decode_descs(...) of them; metas:
    nobj*48 metadata bytes (host)."""
    arr = objs if _is_desc(objs) else decode_descs(objs)
    cfg = slicer._cfg()
    mb = (C.c_uint8 * max(1, len(metas))).from_buffer_copy(metas if metas else b"\0")
    r = lib.te_decode_batch_device(slicer.coder.handle, C.byref(cfg), C.c_void_p(slices.data_ptr()), arr, mb,
                                   len(arr), C.c_void_p(out.data_ptr()), _stream_ptr(stream))
    _check(r, "decode")


def recover_batch(slicer: Slicer, slices, objs: list[tuple[int, int, int, int, int]], metas: bytes, out,
                  stream=None) -> None:
    """Node recover (recover.rs:411-442 `reconstruct`) on the device: objs are (slices_off,
    slice_len, avail_mask, lost, out_off); metas nobj*48 metadata bytes (host)."""
    arr = (_lib.te_recover_object * len(objs))(*[_lib.te_recover_object(*o) for o in objs])
    cfg = slicer._cfg()
    mb = (C.c_uint8 * max(1, len(metas))).from_buffer_copy(metas if metas else b"\0")
    r = lib.te_recover_batch_device(slicer.coder.handle, C.byref(cfg), C.c_void_p(slices.data_ptr()), arr, mb,
                                    len(arr), C.c_void_p(out.data_ptr()), _stream_ptr(stream))
    _check(r, "recover")


def reconstruct(slicer: Slicer, lost: int, peer_slices: list[tuple[int, bytes]]) -> bytes:
    """recover.rs:411-442 `reconstruct`: decode the peers' slices, re-encode, return slice `lost`
    (one object, host bytes in and out, through recover_batch)."""
    import torch
    if not peer_slices:
        raise ValueError("no peer slices provided")
    slen = len(peer_slices[0][1])
    n = slicer.coder.n()
    if not 0 <= lost < n:
        raise ValueError(f"lost slice {lost} out of range")
    host = bytearray(n * slen)
    mask = 0
    for i, d in peer_slices:
        # validate_layout (slicer.rs:79-105): every slice the same length, indices in range, once
        if not 0 <= i < n or mask >> i & 1:
            raise DecodeError("InvalidLayout")
        if len(d) != slen:
            raise DecodeError("InvalidLayout")
        host[i * slen:(i + 1) * slen] = d
        mask |= 1 << i
    dev = torch.frombuffer(host, dtype=torch.uint8).cuda()
    out = torch.empty(slen, dtype=torch.uint8, device="cuda")
    recover_batch(slicer, dev, [(0, slen, mask, lost, 0)], bytes(peer_slices[0][1][-48:]), out)
    torch.cuda.synchronize()
    return out.cpu().numpy().tobytes()


def repair_descs(objs: list[tuple[RepairPlan, dict[int, int], int, bytes]]):
    """Prepared te_repair_object array for repair_batch (build once, reuse; the plans must stay
    alive while it is used)."""
    arr = (_lib.te_repair_object * len(objs))()
    for i, (plan, offs, out_off, meta) in enumerate(objs):
        arr[i].plan = plan.handle.value if hasattr(plan.handle, "value") else plan.handle
        for s in range(20):
            arr[i].helper_off[s] = offs.get(s, 0xFFFFFFFFFFFFFFFF)
        arr[i].out_off = out_off
        for j, b in enumerate(meta):
            arr[i].metadata[j] = b
    return arr


def repair_batch(coder: ClayCoder, helpers, objs, out, stream=None) -> None:
    """objs: (plan, {helper_slice: offset in helpers tensor}, out_off, metadata48) per object, or
    repair_descs(...) of them."""
    arr = objs if _is_desc(objs) else repair_descs(objs)
    r = lib.te_repair_batch_device(coder.handle, C.c_void_p(helpers.data_ptr()), arr, len(arr),
                                   C.c_void_p(out.data_ptr()), _stream_ptr(stream))
    _check(r, "repair")
