"""Device-resident batch entry points over torch tensors (the stream-encode / repair-worker seam).

torch is plumbing here: it owns device memory and the HIP stream; the work is enqueued by
libtapeec.so's te_*_batch_device on that stream.
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import lib
from .slicer import ClayCoder, RepairPlan, Slicer, _check


def _stream_ptr(stream) -> C.c_void_p:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def encode_batch(slicer: Slicer, data, objs: list[tuple[int, int, int, int]], out, stream=None) -> None:
    """objs: (data_off, blob_len, out_off, chunk_index) per object; data/out are uint8 cuda tensors."""
    arr = (_lib.te_object * len(objs))(*[_lib.te_object(*o) for o in objs])
    cfg = slicer._cfg()
    r = lib.te_encode_batch_device(slicer.coder.handle, C.byref(cfg), C.c_void_p(data.data_ptr()), arr, len(objs),
                                   C.c_void_p(out.data_ptr()), _stream_ptr(stream))
    _check(r, "encode")


def encode_batch_host(slicer: Slicer, data, objs: list[tuple[int, int, int, int]], out, window_bytes: int = 0) -> None:
    """Host -> host batched encode (te_encode_batch_host): data/out are host buffers (numpy arrays
    or CPU tensors, pinned for full PCIe rate); objs as for encode_batch, offsets into data/out."""
    arr = (_lib.te_object * len(objs))(*[_lib.te_object(*o) for o in objs])
    cfg = slicer._cfg()
    r = lib.te_encode_batch_host(slicer.coder.handle, C.byref(cfg), C.c_void_p(_host_ptr(data)), arr, len(objs),
                                 C.c_void_p(_host_ptr(out)), window_bytes)
    _check(r, "encode")


def _host_ptr(buf) -> int:
    if hasattr(buf, "data_ptr"):
        assert not buf.is_cuda, "host buffer expected"
        return buf.data_ptr()
    return buf.ctypes.data


def decode_batch(slicer: Slicer, slices, objs: list[tuple[int, int, int, int]], metas: bytes, out,
                 stream=None) -> None:
    """objs: (slices_off, slice_len, avail_mask, out_off); metas: nobj*48 metadata bytes (host)."""
    arr = (_lib.te_decode_object * len(objs))(*[_lib.te_decode_object(o[0], o[1], o[2], 0, o[3]) for o in objs])
    cfg = slicer._cfg()
    mb = (C.c_uint8 * max(1, len(metas))).from_buffer_copy(metas if metas else b"\0")
    r = lib.te_decode_batch_device(slicer.coder.handle, C.byref(cfg), C.c_void_p(slices.data_ptr()), arr, mb,
                                   len(objs), C.c_void_p(out.data_ptr()), _stream_ptr(stream))
    _check(r, "decode")


def repair_batch(coder: ClayCoder, helpers, objs: list[tuple[RepairPlan, dict[int, int], int, bytes]], out,
                 stream=None) -> None:
    """objs: (plan, {helper_slice: offset in helpers tensor}, out_off, metadata48)."""
    arr = (_lib.te_repair_object * len(objs))()
    for i, (plan, offs, out_off, meta) in enumerate(objs):
        arr[i].plan = plan.handle.value if hasattr(plan.handle, "value") else plan.handle
        for s in range(20):
            arr[i].helper_off[s] = offs.get(s, 0xFFFFFFFFFFFFFFFF)
        arr[i].out_off = out_off
        for j, b in enumerate(meta):
            arr[i].metadata[j] = b
    r = lib.te_repair_batch_device(coder.handle, C.c_void_p(helpers.data_ptr()), arr, len(objs),
                                   C.c_void_p(out.data_ptr()), _stream_ptr(stream))
    _check(r, "repair")
