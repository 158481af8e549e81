"""ctypes binding of libtapeec.so (include/tape_ec.h).

The library is built in-tree (tape_amd/libtapeec.so, `make -C tape_amd`).  There is no Python or
CPU fallback for any compute entry point: if the shared object is missing, importing this module
raises, and compute calls on a host without a gfx950 device raise `NoDeviceError`.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TAPE_EC_LIB") or os.path.join(_HERE, "libtapeec.so")  # override: an alternate build
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "tape_ec.h")

TE_OK = 0
TE_ERR_TOO_MUCH_DATA = 1
TE_ERR_EMPTY_INPUT = 2
TE_ERR_NOT_ENOUGH_SLICES = 3
TE_ERR_BAD_ENCODING = 4
TE_ERR_INVALID_LAYOUT = 5
TE_ERR_NOT_ENOUGH_HELPERS = 6
TE_ERR_INVALID_SLICE = 7
TE_ERR_CLAY = 8
TE_ERR_MISSING_HELPER = 9
TE_ERR_MERKLE_TREE_FULL = 10
TE_ERR_MERKLE_INVALID_PROOF = 11
TE_ERR_MERKLE_INVALID_INDEX = 12
TE_ERR_MERKLE_PROOF_LENGTH = 13
TE_ERR_INVALID_ARG = 20
TE_ERR_NO_DEVICE = 21
TE_ERR_HIP = 22
TE_ERR_UNSUPPORTED = 23
TE_ERR_OUT_OF_MEMORY = 24
TE_ERR_BUFFER_TOO_SMALL = 25
META_SIZE = 48


class te_clay_info(C.Structure):
    _fields_ = [(f, C.c_uint32) for f in ("n", "k", "m", "d", "q", "t", "nu", "alpha", "beta")]


class te_slice_metadata(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("version", "blob_len", "stripe_size", "encoding", "params", "chunk_index")]


class te_slicer_cfg(C.Structure):
    _fields_ = [("rotated", C.c_int), ("encoding", C.c_uint64), ("params", C.c_uint64), ("chunk_index", C.c_uint64)]


class te_geometry(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("stripe_size", "num_stripes", "chunk_size", "sub_chunk_size", "slice_len")]


class te_repair_plan_info(C.Structure):
    _fields_ = [("lost", C.c_uint32), ("num_stripes", C.c_uint32), ("d", C.c_uint32), ("beta", C.c_uint32),
                ("chunk_size", C.c_uint64), ("sub_chunk_size", C.c_uint64)]


class te_object(C.Structure):
    _fields_ = [("data_off", C.c_uint64), ("blob_len", C.c_uint64), ("out_off", C.c_uint64),
                ("chunk_index", C.c_uint64)]


class te_decode_object(C.Structure):
    _fields_ = [("slices_off", C.c_uint64), ("slice_len", C.c_uint64), ("avail_mask", C.c_uint32),
                ("pad_", C.c_uint32), ("out_off", C.c_uint64)]


class te_recover_object(C.Structure):
    _fields_ = [("slices_off", C.c_uint64), ("slice_len", C.c_uint64), ("avail_mask", C.c_uint32),
                ("lost", C.c_uint32), ("out_off", C.c_uint64)]


class te_repair_object(C.Structure):
    _fields_ = [("plan", C.c_void_p), ("helper_off", C.c_uint64 * 20), ("out_off", C.c_uint64),
                ("metadata", C.c_uint8 * 48)]


def build(verbose: bool = False) -> str:
    """Compile libtapeec.so for gfx950 with hipcc (make -C tape_amd)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)
    return LIB_PATH


def _load() -> C.CDLL:
    # torch wheels bundle their own HIP runtime with the same soname (libamdhip64.so.7); whichever
    # loads first serves the process.  Load torch's first so torch tensors/streams and our kernels
    # share one runtime (ours is ABI-compatible with it).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C tape_amd` "
                          "(the engine has no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, sz, i = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t, C.c_int
    u32p, szp, u8p = C.POINTER(u32), C.POINTER(sz), C.c_void_p
    pp = C.POINTER(C.c_void_p)
    sig = {
        "te_strerror": (C.c_char_p, [i]),
        "te_device_count": (i, []),
        "te_set_device": (i, [i]),
        "te_clay_bind_device": (i, [vp, i]),
        "te_clay_device": (i, [vp]),
        "te_clay_set_decode_jit": (i, [vp, i, u64]),
        "te_clay_decode_jit_status": (i, [vp, u32, u32p, u32p, u32p]),
        "te_clay_set_decode_store_cap": (i, [vp, u32]),
        "te_clay_decode_store_stats": (i, [vp, u32p, u32p, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)]),
        "te_version": (C.c_char_p, []),
        "te_kernel_timing": (C.c_int, [C.c_int]),
        "te_kernel_time_ms": (C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_uint32)]),
        "te_last_error_detail": (C.c_char_p, []),
        "te_clay_new": (i, [u32, u32, u32, C.POINTER(vp)]),
        "te_clay_from_params": (i, [u64, C.POINTER(vp)]),
        "te_clay_free": (None, [vp]),
        "te_clay_get_info": (i, [vp, C.POINTER(te_clay_info)]),
        "te_clay_chunk_size_for": (sz, [vp, sz]),
        "te_clay_track_chunk_size": (sz, [vp, sz, sz]),
        "te_clay_encode": (i, [vp, u8p, sz, u8p, sz, szp]),
        "te_clay_decode": (i, [vp, pp, sz, u8p, sz]),
        "te_clay_plan_repair": (i, [vp, u32, u32p, sz, u32p, u32p]),
        "te_clay_repair": (i, [vp, u32, u32p, pp, sz, sz, u8p]),
        "te_pick_stripe_size": (sz, [sz]),
        "te_num_stripes": (sz, [sz, sz]),
        "te_shard_to_slice": (u32, [i, u32, u32, u32]),
        "te_slice_to_shard": (u32, [i, u32, u32, u32]),
        "te_slice_metadata_to_bytes": (None, [C.POINTER(te_slice_metadata), u8p]),
        "te_slice_metadata_from_slice": (i, [u8p, sz, C.POINTER(te_slice_metadata)]),
        "te_slicer_geometry": (i, [vp, sz, C.POINTER(te_geometry)]),
        "te_slicer_encode": (i, [vp, C.POINTER(te_slicer_cfg), u8p, sz, u8p, sz]),
        "te_slicer_decode": (i, [vp, C.POINTER(te_slicer_cfg), pp, sz, u8p, sz, szp]),
        "te_repair_plan_from_params": (i, [vp, i, u32, u32p, sz, u64, u64, C.POINTER(vp)]),
        "te_repair_plan_from_slice": (i, [vp, i, u32, u32p, sz, u8p, sz, C.POINTER(vp)]),
        "te_repair_plan_free": (None, [vp]),
        "te_repair_plan_get_info": (i, [vp, C.POINTER(te_repair_plan_info)]),
        "te_repair_plan_stripe": (i, [vp, u32, u32p, u32p, u32p, u32p]),
        "te_extract_repair_data_size": (sz, [vp, u32]),
        "te_extract_repair_data": (i, [vp, u8p, sz, u32, u8p, sz, szp]),
        "te_slicer_repair": (i, [vp, vp, pp, szp, u8p, u8p, sz]),
        "te_repair_plan_helper_request": (i, [vp, u32, u32p, u32p, sz, szp]),
        "te_serve_repair_request": (i, [vp, u8p, sz, u32p, u32p, u32p, sz, u8p, sz, szp]),
        "te_encode_batch_device": (i, [vp, C.POINTER(te_slicer_cfg), vp, C.POINTER(te_object), sz, vp, vp]),
        "te_encode_batch_host": (i, [vp, C.POINTER(te_slicer_cfg), vp, C.POINTER(te_object), sz, vp, sz]),
        "te_balance_object_ranges": (i, [C.POINTER(te_object), sz, sz, C.POINTER(sz)]),
        "te_encode_batch_host_multi": (i, [C.POINTER(vp), sz, C.POINTER(te_slicer_cfg), vp, C.POINTER(te_object), sz,
                                           vp, sz]),
        "te_encode_commit_batch_host": (i, [vp, C.POINTER(te_slicer_cfg), vp, C.POINTER(te_object), sz, vp,
                                            C.c_uint32, vp, vp, vp, sz]),
        "te_stream_writer_new": (i, [C.POINTER(vp), sz, C.POINTER(te_slicer_cfg), C.c_uint32, sz, C.POINTER(vp)]),
        "te_stream_submit": (i, [vp, vp, C.POINTER(te_object), sz, vp, vp, vp, vp, C.POINTER(u64)]),
        "te_stream_wait": (i, [vp, u64]),
        "te_stream_writer_free": (None, [vp]),
        "te_stream_writer_set_hashing": (i, [vp, i]),
        "te_set_commit_hashing": (i, [i]),
        "te_set_host_hash_threads": (i, [i]),
        "te_host_hash_threads": (i, []),
        "te_host_sha_extensions": (i, []),
        "te_host_hash_rate": (C.c_double, []),
        "te_host_hash_lanes": (i, []),
        "te_host_alloc": (i, [sz, C.POINTER(vp)]),
        "te_host_free": (None, [vp]),
        "te_host_register": (i, [vp, sz]),
        "te_host_unregister": (i, [vp]),
        "te_decode_batch_device": (i, [vp, C.POINTER(te_slicer_cfg), vp, C.POINTER(te_decode_object), u8p, sz,
                                       vp, vp]),
        "te_repair_batch_device": (i, [vp, vp, C.POINTER(te_repair_object), sz, vp, vp]),
        "te_recover_batch_device": (i, [vp, C.POINTER(te_slicer_cfg), vp, C.POINTER(te_recover_object), u8p, sz,
                                        vp, vp]),
        "te_hash_leaf": (i, [u8p, sz, u8p]),
        "te_hash_leaves": (i, [u8p, sz, sz, u32, u8p]),
        "te_hash_pair": (i, [u8p, u8p, u8p]),
        "te_empty_subtree_root": (i, [u32, u8p]),
        "te_merkle_root_from_leaf_hashes": (i, [u8p, sz, u32, u8p]),
        "te_merkle_proof_from_leaf_hashes": (i, [u8p, sz, sz, u32, u8p]),
        "te_merkle_verify_leaf_hash": (i, [u8p, u8p, u8p, sz, u64, u32]),
        "te_commit_batch_device": (i, [vp, u64, u64, u32, sz, u32, vp, vp, vp, vp]),
        "te_outer_chunk_bytes": (sz, [u32, sz]),
        "te_outer_encode": (i, [u32, u32, u8p, sz, u8p, sz, szp]),
        "te_outer_decode": (i, [u32, u32, pp, sz, u8p, sz]),
        "te_outer_encode_device": (i, [u32, u32, vp, u64, u32, u64, vp, u64, vp]),
        "te_outer_decode_device": (i, [u32, u32, pp, u64, vp, vp]),
        "te_outer_decode_device_batch": (i, [u32, u32, pp, u32, u64, vp, u64, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = _load()


def declared_symbols() -> list[str]:
    """Every function the public header declares (te_*( ... ) prototypes)."""
    import re
    txt = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(te_[a-z0-9_]+)\s*\(", txt)))


def strerror(code: int) -> str:
    return lib.te_strerror(code).decode()


def device_count() -> int:
    return int(lib.te_device_count())
