"""Python mirror of lib/slicer's public surface (lib/slicer/src/lib.rs:15-27) over libtapeec.so.

Names, argument meaning and error behaviour follow the Rust crate so the parity tests read like
the reference's own tests:

    ErasureCoder::{k,m,n,encode,decode}          lib/slicer/src/coder.rs:14-44
    ClayCoder                                    lib/slicer/src/clay.rs:13-122
    Slicer<ClayCoder>                            lib/slicer/src/slicer.rs:124-387
    RepairPlan / StripeRepair / HelperPlan       lib/slicer/src/repair.rs:16-47
    extract_repair_data                          lib/slicer/src/repair.rs:97-130
    SliceMetadata                                lib/slicer/src/metadata.rs:22-109
    pick_stripe_size / num_stripes / STRIPE_SIZES lib/slicer/src/adaptive.rs:15-49
    EncodeError / DecodeError / RepairError       lib/slicer/src/errors.rs:5-37

Every GF(2^8) computation is executed by the gfx950 kernels of libtapeec.so; on a host without
a device the compute methods raise NoDeviceError (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes as C
import enum
from dataclasses import dataclass, field

from . import _lib
from ._lib import lib

# ---------------------------------------------------------------------------------------------
# constants (adaptive.rs, slicer.rs, lib/core)
# ---------------------------------------------------------------------------------------------
STRIPE_SIZES = (100_000, 1_000_000, 10_000_000)
DEFAULT_STRIPE_SIZE = STRIPE_SIZES[2]
ROTATION_STEP = 7
GROUP_SIZE = 20
SLICE_TREE_HEIGHT = 5


class EngineError(RuntimeError):
    """Engine-level failure (HIP error, unsupported layout, ...)."""

    def __init__(self, code: int, msg: str | None = None):
        self.code = code
        detail = lib.te_last_error_detail().decode() if code in (_lib.TE_ERR_HIP, _lib.TE_ERR_OUT_OF_MEMORY) else ""
        super().__init__(msg or f"{_lib.strerror(code)} (status {code}){': ' + detail if detail else ''}")


class NoDeviceError(EngineError):
    """No gfx950 device: libtapeec has no CPU fallback."""


class EncodeError(Exception):
    """errors.rs:5-11 -- variants TooMuchData, EmptyInput."""

    def __init__(self, variant: str):
        self.variant = variant
        super().__init__(variant)


class DecodeError(Exception):
    """errors.rs:13-23 -- NotEnoughSlices, TooMuchData, BadEncoding, InvalidLayout."""

    def __init__(self, variant: str):
        self.variant = variant
        super().__init__(variant)


class RepairError(Exception):
    """errors.rs:25-37 -- NotEnoughHelpers, InvalidSlice, InvalidLayout, Clay, MissingHelper."""

    def __init__(self, variant: str, detail: str = ""):
        self.variant = variant
        super().__init__(f"{variant}: {detail}" if detail else variant)


_ENC = {_lib.TE_ERR_TOO_MUCH_DATA: "TooMuchData", _lib.TE_ERR_EMPTY_INPUT: "EmptyInput"}
_DEC = {_lib.TE_ERR_NOT_ENOUGH_SLICES: "NotEnoughSlices", _lib.TE_ERR_TOO_MUCH_DATA: "TooMuchData",
        _lib.TE_ERR_BAD_ENCODING: "BadEncoding", _lib.TE_ERR_INVALID_LAYOUT: "InvalidLayout"}
_REP = {_lib.TE_ERR_NOT_ENOUGH_HELPERS: "NotEnoughHelpers", _lib.TE_ERR_INVALID_SLICE: "InvalidSlice",
        _lib.TE_ERR_INVALID_LAYOUT: "InvalidLayout", _lib.TE_ERR_CLAY: "Clay",
        _lib.TE_ERR_MISSING_HELPER: "MissingHelper"}


def _engine_error(code: int) -> EngineError:
    if code == _lib.TE_ERR_NO_DEVICE:
        return NoDeviceError(code)
    return EngineError(code)


def _check(code: int, kind: str) -> None:
    """Raise the reference's error for a status.  kind "recover" (node recover = decode then
    encode) maps through the decode table, then the encode table."""
    if code == 0:
        return
    if kind == "recover":
        if code in _DEC:
            raise DecodeError(_DEC[code])
        if code in _ENC:
            raise EncodeError(_ENC[code])
        raise _engine_error(code)
    table = {"encode": (_ENC, EncodeError), "decode": (_DEC, DecodeError), "repair": (_REP, RepairError)}[kind]
    if code in table[0]:
        if kind == "repair" and code == _lib.TE_ERR_CLAY:  # RepairError::Clay(String), repair.rs:59-62
            raise RepairError("Clay", lib.te_last_error_detail().decode())
        raise table[1](table[0][code])
    raise _engine_error(code)


def _buf(data) -> C.Array:
    b = bytes(data)
    return (C.c_uint8 * max(1, len(b))).from_buffer_copy(b if b else b"\0")


# ---------------------------------------------------------------------------------------------
# profile types (lib/core/src/encoding.rs)
# ---------------------------------------------------------------------------------------------
class EncodingType(enum.IntEnum):
    Unknown = 0
    Basic = 1
    Clay = 2


@dataclass(frozen=True)
class ClayParams:
    """Packed n | k<<8 | d<<16 (encoding.rs:180-239)."""
    packed: int

    @staticmethod
    def new(n: int, k: int, d: int) -> "ClayParams":
        return ClayParams(n | (k << 8) | (d << 16))

    @staticmethod
    def default() -> "ClayParams":
        return ClayParams.new(20, 7, 16)

    def n(self) -> int:
        return self.packed & 0xFF

    def k(self) -> int:
        return (self.packed >> 8) & 0xFF

    def d(self) -> int:
        return (self.packed >> 16) & 0xFF

    def m(self) -> int:
        return max(0, self.n() - self.k())

    def as_u64(self) -> int:
        return self.packed


@dataclass(frozen=True)
class EncodingProfile:
    encoding: int
    params: int

    @staticmethod
    def clay(params: ClayParams) -> "EncodingProfile":
        return EncodingProfile(int(EncodingType.Clay), params.as_u64())

    @staticmethod
    def clay_default() -> "EncodingProfile":
        return EncodingProfile.clay(ClayParams.default())

    def clay_params(self) -> ClayParams:
        return ClayParams(self.params)

    def is_clay(self) -> bool:
        return self.encoding == int(EncodingType.Clay)

    def pack(self) -> bytes:
        return self.encoding.to_bytes(8, "little") + self.params.to_bytes(8, "little")


# ---------------------------------------------------------------------------------------------
# adaptive.rs / slicer.rs free functions
# ---------------------------------------------------------------------------------------------
def pick_stripe_size(blob_len: int) -> int:
    return int(lib.te_pick_stripe_size(blob_len))


def num_stripes(blob_len: int, stripe_size: int) -> int:
    return int(lib.te_num_stripes(blob_len, stripe_size))


class MappingStrategy(enum.Enum):
    Identity = 0
    Rotated = 1


def shard_to_slice(strategy: MappingStrategy, n: int, stripe_idx: int, shard_idx: int) -> int:
    return int(lib.te_shard_to_slice(int(strategy == MappingStrategy.Rotated), n, stripe_idx, shard_idx))


def slice_to_shard(strategy: MappingStrategy, n: int, stripe_idx: int, slice_idx: int) -> int:
    return int(lib.te_slice_to_shard(int(strategy == MappingStrategy.Rotated), n, stripe_idx, slice_idx))


# ---------------------------------------------------------------------------------------------
# SliceMetadata (metadata.rs)
# ---------------------------------------------------------------------------------------------
@dataclass
class SliceMetadata:
    version: int = 0
    blob_len: int = 0
    stripe_size: int = 0
    profile: EncodingProfile = field(default_factory=EncodingProfile.clay_default)
    chunk_index: int = 0

    VERSION = 0
    SIZE = 48

    @staticmethod
    def new(blob_len: int, stripe_size: int) -> "SliceMetadata":
        return SliceMetadata(0, blob_len, stripe_size, EncodingProfile.clay_default(), 0)

    @staticmethod
    def with_profile(blob_len: int, stripe_size: int, profile: EncodingProfile) -> "SliceMetadata":
        return SliceMetadata(0, blob_len, stripe_size, profile, 0)

    def to_bytes(self) -> bytes:
        m = _lib.te_slice_metadata(self.version, self.blob_len, self.stripe_size, self.profile.encoding,
                                   self.profile.params, self.chunk_index)
        out = (C.c_uint8 * 48)()
        lib.te_slice_metadata_to_bytes(C.byref(m), out)
        return bytes(out)

    @staticmethod
    def from_slice(slice_data: bytes) -> "SliceMetadata":
        m = _lib.te_slice_metadata()
        b = _buf(slice_data)
        r = lib.te_slice_metadata_from_slice(b, len(slice_data), C.byref(m))
        _check(r, "decode")
        return SliceMetadata(m.version, m.blob_len, m.stripe_size, EncodingProfile(m.encoding, m.params),
                             m.chunk_index)


# ---------------------------------------------------------------------------------------------
# ClayCoder (clay.rs)
# ---------------------------------------------------------------------------------------------
class ClayCoder:
    """ClayCoder::new(n, k, d) -- raises AssertionError on invalid params like the Rust asserts."""

    def __init__(self, n: int, k: int, d: int):
        assert n > k, "n must be > k"
        assert k > 0, "k must be > 0"
        assert d >= k + 1, "d must be >= k + 1"
        assert d <= n - 1, "d must be <= n - 1"
        h = C.c_void_p()
        r = lib.te_clay_new(n, k, d, C.byref(h))
        if r:
            raise _engine_error(r)
        self._h = h
        info = _lib.te_clay_info()
        lib.te_clay_get_info(h, C.byref(info))
        self._info = info

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.te_clay_free(h)
            self._h = None

    @staticmethod
    def from_params(params: ClayParams) -> "ClayCoder":
        return ClayCoder(params.n(), params.k(), params.d())

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def bind_device(self, device: int) -> None:
        """te_clay_bind_device: run this coder's allocations and launches on `device`."""
        r = lib.te_clay_bind_device(self._h, device)
        if r:
            raise _engine_error(r)

    def device(self) -> int:
        return int(lib.te_clay_device(self._h))

    def set_decode_jit(self, mode: str = "async", min_stripes: int = 1024) -> None:
        """te_clay_set_decode_jit: per-pattern decode kernels off / built in the background /
        built in the decoding call, once a pattern has decoded `min_stripes` stripes."""
        r = lib.te_clay_set_decode_jit(self._h, {"off": 0, "async": 1, "sync": 2}[mode], min_stripes)
        if r:
            raise _engine_error(r)

    def set_decode_store_cap(self, max_patterns: int) -> None:
        """te_clay_set_decode_store_cap: most distinct stripe patterns kept on the device."""
        _check(lib.te_clay_set_decode_store_cap(self.handle, max_patterns), "decode")

    def decode_store_stats(self) -> dict:
        """te_clay_decode_store_stats: the device pattern store's capacity, filled slots, clears,
        grows and over-capacity (arena) calls."""
        cap, used = C.c_uint32(), C.c_uint32()
        cl, gr, ar = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib.te_clay_decode_store_stats(self.handle, C.byref(cap), C.byref(used), C.byref(cl), C.byref(gr),
                                              C.byref(ar)), "decode")
        return {"capacity": cap.value, "used": used.value, "clears": cl.value, "grows": gr.value,
                "arena_calls": ar.value}

    def decode_jit_status(self, timeout_ms: int = 0) -> tuple:
        """(ready, compiling, failed) per-pattern kernels, after waiting up to timeout_ms."""
        v = [C.c_uint32(0) for _ in range(3)]
        r = lib.te_clay_decode_jit_status(self._h, timeout_ms, *[C.byref(x) for x in v])
        if r:
            raise _engine_error(r)
        return tuple(int(x.value) for x in v)

    def k(self) -> int:
        return self._info.k

    def m(self) -> int:
        return self._info.m

    def n(self) -> int:
        return self._info.n

    def d(self) -> int:
        return self._info.d

    def alpha(self) -> int:
        return self._info.alpha

    def beta(self) -> int:
        return self._info.beta

    def chunk_size_for(self, input_len: int) -> int:
        return int(lib.te_clay_chunk_size_for(self._h, input_len))

    def track_chunk_size(self, stripe_size: int, blob_len: int) -> int:
        return int(lib.te_clay_track_chunk_size(self._h, stripe_size, blob_len))

    def encode(self, data: bytes) -> list[bytes]:
        if len(data) == 0:
            raise EncodeError("EmptyInput")
        cs = self.chunk_size_for(len(data))
        out = (C.c_uint8 * (self.n() * cs))()
        got = C.c_size_t()
        r = lib.te_clay_encode(self._h, _buf(data), len(data), out, len(out), C.byref(got))
        _check(r, "encode")
        raw = bytes(out)
        return [raw[i * cs:(i + 1) * cs] for i in range(self.n())]

    def decode(self, chunks: list[tuple[int, bytes]]) -> bytes:
        if len(chunks) < self.k():
            raise DecodeError("NotEnoughSlices")
        cs = len(chunks[0][1])
        keep = []
        ptrs = (C.c_void_p * self.n())()
        for idx, data in chunks:
            if len(data) != cs or not (0 <= idx < self.n()):
                raise DecodeError("BadEncoding")
            b = _buf(data)
            keep.append(b)
            ptrs[idx] = C.cast(b, C.c_void_p)
        out = (C.c_uint8 * (self.k() * cs))()
        r = lib.te_clay_decode(self._h, ptrs, cs, out, len(out))
        _check(r, "decode")
        return bytes(out)

    def plan_repair(self, lost: int, available: list[int]) -> list[tuple[int, list[int]]]:
        av = (C.c_uint32 * max(1, len(available)))(*available)
        hs = (C.c_uint32 * self.d())()
        sc = (C.c_uint32 * self.beta())()
        r = lib.te_clay_plan_repair(self._h, lost, av, len(available), hs, sc)
        _check(r, "repair")
        return [(int(hs[j]), [int(x) for x in sc]) for j in range(self.d())]

    def repair(self, lost: int, helpers: dict[int, bytes], chunk_size: int) -> bytes:
        ids = list(helpers)
        hs = (C.c_uint32 * max(1, len(ids)))(*ids)
        keep = [_buf(helpers[i]) for i in ids]
        ptrs = (C.c_void_p * max(1, len(ids)))(*[C.cast(b, C.c_void_p) for b in keep])
        out = (C.c_uint8 * chunk_size)()
        r = lib.te_clay_repair(self._h, lost, hs, ptrs, len(ids), chunk_size, out)
        _check(r, "repair")
        return bytes(out)


# ---------------------------------------------------------------------------------------------
# Repair plan types (repair.rs:16-47)
# ---------------------------------------------------------------------------------------------
@dataclass
class HelperPlan:
    slice: int
    shard: int
    sub_chunks: list[int]


@dataclass
class StripeRepair:
    stripe: int
    lost_shard: int
    helpers: list[HelperPlan]


class RepairPlan:
    def __init__(self, handle: C.c_void_p):
        self._h = handle
        info = _lib.te_repair_plan_info()
        lib.te_repair_plan_get_info(handle, C.byref(info))
        self.lost = int(info.lost)
        self.num_stripes = int(info.num_stripes)
        self.chunk_size = int(info.chunk_size)
        self.sub_chunk_size = int(info.sub_chunk_size)
        d, b = int(info.d), int(info.beta)
        self.beta = b
        self.stripes: list[StripeRepair] = []
        for s in range(self.num_stripes):
            ls = C.c_uint32()
            hsl = (C.c_uint32 * d)()
            hsh = (C.c_uint32 * d)()
            scs = (C.c_uint32 * (d * b))()
            lib.te_repair_plan_stripe(handle, s, C.byref(ls), hsl, hsh, scs)
            helpers = [HelperPlan(int(hsl[j]), int(hsh[j]), [int(x) for x in scs[j * b:(j + 1) * b]])
                       for j in range(d)]
            self.stripes.append(StripeRepair(s, int(ls.value), helpers))

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib.te_repair_plan_free(h)
            self._h = None


def extract_repair_data(slice_bytes: bytes, plan: RepairPlan, helper: int) -> bytes:
    """Helper-side gather (repair.rs:97-130)."""
    need = int(lib.te_extract_repair_data_size(plan.handle, helper))
    out = (C.c_uint8 * max(1, need))()
    got = C.c_size_t()
    r = lib.te_extract_repair_data(plan.handle, _buf(slice_bytes), len(slice_bytes), helper, out, need,
                                   C.byref(got))
    if r == _lib.TE_ERR_INVALID_LAYOUT:
        raise RepairError("InvalidLayout", "slice too short for chunk / sub-chunk out of bounds")
    _check(r, "repair")
    return bytes(out)[:got.value]


def repair_request(plan: RepairPlan, helper: int) -> list[tuple[int, list[int]]]:
    """per_helper_reqs (network/node/src/features/spool/repair.rs:468-491) for one helper: the
    RepairRequest.stripes (network/protocol/src/api/types.rs:75-85) as [(stripe, sub_chunks)]."""
    cnt = C.c_size_t()
    _check(lib.te_repair_plan_helper_request(plan.handle, helper, None, None, 0, C.byref(cnt)), "repair")
    n = cnt.value
    beta = plan.beta
    st = (C.c_uint32 * max(1, n))()
    sub = (C.c_uint32 * max(1, n * beta))()
    _check(lib.te_repair_plan_helper_request(plan.handle, helper, st, sub, n, C.byref(cnt)), "repair")
    return [(int(st[k]), [int(x) for x in sub[k * beta:(k + 1) * beta]]) for k in range(n)]


def serve_repair_request(coder: ClayCoder, slice_bytes: bytes, stripes: list[tuple[int, list[int]]]) -> bytes:
    """The helper node's extract_repair_data (network/node/src/features/spool/repair.rs:496-553):
    the requested sub-chunks of a stored slice, geometry from the slice's own metadata suffix."""
    ns = len(stripes)
    st = (C.c_uint32 * max(1, ns))(*[s for s, _ in stripes])
    nsub = (C.c_uint32 * max(1, ns))(*[len(z) for _, z in stripes])
    flat = [z for _, zs in stripes for z in zs]
    sub = (C.c_uint32 * max(1, len(flat)))(*flat)
    got = C.c_size_t()
    args = (coder.handle, _buf(slice_bytes), len(slice_bytes), st, nsub, sub, ns)
    r = lib.te_serve_repair_request(*args, None, 0, C.byref(got))
    if r == _lib.TE_ERR_INVALID_LAYOUT:
        raise RepairError("InvalidLayout", _lib.lib.te_last_error_detail().decode())
    if r not in (_lib.TE_OK, _lib.TE_ERR_BUFFER_TOO_SMALL):
        _check(r, "repair")
    out = (C.c_uint8 * max(1, got.value))()
    _check(lib.te_serve_repair_request(*args, out, got.value, C.byref(got)), "repair")
    return bytes(out)[:got.value]


# ---------------------------------------------------------------------------------------------
# Slicer (slicer.rs)
# ---------------------------------------------------------------------------------------------
class Slicer:
    """Slicer<ClayCoder>: striping + metadata + rotation over the GPU Clay engine."""

    def __init__(self, coder: ClayCoder, stripe_size: int = DEFAULT_STRIPE_SIZE,
                 strategy: MappingStrategy = MappingStrategy.Identity,
                 profile: EncodingProfile | None = None, chunk_index: int = 0):
        self.coder = coder
        self.stripe_size = stripe_size
        self.strategy = strategy
        self.profile = profile or EncodingProfile.clay_default()
        self.chunk_index = chunk_index

    # constructors (slicer.rs:138-199)
    @staticmethod
    def new(coder: ClayCoder) -> "Slicer":
        return Slicer(coder)

    @staticmethod
    def with_rotation(coder: ClayCoder) -> "Slicer":
        return Slicer(coder, strategy=MappingStrategy.Rotated)

    @staticmethod
    def with_stripe_size(coder: ClayCoder, stripe_size: int) -> "Slicer":
        return Slicer(coder, stripe_size=stripe_size)

    @staticmethod
    def with_profile(coder: ClayCoder, stripe_size: int, rotated: bool, profile: EncodingProfile) -> "Slicer":
        return Slicer(coder, stripe_size, MappingStrategy.Rotated if rotated else MappingStrategy.Identity, profile)

    @staticmethod
    def clay_default() -> "Slicer":
        return Slicer.with_rotation(ClayCoder.from_params(ClayParams.default()))

    def set_chunk_index(self, index: int) -> None:
        self.chunk_index = index

    def strategy_(self) -> MappingStrategy:
        return self.strategy

    def reconfigure_clay(self, profile: EncodingProfile) -> None:
        if self.profile != profile:
            self.profile = profile
            self.coder = ClayCoder.from_params(profile.clay_params())

    def k(self) -> int:
        return self.coder.k()

    def m(self) -> int:
        return self.coder.m()

    def n(self) -> int:
        return self.coder.n()

    def _cfg(self) -> _lib.te_slicer_cfg:
        return _lib.te_slicer_cfg(int(self.strategy == MappingStrategy.Rotated), self.profile.encoding,
                                  self.profile.params, self.chunk_index)

    def geometry(self, blob_len: int) -> _lib.te_geometry:
        g = _lib.te_geometry()
        lib.te_slicer_geometry(self.coder.handle, blob_len, C.byref(g))
        return g

    def encode(self, data: bytes) -> list[bytes]:
        """Slicer::encode (slicer.rs:237-296)."""
        self.stripe_size = pick_stripe_size(len(data))
        g = self.geometry(len(data))
        n = self.n()
        out = (C.c_uint8 * (n * g.slice_len))()
        cfg = self._cfg()
        r = lib.te_slicer_encode(self.coder.handle, C.byref(cfg), _buf(data), len(data), out, len(out))
        _check(r, "encode")
        raw = bytes(out)
        sl = g.slice_len
        return [raw[i * sl:(i + 1) * sl] for i in range(n)]

    def decode(self, chunks: list[tuple[int, bytes]]) -> bytes:
        """Slicer::decode (slicer.rs:298-364)."""
        if not chunks:
            raise DecodeError("NotEnoughSlices")
        meta = SliceMetadata.from_slice(chunks[0][1])
        if self.stripe_size != meta.stripe_size:
            self.stripe_size = meta.stripe_size
        n = self.n()
        slice_len = len(chunks[0][1])
        ptrs = (C.c_void_p * n)()
        keep = []
        for idx, data in chunks:
            if not (0 <= idx < n):
                raise DecodeError("InvalidLayout")
            if len(data) != slice_len:
                raise DecodeError("InvalidLayout")
            b = _buf(data)
            keep.append(b)
            ptrs[idx] = C.cast(b, C.c_void_p)
        out = (C.c_uint8 * max(1, meta.blob_len))()
        got = C.c_size_t()
        cfg = self._cfg()
        r = lib.te_slicer_decode(self.coder.handle, C.byref(cfg), ptrs, slice_len, out, len(out), C.byref(got))
        _check(r, "decode")
        return bytes(out)[:got.value]

    # repair.rs:137-367
    def repair_plan_from_params(self, lost: int, available: list[int], blob_len: int, stripe_size: int) -> RepairPlan:
        av = (C.c_uint32 * max(1, len(available)))(*available)
        h = C.c_void_p()
        r = lib.te_repair_plan_from_params(self.coder.handle, int(self.strategy == MappingStrategy.Rotated), lost,
                                           av, len(available), blob_len, stripe_size, C.byref(h))
        _check(r, "repair")
        return RepairPlan(h)

    def repair_plan(self, lost: int, available: list[int], reference: bytes) -> RepairPlan:
        av = (C.c_uint32 * max(1, len(available)))(*available)
        h = C.c_void_p()
        r = lib.te_repair_plan_from_slice(self.coder.handle, int(self.strategy == MappingStrategy.Rotated), lost,
                                          av, len(available), _buf(reference), len(reference), C.byref(h))
        _check(r, "repair")
        return RepairPlan(h)

    def repair(self, plan: RepairPlan, helpers: dict[int, bytes], metadata_bytes: bytes) -> bytes:
        n = self.n()
        ptrs = (C.c_void_p * n)()
        lens = (C.c_size_t * n)()
        keep = []
        for sl, data in helpers.items():
            b = _buf(data)
            keep.append(b)
            ptrs[sl] = C.cast(b, C.c_void_p)
            lens[sl] = len(data)
        out_len = plan.num_stripes * plan.chunk_size + 48
        out = (C.c_uint8 * out_len)()
        r = lib.te_slicer_repair(self.coder.handle, plan.handle, ptrs, lens, _buf(metadata_bytes), out, out_len)
        _check(r, "repair")
        return bytes(out)

    def repair_full(self, lost: int, helpers: list[tuple[int, bytes]]) -> bytes:
        if not helpers:
            raise RepairError("NotEnoughHelpers", "needed 1, available 0")
        available = [i for i, _ in helpers]
        reference = helpers[0][1]
        plan = self.repair_plan(lost, available, reference)
        partial = {i: extract_repair_data(s, plan, i) for i, s in helpers}
        if len(reference) < 48:
            raise RepairError("InvalidLayout", "slice too short for metadata")
        return self.repair(plan, partial, reference[-48:])
