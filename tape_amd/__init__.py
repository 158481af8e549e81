"""tape_amd -- MI355X-native drop-in for Tapedrive's lib/slicer hot path (Clay (20,7,16) erasure
coding: Slicer encode, bandwidth-optimal single-slice repair, multi-erasure decode).

The compute lives in libtapeec.so (hand-written gfx950 HIP kernels behind the C ABI of
include/tape_ec.h).  This package is the Python host mirror of the reference's Rust API.
"""
from ._lib import build, device_count, lib  # noqa: F401
from .merkle import MerkleError, commit_batch, commit_slices, hash_leaf, hash_pair  # noqa: F401
from .slicer import (  # noqa: F401
    ClayCoder, ClayParams, DecodeError, EncodeError, EncodingProfile, EncodingType, EngineError, HelperPlan,
    MappingStrategy, NoDeviceError, RepairError, RepairPlan, SliceMetadata, Slicer, StripeRepair,
    DEFAULT_STRIPE_SIZE, GROUP_SIZE, ROTATION_STEP, SLICE_TREE_HEIGHT, STRIPE_SIZES, extract_repair_data,
    repair_request, serve_repair_request, num_stripes, pick_stripe_size, shard_to_slice, slice_to_shard,
)
