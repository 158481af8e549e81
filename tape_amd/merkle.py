"""Python mirror of the slice-commitment step over libtapeec.so.

    hash_leaf / hash_pair / empty_subtree_root      lib/crypto/src/merkle/tree.rs:53-68
    root_from_leaf_hashes::<N>                      tree.rs:344-350
    create_proof_from_leaf_hashes::<N>              tree.rs:353-358, 397-455
    verify_proof                                    tree.rs:462-481
    MerkleError                                     tree.rs:360-366
    BlobEncoder::encode_with_proofs' commitment     sdk/src/codec/encoder.rs:226-234

The single-hash helpers run on the host (a few SHA-256 blocks each); the per-object batch --
a SHA-256 stream per slice, then the tree -- runs in libtapeec's gfx950 kernels (commit_batch).
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import lib
from .slicer import SLICE_TREE_HEIGHT, _engine_error

HASH_SIZE = 32
MAX_MERKLE_TREE_HEIGHT = 32


class MerkleError(Exception):
    """tree.rs:360-366 -- variants TreeFull, InvalidProof, InvalidIndex, ProofLength."""

    def __init__(self, variant: str):
        self.variant = variant
        super().__init__(variant)


_MERKLE = {_lib.TE_ERR_MERKLE_TREE_FULL: "TreeFull", _lib.TE_ERR_MERKLE_INVALID_PROOF: "InvalidProof",
           _lib.TE_ERR_MERKLE_INVALID_INDEX: "InvalidIndex", _lib.TE_ERR_MERKLE_PROOF_LENGTH: "ProofLength"}


def _check(code: int) -> None:
    if code == 0:
        return
    if code in _MERKLE:
        raise MerkleError(_MERKLE[code])
    raise _engine_error(code)


def _out() -> C.Array:
    return (C.c_uint8 * HASH_SIZE)()


def _hashes(hashes) -> C.Array:
    b = b"".join(bytes(h) for h in hashes)
    return (C.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")


def hash_leaf(data: bytes) -> bytes:
    b = bytes(data)
    buf = (C.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")
    out = _out()
    _check(lib.te_hash_leaf(buf, len(b), out))
    return bytes(out)


def hash_leaves(data: bytes, count: int, lanes: int = 0) -> list:
    """hash_leaf of `count` equal-length pieces of `data` (an object's slices), `lanes` of them
    interleaved on this thread (0 = the host's best, te_host_hash_lanes)."""
    b = bytes(data)
    if count <= 0 or len(b) % count:
        raise ValueError("data must split into count equal pieces")
    ln = len(b) // count
    buf = (C.c_uint8 * max(1, len(b))).from_buffer_copy(b or b"\0")
    out = (C.c_uint8 * (HASH_SIZE * count))()
    _check(lib.te_hash_leaves(buf, ln, count, lanes, out))
    o = bytes(out)
    return [o[i * HASH_SIZE:(i + 1) * HASH_SIZE] for i in range(count)]


def hash_pair(left: bytes, right: bytes) -> bytes:
    out = _out()
    _check(lib.te_hash_pair(_hashes([left]), _hashes([right]), out))
    return bytes(out)


def empty_subtree_root(height: int) -> bytes:
    out = _out()
    _check(lib.te_empty_subtree_root(height, out))
    return bytes(out)


def root_from_leaf_hashes(hashes, height: int = SLICE_TREE_HEIGHT) -> bytes:
    out = _out()
    _check(lib.te_merkle_root_from_leaf_hashes(_hashes(hashes), len(hashes), height, out))
    return bytes(out)


def create_proof_from_leaf_hashes(hashes, index: int, height: int = SLICE_TREE_HEIGHT) -> list[bytes]:
    out = (C.c_uint8 * max(1, HASH_SIZE * height))()
    _check(lib.te_merkle_proof_from_leaf_hashes(_hashes(hashes), len(hashes), index, height, out))
    raw = bytes(out)
    return [raw[i * HASH_SIZE:(i + 1) * HASH_SIZE] for i in range(height)]


def verify_leaf_hash(leaf_hash: bytes, root: bytes, proof, index: int, height: int = SLICE_TREE_HEIGHT) -> bool:
    r = lib.te_merkle_verify_leaf_hash(_hashes([leaf_hash]), _hashes([root]), _hashes(proof), len(proof), index, height)
    if r < 0 or r > 1:
        _check(r)
    return r == 1


def verify_proof(data: bytes, root: bytes, proof, index: int, height: int = SLICE_TREE_HEIGHT) -> bool:
    """verify_proof (tree.rs:462-481): hash_leaf(data), then walk the proof."""
    return verify_leaf_hash(hash_leaf(data), root, proof, index, height)


def commit_batch(slices, obj_stride: int, slice_len: int, n: int, nobj: int, leaf_hashes, roots=None,
                 proofs=None, height: int = SLICE_TREE_HEIGHT, stream=None) -> None:
    """Device batch (te_commit_batch_device): uint8 cuda tensors; object o's slice i at
    slices[o*obj_stride + i*slice_len]; leaf_hashes nobj*n*32, roots nobj*32, proofs nobj*n*height*32."""
    from .batch import _stream_ptr
    ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)  # noqa: E731
    r = lib.te_commit_batch_device(ptr(slices), obj_stride, slice_len, n, nobj, height, ptr(leaf_hashes),
                                   ptr(roots), ptr(proofs), _stream_ptr(stream))
    _check(r)


def commit_slices(slices, height: int = SLICE_TREE_HEIGHT):
    """encode_with_proofs' commitment (encoder.rs:226-234) of one object's slices on the device:
    (leaf hashes, root, proofs)."""
    import torch
    n = len(slices)
    slen = len(slices[0])
    if any(len(s) != slen for s in slices):
        raise MerkleError("InvalidProof")
    host = torch.frombuffer(bytearray(b"".join(bytes(s) for s in slices)), dtype=torch.uint8)
    dev = host.to("cuda")
    leaf = torch.empty(n * HASH_SIZE, dtype=torch.uint8, device="cuda")
    root = torch.empty(HASH_SIZE, dtype=torch.uint8, device="cuda")
    proof = torch.empty(max(1, n * height * HASH_SIZE), dtype=torch.uint8, device="cuda")
    commit_batch(dev, n * slen, slen, n, 1, leaf, root, proof, height)
    torch.cuda.synchronize()
    lb, pb = leaf.cpu().numpy().tobytes(), proof.cpu().numpy().tobytes()
    leaves = [lb[i * HASH_SIZE:(i + 1) * HASH_SIZE] for i in range(n)]
    proofs = [[pb[((i * height) + l) * HASH_SIZE:((i * height) + l + 1) * HASH_SIZE] for l in range(height)]
              for i in range(n)]
    return leaves, root.cpu().numpy().tobytes(), proofs
