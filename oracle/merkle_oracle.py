"""CPU restatement of the slice-commitment step -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; it
is the checker for libtapeec's commitment kernels, never the product path.

Follows lib/crypto/src/merkle/tree.rs and the SDK call site sdk/src/codec/encoder.rs:226-234.
SHA-256 itself is hashlib's (FIPS 180-4), standing in for `solana-sha256-hasher::hashv`
(lib/crypto/src/hash.rs:91-98), which hashes the concatenation of its parts.  Pinned by the
reference's only golden vectors, EMPTY_ROOTS (tree.rs:15-48; tests/golden/empty_roots.json).
"""
import hashlib

LEAF_LABEL = b"LEAF"     # tree.rs:11
LEFT_LABEL = b"LEFT"     # tree.rs:9
RIGHT_LABEL = b"RIGHT"   # tree.rs:10
MAX_MERKLE_TREE_HEIGHT = 32  # tree.rs:6
SLICE_TREE_HEIGHT = 5    # lib/core/src/erasure.rs:9


def hashv(parts) -> bytes:  # hash.rs:91-98
    h = hashlib.sha256()
    for p in parts:
        h.update(p)
    return h.digest()


def hash_leaf(data: bytes) -> bytes:  # tree.rs:53-56
    return hashv([LEAF_LABEL, data])


def hash_pair(left: bytes, right: bytes) -> bytes:  # tree.rs:58-62
    return hashv([LEFT_LABEL, left, RIGHT_LABEL, right])


def empty_roots(n: int = MAX_MERKLE_TREE_HEIGHT):  # the derivation in tree.rs:832-841
    out, node = [], hash_leaf(b"")
    for _ in range(n):
        out.append(node)
        node = hash_pair(node, node)
    return out


_EMPTY = empty_roots()


def root_from_leaf_hashes(hashes, height: int) -> bytes:
    """MerkleTree::<N>::new() + add_leaf_hash per leaf (tree.rs:86-153, 344-350)."""
    assert 0 < height <= MAX_MERKLE_TREE_HEIGHT
    if len(hashes) > (1 << height):
        raise ValueError("TreeFull")
    filled = [_EMPTY[i] for i in range(height)]
    root = _EMPTY[height - 1]
    for index, leaf in enumerate(hashes):
        cur, idx = leaf, index
        for level in range(height):
            if idx & 1 == 0:
                filled[level] = cur
                cur = hash_pair(cur, _EMPTY[level])
            else:
                cur = hash_pair(filled[level], cur)
            idx >>= 1
        root = cur
    return root


def create_proof_from_leaf_hashes(hashes, index: int, height: int):
    """create_merkle_proof_hashes (tree.rs:397-455): layers padded with EMPTY_ROOTS[i]."""
    if not hashes or index >= len(hashes) or len(hashes) > (1 << height) or height > MAX_MERKLE_TREE_HEIGHT:
        raise ValueError("InvalidProof")
    layers, cur = [], list(hashes)
    for i in range(height):
        if len(cur) % 2:
            cur.append(_EMPTY[i])
        layers.append(cur)
        cur = [hash_pair(cur[2 * j], cur[2 * j + 1]) for j in range(len(cur) // 2)]
    proof, ci = [], index
    for li in range(height):
        proof.append(layers[li][ci + 1] if ci % 2 == 0 else layers[li][ci - 1])
        ci //= 2
    return proof


def verify_leaf_hash(leaf_hash: bytes, root: bytes, proof, index: int, height: int) -> bool:
    """verify_proof (tree.rs:462-481) from a pre-hashed leaf."""
    if len(proof) != height:
        return False
    node, idx = leaf_hash, index
    for sib in proof:
        node = hash_pair(node, sib) if idx & 1 == 0 else hash_pair(sib, node)
        idx >>= 1
    return node == root


def commit_slices(slices, height: int = SLICE_TREE_HEIGHT):
    """BlobEncoder::encode_with_proofs' commitment (encoder.rs:226-234): leaf hashes, root, proofs."""
    leaves = [hash_leaf(bytes(s)) for s in slices]
    root = root_from_leaf_hashes(leaves, height)
    proofs = [create_proof_from_leaf_hashes(leaves, i, height) for i in range(len(leaves))]
    return leaves, root, proofs
