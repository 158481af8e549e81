"""Slice commitments: oracle pinned by the reference's EMPTY_ROOTS, libtapeec's host
merkle entry points against the oracle, and the reference's own merkle tests
(lib/crypto/src/merkle/tree.rs:488-841) restated.  CPU only (the batch kernel is in
test_gpu_parity.py)."""
import json
import os
import random

import pytest

from oracle import merkle_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden():
    return [bytes.fromhex(h) for h in json.load(open(os.path.join(HERE, "golden", "empty_roots.json")))["empty_roots"]]


@pytest.fixture(scope="module")
def M():
    from tape_amd import merkle
    return merkle


def test_oracle_empty_roots_match_reference(golden):  # tree.rs:15-48 vs the derivation tree.rs:832-841
    assert len(golden) == 32
    assert O.empty_roots() == golden


def test_lib_empty_subtree_root(M, golden):  # empty_subtree_root, tree.rs:64-68
    for h in range(32):
        assert M.empty_subtree_root(h) == golden[h]
    with pytest.raises(Exception):
        M.empty_subtree_root(32)


def test_lib_hashes_match_oracle(M):
    rnd = random.Random(5)
    # every padding case around the 4-byte "LEAF" prefix: the host path assembles block 0 and
    # reads later blocks in place (x86 SHA extensions when present, te_host_sha_extensions)
    for ln in (0, 1, 55, 56, 59, 60, 61, 63, 64, 119, 120, 123, 124, 125, 127, 128, 183, 184, 1000, 715_048):
        d = bytes(rnd.getrandbits(8) for _ in range(ln)) if ln < 5000 else os.urandom(ln)
        assert M.hash_leaf(d) == O.hash_leaf(d), ln
    a, b = bytes(range(32)), bytes(range(32, 64))
    assert M.hash_pair(a, b) == O.hash_pair(a, b)
    assert M.hash_pair(a, b) != M.hash_pair(b, a)


@pytest.mark.parametrize("lanes", [0, 1, 2, 3, 4])
def test_lib_interleaved_leaves_match_oracle(M, lanes):
    # te_hash_leaves: 1-4 messages interleaved round by round (the host pool's tasks); every count
    # leaves a short last group
    rnd = random.Random(11 + lanes)
    for ln in (0, 3, 59, 60, 61, 123, 124, 125, 4096, 70_001):
        for count in (1, 2, 3, 4, 5, 7, 20):
            d = os.urandom(ln * count) if ln > 1000 else bytes(rnd.getrandbits(8) for _ in range(ln * count))
            got = M.hash_leaves(d, count, lanes) if ln else M.hash_leaves(b"", count, lanes)
            want = [O.hash_leaf(d[i * ln:(i + 1) * ln]) for i in range(count)]
            assert got == want, (ln, count)
    with pytest.raises(Exception):
        M.hash_leaves(b"abc", 2)


def test_host_hash_lanes(M):
    from tape_amd import _lib
    assert 1 <= _lib.lib.te_host_hash_lanes() <= 4
    assert _lib.lib.te_hash_leaves(None, 0, 1, 5, None) == _lib.TE_ERR_INVALID_ARG


def test_two_leaves(M):  # tree.rs:503-517
    l1, l2 = M.hash_leaf(b"hello"), M.hash_leaf(b"world")
    assert M.root_from_leaf_hashes([l1, l2], 1) == M.hash_pair(l1, l2)


def test_proofs_four_leaves(M):  # tree.rs:520-547
    data = [b"hello", b"world", b"data", b"test"]
    leaves = [M.hash_leaf(d) for d in data]
    root = M.root_from_leaf_hashes(leaves, 2)
    for i, d in enumerate(data):
        proof = M.create_proof_from_leaf_hashes(leaves, i, 2)
        assert M.verify_proof(d, root, proof, i, 2)
        assert not M.verify_proof(d + b"x", root, proof, i, 2)
        assert not M.verify_proof(d, root, proof, i ^ 1, 2)


def test_missing_leaves_are_empty_leaves(M):  # three_leaves tree.rs:549-566, non_power_of_two :568-588
    h = M.hash_leaf
    assert M.root_from_leaf_hashes([h(b"a"), h(b"b"), h(b"c")], 2) == \
        M.root_from_leaf_hashes([h(b"a"), h(b"b"), h(b"c"), h(b"")], 2)
    assert M.root_from_leaf_hashes([h(b"hello")] * 33, 6) == \
        M.root_from_leaf_hashes([h(b"hello")] * 33 + [h(b"")] * 31, 6)


def test_root_and_proofs_match_oracle(M):  # root_from_leaf_hashes_matches_add_leaf, tree.rs:691-723
    rnd = random.Random(7)
    for height, n in ((5, 20), (5, 1), (5, 32), (1, 2), (3, 5), (6, 33), (12, 100)):
        hs = [bytes(rnd.getrandbits(8) for _ in range(32)) for _ in range(n)]
        root = M.root_from_leaf_hashes(hs, height)
        assert root == O.root_from_leaf_hashes(hs, height)
        for i in range(n):
            p = M.create_proof_from_leaf_hashes(hs, i, height)
            assert p == O.create_proof_from_leaf_hashes(hs, i, height)
            assert M.verify_leaf_hash(hs[i], root, p, i, height)
            assert not M.verify_leaf_hash(hs[i], root, p[:-1], i, height)  # proof length != N


def test_empty_tree_root(M, golden):  # MerkleTree::default().root == EMPTY_ROOTS[N-1], tree.rs:86-104
    assert M.root_from_leaf_hashes([], 5) == golden[4]


def test_merkle_errors(M):  # MerkleError, tree.rs:360-366, 130-133, 405-423
    h = M.hash_leaf(b"x")
    with pytest.raises(M.MerkleError) as e:
        M.root_from_leaf_hashes([h] * 33, 5)
    assert e.value.variant == "TreeFull"
    for args in (([], 0), ([h], 1), ([h] * 33, 0)):
        with pytest.raises(M.MerkleError) as e:
            M.create_proof_from_leaf_hashes(args[0], args[1], 5)
        assert e.value.variant == "InvalidProof"


def test_commit_batch_needs_device():  # no CPU fallback for the batch kernel
    import ctypes as C
    from tape_amd import _lib
    if _lib.device_count() > 0:
        pytest.skip("device present")
    r = _lib.lib.te_commit_batch_device(C.c_void_p(16), 0, 64, 20, 1, 5, C.c_void_p(16), None, None, None)
    assert r == _lib.TE_ERR_NO_DEVICE
