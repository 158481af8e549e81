"""GPU parity of the per-pattern decode kernels (tape_amd/csrc/dec_fixed.hpp + dec_rtc.cpp:
ClayCoder::decode inside Slicer::decode, slicer.rs:298-364, with one erasure pattern's plane
program and decoding matrix compiled in at run time by hipRTC).  The handle is put in sync mode
with a threshold of one stripe, so the first decode of a pattern builds its kernel and runs it;
every output is compared with the original bytes, and the same decode with the kernels off must
agree.  Each pattern costs ~25 s of host compile, so the cases are few and chosen to cover the
program's variety: worst case (13 erasures), random 7-survivor patterns, fewer erasures, ragged
output shares and narrower workgroups (small stripes)."""
import random

import pytest

import tape_amd as T

pytestmark = pytest.mark.gpu
N = 20
MiB = 1024 * 1024


def _jit_slicer():
    s = T.Slicer.new(T.ClayCoder(20, 7, 16))  # unrotated: one pattern for every stripe
    s.coder.set_decode_jit("sync", 1)
    return s


def _check(oracle, s, ln, keep, seed):
    data = oracle.splitmix64_bytes(seed, ln).tobytes()
    sl = s.encode(data)
    before = s.coder.decode_jit_status()[0]
    got = s.decode([(i, sl[i]) for i in keep])
    ready, pending, failed = s.coder.decode_jit_status()
    assert failed == 0 and pending == 0
    assert ready > before, "no pattern kernel was built"
    assert got == data, keep
    ref = T.Slicer.new(T.ClayCoder(20, 7, 16))
    ref.coder.set_decode_jit("off")
    assert ref.decode([(i, sl[i]) for i in keep]) == data


def test_jit_worst_case_4mib(oracle):  # the bench pattern: slices 0..12 erased
    _check(oracle, _jit_slicer(), 4 * MiB, list(range(13, 20)), 0x5EED)


@pytest.mark.parametrize("seed", [1, 2])
def test_jit_random_7_survivors_ragged(oracle, seed):  # 1 MB stripes, the last one partial
    keep = sorted(random.Random(seed).sample(range(N), 7))
    _check(oracle, _jit_slicer(), 2_500_003, keep, seed)


def test_jit_fewer_erasures_small_stripes(oracle):  # 100 kB stripes: 1-wave workgroups
    keep = sorted(random.Random(9).sample(range(N), 11))
    _check(oracle, _jit_slicer(), 250_001, keep, 9)
