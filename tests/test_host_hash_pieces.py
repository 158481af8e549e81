"""hh::LeafLanes (tape_amd/csrc/host_hash.cpp) on the host, no GPU: hashing a slice fed in pieces
(the stream writer hashes a window's row pieces as they land) equals hashing it whole,
for 1-4 interleaved lanes, lengths around the 64-byte block edges and random piece boundaries.
The one-shot hashes themselves are checked against the merkle oracle in test_merkle.py."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.isdir("/opt/rocm/include"),
                    reason="needs g++ and the ROCm headers")
def test_leaf_lanes_pieces(tmp_path):
    exe = str(tmp_path / "leaf_lanes_check")
    src = [os.path.join(HERE, "cpp", "leaf_lanes_check.cpp"), os.path.join(ROOT, "tape_amd", "csrc", "host_hash.cpp")]
    cmd = ["g++", "-O2", "-std=c++20", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROOT, "tape_amd", "csrc"),
           "-I/opt/rocm/include", *src, "-o", exe, "-L/opt/rocm/lib", "-lamdhip64", "-lpthread",
           "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout
