"""rs16::mat_image (tape_amd/csrc/rs16.hpp) on the host, no GPU: the lookup image the OuterCoder
matrix kernel (rs16.hip rs16_matrix_kernel) stages, read the way the kernel reads
it -- 8-row pair entries, the odd 4-row tail group, or the VALU tail row's bit constants for
rows = 8 h + 1 -- reproduces the direct GF(2^16) matrix product for every row count 1..64 at
eight input counts, and the encode matrix (unit-vector encodes) reproduces rs16::encode_column.
The GPU parity of the kernel itself against the oracle is tests/test_gpu_outer.py."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_mat_image_emulated(tmp_path):
    exe = str(tmp_path / "mat_image_check")
    cmd = ["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "tape_amd", "csrc"),
           os.path.join(HERE, "cpp", "mat_image_check.cpp"), "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout
