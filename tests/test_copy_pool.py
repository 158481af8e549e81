"""The per-call host copy pool (tape_amd/csrc/copy_pool.hpp; ADVICE r05 medium: a late worker could
touch the next job's piece list and counters).  A host-only stress program runs many back-to-back
run() calls of different sizes from several threads on one pool and checks every byte, built once
with ThreadSanitizer and once with AddressSanitizer (host code only; no GPU)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "copy_pool_stress.cpp")


@pytest.mark.parametrize("san", ["thread", "address"])
def test_copy_pool_stress_sanitized(tmp_path, san):
    exe = str(tmp_path / f"cp_{san}")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-pthread", SRC, "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1", ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe, "3", "150"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert r.stdout.startswith("ok 450")
    assert "WARNING: ThreadSanitizer" not in r.stderr
