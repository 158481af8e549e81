"""The decode / recover class kernels' relabelling, checked on the host (no GPU): every one of the
77,520 7-of-20 survivor sets of Clay(20,7,16) is decoded by interpreting its class representative's
plane program through the set's relabelling -- the same mapping the generated kernels apply -- with
the set's own 2-bit-field matrix tables, and must give back the data chunks of a stripe encoded by
the oracle; every lost node of one set in 40 is recovered the same way; a neighbouring class's
program must fail (tests/native/dec_class_check.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_class_relabelling_every_survivor_set(tmp_path):
    exe = str(tmp_path / "dec_class_check")
    ora = os.path.join(ROOT, "oracle")
    if not os.path.exists(os.path.join(ora, "libclay_oracle.so")):
        subprocess.run(["make", "-s", "-C", ora], check=True)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++20", "-I", os.path.join(ROOT, "tape_amd", "csrc"),
                        os.path.join(ROOT, "tests", "native", "dec_class_check.cpp"), "-L", ora, "-lclay_oracle",
                        "-Wl,-rpath," + ora, "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe, "40"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    counts = [int(x) for x in r.stdout.split("counts")[1].split()]
    # decode classes by known column-0 nodes a0: C(10, a0) * C(10, 7 - a0) survivor sets each
    assert counts[:8] == [120, 2100, 11340, 25200, 25200, 11340, 2100, 120]
    assert "bad 0" in r.stdout and "wrong-class caught 200/200" in r.stdout


def test_class_programs_load_fusion(tmp_path):
    """Row loads per stripe column of every class program after the load fusions
    (tests/native/dec_class_loads.cpp): pinned, so a change that loses the type-1 or in-row pair
    fusion fails here, on the CPU.  Unfused, a0 = 3 loads 1,330 rows (700 own, 180 known-partner,
    450 type-1 partner); fused, 820."""
    exe = str(tmp_path / "dec_class_loads")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++20", "-I", os.path.join(ROOT, "tape_amd", "csrc"),
                        os.path.join(ROOT, "tests", "native", "dec_class_loads.cpp"), "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    rows = [list(map(int, line.split())) for line in r.stdout.split("\n") if line.strip()]
    assert [x[0] for x in rows] == list(range(24))
    loads = [x[1] for x in rows]
    assert loads[:8] == [1120, 1000, 720, 820, 760, 720, 700, 700]  # decode, a0 = 0..7
    assert max(loads[8:]) <= 820                                      # recover classes
    assert all(x[2] > 0 for x in rows)            # every program has fused type-1 steps
    assert all(x[4] <= 25 for x in rows)          # slots: two workgroups' LDS per CU
    # weighted over the 77,520 survivor sets (class a0 holds C(10, a0) C(10, 7 - a0) of them)
    w = [120, 2100, 11340, 25200, 25200, 11340, 2100, 120]
    assert sum(a * b for a, b in zip(w, loads[:8])) / sum(w) < 790
