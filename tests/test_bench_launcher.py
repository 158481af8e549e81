"""bench.py --gpus N without an external launcher (VERDICT r04 missing #1): the script starts N
worker processes itself, one per GPU, before anything touches the GPU.  On CPU the workers run the
multi-rank plumbing over gloo (`--launcher-check`): process group, rank partition of the object
ids, each rank's SplitMix64 objects and the max-over-ranks time; the objects are checked here
against the oracle's SplitMix64 stream and the partition against SURVEY 8e.
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, gpus=2):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--launcher-check",
                        *extra], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints exactly one line
    return json.loads(lines[0])


def test_gpus_2_spawns_two_ranks():
    from oracle import oracle as O
    L, nobj = 30_011, 3
    line = _run("--objects", str(nobj), "--object-bytes", str(L))
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["backend"] == "gloo"
    ranks = sorted(line["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == [0, 1]
    assert ranks[0]["pid"] != ranks[1]["pid"]            # two worker processes
    assert [(r["first"], r["end"]) for r in ranks] == [(0, nobj), (nobj, 2 * nobj)]
    assert line["max_over_ranks_s"] == 2.0               # rank r reported 1 + r
    for r in ranks:
        for i, gid in enumerate(range(r["first"], r["end"])):
            exp = hashlib.sha256(O.splitmix64_bytes(0x7A9E5EED ^ gid, L).tobytes()).hexdigest()
            assert r["digests"][i] == exp


def test_config5_partition_over_four_ranks():
    """--workload config5: 16,384 objects split into contiguous ranges, 4,096 per rank at N = 4,
    device batches of 2,048 (tiny objects so the check is fast)."""
    from oracle import oracle as O
    L = 16
    line = _run("--workload", "config5", "--object-bytes", str(L), gpus=4)
    assert line["n_gpus"] == 4 and line["world_size"] == 4
    assert line["total_objects"] == 16_384 and line["objects_per_gpu"] == 4_096
    assert line["device_batch_objects"] == 2_048
    ranks = sorted(line["ranks"], key=lambda r: r["rank"])
    assert [(r["first"], r["end"]) for r in ranks] == [(i * 4096, (i + 1) * 4096) for i in range(4)]
    for r in ranks:
        for i in (0, 4095):
            gid = r["first"] + i
            exp = hashlib.sha256(O.splitmix64_bytes(0x7A9E5EED ^ gid, L).tobytes()).hexdigest()
            assert r["digests"][i] == exp


def test_gpus_1_runs_in_process():
    line = _run("--objects", "2", "--object-bytes", "100", gpus=1)
    assert line["n_gpus"] == 1 and line["world_size"] == 1 and len(line["ranks"]) == 1


def _identity(line, steps):
    inj = line["injected"]
    r = inj["rates"]
    assert inj["steps"] == steps
    # value [GiB/s] x ms_per_step = the job's bytes per step, whatever the step count
    assert abs(r["value"] * r["ms_per_step"] * 2**30 / 1e3 - inj["job_bytes_per_step"]) <= 1e-6 * inj["job_bytes_per_step"]
    return r


def test_config5_line_arithmetic_n1_n2_n4():
    """the config-5 line printed one step's bytes over all steps' time.  The
    line's numbers now come from bench.config5_rates; with injected timings (rank r: 83.9 + r ms
    per step) the identity value x ms_per_step = 16,384 objects' bytes must hold at N = 1, 2, 4."""
    L = 16
    for gpus in (1, 2, 4):
        line = _run("--workload", "config5", "--object-bytes", str(L), "--steps", "3", gpus=gpus)
        r = _identity(line, 3)
        assert line["injected"]["job_bytes_per_step"] == 16_384 * L
        assert abs(r["ms_per_step"] - (83.9 + (gpus - 1))) < 1e-9   # max over ranks
        assert len(r["rank_ms_per_step"]) == gpus
        # 8 / N device batches of <= 2,048 objects, 10.43 ms each
        assert abs(r["avg_launch_ms"] - 10.43) < 1e-9


def test_default_line_arithmetic_steps_independent():
    for steps in (1, 5):
        line = _run("--objects", "2", "--object-bytes", "100", "--steps", str(steps), gpus=2)
        r = _identity(line, steps)
        assert line["injected"]["job_bytes_per_step"] == 2 * 2 * 100


def test_step_rates_units():
    sys.path.insert(0, ROOT)
    import bench
    MiB = 1 << 20
    # r05's config-5 N = 1 run: 3 steps of 83.93 ms over 64 GiB -> ~763 GiB/s, not 254
    r = bench.config5_rates(16_384, 4 * MiB, 3, [3 * 0.08393], 3 * 8 * 10.43, 8, 2_048)
    assert 760 < r["value"] < 765
    assert abs(r["avg_launch_ms"] - 10.43) < 1e-9
    exp = bench.ALG_BYTES["encode"] * 2_048 / 10.43e-3 / 1e9
    assert abs(r["achieved"] - exp) < 1e-6 and abs(r["frac"] - exp / bench.PEAK_HBM_GBS) < 1e-9
    r1 = bench.step_rates(1024 * 4 * MiB, 10, 10 * 5.5791e-3, bench.ALG_BYTES["encode"] * 1024, 10 * 5.5639, 10)
    assert abs(r1["value"] - 716.97) < 0.05 and abs(r1["frac"] - 0.4255) < 1e-4
