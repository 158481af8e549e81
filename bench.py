#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X Clay engine (BASELINE.json `metric`).

Workload (BASELINE.json configs[1]): device-resident Slicer::encode of a batch of 1024 x 4 MiB
synthetic objects (SplitMix64, seed 0x7A9E5EED ^ object id) with the production
profile Clay(20,7,16), rotated 1 MB stripes; one "step" = one te_encode_batch_device call over
the whole batch (all 20 slices incl. metadata written to HBM).  Multi-GPU (torchrun): objects
are partitioned across ranks (per-GPU batches, weak scaling), no data-path collective.

Also: --mode repair (config 3), --mode decode (config 4, slices 0..12 erased), --mode commit
(hash_leaf of the 20 slices + merkle root + proofs of every encoded object) and
--mode recover (decode from 7 slices + re-encode, the node's recover path) and
--mode stream (the SDK's stream-write shape -- 64 MiB chunks, encode_with_proofs per
chunk, at most 4 in flight -- host -> host through te_stream_writer).
Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MiB = 1024 * 1024
N = 20
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md chip table (8.0 TB/s spec)
METRIC = "device-resident encode GiB/s, batched 4 MiB objects, 1 MI355X; % HBM peak"
ALG_BYTES = {  # algorithmic HBM bytes per 4 MiB object
    "encode": 4 * MiB + N * 715_048,
    "repair": 16 * 71_500 + 715_048,
    "decode": 7 * 715_048 + 4 * MiB,
    "commit": N * 715_048 + N * 32 + 32 + N * 5 * 32,  # slices read; leaf hashes, root, proofs written
    # the work, not the implementation: 7 peer slices read, the lost slice written (recover.rs:411-442)
    "recover": 7 * 715_048 + 715_048,
}


def splitmix_fill(torch, out_u8, first_obj: int, nobj: int, obj_len: int, seed: int = 0x7A9E5EED):
    """Device-side SplitMix64 stream per object: byte j of object i = word floor(j/8) of
    SplitMix64(seed ^ i), little-endian.  Same stream as oracle.splitmix64_bytes.
    Vectorised over 64 objects per pass (few kernels, so profiles stay small)."""
    words = (obj_len + 7) // 8
    G = -7046029254386353131  # 0x9E3779B97F4A7C15 as int64
    M1 = -4658895280553007687  # 0xBF58476D1CE4E5B9
    M2 = -7723592293110705685  # 0x94D049BB133111EB
    idx = torch.arange(1, words + 1, dtype=torch.int64, device=out_u8.device)

    def lsr(x, k):
        return (x >> k) & ((1 << (64 - k)) - 1)

    view = out_u8[:nobj * obj_len].view(nobj, obj_len)
    for c0 in range(0, nobj, 64):
        c1 = min(nobj, c0 + 64)
        seeds = []
        for i in range(c0, c1):
            s = seed ^ (first_obj + i)
            seeds.append(s - (1 << 64) if s >= 1 << 63 else s)
        sd = torch.tensor(seeds, dtype=torch.int64, device=out_u8.device)
        z = idx[None, :] * G + sd[:, None]
        z = (z ^ lsr(z, 30)) * M1
        z = (z ^ lsr(z, 27)) * M2
        z = z ^ lsr(z, 31)
        view[c0:c1].copy_(z.view(torch.uint8).view(c1 - c0, words * 8)[:, :obj_len])
        del z


def dist_setup(torch, dist, backend: str):
    """One process per GPU (torchrun env).  Objects are partitioned, so the process group is used
    only for the barrier and the max-over-ranks timing -- never on the data path."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            init_rccl(torch, dist, rank, local, world)
        else:
            dist.init_process_group(backend)
    return world, rank, local


RCCL_INIT_TIMEOUT_S = 180


def init_rccl(torch, dist, rank: int, local: int, world: int, timeout_s: float = RCCL_INIT_TIMEOUT_S) -> None:
    """The one place a bench rank brings up RCCL (torch's "nccl" backend on ROCm).  It binds the rank
    to cuda:LOCAL_RANK, creates the process group with a bounded timeout and runs one all_reduce so
    the communicator is built here rather than inside the timed region.  Any failure -- no such
    device, a rendezvous or communicator error, a wrong sum -- prints the rank, its device and the
    error to stderr and exits non-zero, so a first multi-GPU run fails loudly (launch_ranks then
    stops the other ranks) instead of hanging.  This branch has only ever run on the driver's
    8-GPU node; the gloo branch is what the CPU tests exercise."""
    import datetime
    where = f"rank {rank}/{world} on cuda:{local}"
    try:
        ndev = torch.cuda.device_count()
        if local >= ndev:
            raise RuntimeError(f"LOCAL_RANK {local} but only {ndev} visible device(s)")
        torch.cuda.set_device(local)
        try:
            p = torch.cuda.get_device_properties(local)
            where += f" (pci {p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x})"
        except Exception:
            pass
        dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                timeout=datetime.timedelta(seconds=timeout_s))
        t = torch.ones(1, dtype=torch.float64, device=torch.device("cuda", local))
        dist.all_reduce(t)
        torch.cuda.synchronize()
        if int(t.item()) != world:
            raise RuntimeError(f"first all_reduce summed to {t.item()}, expected {world}")
    except BaseException as e:  # SystemExit / KeyboardInterrupt included: report, then leave non-zero
        print(f"[bench] RCCL initialisation failed for {where}: {type(e).__name__}: {e}", file=sys.stderr,
              flush=True)
        os._exit(3)


def step_rates(bytes_per_step: int, steps: int, elapsed_s: float, alg_bytes_per_launch: int | None = None,
               kernel_ms_total: float | None = None, launches: int | None = None) -> dict:
    """The arithmetic of every bench line, in one place (config 5 divided one
    step's bytes by all steps' time).  `bytes_per_step` is the object bytes the whole job (all
    ranks) encodes per step; `elapsed_s` covers `steps` steps (max over ranks).  Then
        value [GiB/s] = bytes_per_step * steps / elapsed_s / 2^30,  ms_per_step = elapsed_s / steps * 1e3,
    so value * ms_per_step * 2^30 / 1e3 == bytes_per_step exactly.  The roofline side: one launch
    (one call's kernels) moves `alg_bytes_per_launch` algorithmic bytes; `kernel_ms_total` is the
    device time of `launches` launches (HIP events on the launch stream)."""
    if steps <= 0 or elapsed_s <= 0:
        raise ValueError("steps and elapsed time must be positive")
    out = {"value": bytes_per_step * steps / elapsed_s / 2**30, "ms_per_step": elapsed_s / steps * 1e3,
           "avg_launch_ms": None, "achieved": None, "frac": None}
    if kernel_ms_total is not None and launches:
        avg_s = kernel_ms_total / launches / 1e3
        out["avg_launch_ms"] = avg_s * 1e3
        if alg_bytes_per_launch and avg_s > 0:
            out["achieved"] = alg_bytes_per_launch / avg_s / 1e9
            out["frac"] = out["achieved"] / PEAK_HBM_GBS
    return out


def config5_rates(total_objects: int, L: int, steps: int, rank_elapsed_s: list, kernel_ms_total: float,
                  batches_per_step: int, device_batch: int) -> dict:
    """Config 5's line values: one step = every rank encodes its whole share (all 16,384 objects
    over the job) in `batches_per_step` device batches of `device_batch` objects."""
    r = step_rates(total_objects * L, steps, max(rank_elapsed_s), ALG_BYTES["encode"] * device_batch
                   if L == 4 * MiB else None, kernel_ms_total, steps * batches_per_step)
    r["rank_ms_per_step"] = [x * 1e3 / steps for x in rank_elapsed_s]
    return r


# The kernels one step of each mode runs on the default workload (rocprofv3 names, prefix match).
# profiles/traffic.json holds per mode the HBM bytes these moved per step, measured by
# scripts/profile_modes.sh + scripts/traffic.py; it is used only while the names still match.
KERNELS = {
    "encode": ["tec::dma::enc_dma_kernel<false>"],
    "repair": ["tec::rfold::rep_fold_kernel"],  # every folded instance (lost column x known set)
    "decode": ["tec::dcls::dec_class_"],  # the decode class kernels (decode_class.hip), side by side
    "commit": ["tec::commit::leaf_kernel", "tec::commit::tree_kernel"],
    "recover": ["tec::dcls::dec_class_"],  # the recover class kernels (decode_class.hip), side by side
    "outer": ["tec::rs16k::rs16_matrix_kernel<9, 32, false>"],  # OuterCoder(17, 50) encode: 17 x 33 matrix
    "outer_decode": ["tec::rs16k::rs16_matrix_kernel<5, 32, true>"],  # 17 restored from 17 (3 launches per step)
}
# launches of a KERNELS entry per bench step (traffic.py scales its per-launch average by this)
LAUNCHES_PER_STEP = {"outer_decode": 3}


def kernel_names(mode: str, decode_jit: str = "async", pattern: str = "worst") -> list:
    # Clay(20,7,16) decode, worst case or random survivor sets: every stripe runs its class's kernel
    # (decode_class.hip); the hipRTC pattern kernels serve other profiles' hot patterns, or callers
    # that ask for them (te_clay_set_decode_jit)
    return KERNELS.get(mode, [])


def traffic_key(mode: str, pattern: str = "worst") -> str:
    """profiles/traffic.json entry of a bench line (random-pattern decode has its own)."""
    return "decode:random" if mode == "decode" and pattern == "random" else mode


def gpu_env(torch, dev) -> dict:
    """The box the line was measured on (two box types answer the same binary 0.41 vs
    0.47): device name, CUs, and from sysfs (best effort, read-only) the current GPU / memory clock
    levels and the compute / memory partition modes of this GPU's PCI function."""
    out = {}
    try:
        p = torch.cuda.get_device_properties(dev)
        out.update(name=p.name, arch=p.gcnArchName, cus=p.multi_processor_count,
                   pci=f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}")
        base = f"/sys/bus/pci/devices/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        for key, fn in (("sclk", "pp_dpm_sclk"), ("mclk", "pp_dpm_mclk"), ("fclk", "pp_dpm_fclk")):
            try:
                lines = open(os.path.join(base, fn)).read().split("\n")
                cur = [l for l in lines if l.strip().endswith("*")]
                out[key] = (cur[0] if cur else " | ".join(l for l in lines if l)).strip()
            except OSError:
                pass
        try:
            out["host_cpu"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
        except (OSError, StopIteration):
            pass
        for key, fn in (("compute_partition", "current_compute_partition"),
                        ("memory_partition", "current_memory_partition")):
            try:
                out[key] = open(os.path.join(base, fn)).read().strip()
            except OSError:
                pass
    except Exception as e:  # never fail a bench line on this
        out["error"] = str(e)[:80]
    return out


def box_ceiling(torch, d_in, in_bytes, d_out, out_bytes, stream, alg_bytes) -> dict | None:
    """This box's HBM ceiling for the encode's byte mix (tape_amd/csrc/hbm_probe.hip, measurement
    only): the step's object bytes read once and slice bytes written once by a compute-free,
    barrier-free streaming kernel on the bench's own buffers, before the timed region.  "blocks":
    contiguous 1 KiB wave-blocks (the best any encode kernel could do); "rows": the output as the
    slices' 1,430-byte sub-chunk rows (what the row shape alone costs).  GB/s = alg bytes / ms."""
    import ctypes as C
    try:
        lib = C.CDLL(os.path.join(ROOT, "tape_amd", "libtecprobe.so"))
    except OSError as e:
        return {"error": str(e)[:100]}
    f = lib.tec_probe_encode_mix
    f.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_void_p,
                  C.POINTER(C.c_float)]
    res = {}
    for name, shape, wgs in (("blocks", 0, 1024), ("blocks", 0, 2048), ("rows", 1, 1024)):
        ms = C.c_float()
        r = f(d_in.data_ptr(), in_bytes, d_out.data_ptr(), out_bytes, shape, wgs, 5, C.c_void_p(stream.cuda_stream),
              C.byref(ms))
        if r:
            return {"error": f"probe failed ({r})"}
        key = f"{name}_ms"
        res[key] = min(res.get(key, 1e9), round(ms.value, 4))
    torch.cuda.synchronize()
    return {"blocks_ms": res["blocks_ms"], "rows_ms": res["rows_ms"],
            "blocks_GBps": round(alg_bytes / res["blocks_ms"] / 1e6, 1),
            "rows_GBps": round(alg_bytes / res["rows_ms"] / 1e6, 1),
            "blocks_frac_of_peak": round(alg_bytes / res["blocks_ms"] / 1e6 / PEAK_HBM_GBS, 4)}


def dev_of(torch, world: int, local: int):
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    return dev


def rank_objects(rank: int, nobj: int) -> tuple[int, int]:
    """Contiguous global object range [first, first + nobj) of this rank (weak scaling)."""
    return rank * nobj, rank * nobj + nobj


def launch_ranks(n: int, argv: list) -> int:
    """`--gpus N` (N > 1) without an external launcher: start N worker processes of this same
    script, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in their
    environment (what torch.distributed.run would set), then wait for all of them.  This process
    never touches the GPU (no torch.cuda call, no libtapeec load) and never re-execs: the workers
    are children.  Rank 0 prints the one JSON line; if any rank fails, the others are stopped (by
    their own PIDs) and the first failing exit code is returned.  The reference's equivalent
    concurrency is the stream writer's worker pool (sdk/src/stream/write.rs:54-57, 329-362)."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TEC_BENCH_LAUNCHED="1")
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE, text=True, bufsize=1))
    # the ranks' stdout: only the JSON line goes to ours; anything else a library prints there
    # (gloo's connection notes, ...) goes to stderr, so the driver reads exactly one line
    import threading

    def pump(p):
        for line in p.stdout:
            (sys.stdout if line.startswith("{") else sys.stderr).write(line)
            (sys.stdout if line.startswith("{") else sys.stderr).flush()
    pumps = [threading.Thread(target=pump, args=(p,), daemon=True) for p in procs]
    for t in pumps:
        t.start()
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print(f"[bench] rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in pending:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    for t in pumps:
        t.join(timeout=10)
    return rc


def launcher_check(args) -> None:
    """`--launcher-check` (CPU, gloo; tests/test_bench_launcher.py): the multi-rank plumbing of a
    bench run without a GPU -- process group, rank partition of the object ids, each rank's
    SplitMix64 objects, the max-over-ranks time -- gathered to rank 0, which prints one JSON line
    with the digests of every rank's objects (the test checks them against the oracle)."""
    import hashlib
    import torch
    import torch.distributed as dist
    world, rank, _ = dist_setup(torch, dist, "gloo")
    share, batch_objs = rank_share(args, world)
    first, end = rank_objects(rank, share)
    L = args.object_bytes
    buf = torch.empty(share * L, dtype=torch.uint8)
    splitmix_fill(torch, buf, first, share, L)
    digests = [hashlib.sha256(buf[i * L:(i + 1) * L].numpy().tobytes()).hexdigest() for i in range(share)]
    t = max_over_ranks(torch, dist, world, 1.0 + rank, torch.device("cpu"))
    # the line arithmetic on injected timings: rank r "took" (83.9 + r) ms per step, its kernels
    # 10.43 ms per device batch -- the same functions the GPU run's line goes through
    steps = args.steps
    rank_el = gather_floats(torch, dist, world, steps * (0.0839 + 0.001 * rank), torch.device("cpu"))
    if args.workload == "config5":
        nbat = share // batch_objs
        rates = config5_rates(share * world, L, steps, rank_el, steps * nbat * 10.43, nbat, batch_objs)
        job_bytes = share * world * L
    else:
        rates = step_rates(share * world * L, steps, max(rank_el), None, steps * 10.43, steps)
        job_bytes = share * world * L
    got = [None] * world
    if world > 1:
        dist.all_gather_object(got, {"rank": rank, "first": first, "end": end, "digests": digests,
                                     "pid": os.getpid()})
    else:
        got = [{"rank": 0, "first": first, "end": end, "digests": digests, "pid": os.getpid()}]
    if rank == 0:
        print(json.dumps({"metric": "launcher check (no GPU)", "n_gpus": world,
                          "world_size": dist.get_world_size() if world > 1 else 1,
                          "backend": dist.get_backend() if world > 1 else None,
                          "objects_per_gpu": share, "device_batch_objects": batch_objs,
                          "total_objects": share * world, "max_over_ranks_s": t, "ranks": got,
                          "injected": {"steps": steps, "job_bytes_per_step": job_bytes, "rates": rates}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


CONFIG5_TOTAL_OBJECTS = 16_384  # BASELINE.json configs[4]: 64 GiB stream of 4 MiB objects over 8 GPUs
CONFIG5_DEVICE_BATCH = 2_048    # one GPU's share at N = 8


def rank_share(args, world: int) -> tuple[int, int]:
    """(objects this rank encodes per step, objects per device batch).  Default: --objects per GPU
    (weak scaling).  --workload config5: the 64 GiB stream of 16,384 objects split over the ranks
    (2,048 per GPU at N = 8; strong scaling), encoded in device batches of <= 2,048 objects."""
    if args.workload == "config5":
        if CONFIG5_TOTAL_OBJECTS % world:
            raise SystemExit(f"--workload config5 needs a world size dividing {CONFIG5_TOTAL_OBJECTS}")
        share = CONFIG5_TOTAL_OBJECTS // world
        return share, min(share, CONFIG5_DEVICE_BATCH)
    return args.objects, args.objects


def coll_dev(dist, dev):
    """Where the timing collectives' tensors live: the GPU under RCCL, the host under gloo."""
    return dev if str(dist.get_backend()) == "nccl" else "cpu"


def max_over_ranks(torch, dist, world: int, seconds: float, dev) -> float:
    if world <= 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=coll_dev(dist, dev))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--objects", type=int, default=1024, help="objects per GPU per step")
    ap.add_argument("--object-bytes", type=int, default=4 * MiB)
    ap.add_argument("--mode", choices=["encode", "repair", "decode", "commit", "recover", "outer", "stream", "percall"],
                    default="encode")
    ap.add_argument("--chunk-bytes", type=int, default=64 * MiB,
                    help="--mode stream: MAX_TRACK_SIZE, the SDK's stream chunk (sdk/src/stream/manifest.rs:22)")
    ap.add_argument("--stream-chunks", type=int, default=64, help="--mode stream: chunks per rank per pass")
    ap.add_argument("--hash-threads", type=int, default=0,
                    help="--mode stream: host hashing pool size (0 = the library's default, min(16, affinity CPUs))")
    ap.add_argument("--in-flight", type=int, default=4,
                    help="--mode stream: MAX_ENCODE_WORKERS, chunk encodes in flight (sdk/src/stream/write.rs:54-57)")
    ap.add_argument("--segments", type=int, default=16,
                    help="--mode outer: snapshot segments per step (OuterCoder(17, 50), 4 MiB chunks)")
    ap.add_argument("--cpu-sample", type=int, default=1024,
                    help="objects in the CPU-baseline sample (0 = skip); 1024 x 4 MiB is ~6-20 s of CPU-thread work "
                         "(16 threads) and checks every GPU output of the default batch")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = min(16, affinity cores): the GPU box grants 16 host cores per GPU (pool rules)")
    ap.add_argument("--copy-objects", type=int, default=-1,
                    help="objects in the copy-inclusive (pinned host -> host) leg, encode mode "
                         "(-1 = the whole per-GPU share, 0 = skip)")
    ap.add_argument("--copy-steps", type=int, default=2)
    ap.add_argument("--decode-jit", choices=["async", "off"], default="async",
                    help="decode / recover: per-pattern decode kernels (hipRTC-built during warm-up) or "
                         "the table-driven kernel only")
    ap.add_argument("--pattern", choices=["worst", "random"], default="worst",
                    help="--mode decode: worst = slices 0..12 erased (config 4); random = each object "
                         "keeps 7 random slices (the sdk downloader's first-k shape, downloader.rs:79-109)")
    ap.add_argument("--unavailable", type=int, default=0, choices=[0, 1],
                    help="--mode repair: 1 = slice (lost + 10) mod 20 is down too, so every stripe's "
                         "helper set skips one node of the other column (a peer outage)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--workload", choices=["default", "config5"], default="default",
                    help="encode mode: default = --objects per GPU (config 2, weak scaling); config5 = the "
                         "64 GiB stream of 16,384 x 4 MiB objects split over the N ranks (2,048 per GPU at "
                         "N = 8), device batches of <= 2,048, plus a copy-inclusive leg per rank")
    ap.add_argument("--sdk-chunks", type=int, default=16,
                    help="encode mode: chunks in the short SDK-shape stream leg (64 MiB chunks, 4 in flight, "
                         "pinned, the library's hashing choice; 0 = skip)")
    ap.add_argument("--launcher-check", action="store_true",
                    help="CPU only (gloo): run the multi-rank plumbing without a GPU (tests)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and env_world is None:
        # no external launcher: one worker process per GPU, started before anything here touches
        # the GPU (this process never initialises HIP)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus and not os.environ.get("TEC_BENCH_LAUNCHED"):
        print(f"[bench] WORLD_SIZE={env_world} from the launcher overrides --gpus {args.gpus}", file=sys.stderr)
    if args.launcher_check:
        return launcher_check(args)

    import numpy as np
    import torch
    import torch.distributed as dist
    import tape_amd as T
    from tape_amd import batch

    # TEC_BENCH_SHARED_GPU=1 (testing the N > 1 paths on a one-GPU box): every rank on cuda:0, the
    # timings exchanged over gloo -- RCCL refuses two ranks on one device
    shared = os.environ.get("TEC_BENCH_SHARED_GPU") == "1"
    world, rank, local = dist_setup(torch, dist, "gloo" if shared else "nccl")
    if shared:
        local = 0
    if args.workload == "config5":
        if args.mode != "encode":
            raise SystemExit("--workload config5 is an encode workload")
        return config5_bench(args, torch, dist, world, rank, dev_of(torch, world, local), np, T, batch)
    dev = dev_of(torch, world, local)
    T.lib.te_set_device(dev.index)

    if args.mode == "outer":
        return outer_bench(args, torch, dist, world, rank, dev)
    if args.mode == "stream":
        return stream_bench(args, torch, dist, world, rank, dev)
    if args.mode == "percall":
        return percall_bench(args, torch, dist, world, rank, dev)
    L, nobj = args.object_bytes, args.objects
    slicer = T.Slicer.clay_default()
    g = slicer.geometry(L)
    per = N * g.slice_len
    first, _ = rank_objects(rank, nobj)
    d_in = torch.empty(nobj * L, dtype=torch.uint8, device=dev)
    splitmix_fill(torch, d_in, first, nobj, L)
    d_out = torch.empty(nobj * per, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    enc_objs = batch.encode_descs([(i * L, L, i * per, 0) for i in range(nobj)])  # built once

    def encode_step():
        batch.encode_batch(slicer, d_in, enc_objs, d_out, stream)

    step = encode_step
    unit_bytes = ALG_BYTES[args.mode] if L == 4 * MiB else None
    if args.mode != "encode":
        encode_step()
        torch.cuda.synchronize()
    if args.mode == "decode":
        metas = b"".join(d_out[i * per + g.slice_len - 48:i * per + g.slice_len].cpu().numpy().tobytes()
                         for i in range(nobj))
        if args.pattern == "random":
            import random
            rnd = random.Random(0x5EED + first)
            masks = [sum(1 << j for j in rnd.sample(range(N), 7)) for _ in range(nobj)]
        else:
            masks = [sum(1 << j for j in range(13, 20))] * nobj
        dec_objs = batch.decode_descs([(i * per, g.slice_len, masks[i], i * L) for i in range(nobj)])
        d_dec = torch.empty(nobj * L, dtype=torch.uint8, device=dev)

        def step():
            batch.decode_batch(slicer, d_out, dec_objs, metas, d_dec, stream)
    elif args.mode == "repair":
        host_out = d_out.cpu().numpy()
        plans, blobs, offs, cur = [], [], [], 0
        for i in range(nobj):
            lost = i % N
            down = (lost + 10) % N if args.unavailable else lost
            avail = [j for j in range(N) if j not in (lost, down)]
            p = slicer.repair_plan_from_params(lost, avail, L, g.stripe_size)
            o = {}
            for h in avail:
                b = T.extract_repair_data(host_out[i * per + h * g.slice_len:i * per + (h + 1) * g.slice_len].tobytes(),
                                          p, h)
                if b:
                    o[h] = cur
                    blobs.append(b)
                    cur += len(b)
            plans.append(p)
            offs.append(o)
        d_help = torch.from_numpy(np.frombuffer(b"".join(blobs), np.uint8).copy()).to(dev)
        d_rep = torch.empty(nobj * g.slice_len, dtype=torch.uint8, device=dev)
        rep_objs = batch.repair_descs([(plans[i], offs[i], i * g.slice_len,
                                        host_out[i * per + g.slice_len - 48:i * per + g.slice_len].tobytes())
                                       for i in range(nobj)])
        del host_out

        def step():
            batch.repair_batch(slicer.coder, d_help, rep_objs, d_rep, stream)

    elif args.mode == "recover":  # lost = i mod 20 from the 7 slices after it (recover.rs:411-442)
        metas = b"".join(d_out[i * per + g.slice_len - 48:i * per + g.slice_len].cpu().numpy().tobytes()
                         for i in range(nobj))
        d_rec = torch.empty(nobj * g.slice_len, dtype=torch.uint8, device=dev)
        rec_objs = [(i * per, g.slice_len, sum(1 << ((i + j) % N) for j in range(1, 8)), i % N, i * g.slice_len)
                    for i in range(nobj)]

        def step():
            batch.recover_batch(slicer, d_out, rec_objs, metas, d_rec, stream)
    elif args.mode == "commit":
        from tape_amd import merkle
        d_leaf = torch.empty(nobj * N * 32, dtype=torch.uint8, device=dev)
        d_root = torch.empty(nobj * 32, dtype=torch.uint8, device=dev)
        d_proof = torch.empty(nobj * N * T.SLICE_TREE_HEIGHT * 32, dtype=torch.uint8, device=dev)

        def step():
            merkle.commit_batch(d_out, per, g.slice_len, N, nobj, d_leaf, d_root, d_proof, T.SLICE_TREE_HEIGHT, stream)

    ceiling = None
    if args.mode == "encode" and unit_bytes:  # this box's HBM on the encode's exact byte mix, same buffers
        ceiling = box_ceiling(torch, d_in, nobj * L, d_out, nobj * per, stream, unit_bytes * nobj)
    if args.mode in ("decode", "recover") and args.decode_jit == "off":
        slicer.coder.set_decode_jit("off")
    # (recover: 20 patterns x ~64 stripes per window -- below the engine's 512-stripe floor for a
    # pattern kernel's own launch, so it runs the shared table-driven launch either way)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    jit = None
    if args.mode in ("decode", "recover"):
        # hot patterns' kernels compile on worker threads from the first decode on; wait for
        # them, then warm up again: one-time work, untimed
        t_jit = time.perf_counter()
        ready, pending, failed = slicer.coder.decode_jit_status()
        while pending:
            ready, pending, failed = slicer.coder.decode_jit_status(timeout_ms=30_000)
            print(f"[bench] pattern kernels: {ready} ready, {pending} compiling, {failed} failed "
                  f"({time.perf_counter() - t_jit:.0f} s)", file=sys.stderr, flush=True)
        jit = {"mode": args.decode_jit, "ready": ready, "failed": failed,
               "compile_wait_s": round(time.perf_counter() - t_jit, 1)}
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # kernel time: HIP events the library records on the launch stream around each call's
    # kernels (te_kernel_timing), read after the timed region
    batch.kernel_time_ms()
    batch.kernel_timing(True)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    mine = time.perf_counter() - t0
    batch.kernel_timing(False)
    kms, kcalls = batch.kernel_time_ms()
    ident = rank_identity(torch, dist, world, dev, mine, kms, args.steps)
    elapsed = ident.pop("max_elapsed_s")

    # one launch = one step's kernels (HIP events on the launch stream)
    rates = step_rates(nobj * world * L, args.steps, elapsed, unit_bytes * nobj if unit_bytes else None,
                       kms, args.steps)
    achieved = rates["achieved"]

    verified = None  # the timed outputs, checked on the device against what they must equal
    if args.mode == "decode":
        verified = bool(torch.equal(d_dec, d_in))
    elif args.mode == "repair":
        sl = g.slice_len
        ref = torch.stack([d_out[i * per + (i % N) * sl:i * per + (i % N + 1) * sl] for i in range(nobj)])
        verified = bool(torch.equal(d_rep.view(nobj, sl), ref))
        del ref
    elif args.mode == "recover":
        sl = g.slice_len
        ref = torch.stack([d_out[i * per + (i % N) * sl:i * per + (i % N + 1) * sl] for i in range(nobj)])
        verified = bool(torch.equal(d_rec.view(nobj, sl), ref))
        del ref
    elif args.mode == "commit":  # first and last object against hashlib (SHA-256 of "LEAF" || slice)
        import hashlib
        ok = True
        for i in (0, nobj - 1):
            lv = d_leaf[i * N * 32:(i + 1) * N * 32].cpu().numpy().tobytes()
            for j in range(N):
                sl = d_out[i * per + j * g.slice_len:i * per + (j + 1) * g.slice_len].cpu().numpy().tobytes()
                ok = ok and lv[j * 32:(j + 1) * 32] == hashlib.sha256(b"LEAF" + sl).digest()
        verified = ok
    commit_sweep = None
    if args.mode == "commit":  # leaf-kernel parallelism = slices in the batch: rate against batch size
        commit_sweep = {}
        for m in (16, 64, 256, 1024, 2048, 4096):
            if m > nobj:
                break
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                merkle.commit_batch(d_out, per, g.slice_len, N, m, d_leaf, d_root, d_proof, T.SLICE_TREE_HEIGHT, stream)
            torch.cuda.synchronize()
            commit_sweep[str(m)] = round(3 * m * L / (time.perf_counter() - t) / 2**30, 2)
    copy_inc = copy_commit = None
    if args.mode == "encode" and args.copy_objects != 0:
        copy_inc = copy_inclusive(args, torch, dist, world, slicer, batch, d_in, d_out, per, L, dev)
        copy_commit = copy_inclusive_commit(args, torch, dist, world, slicer, batch, d_in, d_out, per, L, dev)

    sdk_stream = None
    if args.mode == "encode" and args.copy_objects != 0 and args.sdk_chunks > 0:
        # hand the copy-inclusive legs' pinned blocks (~40 GiB, freed but kept by torch's caching
        # host allocator) back first: with them cached this leg ran 7.2 GiB/s at 33.6 ms per chunk,
        # after the release 13.7 GiB/s at 16.3 ms, as in a fresh process (r05,
        # scripts/sdk_state_probe.py)
        if hasattr(torch._C, "_host_emptyCache"):
            torch._C._host_emptyCache()
        sdk_stream = stream_sdk_short(args, torch, dist, world, rank, dev, T, batch)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0 and args.mode == "encode":  # rank 0 at N=1 only
        cpu = cpu_baseline(args, np, torch, d_in, d_out, per, L)
    if rank == 0 and world == 1 and args.cpu_sample > 0 and args.mode == "commit":
        cpu = cpu_baseline_commit(args, d_out, per, g.slice_len, L)
    if rank == 0 and world == 1 and args.cpu_sample > 0 and args.mode in ("decode", "repair", "recover"):
        if args.mode == "decode":
            cpu = cpu_baseline_mode(args, np, "decode", d_out, per, g.slice_len, L, d_dec, L, masks=masks)
        elif args.mode == "repair":
            lost = [i % N for i in range(nobj)]
            down = [(l + 10) % N if args.unavailable else -1 for l in lost]
            cpu = cpu_baseline_mode(args, np, "repair", d_out, per, g.slice_len, L, d_rep, g.slice_len,
                                    lost=lost, down=down)
        else:
            cpu = cpu_baseline_mode(args, np, "recover", d_out, per, g.slice_len, L, d_rec, g.slice_len,
                                    masks=[o[2] for o in rec_objs], lost=[o[3] for o in rec_objs])
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json)).get(traffic_key(args.mode, args.pattern), {})  # scripts/traffic.py
            if tj.get("objects") == nobj and tj.get("kernels") == kernel_names(args.mode, args.decode_jit, args.pattern):
                traffic = tj.get("hbm_bytes_per_step")
        except Exception:
            traffic = None
    if rank == 0:
        line = {
            "metric": METRIC if args.mode == "encode" else (
                "device-resident slice-commitment GiB/s (hash_leaf x 20 + merkle root + proofs), batched 4 MiB "
                "objects, 1 MI355X" if args.mode == "commit" else
                f"device-resident {args.mode} GiB/s, batched 4 MiB objects, 1 MI355X"),
            "value": round(rates["value"], 3),
            "unit": "GiB/s",
            "n_gpus": world,
            **comm_info(dist, world),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(rates["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (SplitMix64 per object, seed 0x7A9E5EED ^ id), device-resident",
            "config": {"workload": {"encode": "Slicer::encode",
                                    "repair": "Slicer::repair (lost = i mod 20" +
                                              (", slice (i + 10) mod 20 down)" if args.unavailable else ")"),
                                    "decode": "Slicer::decode (slices 0..12 erased)" if args.pattern == "worst" else
                                              "Slicer::decode (7 random slices kept per object)",
                                    "commit": "encode_with_proofs commitment (SHA-256 leaf per slice, height-5 root, 20 proofs)",
                                    "recover": "node recover (the lost slice rebuilt from 7 peer slices, lost = i mod 20)"}[args.mode]
                       + f" of {nobj} x {L} B objects per GPU, Clay(20,7,16) rotated, 1 MB stripes",
                       "objects_per_gpu": nobj, "object_bytes": L, "profile": "clay(20,7,16)",
                       "parallelism": f"objects partitioned over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": rnd_opt(achieved, 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": rnd_opt(rates["frac"], 4),
                         "traffic": traffic,
                         "alg_bytes_per_launch": unit_bytes * nobj if unit_bytes else None,
                         "avg_launch_ms": rnd_opt(rates["avg_launch_ms"], 4),
                         "box_ceiling": ceiling,
                         "box_ceiling_frac": round(achieved / ceiling["blocks_GBps"], 4)
                         if ceiling and achieved else None},
            "cpu_baseline": cpu,
            "gpu": gpu_env(torch, dev),
            "ranks": ident,
            "copy_inclusive": copy_inc,
            "copy_inclusive_encode_commit": copy_commit,
            "stream_sdk_shape": sdk_stream,
            "commit_GiBps_vs_objects": commit_sweep,
            "outputs_verified": verified,
        }
        if jit is not None:
            line["decode_jit"] = jit
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def config5_bench(args, torch, dist, world, rank, dev, np, T, batch):
    """--workload config5 (BASELINE.json configs[4]): the 64 GiB synthetic write
    stream chunked at 4 MiB -- 16,384 objects -- encode partitioned across the N ranks, each rank its
    contiguous range of 16,384 / N objects (2,048 at N = 8) with no data-path collective.  The
    rank's objects are resident in HBM (64 GiB at N = 1); one step encodes all of them in device
    batches of <= 2,048 objects into one 2,048-object slice buffer.  `value` = 64 GiB / the step time
    (max over ranks): the whole job, so `scaling` is "strong".  Then a copy-inclusive leg per rank:
    the rank's objects from pinned host memory to pinned host slices through te_encode_batch_host
    over a host ring of <= 1,024 objects (4 GiB in, 14.6 GB out), every rank at once."""
    L = args.object_bytes
    share, nb = rank_share(args, world)
    first, _ = rank_objects(rank, share)
    slicer = T.Slicer.clay_default()
    g = slicer.geometry(L)
    per = N * g.slice_len
    d_in = torch.empty(share * L, dtype=torch.uint8, device=dev)
    splitmix_fill(torch, d_in, first, share, L)
    d_out = torch.empty(nb * per, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    descs = batch.encode_descs([(i * L, L, i * per, 0) for i in range(nb)])
    views = [d_in[b * nb * L:(b + 1) * nb * L] for b in range(share // nb)]

    def step():
        for v in views:
            batch.encode_batch(slicer, v, descs, d_out, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    batch.kernel_time_ms()
    batch.kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    mine = time.perf_counter() - t0
    batch.kernel_timing(False)
    kms, _ = batch.kernel_time_ms()
    per_rank = gather_floats(torch, dist, world, mine, dev)
    rank_kms = gather_floats(torch, dist, world, kms / max(1, args.steps), dev)
    rank_pci = gather_floats(torch, dist, world, float(pci_id(torch, dev)), dev)
    total = share * world
    rates = config5_rates(total, L, args.steps, per_rank, kms, len(views), nb)
    # the timed outputs of the last batch: decode(slices 13..19) == the objects, on every rank
    metas = b"".join(d_out[i * per + g.slice_len - 48:i * per + g.slice_len].cpu().numpy().tobytes() for i in range(nb))
    dec_objs = batch.decode_descs([(i * per, g.slice_len, sum(1 << j for j in range(13, 20)), i * L) for i in range(nb)])
    d_dec = torch.empty(nb * L, dtype=torch.uint8, device=dev)
    slicer.coder.set_decode_jit("off")
    batch.decode_batch(slicer, d_out, dec_objs, metas, d_dec, stream)
    torch.cuda.synchronize()
    ok = bool(torch.equal(d_dec, views[-1]))
    del d_dec
    oks = gather_floats(torch, dist, world, 1.0 if ok else 0.0, dev)
    # copy-inclusive: pinned host -> host over a ring of <= 1,024 objects, the rank's share streamed through it
    ring = min(share, 1024)
    h_in = torch.empty(ring * L, dtype=torch.uint8).pin_memory()
    h_in.copy_(d_in[:ring * L])
    h_out = torch.empty(ring * per, dtype=torch.uint8).pin_memory()
    hobjs = batch.encode_descs([(i * L, L, i * per, 0) for i in range(ring)])
    batch.encode_batch_host(slicer, h_in, hobjs, h_out)  # warm-up (pipeline buffers)
    if world > 1:
        dist.barrier()
    t = time.perf_counter()
    for _ in range(share // ring):
        batch.encode_batch_host(slicer, h_in, hobjs, h_out)
    cmine = time.perf_counter() - t
    c_rank = gather_floats(torch, dist, world, cmine, dev)
    # the ring's first and last object against a device-resident encode of the same bytes
    batch.encode_batch(slicer, d_in, descs, d_out, stream)
    torch.cuda.synchronize()
    cok = bool(torch.equal(h_out[:per], d_out[:per].cpu()) and
               torch.equal(h_out[(ring - 1) * per:ring * per], d_out[(ring - 1) * per:ring * per].cpu()))
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        import argparse as _ap
        a2 = _ap.Namespace(**vars(args))
        a2.objects = nb
        cpu = cpu_baseline(a2, np, torch, d_in, d_out, per, L)  # d_out now holds the first batch's slices
    if rank == 0:
        print(json.dumps({
            "metric": "device-resident encode GiB/s, 64 GiB stream of 4 MiB objects partitioned over the GPUs "
                      "(BASELINE config 5)",
            "value": round(rates["value"], 3), "unit": "GiB/s", "n_gpus": world,
            **comm_info(dist, world),
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(rates["ms_per_step"], 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (SplitMix64 per object, seed 0x7A9E5EED ^ id), device-resident",
            "config": {"workload": f"Slicer::encode of the 64 GiB stream ({total} x {L} B objects), {share} contiguous "
                                   f"objects per GPU in device batches of {nb}, Clay(20,7,16) rotated, 1 MB stripes",
                       "total_objects": total, "objects_per_gpu": share, "device_batch_objects": nb,
                       "object_bytes": L, "profile": "clay(20,7,16)",
                       "parallelism": f"objects partitioned over {world} GPU(s), no collective"},
            "rank_ms_per_step": [round(x, 3) for x in rates["rank_ms_per_step"]],
            "rank_kernel_ms_per_step": [round(x, 3) for x in rank_kms],
            "rank_pci": [pci_str(int(x)) for x in rank_pci],
            "roofline": {"bound": "hbm", "achieved": rnd_opt(rates["achieved"], 1), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": rnd_opt(rates["frac"], 4),
                         "traffic": None, "alg_bytes_per_launch": ALG_BYTES["encode"] * nb,
                         "avg_launch_ms": rnd_opt(rates["avg_launch_ms"], 4)},
            "cpu_baseline": cpu, "gpu": gpu_env(torch, dev),
            "copy_inclusive": {"value": round(total * L / max(c_rank) / 2**30, 3), "unit": "GiB/s", "pinned": True,
                               "host_ring_objects": ring, "rank_ms": [round(x * 1e3, 1) for x in c_rank],
                               "note": "each rank's share streamed from a pinned host ring of the first `host_ring_objects` "
                                       "objects through te_encode_batch_host, all ranks at once (node PCIe and host "
                                       "memory shared)", "matches_device_resident": cok},
            "outputs_verified": all(x == 1.0 for x in oks)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def rnd_opt(x, nd):
    return None if x is None else round(x, nd)


def pci_id(torch, dev) -> int:
    """The device's PCI address packed as domain << 16 | bus << 8 | device (0 when unknown)."""
    try:
        p = torch.cuda.get_device_properties(dev)
        return (p.pci_domain_id << 16) | (p.pci_bus_id << 8) | p.pci_device_id
    except Exception:
        return 0


def pci_str(v: int) -> str:
    return f"{v >> 16:04x}:{(v >> 8) & 0xFF:02x}:{v & 0xFF:02x}"


def rank_identity(torch, dist, world: int, dev, elapsed_s: float, kernel_ms: float, steps: int) -> dict:
    """Per-rank identity of a line: each rank's wall ms per step, its kernels' ms
    per step and its device's PCI address, so an N > 1 line shows a slow or doubled-up rank."""
    el = gather_floats(torch, dist, world, elapsed_s, dev)
    return {"rank_ms_per_step": [round(x * 1e3 / steps, 4) for x in el],
            "rank_kernel_ms_per_step": [round(x / max(1, steps), 4)
                                        for x in gather_floats(torch, dist, world, kernel_ms, dev)],
            "rank_pci": [pci_str(int(x)) for x in gather_floats(torch, dist, world, float(pci_id(torch, dev)), dev)],
            "max_elapsed_s": max(el)}


def gather_floats(torch, dist, world: int, x: float, dev) -> list:
    """Every rank's value of x (all_gather over the process group; only timings and flags travel)."""
    if world <= 1:
        return [x]
    t = torch.tensor([x], dtype=torch.float64, device=coll_dev(dist, dev))
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def comm_info(dist, world: int) -> dict:
    """The process group as the collective library saw it (RCCL is torch's "nccl" backend on ROCm)."""
    if world <= 1 or not dist.is_initialized():
        return {"world_size": 1, "backend": None}
    return {"world_size": dist.get_world_size(), "backend": str(dist.get_backend())}


def outer_bench(args, torch, dist, world, rank, dev):
    """--mode outer: OuterCoder(17, 50).encode of snapshot segments on the GPU
    (lib/snapshot/src/encode.rs:66-76 -> lib/slicer/src/outer.rs:70-118), 4 MiB chunks (the
    codec's maximum): per segment 17 x 4 MiB of data in, 33 x 4 MiB of recovery chunks out."""
    from tape_amd import outer
    k, n, cb = 17, 50, 4 * MiB
    m, segs = n - k, args.segments
    first, _ = rank_objects(rank, segs)
    d_in = torch.empty(segs * k * cb, dtype=torch.uint8, device=dev)
    splitmix_fill(torch, d_in, first, segs, k * cb)
    d_out = torch.empty(segs * m * cb, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        outer.encode_device(k, m, d_in, cb, segs, k * cb, d_out, m * cb, stream)

    from tape_amd import batch
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    batch.kernel_time_ms()
    batch.kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(torch, dist, world, time.perf_counter() - t0, dev)
    batch.kernel_timing(False)
    kms, _ = batch.kernel_time_ms()
    # the timed output: segment 0 decoded from its 17 parity-only chunks equals its data
    seg0 = [d_out[j * cb:(j + 1) * cb].cpu().numpy().tobytes() for j in range(k)]
    dec = outer.OuterCoder(k, n).decode([(k + j, seg0[j]) for j in range(k)])
    verified = dec == d_in[:k * cb].cpu().numpy().tobytes()
    alg = (k + m) * cb * segs
    er = step_rates(segs * world * k * cb, args.steps, elapsed, alg, kms, args.steps)
    # decode (snapshot reads, outer.rs:126-197) of every segment from its first 17 recovery
    # chunks (all data chunks missing: 17 restored per segment), device-resident
    d_dec = torch.empty(segs * k * cb, dtype=torch.uint8, device=dev)
    addr_out = d_out.data_ptr()

    dec_chunks = [[None] * k + [addr_out + (g * m + j) * cb for j in range(m)] for g in range(segs)]

    def dec_step():  # one te_outer_decode_device_batch call for the read's segments
        outer.decode_device_batch(k, n, dec_chunks, cb, d_dec, k * cb, stream)

    for _ in range(args.warmup):
        dec_step()
    torch.cuda.synchronize()
    batch.kernel_time_ms()
    batch.kernel_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dec_step()
    torch.cuda.synchronize()
    dec_elapsed = max_over_ranks(torch, dist, world, time.perf_counter() - t0, dev)
    batch.kernel_timing(False)
    dkms, _ = batch.kernel_time_ms()
    dec_ok = bool(torch.equal(d_dec, d_in))
    dec_alg = 2 * k * cb * segs  # 17 received chunks read, 17 restored written, per segment
    dr = step_rates(segs * world * k * cb, args.steps, dec_elapsed, dec_alg, dkms, args.steps)
    decode = {"value": round(dr["value"], 3), "unit": "GiB/s",
              "ms_per_step": round(dr["ms_per_step"], 4), "workload": "all 17 data chunks restored "
              "from 17 recovery chunks per segment (one te_outer_decode_device_batch call)",
              "roofline": {"bound": "hbm", "achieved": round(dr["achieved"], 1), "peak": PEAK_HBM_GBS,
                           "unit": "GB/s", "frac": round(dr["frac"], 4),
                           "alg_bytes_per_launch": dec_alg, "avg_launch_ms": round(dr["avg_launch_ms"], 4)},
              "outputs_verified": dec_ok}
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline_outer(args, d_in, d_out, k, m, cb, segs)
    # PMC bytes per step (scripts/profile_modes.sh outer -> traffic.py), when measured at this shape
    traffic = {"outer": None, "outer_decode": None}
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            for key in traffic:
                e = tj.get(key, {})
                if e.get("objects") == segs and e.get("kernels") == KERNELS[key]:
                    traffic[key] = e.get("hbm_bytes_per_step")
        except Exception:
            pass
    decode["roofline"]["traffic"] = traffic["outer_decode"]
    if rank == 0:
        print(json.dumps({
            "metric": "device-resident OuterCoder(17, 50) encode GiB/s of snapshot data, 4 MiB chunks, 1 MI355X",
            "value": round(er["value"], 3), "unit": "GiB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(er["ms_per_step"], 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u16 (GF(2^16))", "data": "synthetic SplitMix64, device-resident",
            "config": {"workload": f"OuterCoder(17, 50).encode of {segs} segments of 17 x 4 MiB per GPU "
                                   "(reed-solomon-simd Leopard GF(2^16) construction, parity unpinned)",
                       "segments_per_gpu": segs, "chunk_bytes": cb, "parallelism": f"segments over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": round(er["achieved"], 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(er["frac"], 4), "traffic": traffic["outer"],
                         "alg_bytes_per_launch": alg, "avg_launch_ms": round(er["avg_launch_ms"], 4)},
            "cpu_baseline": cpu, "outputs_verified": verified, "decode": decode}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_outer(args, d_in, d_out, k, m, cb, segs):
    """The oracle's GF(2^16) encode (oracle/rs16_oracle.c, the crate's algorithm restated) on host
    threads, one segment per task over the first `pre` bytes of each chunk: the code works column by
    column (element e of every shard), so a chunk prefix encodes to the recovery chunks' prefix,
    which is byte-compared with the GPU's."""
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor
    from oracle import rs16 as R
    lib = R._lib()
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    thr = args.cpu_threads or max(1, min(16, cores))
    nseg, pre = min(segs, 16), 1 << 20
    ins = [[d_in[(g * k + j) * cb:(g * k + j) * cb + pre].cpu().numpy() for j in range(k)] for g in range(nseg)]
    outs = [[bytearray(pre) for _ in range(m)] for _ in range(nseg)]

    def one(g):
        ip = (C.c_void_p * k)(*[a.ctypes.data for a in ins[g]])
        op = (C.c_void_p * m)(*[C.addressof((C.c_char * pre).from_buffer(b)) for b in outs[g]])
        return lib.rs16_encode(k, m, pre, ip, op)

    t = time.perf_counter()
    with ThreadPoolExecutor(thr) as ex:
        rcs = list(ex.map(one, range(nseg)))
    el = time.perf_counter() - t
    ok = all(r == 0 for r in rcs)
    for g in range(nseg):
        for j in range(m):
            ok = ok and bytes(outs[g][j]) == d_out[(g * m + j) * cb:(g * m + j) * cb + pre].cpu().numpy().tobytes()
    return {"value": round(nseg * k * pre / el / 2**30, 3), "unit": "GiB/s", "cores": thr, "kind": "port",
            "sample": f"{nseg} segments x 17 chunks, first {pre >> 20} MiB of each (column-wise code: the "
                      "recovery chunks' prefix), oracle rs16_encode per segment on a thread pool",
            "gpu_matches_oracle_on_sample": bool(ok)}


def stream_bench(args, torch, dist, world, rank, dev):
    """--mode stream: the SDK's stream-write shape.  write_bytes / write_stream cut the
    stream into MAX_TRACK_SIZE = 64 MiB chunks (sdk/src/stream/write.rs:219, manifest.rs:22); the
    encode stage keeps at most MAX_ENCODE_WORKERS = 4 chunk encodes in flight and hands them on in
    order (FuturesOrdered, write.rs:54-57, 332-362); each chunk is one encode_with_proofs (slices,
    20 leaf hashes, root, proofs; sdk/src/codec/encoder.rs:220-234).  Here: te_stream_writer, one
    window per chunk, the 5th submitted after the oldest has been waited for; host buffers in a
    ring of 2 x in-flight slots (the chunk source refills them).  Copy-inclusive: chunk bytes in host
    memory, slices + commitments back in host memory.  Legs: the library's choice (auto: these
    9.7 MB slices hash on the host pool as their D2H lands), device hashing forced, pageable host
    buffers; the CPU baseline is the oracle's encode + hashlib per chunk."""
    import collections
    import hashlib
    import numpy as np
    import tape_amd as T
    from tape_amd import batch, merkle
    CB, nch, depth, H = args.chunk_bytes, args.stream_chunks, args.in_flight, T.SLICE_TREE_HEIGHT
    if args.hash_threads:
        batch.set_host_hash_threads(args.hash_threads)
    s = T.Slicer.clay_default()
    g = s.geometry(CB)
    per = N * g.slice_len
    R = 2 * depth
    first, _ = rank_objects(rank, nch)
    d_src = torch.empty(R * CB, dtype=torch.uint8, device=dev)
    splitmix_fill(torch, d_src, first, R, CB)

    def ring(pinned):
        def alloc(n):
            t = torch.empty(n, dtype=torch.uint8)
            return t.pin_memory() if pinned else t
        r = {"in": [alloc(CB) for _ in range(R)], "out": [alloc(per) for _ in range(R)],
             "leaf": [alloc(N * 32) for _ in range(R)], "root": [alloc(32) for _ in range(R)],
             "proof": [alloc(N * H * 32) for _ in range(R)]}
        for k in range(R):
            r["in"][k].copy_(d_src[k * CB:(k + 1) * CB])
        return r

    descs = [batch.encode_descs([(0, CB, 0, first + c)]) for c in range(nch)]

    lat, sub = [], []  # per chunk: submit -> its wait returned (the SDK's FuturesOrdered hand-off); the submit call

    def run(sw, r, chunks):
        inflight = collections.deque()
        t_sub = {}
        del lat[:], sub[:]
        for c in range(chunks):
            k = c % R
            if len(inflight) >= depth:
                t = inflight.popleft()
                sw.wait(t)
                lat.append(time.perf_counter() - t_sub.pop(t))
            t_sub_c = time.perf_counter()
            t = sw.submit(r["in"][k], descs[c], r["out"][k], r["leaf"][k], r["root"][k], r["proof"][k])
            sub.append(time.perf_counter() - t_sub_c)
            t_sub[t] = t_sub_c
            inflight.append(t)
        while inflight:
            t = inflight.popleft()
            sw.wait(t)
            lat.append(time.perf_counter() - t_sub.pop(t))

    def leg(hashing, pinned):
        r = ring(pinned)
        sw = batch.StreamWriter([s], height=H, hashing=hashing)
        run(sw, r, min(nch, R))  # warm-up: buffers, pool
        if world > 1:
            dist.barrier()
        t = time.perf_counter()
        run(sw, r, nch)
        el = max_over_ranks(torch, dist, world, time.perf_counter() - t, dev)
        sw.close()
        return nch * world * CB / el / 2**30, el, r

    legs, ring_auto = {}, None
    for name, hashing, pinned in (("auto_pinned", "auto", True), ("host_hash_pinned", "host", True),
                                  ("device_hash_pinned", "device", True), ("auto_pageable", "auto", False)):
        v, el, r = leg(hashing, pinned)
        ls = sorted(lat)
        legs[name] = {"GiBps": round(v, 3), "ms_per_chunk": round(el / nch * 1e3, 2),
                      "chunk_latency_ms_p50_p90": [round(ls[len(ls) // 2] * 1e3, 2), round(ls[(9 * len(ls)) // 10] * 1e3, 2)]
                      if ls else None,
                      "submit_call_ms_mean_max": [round(sum(sub) / len(sub) * 1e3, 3), round(max(sub) * 1e3, 3)] if sub else None}
        if name == "auto_pinned":
            ring_auto, el_auto = r, el
        else:
            del r
    # the last R chunks of the auto leg: slices against the device-resident Slicer::encode of the
    # same bytes, leaf hashes against hashlib, root and proofs against the library's host merkle
    ok = True
    d_out = torch.empty(per, dtype=torch.uint8, device=dev)
    for c in range(max(0, nch - R), nch):
        k = c % R
        batch.encode_batch(s, d_src[k * CB:(k + 1) * CB], [(0, CB, 0, first + c)], d_out)
        torch.cuda.synchronize()
        ok = ok and torch.equal(ring_auto["out"][k], d_out.cpu())
        lv = ring_auto["leaf"][k].numpy().tobytes()
        sl = ring_auto["out"][k].numpy()
        leaves = []
        for j in range(N):
            h = hashlib.sha256(b"LEAF")
            h.update(memoryview(sl[j * g.slice_len:(j + 1) * g.slice_len]))
            leaves.append(h.digest())
        ok = ok and lv == b"".join(leaves)
        ok = ok and ring_auto["root"][k].numpy().tobytes() == merkle.root_from_leaf_hashes(leaves, H)
        pv = ring_auto["proof"][k].numpy().tobytes()
        for j in range(N):
            ok = ok and pv[j * H * 32:(j + 1) * H * 32] == b"".join(merkle.create_proof_from_leaf_hashes(leaves, j, H))
    # one thread's leaf-hash rate over one chunk's 20 slices at 1-4 interleaved lanes (te_hash_leaves;
    # the pool runs te_host_hash_lanes of them per task)
    lane_rate, pool_rate = [], None
    if rank == 0:
        import ctypes as C
        sl = ring_auto["out"][0]
        hout = (C.c_uint8 * (32 * N))()
        for L in range(1, 5):
            t = time.perf_counter()
            T.lib.te_hash_leaves(C.cast(sl.data_ptr(), C.POINTER(C.c_uint8)), g.slice_len, N, L, hout)
            lane_rate.append(round(N * g.slice_len / (time.perf_counter() - t) / 1e9, 3))
        # the pool's share of host cores hashing at once: one thread per te_host_hash_lanes slices
        # of the ring's chunks (ctypes drops the GIL), as the pool's tasks do
        import threading
        lanes = T.lib.te_host_hash_lanes()
        jobs = [(k, i0) for k in range(R) for i0 in range(0, N, lanes)]
        nthr = batch.host_hash_threads()
        outs = [(C.c_uint8 * (32 * N))() for _ in range(nthr)]

        def worker(w):
            for k, i0 in jobs[w::nthr]:
                base = ring_auto["out"][k].data_ptr() + i0 * g.slice_len
                T.lib.te_hash_leaves(C.cast(base, C.POINTER(C.c_uint8)), g.slice_len, min(lanes, N - i0), lanes, outs[w])
        ths = [threading.Thread(target=worker, args=(w,)) for w in range(nthr)]
        t = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        pool_rate = round(R * N * g.slice_len / (time.perf_counter() - t) / 1e9, 2)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_baseline_stream(args, ring_auto, CB, R, first)
    if rank == 0:
        print(json.dumps({
            "metric": "copy-inclusive stream write GiB/s (64 MiB chunks, encode_with_proofs per chunk, <= 4 in flight), "
                      "1 MI355X",
            "value": legs["auto_pinned"]["GiBps"], "unit": "GiB/s", "n_gpus": world, "steps": nch, "warmup": min(nch, R),
            "ms_per_step": round(el_auto / nch * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (SplitMix64 per chunk), host memory in and out (copy-inclusive)",
            "config": {"workload": f"stream of {nch} x {CB} B chunks per GPU, one encode_with_proofs window per chunk, "
                                   f"{depth} in flight (te_stream_writer)", "chunk_bytes": CB,
                       "slice_len": g.slice_len, "in_flight": depth, "profile": "clay(20,7,16)",
                       "host_hash_threads": batch.host_hash_threads(),
                       "host_hash_GBps_per_thread": round(T.lib.te_host_hash_rate() / 1e9, 3),
                       "host_hash_lanes": T.lib.te_host_hash_lanes(),
                       "host_hash_GBps_one_thread_at_lanes_1_to_4": lane_rate,
                       "host_hash_GBps_all_threads": pool_rate,
                       "host_sha_extensions": bool(T.lib.te_host_sha_extensions()),
                       "parallelism": f"chunks partitioned over {world} GPU(s)"},
            "legs": legs, "roofline": None, "cpu_baseline": cpu, "gpu": gpu_env(torch, dev),
            "outputs_verified": bool(ok)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def stream_sdk_short(args, torch, dist, world, rank, dev, T, batch) -> dict:
    """The SDK's stream-write shape as a short leg of the default encode line: a
    stream of `--sdk-chunks` x 64 MiB chunks (MAX_TRACK_SIZE, sdk/src/stream/manifest.rs:22), one
    encode_with_proofs window per chunk through te_stream_writer, at most 4 in flight
    (MAX_ENCODE_WORKERS, sdk/src/stream/write.rs:54-57, 332-362), pinned host buffers in a ring of
    8 slots, the library's hashing choice (host cores for these 9.7 MB slices).  Copy-inclusive:
    chunk bytes in host memory, slices + leaf hashes + roots + proofs back in host memory.  The last
    chunk is checked against a device-resident encode and hashlib; the CPU figure is the oracle's
    encode + hashlib of 4 chunks on 4 threads (the SDK's own worker count)."""
    import collections
    import hashlib
    CB, nch, depth, H = 64 * MiB, args.sdk_chunks, 4, T.SLICE_TREE_HEIGHT
    s = T.Slicer.clay_default()
    g = s.geometry(CB)
    per = N * g.slice_len
    R = 2 * depth
    first, _ = rank_objects(rank, nch)
    d_src = torch.empty(R * CB, dtype=torch.uint8, device=dev)
    splitmix_fill(torch, d_src, first, R, CB)
    pin = lambda n: torch.empty(n, dtype=torch.uint8).pin_memory()
    r = {"in": [pin(CB) for _ in range(R)], "out": [pin(per) for _ in range(R)],
         "leaf": [pin(N * 32) for _ in range(R)], "root": [pin(32) for _ in range(R)],
         "proof": [pin(N * H * 32) for _ in range(R)]}
    for k in range(R):
        r["in"][k].copy_(d_src[k * CB:(k + 1) * CB])
    descs = [batch.encode_descs([(0, CB, 0, first + c)]) for c in range(nch)]
    sw = batch.StreamWriter([s], height=H, hashing="auto")
    lat = []

    def run(chunks):
        inflight, t_sub = collections.deque(), {}
        del lat[:]
        for c in range(chunks):
            k = c % R
            if len(inflight) >= depth:
                t = inflight.popleft()
                sw.wait(t)
                lat.append(time.perf_counter() - t_sub.pop(t))
            t_sub_c = time.perf_counter()
            t = sw.submit(r["in"][k], descs[c], r["out"][k], r["leaf"][k], r["root"][k], r["proof"][k])
            t_sub[t] = t_sub_c
            inflight.append(t)
        while inflight:
            t = inflight.popleft()
            sw.wait(t)
            lat.append(time.perf_counter() - t_sub.pop(t))

    run(min(nch, R))  # warm-up: buffers, hashing pool
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run(nch)
    el = max_over_ranks(torch, dist, world, time.perf_counter() - t0, dev)
    sw.close()
    k = (nch - 1) % R
    d_out = torch.empty(per, dtype=torch.uint8, device=dev)
    batch.encode_batch(s, d_src[k * CB:(k + 1) * CB], [(0, CB, 0, first + nch - 1)], d_out)
    torch.cuda.synchronize()
    ok = bool(torch.equal(r["out"][k], d_out.cpu()))
    sl = r["out"][k].numpy()
    lv = r["leaf"][k].numpy().tobytes()
    for j in range(N):
        h = hashlib.sha256(b"LEAF")
        h.update(memoryview(sl[j * g.slice_len:(j + 1) * g.slice_len]))
        ok = ok and lv[j * 32:(j + 1) * 32] == h.digest()
    ls = sorted(lat)
    out = {"value": round(nch * world * CB / el / 2**30, 3), "unit": "GiB/s", "chunks_per_gpu": nch,
           "chunk_bytes": CB, "in_flight": depth, "pinned": True, "hashing": "auto (host cores for 64 MiB chunks)",
           "ms_per_chunk": round(el / nch * 1e3, 2),
           "chunk_latency_ms_p50_p90": [round(ls[len(ls) // 2] * 1e3, 2), round(ls[(9 * len(ls)) // 10] * 1e3, 2)],
           "host_hash_threads": batch.host_hash_threads(), "outputs_verified": ok, "cpu_baseline": None}
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        from concurrent.futures import ThreadPoolExecutor
        from oracle import oracle as O
        from oracle import merkle_oracle as MO
        clay = O.OracleClay(20, 7, 16)

        def one(kk):
            slc = O.slicer_encode_np(clay, r["in"][kk].numpy(), chunk_index=first + kk)
            leaves = [hashlib.sha256(b"LEAF" + slc[j].tobytes()).digest() for j in range(N)]
            return MO.root_from_leaf_hashes(leaves, H)
        t = time.perf_counter()
        with ThreadPoolExecutor(4) as ex:
            list(ex.map(one, range(4)))
        out["cpu_baseline"] = {"value": round(4 * CB / (time.perf_counter() - t) / 2**30, 3), "unit": "GiB/s",
                               "cores": 4, "kind": "port",
                               "sample": "4 x 64 MiB chunks on 4 threads (the SDK's MAX_ENCODE_WORKERS): oracle "
                                         "Slicer::encode + hashlib SHA-256 leaves + merkle root"}
    del d_src, r
    return out


def percall_bench(args, torch, dist, world, rank, dev):
    """--mode percall: the unchanged callers' shape.  lib/slicer's callers use one
    object per call with pageable Vec<u8>s: Slicer::encode per track (sdk/src/track/write.rs:273-308,
    objects <= 64 MiB), Slicer::repair per lost slice (network/node/src/features/spool/repair.rs:
    312-339), Slicer::decode per read.  Times te_slicer_encode / te_slicer_decode (7 slices, the
    worst case 13..19) / te_slicer_repair (lost 0, every other slice a helper) per call at 4 MiB and
    64 MiB, with pageable buffers and with te_host_alloc'd ones, beside the oracle on one thread
    (cpu_baseline; the reference itself is single-threaded per call).  Each output is checked."""
    import ctypes as C
    import numpy as np
    import tape_amd as T
    from tape_amd import batch
    from tape_amd._lib import lib
    s = T.Slicer.clay_default()
    cfg, hdl = s._cfg(), s.coder.handle
    ptr = lambda a: C.c_void_p(a.ctypes.data)
    res, ok, cpu = {}, True, {}
    for L in (4 * MiB, 64 * MiB):
        g = s.geometry(L)
        sl, per = g.slice_len, N * g.slice_len
        d = torch.empty(L, dtype=torch.uint8, device=dev)
        splitmix_fill(torch, d, 0, 1, L)
        src = d.cpu().numpy()
        avail = list(range(1, N))
        plan = s.repair_plan_from_params(0, avail, L, g.stripe_size)
        reps = 20 if L <= 4 * MiB else 5
        for kind in ("pageable", "pinned"):
            alloc = (lambda n: np.empty(n, np.uint8)) if kind == "pageable" else batch.host_empty
            data, out, dec, rep = alloc(L), alloc(per), alloc(L), alloc(sl)
            data[:] = src

            def enc():
                assert lib.te_slicer_encode(hdl, C.byref(cfg), ptr(data), L, ptr(out), per) == 0
            enc()
            ptrs = (C.c_void_p * N)()
            for i in range(13, 20):
                ptrs[i] = out.ctypes.data + i * sl
            got = C.c_size_t()

            def dcd():
                assert lib.te_slicer_decode(hdl, C.byref(cfg), ptrs, sl, ptr(dec), L, C.byref(got)) == 0
            blobs = [T.extract_repair_data(out[h * sl:(h + 1) * sl].tobytes(), plan, h) for h in avail]
            hbuf = alloc(sum(len(b) for b in blobs))
            hp, hl = (C.c_void_p * N)(), (C.c_size_t * N)()
            at = 0
            for h, b in zip(avail, blobs):
                hbuf[at:at + len(b)] = np.frombuffer(b, np.uint8)
                hp[h], hl[h] = hbuf.ctypes.data + at, len(b)
                at += len(b)
            meta = (C.c_uint8 * 48).from_buffer_copy(out[sl - 48:sl].tobytes())

            def rpr():
                assert lib.te_slicer_repair(hdl, plan.handle, hp, hl, meta, ptr(rep), sl) == 0
            row = {}
            for name, fn in (("encode", enc), ("decode", dcd), ("repair", rpr)):
                fn()
                t = time.perf_counter()
                for _ in range(reps):
                    fn()
                ms = (time.perf_counter() - t) / reps * 1e3
                # the calls' device time alone (HIP events around each call's kernels), in a
                # second pass so the events do not touch the timed one
                batch.kernel_time_ms()
                batch.kernel_timing(True)
                for _ in range(reps):
                    fn()
                batch.kernel_timing(False)
                kms, kn = batch.kernel_time_ms()
                row[name] = {"ms_per_call": round(ms, 3), "object_GiBps": round(L / (ms / 1e3) / 2**30, 3),
                             "kernel_ms_per_call": round(kms / max(1, reps), 3)}
            ok = ok and np.array_equal(dec, src) and np.array_equal(rep, out[:sl])
            res[f"{L >> 20}MiB_{kind}"] = row
        if rank == 0 and args.cpu_sample > 0:
            cpu[f"{L >> 20}MiB"] = cpu_baseline_percall(src, out, sl, L, g.stripe_size)
            ok = ok and cpu[f"{L >> 20}MiB"].pop("encode_equal")
    if rank == 0:
        print(json.dumps({
            "metric": "per-call Slicer::encode / decode / repair ms, one object per call, host buffers, 1 MI355X",
            "value": res["4MiB_pageable"]["encode"]["ms_per_call"], "unit": "ms", "n_gpus": world, "steps": None,
            "warmup": 1, "ms_per_step": res["4MiB_pageable"]["encode"]["ms_per_call"], "higher_is_better": False,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (SplitMix64), host memory",
            "config": {"workload": "te_slicer_encode / te_slicer_decode (slices 13..19) / te_slicer_repair (lost 0, "
                                   "19 helpers), one object per call, 4 MiB and 64 MiB", "profile": "clay(20,7,16)"},
            "calls": res, "roofline": None, "cpu_baseline": cpu, "outputs_verified": bool(ok)}), flush=True)


def cpu_baseline_percall(src, out, sl, L, stripe):
    """The oracle (C restatement of lib/slicer) per call on one thread: encode, decode from the same
    7 slices, repair of slice 0 from the other 19 (kind "port")."""
    from oracle import oracle as O
    clay = O.OracleClay(20, 7, 16)
    t = time.perf_counter()
    exp = O.slicer_encode_np(clay, src)
    te = time.perf_counter() - t
    slices = {i: out[i * sl:(i + 1) * sl].tobytes() for i in range(13, 20)}
    t = time.perf_counter()
    O.slicer_decode(clay, slices)
    td = time.perf_counter() - t
    cs, stripes = O.repair_plan(clay, 0, list(range(1, N)), L, stripe)
    helpers = {h: O.extract_repair_data(out[h * sl:(h + 1) * sl].tobytes(), cs, clay.alpha, stripes, h)
               for h in range(1, N)}
    t = time.perf_counter()
    O.slicer_repair(clay, cs, stripes, helpers, out[sl - 48:sl].tobytes())
    tr = time.perf_counter() - t
    return {"encode_ms": round(te * 1e3, 2), "decode_ms": round(td * 1e3, 2), "repair_ms": round(tr * 1e3, 2),
            "cores": 1, "kind": "port", "encode_equal": bool((exp.reshape(-1) == out).all())}


def cpu_baseline_stream(args, r, CB, R, first=0):
    """The reference's stream encode on host cores: per chunk the oracle's Slicer::encode (C
    restatement, AVX2 region multiply) + hashlib SHA-256 leaves + merkle root and proofs (the
    oracle's), one chunk per thread: on 16 threads (the GPU's host share) and on MAX_ENCODE_WORKERS
    = 4 threads, the SDK's own concurrency (write.rs:54-57).  Sample: R chunks per thread count."""
    from concurrent.futures import ThreadPoolExecutor
    import hashlib
    from oracle import oracle as O
    from oracle import merkle_oracle as MO
    clay = O.OracleClay(20, 7, 16)
    nch = args.stream_chunks
    # the chunk each ring slot held last (its metadata suffix names that chunk's index)
    chunk_of = [first + k + R * ((nch - 1 - k) // R) for k in range(R)]

    def one(k):
        sl = O.slicer_encode_np(clay, r["in"][k].numpy(), chunk_index=chunk_of[k])
        leaves = []
        for j in range(N):
            h = hashlib.sha256(b"LEAF")
            h.update(memoryview(sl[j]))
            leaves.append(h.digest())
        root = MO.root_from_leaf_hashes(leaves, 5)
        _ = [MO.create_proof_from_leaf_hashes(leaves, i, 5) for i in range(N)]
        return root

    res = {}
    cores = len(os.sched_getaffinity(0))
    for thr in (min(16, cores), 4, 1):
        jobs = list(range(R)) * (2 if thr == 16 else 1) if thr > 1 else [0]
        t = time.perf_counter()
        with ThreadPoolExecutor(thr) as ex:
            roots = list(ex.map(one, jobs))
        res[thr] = len(jobs) * CB / (time.perf_counter() - t) / 2**30
    ok = roots[0] == r["root"][0].numpy().tobytes()
    return {"value": round(res[min(16, cores)], 3), "unit": "GiB/s", "cores": min(16, cores), "kind": "port",
            "sample": f"{R * 2} x 64 MiB chunks on {min(16, cores)} threads (one chunk per thread): oracle Slicer::encode "
                      "+ hashlib SHA-256 leaves + merkle root and proofs",
            "sdk_4_workers_GiBps": round(res[4], 3), "single_thread_GiBps": round(res[1], 3),
            "affinity_cores": cores, "root_matches_gpu": bool(ok)}


def cpu_baseline_mode(args, np, mode, d_out, per, slice_len, L, d_gpu, out_stride, masks=None, lost=None, down=None):
    """CPU baseline of the decode / repair / recover lines (the oracle, kind "port": the reference's
    Rust crate cannot run here): the same objects and the same survivor / lost / down choices as the
    GPU step, one object per thread on the GPU's host share (16 threads), then the same entry point
    on one thread over 16 objects; the oracle's outputs are byte-compared with the GPU's timed
    outputs of the sample.  Rate in GiB/s of objects, as `value`."""
    from oracle import oracle as O
    cores = len(os.sched_getaffinity(0))
    thr = args.cpu_threads or max(1, min(16, cores))
    m = min(args.cpu_sample, args.objects)
    host = d_out[:m * per].cpu().numpy()
    clay = O.OracleClay(20, 7, 16)
    out = np.zeros(m * out_stride, np.uint8)
    sel = lambda v, k: None if v is None else list(v)[:k]
    t = time.perf_counter()
    bad = O.slicer_many(clay, mode, host, per, slice_len, m, out, out_stride, thr, sel(masks, m), sel(lost, m),
                        sel(down, m))
    wall = time.perf_counter() - t
    match = bad == 0 and bool(np.array_equal(d_gpu[:m * out_stride].cpu().numpy(), out))
    m1 = min(m, 16)
    t = time.perf_counter()
    O.slicer_many(clay, mode, host, per, slice_len, m1, out, out_stride, 1, sel(masks, m1), sel(lost, m1), sel(down, m1))
    single = m1 * L / (time.perf_counter() - t) / 2**30
    what = {"decode": "Slicer::decode from the same 7 slices per object",
            "repair": "plan + helper sub-chunk gather + Slicer::repair of the same lost slice per object",
            "recover": "Slicer::decode from the same 7 slices + Slicer::encode, keep the lost slice (recover.rs:411-442)"}
    return {"value": round(m * L / wall / 2**30, 4), "unit": "GiB/s", "cores": thr, "kind": "port",
            "sample": f"{m} x 4 MiB objects (first {m} of the batch), {thr} threads, one object per thread: oracle "
                      f"{what[mode]} (oracle/clay_oracle.c oc_slicer_many)",
            "single_thread_GiBps": round(single, 4), "single_thread_objects": m1, "affinity_cores": cores,
            "gpu_matches_oracle_on_sample": match}


def cpu_baseline_commit(args, d_out, per, slice_len, L):
    """CPU commitment of a bounded sample (the oracle: hashlib SHA-256, as the SDK's
    solana-sha256-hasher would run it), one object per thread."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import merkle_oracle as O
    ncpu = len(os.sched_getaffinity(0))
    threads = args.cpu_threads or min(16, ncpu)
    k = min(args.cpu_sample, d_out.numel() // per)
    host = d_out[:k * per].cpu().numpy()
    objs = [[host[i * per + j * slice_len:i * per + (j + 1) * slice_len].tobytes() for j in range(N)] for i in range(k)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(O.commit_slices, objs))
    dt = time.perf_counter() - t0
    return {"value": round(k * L / dt / 2**30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{k} x 4 MiB objects' 20 slices, {threads} threads, one object per thread (hashlib SHA-256)"}


def copy_share(args, world: int) -> int:
    """Objects per rank in the copy-inclusive legs: the whole share on one GPU (config 5's
    per-GPU share when --objects 2048); 256 per rank at N > 1, where every rank's pinned in/out
    buffers (18.5 MB per object) share the node's host memory and PCIe."""
    if args.copy_objects >= 0:
        return min(args.copy_objects, args.objects)
    return args.objects if world == 1 else min(args.objects, 256)


def copy_inclusive(args, torch, dist, world, slicer, batch, d_in, d_out, per, L, dev):
    """Copy-inclusive encode rate: pinned host object bytes in, pinned host
    slices out, through te_encode_batch_host (3-slot H2D / kernel / D2H pipeline).  Reported
    beside `value`, never as it.  Every rank runs it at once (max over ranks), so at N>1 it
    includes the host-memory / PCIe contention of the node."""
    m = copy_share(args, world)
    h_in = torch.empty(m * L, dtype=torch.uint8).pin_memory()
    h_in.copy_(d_in[:m * L])
    h_out = torch.empty(m * per, dtype=torch.uint8).pin_memory()
    objs = batch.encode_descs([(i * L, L, i * per, 0) for i in range(m)])
    batch.encode_batch_host(slicer, h_in, objs, h_out)  # warm-up (pipeline buffers)
    if world > 1:
        dist.barrier()
    t = time.perf_counter()
    for _ in range(args.copy_steps):
        batch.encode_batch_host(slicer, h_in, objs, h_out)
    el = time.perf_counter() - t
    el = max_over_ranks(torch, dist, world, el, dev)
    # same bytes as the device-resident run: first and last object
    ok = bool(torch.equal(h_out[:per], d_out[:per].cpu()) and
              torch.equal(h_out[(m - 1) * per:m * per], d_out[(m - 1) * per:m * per].cpu()))
    # the PCIe legs alone (whole share, pinned, one DMA each way): what bounds the pipeline
    torch.cuda.synchronize()
    t = time.perf_counter()
    d_in[:m * L].copy_(h_in, non_blocking=True)
    torch.cuda.synchronize()
    h2d = m * L / (time.perf_counter() - t) / 1e9
    t = time.perf_counter()
    h_out.copy_(d_out[:m * per], non_blocking=True)
    torch.cuda.synchronize()
    d2h = m * per / (time.perf_counter() - t) / 1e9
    return {"value": round(m * world * args.copy_steps * L / el / 2**30, 3), "unit": "GiB/s",
            "objects_per_gpu": m, "steps": args.copy_steps, "pinned": True,
            "ms_per_step": round(el / args.copy_steps * 1e3, 3),
            "h2d_bytes_per_object": L, "d2h_bytes_per_object": per,
            "h2d_GBps": round(h2d, 2), "d2h_GBps": round(d2h, 2),
            # PCIe ceilings: both directions at once (full duplex) / one after the other
            "pcie_duplex_bound_GiBps": round(min(h2d * 1e9 / L, d2h * 1e9 / per) * L / 2**30, 3),
            "pcie_serial_bound_GiBps": round(m * L / (m * L / (h2d * 1e9) + m * per / (d2h * 1e9)) / 2**30, 3),
            "matches_device_resident": ok}


def copy_inclusive_commit(args, torch, dist, world, slicer, batch, d_in, d_out, per, L, dev):
    """Copy-inclusive encode + commitments: BlobEncoder::encode_with_proofs per object
    (sdk/src/codec/encoder.rs:220-260) as the stream writer runs it (sdk/src/stream/write.rs:
    332-362), through te_encode_commit_batch_host: pinned object bytes in; slices, leaf hashes,
    roots and proofs out.  Per group size (window_bytes: the slices a leaf launch hashes at once,
    whose time is one slice's SHA-256 whatever the group size)."""
    m = copy_share(args, world)
    N, H = 20, 5
    h_in = torch.empty(m * L, dtype=torch.uint8).pin_memory()
    h_in.copy_(d_in[:m * L])
    h_out = torch.empty(m * per, dtype=torch.uint8).pin_memory()
    leaf = torch.empty(m * N * 32, dtype=torch.uint8).pin_memory()
    root = torch.empty(m * 32, dtype=torch.uint8).pin_memory()
    proof = torch.empty(m * N * H * 32, dtype=torch.uint8).pin_memory()
    objs = batch.encode_descs([(i * L, L, i * per, 0) for i in range(m)])
    res = {}
    for wgib in (2, 4, 8):
        wb = wgib << 30
        batch.encode_commit_batch_host(slicer, h_in, objs, h_out, leaf, root, proof, window_bytes=wb)  # warm-up
        if world > 1:
            dist.barrier()
        t = time.perf_counter()
        for _ in range(args.copy_steps):
            batch.encode_commit_batch_host(slicer, h_in, objs, h_out, leaf, root, proof, window_bytes=wb)
        el = max_over_ranks(torch, dist, world, time.perf_counter() - t, dev)
        res[f"window_{wgib}GiB_GiBps"] = round(m * world * args.copy_steps * L / el / 2**30, 3)
    # the first object's slices and commitments against the device-resident encode + hashlib
    import hashlib
    ok = bool(torch.equal(h_out[:per], d_out[:per].cpu()))
    sl_len = per // N
    for i in range(N):
        sl = h_out[i * sl_len:(i + 1) * sl_len].numpy().tobytes()
        ok = ok and leaf[i * 32:(i + 1) * 32].numpy().tobytes() == hashlib.sha256(b"LEAF" + sl).digest()
    best = max(res.values())
    # te_stream_writer: the same work as per-window submissions, the stream writer's
    # shape (sdk/src/stream/write.rs:332-362): windows of `wobj` objects, at most 4 in flight (the
    # SDK's FuturesOrdered depth), each waited for in order before the 5th is submitted
    stream = {}
    # hashing groups of 8 GiB (objects + slices): a leaf launch costs one slice's SHA-256 (~29 ms)
    # whatever the group size, so a group must hold >= ~13 GiB/s x 29 ms of objects (4 GiB groups
    # closed at half hold ~116 objects and ran 7.3-12 GiB/s; 8 GiB ones 11.3-13.0)
    sw = batch.StreamWriter([slicer], height=H, group_bytes=8 << 30)

    def run_stream(wobj):
        wins = [(a, min(m, a + wobj)) for a in range(0, m, wobj)]
        t = 0
        for a, b in wins:
            objs_w = batch.encode_descs([(i * L, L, i * per, 0) for i in range(a, b)])
            t = sw.submit(h_in, objs_w, h_out, leaf[a * N * 32:], root[a * 32:], proof[a * N * H * 32:])
            if t > 4:
                sw.wait(t - 4)
        sw.wait(t)

    # the library's per-window choice of who hashes (auto), and each side forced
    for hashing in ("auto", "device", "host"):
        sw.set_hashing(hashing)
        for wobj in (64, 128, 256):
            if wobj > m:
                continue
            run_stream(wobj)  # warm-up (buffers)
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.copy_steps):
                run_stream(wobj)
            el = max_over_ranks(torch, dist, world, time.perf_counter() - t0, dev)
            key = f"window_{wobj}_objects_GiBps" + ("" if hashing == "auto" else f"_{hashing}_hashing")
            stream[key] = round(m * world * args.copy_steps * L / el / 2**30, 3)
    sw.close()
    ok2 = bool(torch.equal(h_out[:per], d_out[:per].cpu()))
    return {"value": best, "unit": "GiB/s", "objects_per_gpu": m, "steps": args.copy_steps, "pinned": True,
            "tree_height": H, "proofs": True, "by_window": res, "matches_device_resident": ok and ok2,
            "stream_writer": {"in_flight": 4, "group_bytes": 8 << 30, **stream}}


def cpu_baseline(args, np, torch, d_in, d_out, per, L):
    """Oracle (C restatement of lib/slicer's Slicer::encode) on the host cores, bounded sample of
    the same workload; its outputs double as a bit-exact check of the GPU outputs."""
    from oracle import oracle as O
    try:
        cores = len(os.sched_getaffinity(0))
    except Exception:
        cores = os.cpu_count() or 1
    thr = args.cpu_threads or max(1, min(16, cores))  # the box's CPU share per GPU is 16 cores
    m = min(args.cpu_sample, args.objects)
    host_in = d_in[:m * L].cpu().numpy()
    clay = O.OracleClay(20, 7, 16)
    out = np.zeros(m * per, np.uint8)
    t = time.perf_counter()
    O.encode_many(clay, host_in, L, m, out, per, thr)
    wall = time.perf_counter() - t
    gpu = d_out[:m * per].cpu().numpy()
    match = bool(np.array_equal(gpu, out))
    # the same code path on one thread (the single-thread figure came from
    # another entry point), over >= 8 objects
    m1 = min(m, 16)
    t = time.perf_counter()
    O.encode_many(clay, host_in, L, m1, out, per, 1)
    single = m1 * L / (time.perf_counter() - t) / 2**30
    # and on every core this process may use (the whole host, not the GPU's 16-core share)
    all_cores = None
    if cores > thr:
        t = time.perf_counter()
        O.encode_many(clay, host_in, L, m, out, per, cores)
        all_cores = round(m * L / (time.perf_counter() - t) / 2**30, 4)
    return {"value": round(m * L / wall / 2**30, 4), "unit": "GiB/s", "cores": thr, "kind": "port",
            "sample": f"{m} x 4 MiB objects (first {m} of the batch), {thr} threads, one object per thread; "
                      "oracle/clay_oracle.c: the Clay layering restated in C over an AVX2 nibble-shuffle GF(2^8) "
                      "region multiply -- the method of reed-solomon-erasure's simd-accel C kernel, which the "
                      "reference's Cargo.lock enables (cc + libc resolved)",
            "single_thread_GiBps": round(single, 4), "single_thread_objects": m1,
            "all_affinity_cores_GiBps": all_cores, "affinity_cores": cores,
            "gpu_matches_oracle_on_sample": match}


if __name__ == "__main__":
    main()
