"""N>1 path of bench.py on CPU: world_size-2 gloo process group.

The path shards by object: each rank owns a contiguous global object range, generates those
objects' SplitMix64 bytes itself and encodes them with no data-path collective; the process group
carries only the barrier and the max-over-ranks time.  Here the per-rank encode is the oracle
(CPU test only); the GPU path under the same partition is what bench.py runs with torchrun.
"""
import hashlib
import os
import socket
import sys

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

OBJ = 30_011   # odd size: ragged last stripe
NOBJ = 3       # objects per rank


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import bench
    from oracle import oracle as O
    w, r, _ = bench.dist_setup(torch, dist, "gloo")
    assert (w, r) == (world, rank)
    first, end = bench.rank_objects(r, NOBJ)
    buf = torch.empty(NOBJ * OBJ, dtype=torch.uint8)
    bench.splitmix_fill(torch, buf, first, NOBJ, OBJ)
    clay = O.OracleClay(20, 7, 16)
    hashes = []
    for i in range(NOBJ):
        sl = O.slicer_encode(clay, buf[i * OBJ:(i + 1) * OBJ].numpy().tobytes())
        hashes.append(hashlib.sha256(b"".join(sl)).hexdigest())
    t = bench.max_over_ranks(torch, dist, w, 1.0 + r, torch.device("cpu"))
    got = [None] * w
    dist.all_gather_object(got, (first, end, hashes, t, buf.numpy().tobytes()))
    dist.destroy_process_group()
    if r == 0:
        q.put(got)


def test_two_rank_partition_gloo():
    from oracle import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ranges = sorted((g[0], g[1]) for g in got)
    assert ranges == [(0, NOBJ), (NOBJ, 2 * NOBJ)]           # contiguous, disjoint, complete
    assert all(g[3] == float(world) for g in got)             # max over ranks
    clay = O.OracleClay(20, 7, 16)
    for first, end, hashes, _, raw in got:
        for i, gid in enumerate(range(first, end)):
            data = O.splitmix64_bytes(0x7A9E5EED ^ gid, OBJ).tobytes()   # SURVEY 8d stream
            assert raw[i * OBJ:(i + 1) * OBJ] == data
            assert hashlib.sha256(b"".join(O.slicer_encode(clay, data))).hexdigest() == hashes[i]
