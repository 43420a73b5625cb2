"""Multi-process path on CPU (gloo, world_size 2): each rank owns a contiguous
range of global group ids (bench.py's weak/strong sharding), steps it with the
oracle, and the per-step counters and digests all-reduce to exactly the
single-process result (config 4's contract: partitioning changes nothing)."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from helpers import abi

KW = dict(abi.CONFIGS[3], G=600, churn_ppm=20_000)
STEPS = 150


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G = KW["G"]
    n = G // world + (1 if rank < G % world else 0)
    g0 = rank * (G // world) + min(rank, G % world)
    o = O.Oracle(abi.make_params(log_cap=96, **dict(KW, G=n, g0=g0)))
    c = torch.from_numpy(o.step(STEPS)[:, : abi.NUM_COUNTERS].copy())
    dist.all_reduce(c)                                   # the batched counter all-reduce
    d = torch.tensor([o.digest()], dtype=torch.uint64).view(torch.int64)
    dist.all_reduce(d)                                   # int64 sum wraps like the u64 digest sum
    if rank == 0:
        q.put((c.numpy(), int(d.view(torch.uint64).item()) if hasattr(torch, "uint64") else int(d.item())))
    dist.destroy_process_group()


def test_two_rank_sharding_equals_single():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    counters, digest = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = O.Oracle(abi.make_params(log_cap=96, **KW))
    cf = full.step(STEPS)[:, : abi.NUM_COUNTERS]
    np.testing.assert_array_equal(counters, cf)
    assert digest % (1 << 64) == full.digest()


def rehearsal_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    # uneven shards whose own counts differ (600 vs 601 repeats of 20 steps)
    own = bench.rehearsal_count(50.0, 125_001 - 2 * rank, 20)
    q.put((rank, own, bench.rehearsal_count(50.0, 125_001 - 2 * rank, 20, coll=True)))
    dist.destroy_process_group()


def test_rehearsal_count_agreed_over_ranks():
    """bench.py's rehearsal repeats a launch sequence that holds the RCCL
    counter all-reduce, so every rank must run the same number of repeats:
    ranks whose own counts differ agree on the MAX."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=rehearsal_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][1] != got[1][1]                       # the ranks' own counts differ
    assert got[0][2] == got[1][2] == max(got[0][1], got[1][1])
