"""bench.py's collective branch on one MI355X (marker `gpu`).

The driver runs config 4 (10^6 x 5 sharded over 2/4/8 GPUs) with one RCCL
communicator per node; a one-GPU box can still execute every line of that
branch at WORLD_SIZE 1 (RAFT_BENCH_FORCE_COLLECTIVE=1): the `nccl` (RCCL)
process group created with device_id, the all_reduce of the counter rows
inside the timed region (the default, --allreduce end: once, on the engine
stream after the last launch; inline: per chunk on a side stream, in series
with the launches; after: the diagnostic off the clock), and the MAX /
all-gather reductions of the elapsed and kernel times.  The
all-reduced rows must equal this rank's own rows and the CPU oracle's
counters for the same global groups and steps.  bench.main runs in this
process (no child process once the GPU is initialised).
"""
import importlib.util
import os

import numpy as np
import pytest

import oracle as O
from helpers import abi

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)


@pytest.mark.parametrize("backend,mode", [("nccl", None), ("nccl", "inline"), ("nccl", "after"), ("gloo", None)])
def test_forced_collective_at_one_rank(backend, mode, monkeypatch):
    monkeypatch.setenv("RAFT_BENCH_FORCE_COLLECTIVE", "1")
    monkeypatch.setenv("RAFT_BENCH_BACKEND", backend)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    G, warm, steps = 24_000, 40, 800          # two 400-step launches: two all-reduce chunks at --reduce-every 400
    res = {}
    argv = ["--groups", str(G), "--steps", str(steps), "--warmup", str(warm), "--stream-steps", "0",
            "--reduce-every", "400", "--no-cpu-baseline"] + (["--allreduce", mode] if mode else [])
    rc = bench.main(argv, result=res)
    assert rc == 0
    out = res["out"]
    col = out["config"]["collective"]
    assert (col["backend"], col["ranks"], col["forced_at_one_rank"]) == (backend, 1, True)
    # the default in-clock all-reduce over RCCL is the engine's own native call
    native = backend == "nccl" and mode is None
    assert col["counter_allreduce"].startswith("raft_engine_allreduce_counters") == native
    # the default is the in-clock mode: one all-reduce of the timed rows before the closing sync
    want = {None: "timed_region_once", "inline": 400, "after": "after_timed_region_diagnostic"}[mode]
    assert out["config"]["counter_allreduce_every"] == want
    if mode is None:
        ar = out["timing"]["allreduce_ms"]
        assert ar is not None and 0 < ar < out["timing"]["wall_ms"], "the all-reduce runs inside the clock"
    assert out["valid"] and out["value"] > 0
    # the kernel times come from an exact replay of the timed launches after the clock
    assert out["timing"]["kernel_timing"] == "replay" and out["timing"]["replay_counters_equal"] is True
    assert out["roofline"]["kernel_avg_ms"] > 0
    ca, cl = res["counters_all"], res["counters_local"]
    assert np.array_equal(ca, cl), "a one-rank all-reduce must return this rank's rows"
    kw = dict(abi.CONFIGS[3], G=G)
    o = O.Oracle(abi.make_params(log_cap=out["config"]["log_cap"], **kw))
    co = o.step(warm + steps, nthreads=min(16, os.cpu_count() or 1))[:, : abi.NUM_COUNTERS]
    assert np.array_equal(res["warmup_counters"], co[:warm])
    assert np.array_equal(ca, co[warm:]), "all-reduced counter rows differ from the oracle's"


def test_native_counter_allreduce_at_one_rank():
    """raft_engine_allreduce_counters on a one-rank communicator of the
    engine's own (raft_comm_*): out of place and in place it returns the rows
    it was given, ordered after the engine's step launches on its stream; zero
    rows is a no-op."""
    import torch
    eng_mod = importlib.import_module("raft-kotlin_amd.engine")
    e = eng_mod.RaftEngine(abi.make_params(**dict(abi.CONFIGS[3], G=2000)))
    comm = eng_mod.RaftComm(eng_mod.RaftComm.unique_id(), 1, 0, 0)
    try:
        dev = torch.device("cuda", 0)
        n = 30
        rows = torch.zeros((n, abi.COUNTER_STRIDE), dtype=torch.int64, device=dev)
        out = torch.full_like(rows, -7)
        torch.cuda.synchronize(dev)
        e.step_async(n, rows.data_ptr())
        e.allreduce_counters(comm, rows.data_ptr(), out.data_ptr(), n)
        e.sync()
        assert int(rows.abs().sum()) > 0
        assert torch.equal(out, rows), "out of place"
        keep = rows.clone()
        e.allreduce_counters(comm, rows.data_ptr(), rows.data_ptr(), n)
        e.allreduce_counters(comm, rows.data_ptr(), out.data_ptr(), 0)
        e.sync()
        assert torch.equal(rows, keep), "in place"
    finally:
        comm.close()
        e.close()
