"""In-process A/B of the short shard's fixed costs (config 4's 1/8 shard, the
driver's 20-step command): ONE engine, the bench's own timed region
(bench.timed_leg: warmup, barrier + sync, the launches, the counter
all-reduce inside the clock, the closing sync) repeated --reps times per
variant, the variants interleaved and each repetition from step 0
(raft_engine_reset), so box-to-box and run-to-run drift cancel.  Variants:
where the timestamps are (--kernel-timing region: on the timed launches and
around the all-reduce, inside the clock; replay: none inside the clock, the
times from a replay after it) x the closing wait (--sync block / spin).
With --collective the one-rank RCCL all-reduce runs inside the clock (the
bench's RAFT_BENCH_FORCE_COLLECTIVE).
Prints one JSON line: the median wall / stream-event / kernel times per variant.

    python scripts/shard_ab.py --groups 125000 --reps 15 --collective
"""
import argparse
import importlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

abi = bench.abi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=125_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--collective", action="store_true")
    ap.add_argument("--variants", default="region_block,replay_block,replay_spin")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    eng_mod = importlib.import_module("raft-kotlin_amd.engine")
    dev = torch.device("cuda", 0)
    comm = None
    if a.collective:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=dev, init_method=f"tcp://127.0.0.1:{bench.free_port()}",
                                rank=0, world_size=1)
        comm = eng_mod.RaftComm(eng_mod.RaftComm.unique_id(), 1, 0, 0)
    kw = dict(abi.CONFIGS[3], G=a.groups)
    L = bench.launch_length(a.steps, abi.bench_steps_per_launch(5, 0, 0, abi.step_net_of(kw)))
    eng = eng_mod.RaftEngine(abi.make_params(log_cap=64 + a.steps + a.warmup, steps_per_launch=L, **kw))
    out = {v: [] for v in a.variants.split(",")}
    for rep in range(a.reps):
        for v in out:
            kt, sync = v.split("_")
            args = bench.parse_args(["--steps", str(a.steps), "--warmup", str(a.warmup), "--sync", sync,
                                     "--kernel-timing", kt])
            eng.reset()
            leg = bench.timed_leg(eng, args, L, a.collective, dev, 1, comm)
            out[v].append({"wall_ms": leg["wall"] * 1e3, "ev_ms": leg["ev_ms"], "kern_ms": leg["kern_avg_ms"],
                           "allreduce_ms": leg["allreduce_ms"]})
    def med(rows, k):
        xs = [x[k] for x in rows if x[k] is not None]
        return statistics.median(xs) if xs else None
    res = {v: {k: med(rows, k) for k in ("wall_ms", "ev_ms", "kern_ms", "allreduce_ms")} |
           {"wall_ms_all": [round(x["wall_ms"], 4) for x in rows]} for v, rows in out.items()}
    print(json.dumps({"groups": a.groups, "steps": a.steps, "reps": a.reps, "collective": a.collective,
                      "variants": res}))
    eng.close()
    if comm is not None:
        comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
