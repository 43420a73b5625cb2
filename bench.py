#!/usr/bin/env python3
"""bench.py — Raft group-steps/sec of the MI355X batched Raft engine.

Workload (BASELINE.json configs[2], "config 3"): 10^6 five-replica groups per
GPU, seeded 5% message drop, leader-isolation churn (1e-3 per group-step, 15
steps), one client command per group-step with probability 1/4.  A "step" is
one lockstep heartbeat period of every group: timers, the
RequestVote phase, the AppendEntries/commit phase and client commands, with
all state resident in HBM before the timed region starts.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: one process per GPU, each owns its own contiguous range of global
group ids (weak scaling; no data-path collective).  The per-step global
counters (commits, leaders, safety flags, ...) are all-reduced over RCCL in
batches on a side stream.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

abi = importlib.import_module("raft-kotlin_amd.abi")

METRIC = "Raft group-steps/sec (whole node) at 1M×5-replica groups; % of HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# per replica: 10 canonical fields + the log-tail cache (t1, t2, c1) + the
# primary-session column (nextIndex, matchIndex); per group: 3 harness words
REPLICA_BYTES = 4 * (abi.NUM_FIELDS + 3) + 8
GROUP_BYTES = 4 * 3


def algorithmic_bytes(c: np.ndarray, G: int, R: int) -> float:
    """SURVEY.md §8(d)'s algorithmic HBM bytes of the counted group-steps (the
    contract's per-unit figure x the units processed):

        B = 2·R·37 + 2·8R·H + 4·P_L + 8·E_L + 4·P_F + 8·E_W + 4·V + 8·C  per group-step

    37 B of canonical scalar state per replica read and written every step,
    the leader sessions that ticked (H, 2R int32 each, read and written),
    prevLogTerm reads at the leader (P_L) and follower (P_F), entries read at
    the leader (E_L) and written at the follower (E_W), last-log-term reads of
    the vote path (V) and client commands appended (C).  Every event count is
    the kernel's own counter, summed over the steps of `c`."""
    ix = abi.C_INDEX
    s = lambda n: float(c[:, ix[n]].sum())  # noqa: E731
    return (2.0 * R * 37 * G * c.shape[0] + 2 * 8 * R * s("sessions_ticked")
            + 4 * s("prev_reads_leader") + 8 * s("entry_reads_leader") + 4 * s("prev_reads_follower")
            + 8 * s("entry_writes") + 4 * s("vote_log_reads") + 8 * s("commands"))


def state_crossing_bytes(c: np.ndarray, G: int, R: int, launches: int) -> float:
    """The bytes a launch of THIS kernel must move, a lower
    bound: the group state (fields, tail cache, primary-session column, harness
    words) read and written once per launch, plus every log entry a handler or
    appendCommand stores.  A fused launch carries the state across its K steps
    in VGPRs, so this is far below the algorithmic bytes of its K steps."""
    ix = abi.C_INDEX
    state = 2.0 * G * (R * REPLICA_BYTES + GROUP_BYTES) * launches
    log = 8.0 * (c[:, ix["entry_writes"]].sum() + c[:, ix["commands"]].sum())
    return state + log


def load_traffic(workload: dict):
    """HBM traffic per launch measured by rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
    for this exact workload (scripts/traffic.sh -> profiles/traffic.json), or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            rows = json.load(f)
    except (OSError, ValueError):
        return None
    for row in rows:
        if all(row.get(k) == v for k, v in workload.items()):
            return row
    return None


def cpu_baseline(args, kw, log_cap, total_steps):
    """Oracle (scalar C restatement of the reference) on a bounded sample of
    the same workload, on this host's cores (rank 0, N=1 only).  The sample
    is a contiguous range of the same global groups, run for the same number
    of steps as the GPU (so logs grow exactly as they do there); its size is
    calibrated so that the timed part takes about --cpu-seconds."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    # calibration: a short run of a small sample
    probe = O.Oracle(abi.make_params(log_cap=log_cap, **dict(kw, G=args.cpu_groups)))
    t0 = time.perf_counter()
    probe.step(args.cpu_chunk, nthreads=threads, counters=False)
    rate = args.cpu_groups * args.cpu_chunk / max(1e-6, time.perf_counter() - t0)
    probe.close()

    def timed(G, nthreads):
        o = O.Oracle(abi.make_params(log_cap=log_cap, **dict(kw, G=G)))
        o.step(args.warmup, nthreads=nthreads, counters=False)
        t0 = time.perf_counter()
        done = 0
        while done < total_steps - args.warmup:
            k = min(args.cpu_chunk * 10, total_steps - args.warmup - done)
            o.step(k, nthreads=nthreads, counters=True)
            done += k
        dt = time.perf_counter() - t0
        o.close()
        return G * done / dt, dt

    G = int(min(kw["G"], max(threads * 64, rate * args.cpu_seconds / total_steps)))
    value, dt = timed(G, threads)
    # the single-thread rate on a smaller sample of the same groups
    G1 = int(min(kw["G"], max(64, rate / threads * args.cpu_seconds_1t / total_steps)))
    value1, dt1 = timed(G1, 1)
    return {"value": value, "unit": "group-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/raft_oracle.c (scalar C restatement of RaftServer.kt/Commons.kt), global groups "
                      f"0..{G - 1} of the same config for the same {total_steps} steps as the GPU "
                      f"({args.warmup} untimed), {dt:.1f} s, pthreads over groups",
            "single_thread": {"value": value1, "unit": "group-steps/s", "cores": 1,
                              "sample": f"global groups 0..{G1 - 1}, same steps, {dt1:.1f} s"},
            "host_cpus": os.cpu_count()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10_000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--groups", type=int, default=1_000_000, help="groups per GPU")
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 5])
    ap.add_argument("--mode", choices=["reference", "textbook"], default="reference",
                    help="protocol mode: the reference's handlers (parity) or the opt-in textbook rules")
    ap.add_argument("--steps-per-launch", type=int, default=512,
                    help="lockstep steps fused into one kernel launch (state stays in VGPRs)")
    ap.add_argument("--stream-steps", type=int, default=200,
                    help="steps of the streaming leg (1 step per launch: the HBM-bound formulation)")
    ap.add_argument("--log-cap", type=int, default=0)
    ap.add_argument("--reduce-every", type=int, default=512,
                    help="steps per counter all-reduce (and per step_async call: keep it a multiple of --steps-per-launch)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-groups", type=int, default=20_000, help="calibration sample for the CPU baseline")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-seconds-1t", type=float, default=5.0, help="target seconds of the single-thread CPU leg")
    ap.add_argument("--cpu-chunk", type=int, default=20)
    ap.add_argument("--warmup-cpu", type=int, default=40)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a one-GPU box (never set by the driver):
    # RAFT_BENCH_BACKEND=gloo with RAFT_BENCH_ONE_DEVICE=1 runs every rank on
    # cuda:0 with gloo collectives, which exercises the N > 1 path end to end
    backend = os.environ.get("RAFT_BENCH_BACKEND", "nccl")
    if os.environ.get("RAFT_BENCH_ONE_DEVICE") == "1":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    eng_mod = importlib.import_module("raft-kotlin_amd.engine")
    kw = dict(abi.CONFIGS[args.config])
    R = kw["R"]
    if args.scaling == "weak":
        G_local = args.groups
        g0 = rank * G_local
    else:
        G_local = args.groups // world + (1 if rank < args.groups % world else 0)
        g0 = rank * (args.groups // world) + min(rank, args.groups % world)
    total_steps = args.warmup + args.steps + args.stream_steps
    # physical slots a replica can fill: ~0.3 per step at config 3's command
    # rate, up to one per step where every leader takes a command each step
    log_cap = args.log_cap or int(64 + (1.0 if kw["cmd_ppm"] >= 1_000_000 else 0.3) * total_steps)
    spl = args.steps_per_launch
    mode = abi.MODE_TEXTBOOK if args.mode == "textbook" else abi.MODE_REFERENCE
    params = abi.make_params(log_cap=log_cap, steps_per_launch=spl, mode=mode, **dict(kw, G=G_local, g0=g0))
    eng = eng_mod.RaftEngine(params, device=local)
    stream = torch.cuda.ExternalStream(eng.stream, device=dev)
    counters = torch.zeros((args.steps, abi.COUNTER_STRIDE), dtype=torch.int64, device=dev)
    wcount = torch.zeros((max(1, args.warmup), abi.COUNTER_STRIDE), dtype=torch.int64, device=dev)

    # ---- warmup (untimed) ----
    if args.warmup:
        eng.step_async(args.warmup, wcount.data_ptr())
    eng.sync()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()

    # ---- timed region ----
    comm_stream = torch.cuda.Stream(device=dev)
    eng.set_kernel_timing(True)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    ev0.record(stream)
    done = 0
    while done < args.steps:
        k = min(args.reduce_every, args.steps - done)
        eng.step_async(k, counters[done].data_ptr())
        if world > 1:
            # the only collective: the batched per-step counter all-reduce,
            # off the critical path on a side stream (counters never feed back)
            ev = torch.cuda.Event()
            ev.record(stream)
            comm_stream.wait_event(ev)
            with torch.cuda.stream(comm_stream):
                dist.all_reduce(counters[done:done + k])
        done += k
    ev1.record(stream)
    eng.sync()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)
    kern_ms, launches = eng.kernel_time()
    eng.set_kernel_timing(False)

    elapsed = max(wall, ev_ms / 1e3)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    c_all = counters.cpu().numpy()[:, : abi.NUM_COUNTERS]     # already global if world > 1
    local_counts = None
    if world == 1:
        local_counts = c_all
    total_groups = G_local * world if args.scaling == "weak" else args.groups
    value = total_groups * args.steps / elapsed

    # roofline of the dominant kernel (step_kernel), from this rank's counters
    if world > 1:
        # the all-reduced counters are global; scale to this rank's share
        local_counts = c_all * (G_local / total_groups)
    kern_avg_ms = kern_ms / max(1, launches)
    kern_s = kern_ms / 1e3
    bytes_alg = algorithmic_bytes(local_counts, G_local, R)
    bytes_state = state_crossing_bytes(local_counts, G_local, R, launches)
    achieved = bytes_alg / kern_s / 1e9 if launches else 0.0
    achieved_state = bytes_state / kern_s / 1e9 if launches else 0.0
    overflow = int(c_all[:, abi.C_INDEX["log_overflow"]].sum())
    K = spl or 1
    tr = load_traffic({"config": args.config, "groups": G_local, "steps_per_launch": K})

    # ---- streaming leg (untimed for `value`): one step per launch, so every
    # launch streams the whole group state HBM -> VGPRs -> HBM.  Its roofline
    # is the HBM-bound formulation of the same step. ----
    stream = None
    if args.stream_steps > 0:
        eng.set_steps_per_launch(1)
        sc = torch.zeros((args.stream_steps, abi.COUNTER_STRIDE), dtype=torch.int64, device=dev)
        eng.set_kernel_timing(True)
        eng.step_async(args.stream_steps, sc.data_ptr())
        eng.sync()
        s_ms, s_n = eng.kernel_time()
        eng.set_kernel_timing(False)
        cs = sc.cpu().numpy()[:, : abi.NUM_COUNTERS]
        s_avg = s_ms / max(1, s_n)
        s_bytes = algorithmic_bytes(cs, G_local, R) / max(1, s_n)
        s_state = state_crossing_bytes(cs, G_local, R, s_n) / max(1, s_n)
        s_ach = s_bytes / (s_avg / 1e3) / 1e9
        s_tr = load_traffic({"config": args.config, "groups": G_local, "steps_per_launch": 1})
        stream = {"steps_per_launch": 1, "steps": args.stream_steps, "kernel_avg_ms": s_avg,
                  "alg_bytes_per_launch": s_bytes, "achieved": s_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": s_ach / HBM_PEAK_GBS, "traffic": s_tr["bytes_per_launch"] if s_tr else None,
                  "state_bytes_per_launch": s_state,
                  "achieved_state_crossing": s_state / (s_avg / 1e3) / 1e9,
                  "frac_state_crossing": s_state / (s_avg / 1e3) / 1e9 / HBM_PEAK_GBS,
                  "kernel_group_steps_per_s": G_local / (s_avg / 1e3)}

    # ---- safety flags (untimed): the run's counter-borne flags plus the
    # Log Matching check over committed prefixes ----
    mism = eng.check_log_matching()
    if world > 1:
        t = torch.tensor([mism], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        mism = int(t.item())
    safety = {
        "log_matching_mismatched_groups": mism,
        "commit_regressions": int(c_all[:, abi.C_INDEX["commit_regressions"]].sum()),
        "dual_leader_group_steps": int(c_all[:, abi.C_INDEX["dual_leader_groups"]].sum()),
        "log_overflow": overflow,
        "note": "observations of the reference's protocol (quirks Q4/Q9 do not preserve these "
                "properties); over the timed steps, Log Matching at the end of the run",
    }

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "group-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (seeded Philox harness: drops, churn, commands)",
        "config": {
            "workload": f"config{args.config}: {G_local} groups/GPU x {R} replicas"
                        + {3: ", 5% drop, leader-isolation churn 1e-3 x 15 steps, 1/4 command per group-step",
                           5: ", 2-way partitions 25 of every 50 steps, 1 command per step to every leader",
                           2: ", no faults, 1/4 command per group-step"}[args.config]
                        + (", textbook mode" if mode else ""),
            "groups_total": total_groups, "replicas": R, "log_cap": log_cap,
            "steps_per_launch": K, "parallelism": f"shard-by-group x{world}",
            "counter_allreduce_every": args.reduce_every if world > 1 else None,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": tr["bytes_per_launch"] if tr else None,
            "kernel": f"step_kernel<{R}> x{K} fused steps", "kernel_avg_ms": kern_avg_ms, "launches": launches,
            "alg_bytes_per_launch": bytes_alg / max(1, launches),
            "alg_bytes_per_group_step": bytes_alg / max(1, G_local * local_counts.shape[0]),
            "traffic_source": tr["source"] if tr else None,
            "state_bytes_per_launch": bytes_state / max(1, launches),
            "achieved_state_crossing": achieved_state,
            "frac_state_crossing": achieved_state / HBM_PEAK_GBS,
            "note": "achieved = SURVEY.md §8(d) algorithmic bytes per group-step (event counts from the "
                    "kernel's counters) x the group-steps of one launch / the launch's average duration. "
                    "A fused launch keeps every replica in VGPRs for its K steps, so the HBM bytes it really "
                    "moves (traffic, PMC) are far below the algorithmic bytes and the kernel is "
                    "VALU-issue bound; achieved_state_crossing prices only the state a launch must move. "
                    "roofline_streaming is the same step at one step per launch",
        },
        "roofline_streaming": stream,
        "valid": overflow == 0,
        "safety": safety,
        "counters_last_step": {n: int(v) for n, v in zip(abi.COUNTER_NAMES, c_all[-1])},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, dict(kw, mode=mode), log_cap, args.warmup + args.steps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
