#!/usr/bin/env python3
"""bench.py — Raft group-steps/sec of the MI355X batched Raft engine.

Workload (BASELINE.json configs[2], "config 3"): 10^6 five-replica groups,
seeded 5% message drop, leader-isolation churn (1e-3 per group-step, 15
steps), one client command per group-step with probability 1/4.  A "step" is
one lockstep heartbeat period of every group: timers, the
RequestVote phase, the AppendEntries/commit phase and client commands, with
all state resident in HBM before the timed region starts.  Before the W
warmup steps, an untimed rehearsal runs the timed launches on scratch counter
rows and resets the engine to step 0, repeated for >= --rehearse-ms (50 ms),
so a short timed region does not run on the GPU's idle clocks; the warmup and
the timed K steps then run from the same state as without it.  Nothing inside
the clock is instrumented: kernel and all-reduce times come from a replay of
the same launches after it (--kernel-timing replay).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: one process per GPU.  With --gpus N > 1 and no torch.distributed
environment, this script spawns the N rank processes itself (fresh
interpreters; the parent makes no HIP or torch.cuda call) and exits with their
status.  Groups never talk across GPUs, so the path shards with no data-path
exchange.  By default `value` is BASELINE.json configs[3] ("config 4"): the
same 10^6 groups split into contiguous global-id ranges over the N GPUs
(strong scaling, `value` = 10^6 x steps / the MAX of the ranks' times).  The
line then also carries `weak_scaling`, measured in the same job: every GPU its
own 10^6 groups, timed the same way, whose rank-0 counter rows must equal the
strong leg's all-reduced rows (the same global groups).  --scaling weak swaps
the two (the strong leg is then `config4_strong`).  The only collective is the
all-reduce of the per-step counter rows over RCCL: one all-reduce of all the
timed rows, enqueued on the engine stream after the last launch and inside the
timed region (SURVEY.md §8(e)'s batching: one collective per region; its own
time is `timing.allreduce_ms`).  --allreduce inline: one per --reduce-every
chunk, in series with the launches; --allreduce after: once the clock has
stopped (a diagnostic: the line then times the kernels without the collective).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

abi = importlib.import_module("raft-kotlin_amd.abi")

METRIC = "Raft group-steps/sec (whole node) at 1M×5-replica groups; % of HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# VALU issue peak: 1024 SIMDs (256 CUs x 4), a wave64 VALU instruction issues
# over 2 cycles on a 32-lane SIMD (MI355X_MICROARCH.md), 2.4 GHz max clock
SIMDS, CLOCK_HZ, VALU_CYCLES = 1024, 2.4e9, 2
VALU_PEAK_GIPS = SIMDS * CLOCK_HZ / VALU_CYCLES / 1e9
# per replica: 10 canonical fields + the log-tail cache (t1, t2, c1) + the
# primary-session column (nextIndex, matchIndex) in 4 int32 quads; per group: 3 harness words
REPLICA_BYTES, GROUP_BYTES = abi.REPLICA_STATE_BYTES, abi.GROUP_STATE_BYTES
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_rows.json")
# group-steps/s the rehearsal count assumes (above every measured rate: its
# repeats last at least --rehearse-ms)
REHEARSE_RATE = 3.0e10
SCHEDULES = {"auto": abi.SCHED_AUTO, "one": abi.SCHED_ONE_PER_WAVE, "balanced": abi.SCHED_BALANCED}


def NET_NAMES(net: int) -> list:
    """The network faults / harness a step kernel is built for (raft_step.h NET_*)."""
    return [n for b, n in ((abi.NET_DROP, "drops"), (abi.NET_PART, "partitions"), (abi.NET_ISO, "isolation_churn"),
                           (abi.NET_CMDLOW, "commands_to_lowest_leader_compiled_in")) if net & b]


def kernel_source_id() -> str:
    """Short hash of the step kernel's sources: a PMC row describes one kernel
    build, so bench.py attaches it only to a run of the same sources (the
    loaded library carries the same id, raft_build_kernel_source_id)."""
    return importlib.import_module("raft-kotlin_amd.build").kernel_source_id()


def library_source_id() -> str:
    """Short hash of everything the library is built from."""
    return importlib.import_module("raft-kotlin_amd.build").library_source_id()


def batch_source_id() -> str:
    """Short hash of the handler batches' sources: their PMC rows are keyed on
    it (their kernels are not the step kernel's)."""
    return importlib.import_module("raft-kotlin_amd.build").batch_source_id()


def shard(total: int, world: int, rank: int, scaling: str) -> tuple[int, int]:
    """(first global group id, groups) of `rank`.  strong: `total` groups split
    into contiguous ranges (the first total % world ranks take one more);
    weak: every rank owns its own `total` groups."""
    if scaling == "weak":
        return rank * total, total
    base, extra = divmod(total, world)
    return rank * base + min(rank, extra), base + (1 if rank < extra else 0)


def launch_length(steps: int, spl: int) -> int:
    """Steps per launch of the timed region: the largest divisor of `steps`
    that is <= spl, so every timed launch has the same length (its roofline
    and PMC row then describe every launch); spl itself when no divisor
    within a factor 4 of it exists."""
    for d in range(min(spl, steps), 0, -1):
        if steps % d == 0:
            return d if d * 4 >= min(spl, steps) else min(spl, steps)
    return max(1, min(spl, steps))


def launch_plan(n: int, k: int) -> list[int]:
    """Launch lengths of raft_engine_step_async(n) at steps_per_launch k."""
    out = []
    while n > 0:
        out.append(min(k, n))
        n -= out[-1]
    return out


def available_cpus() -> int:
    """CPUs this process may really use: its affinity set, capped by a cgroup
    CPU quota (a GPU box's share of the host is a quota, while os.cpu_count()
    shows every CPU of the machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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


def load_pmc(key: dict):
    """The rocprofv3 PMC row (scripts/pmc_bench.sh -> profiles/pmc_rows.json)
    of exactly this workload and launch length, or None: HBM bytes per launch
    (FETCH_SIZE + WRITE_SIZE, separate passes, calibrated factors) and SQ
    instruction counts per launch."""
    try:
        rows = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None
    for row in rows:
        if all(row.get(k) == v for k, v in key.items()) and \
                row.get("ae_max_entries", 0) == key.get("ae_max_entries", 0):
            return row
    return None


def cycle_split(pmc):
    """The disjoint split of the step kernel's wave cycles from the PMC row
    (MI355X_MICROARCH.md, SQ block): issuing (SQ_ACTIVE_INST_ANY), parked on
    s_waitcnt / barrier (SQ_WAIT_ANY) and ready but not issued
    (SQ_WAIT_INST_ANY); they sum to about SQ_WAVE_CYCLES.  None when the row
    lacks that pass."""
    raw = (pmc or {}).get("pmc_raw") or {}
    need = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")
    if not all(raw.get(k) for k in need):
        return None
    wc = raw["SQ_WAVE_CYCLES"]
    out = {"issuing": raw["SQ_ACTIVE_INST_ANY"] / wc, "waitcnt_or_barrier": raw["SQ_WAIT_ANY"] / wc,
           "ready_not_issued": raw["SQ_WAIT_INST_ANY"] / wc,
           "sum": (raw["SQ_ACTIVE_INST_ANY"] + raw["SQ_WAIT_ANY"] + raw["SQ_WAIT_INST_ANY"]) / wc}
    if raw.get("SQ_WAIT_INST_LDS"):
        out["lds_issue_stall"] = raw["SQ_WAIT_INST_LDS"] / wc
    for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
              "SQ_ACTIVE_INST_MISC", "SQ_INST_CYCLES_SALU"):
        if raw.get(k):
            out[k.lower()[3:] + "_per_wave_cycle"] = raw[k] / wc
    return out


def grid_fill(G: int, R: int, L: int, seven: bool) -> str:
    """How the step kernel's waves (one per 64 // R groups) fill the chip: 7
    resident waves per SIMD for the 7-wave kernels whose counter rows fit 7
    workgroups' LDS (launches of at most STEP_K_7WG steps, or longer ones run
    as 400-step epochs), else 6."""
    waves = -(-G // (64 // R))
    lds6 = abi.BENCH_STEPS_PER_LAUNCH < L <= abi.LDS_MAX_STEPS_PER_LAUNCH
    slots = SIMDS * (7 if seven and not lds6 else 6)
    if waves < slots:
        return (f"{waves} waves < the {slots} resident wave slots of one MI355X: the grid cannot fill "
                f"the chip ({waves / slots:.0%} of the slots), so this rate is not the kernel's throughput")
    return f"{waves} waves = {waves / slots:.2f} rounds of the {slots} resident wave slots"


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int) -> int:
    """Run this script as n rank processes on this node (one per GPU) and
    return their combined exit status.  Called before anything touches a GPU:
    the children are fresh interpreters, never an exec of this process."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # only rank 0 writes the result line to stdout; the others' output goes to stderr
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:                                   # one rank failed: the others would hang in a collective
                rc = bad[0]
                break
            time.sleep(0.05)
        rc = rc or next((p.returncode for p in procs if p.returncode not in (None, 0)), 0)
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return rc if rc >= 0 else 128 - rc


def legs():
    """scripts/bench_legs.py (the legs beside the timed region), imported on
    first use against THIS module (bench.py may be running as __main__)."""
    if __name__ in sys.modules:
        sys.modules.setdefault("bench", sys.modules[__name__])
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    return importlib.import_module("bench_legs")


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10_000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--groups", type=int, default=None,
                    help="total groups (strong scaling) or groups per GPU (weak scaling); default: the "
                         "configuration's own (BASELINE.json: 10^6 for config 3, 10^5 for 5, 10^4 for 2)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="strong (config 4, BASELINE.json configs[3]): --groups split over the GPUs; weak: --groups "
                         "per GPU")
    ap.add_argument("--no-side-leg", "--no-strong-leg", dest="no_side_leg", action="store_true",
                    help="N > 1, config 3: skip the other scaling's leg (weak beside a strong job, strong beside a "
                         "weak one)")
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 5])
    ap.add_argument("--mode", choices=["reference", "textbook"], default="reference",
                    help="protocol mode: the reference's handlers (parity) or the opt-in textbook rules")
    ap.add_argument("--ae-max-entries", type=int, default=0,
                    help="textbook mode: entries per AppendEntries request (0/1 = one, the reference's shape)")
    ap.add_argument("--steps-per-launch", type=int, default=0,
                    help="upper bound of the lockstep steps fused into one kernel launch (state stays in VGPRs); "
                         "0 = the kernel variant's default (abi.bench_steps_per_launch)")
    ap.add_argument("--subranges", type=int, default=0,
                    help="step-kernel launch sub-ranges, each on its own stream (0 = the engine's automatic choice)")
    ap.add_argument("--schedule-workgroups", type=int, default=0,
                    help="workgroups of a balanced launch (0 = the resident workgroups; tuning)")
    ap.add_argument("--schedule", choices=["auto", "one", "balanced"], default="auto",
                    help="step-kernel schedule (raft_params.schedule): balanced when the chunks outnumber the "
                         "resident wave slots (auto), one chunk per wave, or balanced")
    ap.add_argument("--stream-steps", type=int, default=200,
                    help="steps of the streaming leg (1 step per launch: the HBM-bound formulation)")
    ap.add_argument("--log-cap", type=int, default=0)
    ap.add_argument("--log-window", type=int, default=-1,
                    help="ring slots per replica (power of two; 0 = keep every physical slot); default: every slot "
                         "while that fits 60%% of HBM, else 256 for configs 2 and 3 (DESIGN.md §4.2)")
    ap.add_argument("--reduce-every", type=int, default=512,
                    help="steps per step_async call and per inline counter all-reduce (rounded to whole launches)")
    ap.add_argument("--allreduce", choices=["end", "inline", "after"], default="end",
                    help="N > 1: all-reduce the timed region's per-step counter rows once, on the engine stream "
                         "after the last launch, inside the timed region (end); per --reduce-every chunk, in series "
                         "with the launches (inline); or once the clock has stopped (after: a diagnostic that "
                         "leaves the collective off the clock)")
    ap.add_argument("--kernel-timing", choices=["replay", "region"], default="replay",
                    help="where the step kernel's per-launch time comes from: an exact replay of the timed launches "
                         "after the clock, each launch carrying its own timestamps (replay), or the timed region's "
                         "own launches (region: the timestamps are then inside the clock)")
    ap.add_argument("--no-rehearse", dest="rehearse", action="store_false",
                    help="skip the untimed rehearsal of the timed launches (then raft_engine_reset) before the warmup")
    ap.add_argument("--rehearse-ms", type=float, default=50.0,
                    help="the rehearsal's length: repeats of REHEARSE_RATE-priced work lasting at least this")
    ap.add_argument("--sync", choices=["spin", "block"], default="block",
                    help="how the host waits for the timed region's last work before the closing device sync: "
                         "poll its event (spin) or the runtime's blocking wait alone (block)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-general-leg", action="store_true",
                    help="N = 1: skip the general_kernel leg (the main leg on the run-time-decided kernel)")
    ap.add_argument("--handler-batch", type=int, default=1_000_000,
                    help="messages per single-handler batch of the handler_batch leg (0 = skip the leg)")
    ap.add_argument("--handler-reps", type=int, default=20)
    ap.add_argument("--handler-parity", type=int, default=20_000,
                    help="messages of each kind in the handler leg's oracle-checked batch")
    ap.add_argument("--handler-span", type=int, default=1024, help="groups the parity batch spans")
    ap.add_argument("--cpu-groups", type=int, default=20_000, help="calibration sample for the CPU baseline")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target seconds of the SoA leg on every core")
    ap.add_argument("--cpu-seconds-1t", type=float, default=3.0, help="target seconds of each single-thread leg")
    ap.add_argument("--cpu-chunk", type=int, default=20)
    ap.add_argument("--cpu-steady-at", type=int, default=9_600,
                    help="the CPU baseline's steady-state window starts at this step (state from the GPU engine)")
    ap.add_argument("--cpu-steady-steps", type=int, default=400, help="steps timed in that window (0 = skip)")
    ap.add_argument("--cpu-steady-groups", type=int, default=50_000, help="groups of the steady-state sample")
    ap.add_argument("--plan-file", default="",
                    help="write the step-kernel launch sequence (leg, steps) and the workload key as JSON, for "
                         "attributing rocprofv3 dispatches (scripts/pmc_bench.sh)")
    ap.add_argument("--traffic-probe", action="store_true",
                    help="after the timed legs (untimed): raft_engine_traffic_probe dispatches (the step kernel's own "
                         "state and log-store access patterns over known bytes), recorded in --plan-file for "
                         "calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE in the same process (scripts/pmc_bench.sh)")
    ap.add_argument("--plan-only", action="store_true",
                    help="no GPU: start the ranks, agree on the shards over gloo, print them (tests)")
    args = ap.parse_args(argv)
    args.groups = abi.CONFIGS[args.config]["G"] if args.groups is None else args.groups
    return args


def rehearsal_count(rehearse_ms, groups, steps, coll=False, dev="cpu"):
    """The rehearsal's repeats: this rank's group-steps priced at REHEARSE_RATE
    fill rehearse_ms; with `coll` the MAX over the ranks, so every rank runs
    the same number of the repeats' collectives (tests/test_dist_cpu.py)."""
    n = max(1, math.ceil(rehearse_ms / 1e3 * REHEARSE_RATE / max(1, groups * steps)))
    if coll:
        import torch, torch.distributed as dist  # noqa: E401
        t = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n = int(t.item())
    return n


def timed_leg(eng, args, chunk, coll, dev, world, comm=None):
    """Warmup (untimed), then the timed region of `args.steps` lockstep steps on
    `eng`: enqueued in chunks of `chunk` steps, bracketed by a barrier and a
    device sync on both sides.  When `coll`, the counter rows are all-reduced
    over the ranks: by default (--allreduce end) once, on the engine stream
    after the last launch and before the closing sync, so the collective is
    inside the clock; per chunk in series with the launches (inline); or after
    the clock stops (after, a diagnostic).  With `comm` (the engine's own RCCL
    communicator, engine.RaftComm) the in-clock all-reduce is one native call,
    raft_engine_allreduce_counters, out of place; else torch.distributed's
    all_reduce after a row copy.  Returns this rank's clock, the
    stream-event, step-kernel and all-reduce times, the job's elapsed time (MAX
    over ranks) and the counter rows (this rank's, all ranks', warmup)."""
    import torch
    import torch.distributed as dist
    stream = torch.cuda.ExternalStream(eng.stream, device=dev)
    counters = torch.zeros((args.steps, abi.COUNTER_STRIDE), dtype=torch.int64, device=dev)
    gcounters = torch.zeros_like(counters) if coll else counters
    wcount = torch.zeros((max(1, args.warmup), abi.COUNTER_STRIDE), dtype=torch.int64, device=dev)
    mode = args.allreduce if coll else None
    plan = [(q, min(chunk, args.steps - q)) for q in range(0, args.steps, chunk)]
    rehearsals = 0

    # ---- rehearsal (untimed, before the warmup): the timed region's launches
    # and its all-reduce on scratch rows, then raft_engine_reset to step 0, so
    # the launch shapes' and the collective's first use (~8 us at the 1/8
    # shard, profiles/r6_e) and the GPU's idle clocks (a short first region's
    # kernel ran ~4 % slow, r6_g) stay off the clock; repeated for at least
    # --rehearse-ms, the count fixed by the planned work (rehearsal_count)
    if args.rehearse and args.steps:
        scratch, sglob = torch.zeros_like(counters), torch.zeros_like(counters)
        rehearsals = rehearsal_count(args.rehearse_ms, eng.G, args.steps, coll, dev)
        for _ in range(rehearsals):
            for done, k in plan:
                eng.step_async(k, scratch[done].data_ptr())
            if mode == "end" and comm is not None:
                eng.allreduce_counters(comm, scratch.data_ptr(), sglob.data_ptr(), args.steps)
            eng.sync()
            eng.reset()
        del scratch, sglob

    # ---- warmup (untimed) ----
    comm_stream = torch.cuda.Stream(device=dev)
    if args.warmup:
        eng.step_async(args.warmup, wcount.data_ptr())
    if coll:
        # the counter all-reduce's first use (communicator and stream setup)
        # belongs to the warmup: the warmup rows all-reduced twice, on the
        # stream the timed region will use
        wglob = torch.zeros_like(wcount)
        wst = stream if mode == "end" else comm_stream
        if mode != "end":
            wev = torch.cuda.Event()
            wev.record(stream)
            comm_stream.wait_event(wev)
        if comm is not None and mode == "end":
            for _ in range(2):
                eng.allreduce_counters(comm, wcount.data_ptr(), wglob.data_ptr(), max(1, args.warmup))
        else:
            with torch.cuda.stream(wst):
                for _ in range(2):
                    wglob.copy_(wcount)
                    dist.all_reduce(wglob)
    eng.sync()
    torch.cuda.synchronize(dev)
    if coll:
        dist.barrier()

    # ---- timed region ----
    # The launches' own start / stop timestamps (hipExtLaunchKernelGGL events)
    # cost ~10 us of host time at the first launch (profiles/r6_b shard_ab):
    # by default (--kernel-timing replay) the timed region carries no event at
    # all, and the kernel and all-reduce times come from an exact replay of
    # the same launches after the clock (below); --kernel-timing region times
    # the region's own.
    # RAFT_BENCH_NO_KERNEL_EVENTS=1: no kernel times at all (A/B runs).
    no_ev = os.environ.get("RAFT_BENCH_NO_KERNEL_EVENTS") == "1"
    timing = args.kernel_timing == "region" and not no_ev
    eng.set_kernel_timing(timing)
    ev1 = torch.cuda.Event(enable_timing=True)
    ar0 = torch.cuda.Event(enable_timing=True)
    ar1 = torch.cuda.Event(enable_timing=True)
    # the chunks' counter rows and events, made before the clock starts (torch
    # tensor indexing in the loop put ~80 us of host time ahead of the first
    # launch, 6 % of the driver's 20-step run)
    rows = [counters[q].data_ptr() for q, _ in plan]
    inline = mode == "inline"
    chunk_ev = [torch.cuda.Event() for _ in plan] if inline else []
    # torch creates an event's HIP event at its first record: done here, so
    # the records inside the clock are plain hipEventRecord calls (the lazy
    # creation put ~2 us of host time ahead of the first launch)
    for e in (ev1, ar0, ar1, *chunk_ev):
        e.record(stream)
    torch.cuda.synchronize(dev)
    if coll:
        dist.barrier()
    # (no marker ahead of the first launch: the stream-event time starts at
    # that launch's own start timestamp, raft_engine_timed_span)
    t0 = time.perf_counter()
    for ci, (done, k) in enumerate(plan):
        eng.step_async(k, rows[ci])
        if inline:
            # --allreduce inline: the per-step counter rows all-reduced per
            # chunk on a side stream, the next launch waiting for it: a
            # balanced launch holds exactly the workgroups the GPU keeps
            # resident, so an RCCL kernel running beside it displaces some of
            # them into a second round (1.9e10 -> 1.3e10 group-steps/s at one
            # rank)
            chunk_ev[ci].record(stream)
            comm_stream.wait_event(chunk_ev[ci])
            with torch.cuda.stream(comm_stream):
                gcounters[done:done + k].copy_(counters[done:done + k])
                dist.all_reduce(gcounters[done:done + k])
            if done + k < args.steps:
                eng.wait_stream(comm_stream.cuda_stream)
    # the clock's own instrumentation: none with --kernel-timing replay (the
    # all-reduce's events too are recorded around its replay, below)
    instr = timing or no_ev

    def allreduce_end(src, dst, events):
        if events:
            ar0.record(stream)
        if comm is not None:
            eng.allreduce_counters(comm, src.data_ptr(), dst.data_ptr(), args.steps)
        else:
            with torch.cuda.stream(stream):
                dst.copy_(src)
                dist.all_reduce(dst)
        if events:
            ar1.record(stream)
    if mode == "end":
        # the default: every timed row all-reduced once, in series on the
        # engine stream after the last launch's counter reduction (nothing
        # runs beside the RCCL kernel), before the closing sync.  The copy
        # keeps this rank's own rows for its roofline.
        allreduce_end(counters, gcounters, instr)
    if instr or args.sync == "spin":
        ev1.record(stream)
    if args.sync == "spin":
        # the host polls the region's last event before the closing device
        # sync: a blocking wait sleeps on an interrupt once the runtime's short
        # active wait times out, and wakes ~15 us after the GPU is done
        while not ev1.query():
            pass
    torch.cuda.synchronize(dev)                 # the device: the engine's streams and the counter all-reduce
    wall = time.perf_counter() - t0             # this rank's clock; the job's time is the MAX over ranks (below)
    if coll:
        dist.barrier()
        if mode == "after":
            # --allreduce after (a diagnostic): the rows of every rank summed
            # once the clock has stopped, so the line times the kernels alone
            t_ar = time.perf_counter()
            gcounters.copy_(counters)
            dist.all_reduce(gcounters)
            torch.cuda.synchronize(dev)
            after_ms = (time.perf_counter() - t_ar) * 1e3
    ev_ms = eng.timed_span(ev1.cuda_event) if timing else None
    allreduce_ms = ar0.elapsed_time(ar1) if mode == "end" and instr else (after_ms if mode == "after" else None)
    kern_ms, launches = eng.kernel_time()
    eng.set_kernel_timing(False)
    replay_equal = None
    if args.kernel_timing == "replay" and not no_ev:
        # the timed region's launches again, from step 0 (raft_engine_reset: a
        # deterministic replay to the same state), each carrying its own
        # timestamps: the step kernel's time per launch without instrumenting
        # the clock; the replay's counter rows must equal the region's
        rcount = torch.zeros_like(counters)
        eng.reset()
        if args.warmup:
            eng.step_async(args.warmup, wcount.data_ptr())
        eng.sync()
        eng.set_kernel_timing(True)
        for done, k in plan:
            eng.step_async(k, rcount[done].data_ptr())
        if mode == "end":                         # the all-reduce's time, from its replay
            allreduce_end(rcount, torch.zeros_like(gcounters), True)
        kern_ms, launches = eng.kernel_time()
        eng.set_kernel_timing(False)
        if mode == "end":
            allreduce_ms = ar0.elapsed_time(ar1)
        replay_equal = bool(torch.equal(rcount, counters))

    elapsed = max(wall, ev_ms / 1e3) if ev_ms is not None else wall
    kern_avg_ms = kern_ms / max(1, launches)
    if coll:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ka = torch.tensor([kern_avg_ms], dtype=torch.float64, device=dev)
        kall = [torch.zeros_like(ka) for _ in range(world)]
        dist.all_gather(kall, ka)
        kern_avg_per_rank = [float(x.item()) for x in kall]
    else:
        kern_avg_per_rank = [kern_avg_ms]
    return {"wall": wall, "ev_ms": ev_ms, "kern_ms": kern_ms, "launches": launches, "elapsed": elapsed,
            "kern_avg_ms": kern_avg_ms, "kern_avg_per_rank": kern_avg_per_rank, "allreduce_ms": allreduce_ms,
            "counters": counters, "gcounters": gcounters, "wcount": wcount, "replay_counters_equal": replay_equal,
            "rehearsals": rehearsals}


def main(argv=None, result=None):
    """The bench.  `result` (a dict, in-process callers such as the GPU tests)
    receives the output line's object and the raw counter rows."""
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return spawn_ranks(args.gpus)                 # the parent never touches a GPU
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr, flush=True)
        return 2
    if args.plan_only:
        legs().plan_only(args, world, rank)
        return 0

    import torch
    import torch.distributed as dist

    # rehearsal knobs for a one-GPU box (never set by the driver):
    # RAFT_BENCH_BACKEND=gloo with RAFT_BENCH_ONE_DEVICE=1 runs every rank on
    # cuda:0 with gloo collectives, which exercises the N > 1 path end to end
    # RAFT_BENCH_FORCE_COLLECTIVE=1 runs the collective branch at WORLD_SIZE 1:
    # a one-rank communicator (RCCL by default), the counter
    # all-reduce and the elapsed / kernel-time reductions, so the
    # multi-GPU path executes on a one-GPU box (tests/test_gpu_bench.py)
    backend = os.environ.get("RAFT_BENCH_BACKEND", "nccl")
    if os.environ.get("RAFT_BENCH_ONE_DEVICE") == "1":
        local = 0
    coll = world > 1 or os.environ.get("RAFT_BENCH_FORCE_COLLECTIVE") == "1"
    if coll:
        torch.cuda.set_device(local)
        init = {} if world > 1 else {"init_method": f"tcp://127.0.0.1:{free_port()}", "rank": 0, "world_size": 1}
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), **init)
        else:
            dist.init_process_group(backend, **init)
    dev = torch.device("cuda", local)

    eng_mod = importlib.import_module("raft-kotlin_amd.engine")
    # the counter all-reduce's own RCCL communicator (engine.RaftComm): one
    # native call inside the clock instead of torch's all_reduce (whose host
    # path is ~150 us, exposed on a short shard, profiles/r5_d); the id goes
    # to the ranks over the torch process group.  RAFT_BENCH_TORCH_ALLREDUCE=1
    # keeps torch's all_reduce (and the gloo rehearsal always does: RCCL
    # refuses two ranks on one GPU)
    comm = None
    if coll and backend == "nccl" and os.environ.get("RAFT_BENCH_TORCH_ALLREDUCE") != "1":
        uid = eng_mod.RaftComm.unique_id() if rank == 0 else bytes(abi.COMM_ID_BYTES)
        t = torch.tensor(list(uid), dtype=torch.uint8, device=dev)
        dist.broadcast(t, 0)
        comm = eng_mod.RaftComm(bytes(t.cpu().tolist()), world, rank, local)
    kw = dict(abi.CONFIGS[args.config])
    R = kw["R"]
    g0, G_local = shard(args.groups, world, rank, args.scaling)
    groups_per_rank = [shard(args.groups, world, q, args.scaling)[1] for q in range(world)]
    total_groups = sum(groups_per_rank)
    total_steps = args.warmup + args.steps + args.stream_steps
    # physical slots a replica can fill: ~0.3 per step at config 3's command
    # rate, up to one per step where every leader takes a command each step
    log_cap = args.log_cap or int(64 + (1.0 if kw["cmd_ppm"] >= 1_000_000 else 0.3) * total_steps)
    window = args.log_window
    if window < 0:
        # every physical slot (no window checks in the kernel) while that log
        # fits in 60 % of this GPU's HBM; else the 256-slot ring (configs 2
        # and 3 never access more than 48 slots below physLen; config 5's
        # ghost-tail gaps reach thousands of slots, so it is always flat)
        flat = -(-G_local // (64 // R)) * 64 * log_cap * 8
        hbm = torch.cuda.get_device_properties(dev).total_memory
        window = 0 if args.config == 5 or flat <= 0.6 * hbm else 256
    log_cap = max(log_cap, window)                          # the window never exceeds the physLen limit
    mode = abi.MODE_TEXTBOOK if args.mode == "textbook" else abi.MODE_REFERENCE
    net = abi.step_net_of(kw)
    spl = args.steps_per_launch or abi.bench_steps_per_launch(R, mode, window, net, G_local, SIMDS)
    L = launch_length(args.steps, spl)                      # every timed launch has L steps
    chunk = L * max(1, args.reduce_every // L)               # steps per step_async call / all-reduce
    # launch sub-ranges: 0 = the engine's automatic choice (one on the balanced
    # schedule; three for a partitions-only workload)
    subranges = args.subranges
    params = abi.make_params(log_cap=log_cap, log_window=window, steps_per_launch=L, mode=mode, subranges=subranges,
                             schedule=SCHEDULES[args.schedule], schedule_workgroups=args.schedule_workgroups,
                             ae_max_entries=args.ae_max_entries, **dict(kw, G=G_local, g0=g0))
    eng = eng_mod.RaftEngine(params, device=local)
    nsub = eng.subranges                                     # launch sub-ranges of the warmup and timed legs
    hbm_bytes_engine = eng.device_bytes
    leg = timed_leg(eng, args, chunk, coll, dev, world, comm)
    wall, ev_ms, kern_ms, launches = leg["wall"], leg["ev_ms"], leg["kern_ms"], leg["launches"]
    elapsed, kern_avg_ms, kern_avg_per_rank = leg["elapsed"], leg["kern_avg_ms"], leg["kern_avg_per_rank"]
    counters, gcounters, wcount = leg["counters"], leg["gcounters"], leg["wcount"]

    kinfo = eng.kernel_info()                                # the timed leg's last launch
    kernel_variant = {"net": kinfo["net"], "net_bits": NET_NAMES(kinfo["net"]), "textbook": bool(kinfo["textbook"]),
                      "ring": bool(kinfo["ring"]), "schedule": "balanced" if kinfo["balanced"] else "one_per_wave",
                      "workgroups": kinfo["workgroups"], "resident_workgroups": kinfo["resident_workgroups"],
                      # the loaded library's own provenance (build.py ids compiled in)
                      "kernel_source_id": abi.build_ids()["kernel_source_id"],
                      "library_source_id": abi.build_ids()["library_source_id"]}
    c_all = gcounters.cpu().numpy()[:, : abi.NUM_COUNTERS]    # all ranks' groups
    c_loc = counters.cpu().numpy()[:, : abi.NUM_COUNTERS]     # this rank's groups (before the all-reduce)
    value = total_groups * args.steps / elapsed

    # roofline of the dominant kernel (step_kernel), from this rank's own counters
    timed_plan = [x for q in range(0, args.steps, chunk) for x in launch_plan(min(chunk, args.steps - q), L)]
    kern_s = kern_ms / 1e3
    bytes_alg = algorithmic_bytes(c_loc, G_local, R)
    bytes_state = state_crossing_bytes(c_loc, G_local, R, launches)
    achieved = bytes_alg / kern_s / 1e9 if launches else 0.0
    achieved_state = bytes_state / kern_s / 1e9 if launches else 0.0
    overflow = int(c_all[:, abi.C_INDEX["log_overflow"]].sum())
    wmiss = int(c_all[:, abi.C_INDEX["log_window_miss"]].sum())
    wc = wcount.cpu().numpy()[: args.warmup, : abi.NUM_COUNTERS]      # this rank's untimed legs count too
    bad_untimed = int(wc[:, abi.C_INDEX["log_overflow"]].sum() + wc[:, abi.C_INDEX["log_window_miss"]].sum())
    pmc_key = {"config": args.config, "mode": args.mode, "groups": G_local, "launch_steps": L,
               "warmup": args.warmup, "steps": args.steps, "log_window": window,
               "kernel_src": kernel_source_id()}
    if args.ae_max_entries > 1:
        pmc_key["ae_max_entries"] = args.ae_max_entries
    pmc = load_pmc(dict(pmc_key, leg="timed")) if len(set(timed_plan)) == 1 else None
    traffic = pmc["hbm_bytes_per_launch"] if pmc else None
    roofline_valu = None
    if pmc and pmc.get("valu_per_launch"):
        ips = pmc["valu_per_launch"] / (kern_avg_ms / 1e3) / 1e9
        clk = pmc.get("effective_clock_ghz") or CLOCK_HZ / 1e9
        roofline_valu = {
            "bound": "valu", "achieved": ips, "peak": VALU_PEAK_GIPS, "unit": "G wave-instructions/s",
            "frac": ips / VALU_PEAK_GIPS,
            # per chunk-step: one wave's 64 // R groups for one step (a launch of
            # the balanced schedule runs fewer, longer-lived waves than chunks)
            "valu_per_wave_step": pmc["valu_per_launch"] / (-(-G_local // (64 // R)) * L),
            "salu_per_wave_step": pmc["salu_per_launch"] / (-(-G_local // (64 // R)) * L),
            "valu_per_simd_cycle": pmc["valu_per_launch"] / (SIMDS * CLOCK_HZ * kern_avg_ms / 1e3),
            "simd_cycles_per_valu": SIMDS * clk * 1e9 * kern_avg_ms / 1e3 / pmc["valu_per_launch"],
            "effective_clock_ghz": clk,
            "cycle_split": cycle_split(pmc),
            "source": pmc["source"],
            "note": "SQ_INSTS_VALU of this exact launch and kernel build (rocprofv3 --pmc) / the live launch time; "
                    "peak = 1024 SIMDs x 2.4 GHz / 2 cycles (the cheapest VALU); this mix averages ~2.6 cycles per "
                    "VALU plus ~2 per SALU (DESIGN.md §4.6); cycle_split: SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY / "
                    "SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES",
        }

    # ---- the general kernel (untimed for `value`): the warmup and timed legs
    # replayed from step 0, ending at the same state ----
    general = None
    if world == 1 and not coll and not args.no_general_leg and net != abi.NET_ALL:
        general = legs().general_kernel_leg(eng, args, chunk, dev, c_loc, kern_avg_ms)

    # ---- streaming leg (untimed for `value`): one step per launch, the
    # HBM-bound formulation of the same step (bench_legs.streaming_leg) ----
    streaming, bad_stream = legs().streaming_leg(eng, args, dev, G_local, R, pmc_key) if args.stream_steps > 0 else (None, 0)
    bad_untimed += bad_stream

    # ---- traffic probes (untimed, --traffic-probe): the step kernel's own
    # access patterns over known bytes, for the PMC byte factors ----
    probes = []
    if args.traffic_probe:
        for kind in ((0, 1) if window == 0 else (0,)):
            for _ in range(3):
                probes.append([kind, *eng.traffic_probe(kind)])
    if args.plan_file and rank == 0:
        # [leg, steps, dispatches]: a launch of the warmup / timed legs is one
        # step-kernel dispatch per sub-range; the streaming leg runs one range.
        # Each timed_leg: the rehearsal (the timed launches), the warmup, the
        # timed launches, then the replay of warmup + timed (kernel timing)
        def leg_seq(name, reps):
            w = [[f"{name}warmup", x, nsub] for x in launch_plan(args.warmup, L)]
            t = [[f"{name}timed" if name else "timed", x, nsub] for x in timed_plan]
            r = [[f"{name}rehearsal", x, nsub] for x in timed_plan] * reps
            rp = ([[f"{name}replay_warmup", x, nsub] for x in launch_plan(args.warmup, L)]
                  + [[f"{name}replay", x, nsub] for x in timed_plan]) if args.kernel_timing == "replay" else []
            return r + w + t + rp
        seq = leg_seq("", leg["rehearsals"])
        if general is not None:                   # the general kernel runs the same leg from step 0
            seq += [["general" if x[0] == "general_timed" else x[0], *x[1:]]
                    for x in leg_seq("general_", general["rehearsals"])]
        seq += [["streaming", 1, 1]] * args.stream_steps
        ix = abi.C_INDEX
        stores = float(c_loc[:, ix["entry_writes"]].sum() + c_loc[:, ix["commands"]].sum()) / max(1, launches)
        json.dump({"key": pmc_key, "stream_steps": args.stream_steps, "R": R, "launches": seq, "probes": probes,
                   "state_bytes_per_launch": 2 * G_local * (R * REPLICA_BYTES + GROUP_BYTES),
                   "log_stores_per_timed_launch": stores},
                  open(args.plan_file, "w"))

    # ---- safety flags (untimed): the run's counter-borne flags plus the
    # Log Matching check over committed prefixes ----
    mism = eng.check_log_matching()
    if coll:
        t = torch.tensor([mism, bad_untimed], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        mism, bad_untimed = int(t[0].item()), int(t[1].item())
    safety = {
        "log_matching_mismatched_groups": mism,
        "commit_regressions": int(c_all[:, abi.C_INDEX["commit_regressions"]].sum()),
        "dual_leader_group_steps": int(c_all[:, abi.C_INDEX["dual_leader_groups"]].sum()),
        "log_overflow": overflow,
        "log_window_misses": wmiss,
        "untimed_overflow_or_window_misses": bad_untimed,
        "note": "observations of the reference's protocol (quirks Q4/Q9 do not preserve these "
                "properties); over the timed steps, Log Matching at the end of the run",
    }

    # the other scaling's leg: weak beside config 4 (the default), config 4 beside a weak job
    side = None
    if world > 1 and args.config == 3 and not args.no_side_leg:
        eng.close()
        eng = None
        other = "weak" if args.scaling == "strong" else "strong"
        side = legs().side_leg(args, kw, mode, world, rank, local, dev, coll, log_cap, L, chunk, other,
                        (c_all if other == "weak" else c_loc) if rank == 0 else None, comm)

    cfg_name = "config4" if world > 1 and args.config == 3 and args.scaling == "strong" else f"config{args.config}"
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
            "workload": (f"{cfg_name}: {total_groups} groups x {R} replicas"
                         + (f" sharded by contiguous group id over {world} GPUs" if world > 1 else "")
                         if world == 1 or args.scaling == "strong" else
                         f"{cfg_name} on every GPU (weak scaling): {G_local} groups x {R} replicas per GPU, "
                         f"{world} GPUs, {total_groups} groups in contiguous global-id ranges")
                        + {3: ", 5% drop, leader-isolation churn 1e-3 x 15 steps, 1/4 command per group-step",
                           5: ", 2-way partitions 25 of every 50 steps, 1 command per step to every leader",
                           2: ", no faults, 1/4 command per group-step"}[args.config]
                        + (", textbook mode" if mode else "")
                        + (f", up to {args.ae_max_entries} entries per AppendEntries" if args.ae_max_entries > 1 else ""),
            "groups_total": total_groups, "groups_per_rank": groups_per_rank, "replicas": R, "log_cap": log_cap,
            "log_window": window, "hbm_bytes_engine": hbm_bytes_engine,
            "steps_per_launch": L, "launches": launches, "parallelism": f"shard-by-group x{world}",
            "subranges": nsub,
            "step_waves_per_rank": -(-G_local // (64 // R)),
            "grid_fill": grid_fill(G_local, R, L, R <= 5 or (R == 7 and net == abi.NET_PART)),
            "counter_allreduce_every": ({"end": "timed_region_once", "inline": chunk,
                                         "after": "after_timed_region_diagnostic"}[args.allreduce] if coll else None),
            "collective": ({"backend": backend, "ranks": world, "forced_at_one_rank": world == 1,
                            "counter_allreduce": ("raft_engine_allreduce_counters (the engine's RCCL communicator)"
                                                  if comm is not None and args.allreduce == "end" else
                                                  "torch.distributed.all_reduce")} if coll else None),
        },
        "roofline": {
            "bound": "alg_equiv", "basis": "alg_equiv", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_frac": traffic / (kern_avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS if traffic else None,
            "kernel": f"step_kernel<{R}> x{L} fused steps", "launch_steps": L,
            "kernel_variant": kernel_variant,
            "kernel_avg_ms": kern_avg_ms, "kernel_avg_ms_per_rank": kern_avg_per_rank, "launches": launches,
            "alg_bytes_per_launch": bytes_alg / max(1, launches),
            "alg_bytes_per_group_step": bytes_alg / max(1, G_local * c_loc.shape[0]),
            "pmc_source": pmc["source"] if pmc else None,
            # the PMC counts behind `traffic`: raw FETCH_SIZE / WRITE_SIZE
            # kilobytes per launch and the byte factors of the same process's
            # traffic probes (scripts/pmc_parse.py probe_factors)
            "traffic_raw_kb": ({"fetch": pmc.get("fetch_kb_raw"), "write": pmc.get("write_kb_raw")} if pmc else None),
            "traffic_split": ({"fetch_bytes": pmc.get("fetch_bytes_per_launch"),
                               "write_bytes": pmc.get("write_bytes_per_launch"),
                               "log_stores": pmc.get("log_stores_per_launch"),
                               "fetch_factor": pmc.get("fetch_factor"), "write_factor": pmc.get("write_factor"),
                               "probes": pmc.get("traffic_probes")} if pmc else None),
            "state_bytes_per_launch": bytes_state / max(1, launches),
            "achieved_state_crossing": achieved_state,
            "frac_state_crossing": achieved_state / HBM_PEAK_GBS,
            "note": "alg_equiv: SURVEY.md §8(d) algorithmic bytes per group-step (this rank's own kernel counters) "
                    "x the group-steps of one launch / the launch's average duration; the fused launch keeps the "
                    "replicas in VGPRs, so its real HBM bytes (traffic, PMC) are far below: traffic_frac is the "
                    "measured HBM fraction, bound_by / roofline_valu the binding resource",
        },
        "roofline_valu": roofline_valu,
        # what binds the fused launch (roofline is §8(d)'s algorithmic-bytes
        # figure, not an HBM measurement): instruction issue, DESIGN.md §4.6
        "bound_by": {"resource": "SIMD instruction issue (VALU + SALU, ~2.6 + ~2.0 SIMD-cycles each)",
                     "valu_frac_of_nominal": roofline_valu["frac"] if roofline_valu else None,
                     "hbm_traffic_frac": (traffic / (kern_avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS if traffic else None)},
        "general_kernel": general,
        "roofline_streaming": streaming,
        "timing": {"wall_ms": wall * 1e3, "stream_event_ms": ev_ms, "step_kernel_ms_total": kern_ms,
                   "allreduce_ms": leg["allreduce_ms"], "kernel_timing": args.kernel_timing,
                   "replay_counters_equal": leg["replay_counters_equal"],
                   "rehearsals": leg["rehearsals"], "rehearse_ms": args.rehearse_ms,
                   "note": "each rank's wall clock from after the opening barrier + device sync to after its closing "
                           "device sync (the job's time is the MAX over ranks); nothing inside it is instrumented "
                           "(kernel_timing replay): the kernel and all-reduce times come from the same launches "
                           "replayed from step 0 after the clock, whose counter rows equal the region's; before the "
                           "warmup an untimed rehearsal of the timed launches (then a reset) runs for >= "
                           "--rehearse-ms, so the GPU leaves its idle clocks (DESIGN.md §5)"},
        "valid": overflow == 0 and wmiss == 0 and bad_untimed == 0,
        "safety": safety,
        "counters_last_step": {n: int(v) for n, v in zip(abi.COUNTER_NAMES, c_all[-1])},
    }
    if side is not None:
        out["weak_scaling" if side["scaling"] == "weak" else "config4_strong"] = side
    if args.handler_batch > 0 and world == 1 and not coll:
        out["handler_batch"] = legs().handler_batch_leg(eng, args, dict(kw, mode=mode, ae_max_entries=args.ae_max_entries),
                                                 log_cap, dev, G_local, R)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = legs().cpu_baseline(args, dict(kw, mode=mode, ae_max_entries=args.ae_max_entries), log_cap,
                                                  args.warmup + args.steps, device=local)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if result is not None:
        result.update(out=out, counters_all=c_all, counters_local=c_loc,
                      warmup_counters=wcount.cpu().numpy()[: args.warmup, : abi.NUM_COUNTERS])
    if eng is not None:
        eng.close()
    if comm is not None:
        comm.close()
    if coll:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
