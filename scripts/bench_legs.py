"""bench.py's legs beside the timed region (its driver path is bench.main and
bench.timed_leg): the CPU baseline, the drop-in handler batches, the general
kernel, the other scaling's leg of an N > 1 job and the rank plumbing without a
GPU.  Each returns the object bench.py puts into its output line."""
from __future__ import annotations

import importlib
import json
import os
import sys
import time

import numpy as np

import bench
from bench import (ROOT, HBM_PEAK_GBS, SCHEDULES, abi, algorithmic_bytes, available_cpus, cpu_model, grid_fill,
                   load_pmc, shard, state_crossing_bytes, timed_leg)


def streaming_leg(eng, args, dev, G, R, pmc_key):
    """One step per launch (--stream-steps launches, one sub-range): every
    launch streams the whole group state HBM -> VGPRs -> HBM, the HBM-bound
    formulation SURVEY.md §8(d) prices.  Returns (its roofline object, the
    overflow / window-miss count of its steps)."""
    import torch
    eng.set_steps_per_launch(1)
    eng.set_subranges(1)                      # one full-grid launch per step
    sc = torch.zeros((args.stream_steps, abi.COUNTER_STRIDE), dtype=torch.int64, device=dev)
    eng.set_kernel_timing(True)
    eng.step_async(args.stream_steps, sc.data_ptr())
    eng.sync()
    s_ms, s_n = eng.kernel_time()
    eng.set_kernel_timing(False)
    cs = sc.cpu().numpy()[:, : abi.NUM_COUNTERS]
    s_avg = s_ms / max(1, s_n)
    s_bytes = algorithmic_bytes(cs, G, R) / max(1, s_n)
    s_state = state_crossing_bytes(cs, G, R, s_n) / max(1, s_n)
    s_ach = s_bytes / (s_avg / 1e3) / 1e9
    s_pmc = load_pmc(dict(pmc_key, launch_steps=1, leg="streaming", stream_steps=args.stream_steps))
    bad = int(cs[:, abi.C_INDEX["log_overflow"]].sum() + cs[:, abi.C_INDEX["log_window_miss"]].sum())
    out = {"steps_per_launch": 1, "steps": args.stream_steps, "kernel_avg_ms": s_avg,
           "alg_bytes_per_launch": s_bytes, "achieved": s_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": s_ach / HBM_PEAK_GBS,
           "traffic": s_pmc["hbm_bytes_per_launch"] if s_pmc else None,
           "traffic_frac": (s_pmc["hbm_bytes_per_launch"] / (s_avg / 1e3) / 1e9 / HBM_PEAK_GBS if s_pmc else None),
           "state_bytes_per_launch": s_state,
           "achieved_state_crossing": s_state / (s_avg / 1e3) / 1e9,
           "frac_state_crossing": s_state / (s_avg / 1e3) / 1e9 / HBM_PEAK_GBS,
           "kernel_group_steps_per_s": G / (s_avg / 1e3)}
    return out, bad


def cpu_baseline(args, kw, log_cap, total_steps, device=0):
    """The CPU path on a bounded sample of the same workload, on this host's
    cores (rank 0, N=1 only): the SoA backend (oracle/raft_soa.cpp, the same
    step laid out as structure-of-arrays, std::thread over groups; `value`)
    and the scalar oracle (oracle/raft_oracle.c, one object per replica,
    pthreads over groups), each with every usable core and with one.  Both
    restate the reference's algorithm (the Kotlin itself cannot run here) and
    are bit-exact with each other and the engine.  A sample is a contiguous
    range of the same global groups, run for the same number of steps as the
    GPU (so logs grow exactly as they do there), sized by a short calibration
    run to take about --cpu-seconds (--cpu-seconds-1t single-threaded).

    soa_steady / soa_steady_1t: the same SoA backend on the steady-state phase
    mix (leader ticks dominate; the cold-start window above is the first
    election storm): --cpu-steady-groups global groups are run on the GPU engine to
    step --cpu-steady-at, their state and logs restored into the SoA backend,
    and --cpu-steady-steps steps timed there; the engine runs the same steps
    from the same state and the two digests must agree (matches_engine)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = args.cpu_threads or available_cpus()
    impls = {"soa": O.Soa, "oracle": O.Oracle} if kw.get("mode", 0) == abi.MODE_REFERENCE else {"oracle": O.Oracle}

    def rate_of(cls, nthreads):
        probe = cls(abi.make_params(log_cap=log_cap, **dict(kw, G=args.cpu_groups)))
        t0 = time.perf_counter()
        probe.step(args.cpu_chunk, nthreads=nthreads, counters=False)
        r = args.cpu_groups * args.cpu_chunk / max(1e-6, time.perf_counter() - t0)
        probe.close()
        return r

    def timed(cls, nthreads, seconds):
        rate = rate_of(cls, nthreads)
        G = int(min(kw["G"], max(nthreads * 64, rate * seconds / total_steps)))
        o = cls(abi.make_params(log_cap=log_cap, **dict(kw, G=G)))
        o.step(args.warmup, nthreads=nthreads, counters=False)
        t0 = time.perf_counter()
        done = 0
        while done < total_steps - args.warmup:
            k = min(args.cpu_chunk * 10, total_steps - args.warmup - done)
            o.step(k, nthreads=nthreads, counters=True)
            done += k
        dt = time.perf_counter() - t0
        o.close()
        return {"value": G * done / dt, "unit": "group-steps/s", "cores": nthreads,
                "sample": f"global groups 0..{G - 1}, the same {total_steps} steps as the GPU "
                          f"({args.warmup} untimed), {dt:.1f} s"}

    def steady(nthreads):
        eng_mod = importlib.import_module("raft-kotlin_amd.engine")
        G, t0, n = args.cpu_steady_groups, args.cpu_steady_at, args.cpu_steady_steps
        cap = int(64 + 0.3 * (t0 + n)) if kw["cmd_ppm"] < 1_000_000 else 64 + t0 + n
        p = abi.make_params(log_cap=cap, **dict(kw, G=G))
        e = eng_mod.RaftEngine(p, device=device)
        e.step(t0, counters=False)                       # the GPU gets the sample to the window's start
        o = O.Soa(abi.make_params(log_cap=cap, **dict(kw, G=G)))
        o.write_state(e.read_state())
        o.write_log(*e.read_log())
        o.set_step_index(t0)
        t = time.perf_counter()
        o.step(n, nthreads=nthreads, counters=True)
        dt = time.perf_counter() - t
        e.step(n, counters=False)
        same = e.digest() == o.digest()
        e.close()
        o.close()
        return {"value": G * n / dt, "unit": "group-steps/s", "cores": nthreads, "matches_engine": same,
                "window": [t0, t0 + n],
                "sample": f"global groups 0..{G - 1}, steps {t0}..{t0 + n} (the steady state: state and logs at step "
                          f"{t0} from the GPU engine), {dt:.2f} s"}

    legs = {}
    for name, cls in impls.items():
        legs[name] = timed(cls, threads, args.cpu_seconds if name == "soa" else args.cpu_seconds / 2)
        legs[name + "_1t"] = timed(cls, 1, args.cpu_seconds_1t)
    if "soa" in impls and args.cpu_steady_steps > 0:
        legs["soa_steady"] = steady(threads)
        legs["soa_steady_1t"] = steady(1)
    best = legs["soa"] if "soa" in legs else legs["oracle"]
    return {"value": best["value"], "unit": "group-steps/s", "cores": threads, "kind": "port",
            "sample": ("oracle/raft_soa.cpp, the SoA CPU backend (bit-exact with the scalar restatement of "
                       "RaftServer.kt/Commons.kt), std::thread over groups; " if "soa" in legs else
                       "oracle/raft_oracle.c (scalar C restatement of RaftServer.kt/Commons.kt), pthreads; ")
                      + best["sample"],
            "legs": legs, "host_cpus": os.cpu_count(), "cpu_model": cpu_model()}

def handler_requests(rng, n, G, R, max_term):
    """n random single-handler messages over the engine's G x R replicas:
    (group, dst, vote requests [n, 4], append requests [n, 8] as int32 bit
    patterns).  Vote fields are drawn around the run's terms; half the appends
    carry prevLogIndex -1 (the consistency check passes and, with an entry,
    Log.add(0) overwrites and truncates: Q2), half a random prevLogIndex below
    64 with a random prevLogTerm (mostly rejected)."""
    group = rng.integers(0, G, n, dtype=np.int64)
    dst = rng.integers(0, R, n).astype(np.int32)
    vote = np.stack([rng.integers(0, 2 * max_term + 2, n), rng.integers(1, R + 1, n), rng.integers(0, 4000, n),
                     rng.integers(0, max_term + 1, n)], axis=1).astype(np.int32)
    prev = np.where(rng.random(n) < 0.5, -1, rng.integers(0, 64, n))
    app = np.stack([rng.integers(0, 2 * max_term + 2, n), rng.integers(1, R + 1, n), prev,
                    rng.integers(0, max_term + 1, n), rng.integers(0, 2, n), rng.integers(0, max_term + 1, n),
                    rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.int64), rng.integers(0, 4000, n)],
                   axis=1).astype(np.int64).astype(np.uint32).view(np.int32)
    return group, dst, vote, app

# the handler batches' algorithmic bytes per message: what
# the reference's handler itself reads and writes.  The message in (group 8 +
# replica 4 + request 16 / 32) and the response out (8 / 12).  vote()
# (RaftServer.kt:228-251) reads 6 fields (term, votedFor, state, lastIndex,
# physLen, the consumer flags) and log[lastIndex-1].term, and writes at most 5
# (term, votedFor, state, flags, the re-armed timer).  append() (:253-287)
# reads 7 (those plus commitIndex) and log[prev].term, writes at most 8 (plus
# commitIndex, lastIndex, physLen) and one entry.
HANDLER_ALG_BYTES = {"vote": 12 + 16 + 8 + 4 * 6 + 4 * 5 + 4,
                     "append": 12 + 32 + 12 + 4 * 7 + 4 * 8 + 4 + 8}
HANDLER_PMC_FILE = os.path.join(ROOT, "profiles", "pmc_handler.json")

def handler_parity(eng, O, params_kw, log_cap, kind, G, R, n_msgs, span, seed):
    """The handler batch against the oracle's handlers on n_msgs messages over
    `span` contiguous groups (several messages per replica, so runs of
    messages to one replica are exercised): the span's state and logs copied
    into one oracle, the batch applied by both, every response, state field
    and log slot compared.  Returns (messages, mismatches)."""
    import torch
    rng = np.random.default_rng(seed)
    ga = int(rng.integers(0, max(1, G - span)))
    st = eng.read_state(ga, span)
    max_term = int(st[:, [r * abi.NUM_FIELDS + abi.F_INDEX["term"] for r in range(R)]].max())
    group, dst, vote, app = handler_requests(rng, n_msgs, span, R, max_term)
    group = group + ga
    req = vote if kind == "vote" else app
    t0, c0 = eng.read_log(ga, span)
    o = O.Oracle(abi.make_params(log_cap=log_cap, **dict(params_kw, G=span, g0=eng.g0 + ga)))
    o.write_state(st)
    o.write_log(t0, c0)
    o.step_index = eng.step_index
    dev = torch.device("cuda", eng.device)
    w = 2 if kind == "vote" else 3
    d_resp = torch.zeros((n_msgs, w), dtype=torch.int32, device=dev)
    d_in = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (group, dst, req)]
    fn = eng.vote_batch_dev if kind == "vote" else eng.append_batch_dev
    fn(*(x.data_ptr() for x in d_in), d_resp.data_ptr(), n_msgs, after_stream=torch.cuda.current_stream(dev).cuda_stream)
    resp = d_resp.cpu().numpy()
    bad = 0
    for m in range(n_msgs):
        q, g = req[m], int(group[m]) - ga
        if kind == "vote":
            want = o.vote(g, int(dst[m]), *(int(x) for x in q))
            bad += (int(resp[m, 0]), int(resp[m, 1])) != (int(want[0]), int(want[1]))
        else:
            qq = q.view(np.uint32).astype(np.int64)
            t_, s_, st_ = o.append(g, int(dst[m]), int(q[0]), int(q[1]), int(q[2]), int(q[3]),
                                   (int(q[5]), int(qq[6])) if q[4] else None, int(q[7]))
            bad += tuple(int(x) for x in resp[m]) != (int(t_), int(s_), int(st_))
    es, (et, ec) = eng.read_state(ga, span), eng.read_log(ga, span)
    os_, (ot, oc) = o.read_state(), o.read_log()
    bad += int(np.count_nonzero(np.any(es != os_, axis=1)))
    phys = es[:, [r * abi.NUM_FIELDS + abi.F_INDEX["phys"] for r in range(R)]]
    slot = np.arange(log_cap)[None, None, :] < phys[:, :, None]
    bad += int(np.count_nonzero(((et != ot) | (ec != oc)) & slot))
    o.close()
    return n_msgs, bad

def handler_batch_leg(eng, args, params_kw, log_cap, dev, G, R):
    """The drop-in service path (RaftServer.vote() / append(), RaftServer.kt:228-287):
    raft_vote_batch_dev / raft_append_batch_dev on n random messages already
    in HBM (the bucketed path: a stable partition of each tile into buckets of
    consecutive replicas, a workgroup per bucket sorting its messages in LDS,
    one lane per replica run), and the same
    through the host entry points (from pageable arrays through pinned
    staging, and from page-locked arrays by direct DMA).  Parity: a batch of
    --handler-parity messages of each kind on a span of groups against the
    oracle's handlers (handler_parity).  Roofline: the algorithmic bytes per
    message (HANDLER_ALG_BYTES) at the measured rate, and the rocprofv3 row of
    the same batch (profiles/pmc_handler.json, scripts/pmc_handler.sh) when
    one matches this kernel build."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    n = args.handler_batch
    st = eng.read_state()
    max_term = int(st[:, [r * abi.NUM_FIELDS + abi.F_INDEX["term"] for r in range(R)]].max())
    rng = np.random.default_rng(12345)
    group, dst, vote, app = handler_requests(rng, n, G, R, max_term)
    try:
        pmc_rows = json.load(open(HANDLER_PMC_FILE))
    except (OSError, ValueError):
        pmc_rows = []
    src = abi.build_ids()["batch_source_id"]               # the loaded library's (its compile-time knobs included)
    path = eng.batch_path
    out = {"messages_per_batch": n, "groups": G, "replicas": R}
    for kind, req, resp_w in (("vote", vote, 2), ("append", app, 3)):
        msgs, bad = handler_parity(eng, O, params_kw, log_cap, kind, G, R, args.handler_parity,
                                   min(G, args.handler_span), 777 if kind == "vote" else 778)
        d_group = torch.from_numpy(group).to(dev)
        d_dst = torch.from_numpy(dst).to(dev)
        d_req = torch.from_numpy(np.ascontiguousarray(req)).to(dev)
        d_resp = torch.zeros((n, resp_w), dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        fn = eng.vote_batch_dev if kind == "vote" else eng.append_batch_dev
        ptrs = (d_group.data_ptr(), d_dst.data_ptr(), d_req.data_ptr(), d_resp.data_ptr(), n)
        fn(*ptrs)                                                       # warm (staging sized)
        # timed: device-resident batches (each call returns after its batch finished)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.handler_reps):
            fn(*ptrs)
        dt_dev = time.perf_counter() - t0
        # timed: host buffers (pinned staging + PCIe both ways)
        hfn = eng.vote_batch if kind == "vote" else eng.append_batch
        t0 = time.perf_counter()
        reps_h = max(1, args.handler_reps // 4)
        for _ in range(reps_h):
            hfn(group, dst, req)
        dt_host = time.perf_counter() - t0
        # timed: page-locked host buffers (the engine's DMA reads and writes
        # the caller's arrays directly, no staging copy)
        pin = [torch.from_numpy(np.ascontiguousarray(a)).pin_memory() for a in (group, dst, req)]
        pout = torch.zeros((n, resp_w), dtype=torch.int32).pin_memory()
        pg, pd, pq, po = pin[0].numpy(), pin[1].numpy(), pin[2].numpy(), pout.numpy()
        hfn(pg, pd, pq, out=po)
        t0 = time.perf_counter()
        for _ in range(args.handler_reps):
            hfn(pg, pd, pq, out=po)
        dt_pin = time.perf_counter() - t0
        rate = n * args.handler_reps / dt_dev
        ach = HANDLER_ALG_BYTES[kind] * rate / 1e9
        pmc = next((r for r in pmc_rows if (r["kind"], r["n"], r["groups"], r["replicas"], r.get("batch_src"),
                                            r.get("batch_path", 0)) == (kind, n, G, R, src, path)), None)
        out[kind] = {"messages_per_s_device": rate,
                     "ms_per_batch_device": dt_dev * 1e3 / args.handler_reps,
                     "messages_per_s_host_buffers": n * reps_h / dt_host,
                     "ms_per_batch_host_buffers": dt_host * 1e3 / reps_h,
                     "messages_per_s_pinned_host": n * args.handler_reps / dt_pin,
                     "ms_per_batch_pinned_host": dt_pin * 1e3 / args.handler_reps,
                     "roofline": {"bound": "hbm", "alg_bytes_per_message": HANDLER_ALG_BYTES[kind],
                                  "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": ach / HBM_PEAK_GBS,
                                  "traffic_bytes_per_message": pmc["hbm_bytes_per_message"] if pmc else None,
                                  "handler_kernel_traffic_bytes_per_message":
                                      pmc["handler_kernel_hbm_bytes_per_message"] if pmc else None,
                                  "traffic_frac": (pmc["hbm_bytes_per_message"] * rate / 1e9 / HBM_PEAK_GBS
                                                   if pmc else None),
                                  "pmc_source": pmc["source"] if pmc else None},
                     "parity_messages": msgs, "parity_span_groups": min(G, args.handler_span),
                     "parity_mismatches": int(bad)}
    out["note"] = ("raft_*_batch_dev on HBM-resident messages: per call a tile kernel (each tile's messages "
                   "partitioned stably into buckets of consecutive replicas), the handler kernel (a workgroup per bucket: "
                   "its messages gathered in batch order, sorted by replica in LDS, one lane per replica run) and "
                   "one status synchronisation; _host_buffers: the same through the host entry points from pageable "
                   "arrays (multi-threaded copy into engine-owned pinned staging, PCIe both ways); _pinned_host: from "
                   "page-locked arrays, which the DMA reads and writes directly. The engine holds the bench run's "
                   "final state; the messages are random (bench.handler_requests). roofline: the algorithmic bytes "
                   "per message (HANDLER_ALG_BYTES: message in, response out, the fields the reference's handler reads "
                   "and writes, its log[lastIndex-1] / log[prev] term read and an append's entry write) at the device rate; traffic: rocprofv3 "
                   "FETCH_SIZE + WRITE_SIZE of every kernel of the batch per message. Parity: a separate batch of "
                   "parity_messages messages over a span of groups, replayed by the oracle's handlers")
    return out

def side_leg(args, kw, mode, world, rank, local, dev, coll, log_cap, L, chunk, scaling, main_rows, comm=None):
    """The other scaling's leg of an N > 1 config-3 job, warmed up and timed
    exactly like the main leg (timed_leg).  Rank 0's weak shard holds global
    groups 0..groups-1, which the strong split covers over all ranks, so the
    strong leg's all-reduced counter rows must equal rank 0's weak-shard rows:
    beside a strong job (the default) this leg is weak scaling (every GPU its
    own --groups groups) and `main_rows` are the strong leg's all-reduced rows;
    beside a weak job it is config 4 (`main_rows`: rank 0's weak rows)."""
    eng_mod = importlib.import_module("raft-kotlin_amd.engine")
    import torch
    R = kw["R"]
    g0, G = shard(args.groups, world, rank, scaling)
    per_rank = [shard(args.groups, world, q, scaling)[1] for q in range(world)]
    total = sum(per_rank)
    flat = -(-G // (64 // R)) * 64 * log_cap * 8
    window = 0 if flat <= 0.6 * torch.cuda.get_device_properties(dev).total_memory else 256
    params = abi.make_params(log_cap=max(log_cap, window), log_window=window, steps_per_launch=L, mode=mode,
                             subranges=args.subranges, schedule=SCHEDULES[args.schedule], schedule_workgroups=args.schedule_workgroups,
                             ae_max_entries=args.ae_max_entries, **dict(kw, G=G, g0=g0))
    eng = eng_mod.RaftEngine(params, device=local)
    nsub = eng.subranges
    try:
        leg = timed_leg(eng, args, chunk, coll, dev, world, comm)
    finally:
        eng.close()
    c_all = leg["gcounters"].cpu().numpy()[:, : abi.NUM_COUNTERS]
    c_loc = leg["counters"].cpu().numpy()[:, : abi.NUM_COUNTERS]
    wc = leg["wcount"].cpu().numpy()[: args.warmup, : abi.NUM_COUNTERS]
    bad = int(c_all[:, abi.C_INDEX["log_overflow"]].sum() + c_all[:, abi.C_INDEX["log_window_miss"]].sum()
              + wc[:, abi.C_INDEX["log_overflow"]].sum() + wc[:, abi.C_INDEX["log_window_miss"]].sum())
    out = {"value": total * args.steps / leg["elapsed"], "unit": "group-steps/s", "scaling": scaling,
           "ms_per_step": leg["elapsed"] * 1e3 / args.steps, "groups_total": total, "groups_per_rank": per_rank,
           "steps_per_launch": L, "subranges": nsub, "log_window": window,
           "step_waves_per_rank": -(-G // (64 // R)),
           "grid_fill": grid_fill(G, R, L, R <= 5 or (R == 7 and abi.step_net_of(kw) == abi.NET_PART)),
           "kernel_avg_ms_per_rank": leg["kern_avg_per_rank"],
           "timing": {"wall_ms": leg["wall"] * 1e3, "stream_event_ms": leg["ev_ms"],
                      "step_kernel_ms_total": leg["kern_ms"], "allreduce_ms": leg["allreduce_ms"]},
           "valid": bad == 0}
    if scaling == "weak":
        out["note"] = ("weak scaling in the same job: every GPU its own --groups groups (contiguous global-id "
                       "ranges), the same steps, warmup and timing as the main leg; "
                       "counters_equal_strong_allreduced: rank 0's rows (global groups 0..groups-1) equal the "
                       "strong leg's all-reduced rows, which cover the same groups")
        if main_rows is not None:
            out["counters_equal_strong_allreduced"] = bool(np.array_equal(c_loc, main_rows))
    else:
        out["note"] = ("config 4 in the same job: the groups split by contiguous global id over the GPUs, the same "
                       "steps, warmup and timing as the main leg; counters_equal_rank0_weak_shard: its all-reduced "
                       "per-step counter rows equal rank 0's weak-leg rows, which cover the same global groups")
        if main_rows is not None:
            out["counters_equal_rank0_weak_shard"] = bool(np.array_equal(c_all, main_rows))
    return out

def general_kernel_leg(eng, args, chunk, dev, main_rows, main_kern_avg_ms):
    """The main leg again on the same engine (reset to step 0) with the
    general step kernel, which decides every network fault and the command
    harness at run time (raft_params.kernel = RAFT_KERNEL_GENERAL), where the
    main leg ran the kernel built for the workload (config 3: drops and churn,
    no partitions, commands to the lowest LEADER compiled in).  Same warmup,
    steps and launches; its counter rows must equal the main leg's."""
    eng.set_kernel(abi.KERNEL_GENERAL)
    eng.reset()
    try:
        leg = timed_leg(eng, args, chunk, False, dev, 1)
        info = eng.kernel_info()
    finally:
        eng.set_kernel(abi.KERNEL_AUTO)
    rows = leg["counters"].cpu().numpy()[:, : abi.NUM_COUNTERS]
    return {"value": eng.G * args.steps / leg["elapsed"], "unit": "group-steps/s",
            "kernel_net": info["net"], "kernel_avg_ms": leg["kern_avg_ms"],
            "kernel_time_vs_specialised": leg["kern_avg_ms"] / main_kern_avg_ms if main_kern_avg_ms else None,
            "counters_equal_main_leg": bool(np.array_equal(rows, main_rows)), "rehearsals": leg["rehearsals"],
            "note": "the same warmup, steps and launches on the same engine (reset to step 0) with the general "
                    "step kernel (NET_ALL: drops, partitions and isolation churn decided at run time, the command "
                    "harness read from the parameters); the main leg's kernel is built for the workload "
                    "(roofline.kernel_variant)"}

def plan_only(args, world, rank):
    """The rank/shard plumbing without a GPU (tests/test_bench_cpu.py)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    g0, n = shard(args.groups, world, rank, args.scaling)
    t = torch.tensor([rank, g0, n], dtype=torch.int64)
    rows = [torch.zeros_like(t) for _ in range(world)]
    if world > 1:
        dist.all_gather(rows, t)
    else:
        rows = [t]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "scaling": args.scaling,
                          "shards": [[int(x) for x in r.tolist()] for r in rows]}), flush=True)
    if world > 1:
        dist.destroy_process_group()
