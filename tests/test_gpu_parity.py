"""HIP engine vs the CPU oracle: bit-exact parity on the GPU (marker `gpu`).

Every comparison is exact (integer state machine): per-step counters, state
digests, full canonical state and logs up to physLen.  Sizes are chosen so the
oracle finishes in seconds; the full-size configuration is checked on a random
sample of groups (the oracle can run any subset of global group ids, since
groups are independent and all randomness is keyed by the global id).
"""
import ctypes as C
import importlib
import os

import numpy as np
import pytest

import oracle as O
from helpers import (abi, assert_same_logs, assert_same_state, blank_groups, fld, log_matching_flags, set_fld,
                     set_session, session)

pytestmark = pytest.mark.gpu

eng_mod = importlib.import_module("raft-kotlin_amd.engine")
RaftEngine = eng_mod.RaftEngine

NTHREADS = min(16, os.cpu_count() or 1)


def pair(**kw):
    p = abi.make_params(**kw)
    return RaftEngine(p), O.Oracle(abi.make_params(**kw))


def run_lockstep(e, o, steps, chunk, label, digest_every=1):
    done = 0
    while done < steps:
        k = min(chunk, steps - done)
        ce = e.step(k)
        co = o.step(k, nthreads=NTHREADS)[:, : abi.NUM_COUNTERS]
        if not np.array_equal(ce, co):
            bad = np.argwhere(ce != co)[0]
            raise AssertionError(f"{label}: counters differ at step {done + bad[0]} "
                                 f"({abi.COUNTER_NAMES[bad[1]]}): {ce[tuple(bad)]} vs {co[tuple(bad)]}")
        done += k
        if digest_every and (done // chunk) % digest_every == 0 and e.digest() != o.digest():
            se, so = e.read_state(), o.read_state()
            assert_same_state(se, so, e.R, f"{label} @ step {done}")
            assert_same_logs(se, e.read_log(), o.read_log(), e.R, f"{label} @ step {done}")
            raise AssertionError(f"{label}: digest differs after step {done} with equal state and logs")
    se, so = e.read_state(), o.read_state()
    assert_same_state(se, so, e.R, label)
    assert_same_logs(se, e.read_log(), o.read_log(), e.R, label)
    assert e.digest() == o.digest()
    ov = int(np.sum(se[:, [r * abi.NUM_FIELDS + abi.F_INDEX["phys"] for r in range(e.R)]] >= e.cap))
    return se, ov


def check_log_matching(e, o, label):
    """The kernel's Log Matching flags vs the numpy restatement on the oracle's logs."""
    so = o.read_state()
    t, c = o.read_log()
    want = log_matching_flags(so, t, c, e.R, int(e.p.log_window))
    n, got = e.check_log_matching(flags=True)
    assert np.array_equal(got, want), f"{label}: log-matching flags differ in {np.count_nonzero(got != want)} groups"
    assert n == int(want.sum())
    return n


def test_log_matching_check_crafted():
    """Flags exactly the groups whose replicas differ inside both committed prefixes."""
    R, G, cap = 3, 6, 16
    e = RaftEngine(abi.make_params(R=R, G=G, log_cap=cap))
    w = blank_groups(G, R)
    t = np.zeros((G, R, cap), np.int32)
    c = np.zeros((G, R, cap), np.uint32)
    for g in range(G):
        for r in range(R):
            set_fld(w, R, r, "last", 8)
            set_fld(w, R, r, "phys", 8)
            set_fld(w, R, r, "commit", 6)
            t[g, r, :8] = np.arange(1, 9)
            c[g, r, :8] = 100 + np.arange(8)
    c[1, 2, 5] += 1                      # inside every committed prefix -> flagged
    t[2, 1, 6] = 99                      # beyond the committed prefixes -> not flagged
    set_fld(w[3:4], R, 0, "commit", 3)   # replica 0's prefix is short ...
    t[3, 0, 3] = 99                      # ... so index 3 of it is not covered -> not flagged
    set_fld(w[4:5], R, 1, "last", 5)     # commit 6 > lastIndex 5 clamps to 5 ...
    t[4, 1, 5] = 77                      # ... so index 5 is not covered -> not flagged
    t[5, 0, 0] = 42                      # index 0 -> flagged
    e.write_state(w)
    e.write_log(t, c)
    n, f = e.check_log_matching(flags=True)
    want = log_matching_flags(w, t, c, R)
    assert list(f) == list(want)
    assert n == 2 and list(np.nonzero(f)[0]) == [1, 5]


def test_init_state_matches_oracle():
    e, o = pair(R=5, G=1000, seed=9, log_cap=16)
    assert_same_state(e.read_state(), o.read_state(), 5, "init")
    assert e.digest() == o.digest()


def test_config1_cluster_1000_commands():
    """BASELINE config 1: one 5-node cluster, election + 1000 replicated commands."""
    kw = dict(abi.CONFIGS[1])
    e, o = pair(log_cap=1100, **kw)
    steps = 0
    while True:
        run_lockstep(e, o, 50, 50, "config1")
        steps += 50
        s = e.read_state()[0]
        leaders = [r for r in range(5) if fld(s, 5, r, "role") == abi.LEADER]
        if leaders and fld(s, 5, leaders[0], "commit") >= 1000:
            break
        assert steps < 3000
    assert all(fld(s, 5, r, "commit") >= 999 for r in range(5))


def test_config2_parity_every_step():
    """BASELINE config 2 at full size: 10^4 x 3, no faults, 10^3 steps, parity every step."""
    kw = dict(abi.CONFIGS[2])
    e, o = pair(log_cap=400, **kw)
    run_lockstep(e, o, abi.CONFIG_STEPS[2], 10, "config2", digest_every=1)


@pytest.mark.parametrize("window", [0, 64])
def test_config3_drops_churn_reduced(window):
    """BASELINE config 3 semantics (5% drop + leader-isolation churn) at reduced
    G/steps, with every physical slot kept and on a 64-slot ring (the logs
    wrap ~10 times; no access misses it)."""
    kw = dict(abi.CONFIGS[3])
    kw.update(G=20_000, churn_ppm=5_000)
    e, o = pair(log_cap=768, log_window=window, **kw)
    se, ov = run_lockstep(e, o, 2_000, 100, f"config3 W={window}", digest_every=5)
    assert ov == 0
    check_log_matching(e, o, "config3")


def test_config5_partitions_reduced():
    """BASELINE config 5 semantics (R=7, partitions, commands to every leader) at reduced G/steps."""
    kw = dict(abi.CONFIGS[5])
    kw.update(G=2_000)
    e, o = pair(log_cap=2600, **kw)
    run_lockstep(e, o, 1_500, 100, "config5", digest_every=3)
    check_log_matching(e, o, "config5")


@pytest.mark.parametrize("R", [1, 2, 3, 4, 5, 6, 7, 8])
def test_other_replica_counts(R):
    """Drops, churn and partitions at every R: pins every staged and unstaged
    drop-word chunk layout of the reference kernel (R = 5, 7 included)."""
    e, o = pair(R=R, G=3000, seed=100 + R, log_cap=300, drop_ppm=100_000, churn_ppm=20_000, churn_steps=15,
                cmd_ppm=500_000, partition_period=40, partition_len=10)
    run_lockstep(e, o, 400, 50, f"R={R}")


NET_CASES = [(3, "drops+churn"), (5, "drops+churn"), (7, "drops+churn"), (5, "drops"), (3, "partitions"),
             (5, "partitions"), (7, "partitions"), (7, "partitions+churn"), (5, "none"), (5, "churn"),
             (5, "drops+all-leaders"), (5, "drops+limit")]


@pytest.mark.parametrize("R,faults", NET_CASES, ids=[f"{r}-{f}" for r, f in NET_CASES])
def test_network_fault_kernels(R, faults):
    """The step kernels built for the workload's network faults (raft_step.h
    NET_*: the engine picks them at R = 3, 5, 7 from raft_params), each
    against the oracle: drops (with and without isolation churn) on the
    drops + isolation kernel, partitions alone and no faults at all on the
    partitions-only kernel, and the mixes that need the NET_ALL kernel."""
    kw = dict(R=R, G=3000, seed=200 + R, log_cap=300, cmd_ppm=500_000)
    if "churn" in faults:
        kw.update(churn_ppm=20_000, churn_steps=15)
    if "drops" in faults:
        kw.update(drop_ppm=100_000)
    if "partitions" in faults:
        kw.update(partition_period=40, partition_len=10)
    if "all-leaders" in faults:
        kw.update(cmd_mode=abi.CMD_ALL_LEADERS)
    if "limit" in faults:
        kw.update(cmd_limit=30)
    low = abi.NET_DROP | abi.NET_ISO | abi.NET_CMDLOW
    want = {"drops+churn": low, "drops": low, "partitions": abi.NET_PART, "none": abi.NET_PART,
            "partitions+churn": abi.NET_ALL, "churn": abi.NET_ALL, "drops+all-leaders": abi.NET_ALL,
            "drops+limit": abi.NET_ALL}[faults]
    assert abi.step_net_of(kw) == want
    e, o = pair(**kw)
    run_lockstep(e, o, 400, 50, f"R={R} {faults}")


@pytest.mark.parametrize("mode", [abi.MODE_REFERENCE, abi.MODE_TEXTBOOK])
def test_log_overflow_on_engine(mode):
    """S-12 on the GPU: a log_cap too small for the run.  Appends beyond it
    are refused and counted (RAFT_C_LOG_OVERFLOW) in the same steps as the
    oracle counts them (tests/test_oracle_kats.py pins the oracle's rule), and
    the state and logs stay equal."""
    kw = dict(abi.CONFIGS[3], G=4000, churn_ppm=20_000, cmd_ppm=1_000_000, log_cap=40, mode=mode)
    e, o = pair(**kw)
    run_lockstep(e, o, 300, 50, f"overflow mode={mode}")
    e2 = RaftEngine(abi.make_params(**kw))
    c = e2.step(300)
    assert c[:, abi.C_INDEX["log_overflow"]].sum() > 0, "the run must overflow its log_cap"


def test_steps_per_launch_invariance():
    kw = dict(abi.CONFIGS[3])
    kw.update(G=5000, churn_ppm=10_000)
    digests = []
    # 600 = one full 512-step launch + 88; 433 / 434: the longest launch at 7
    # workgroups per CU and the shortest at 6 (STEP_K_7WG, raft_engine.hip)
    for k in (1, 7, 32, 128, abi.BENCH_STEPS_PER_LAUNCH, 433, 434, abi.LDS_MAX_STEPS_PER_LAUNCH, 600):
        e = RaftEngine(abi.make_params(log_cap=400, steps_per_launch=k, **kw))
        c = e.step(600)
        # one chunk per wave: a launch beyond the LDS rows is cut to 512 steps
        assert e.kernel_info()["steps"] == (88 if k == 600 else 600 % k or k)
        digests.append((e.digest(), c.tobytes()))
    # the balanced schedule (forced at this size): 450 steps per launch (LDS
    # rows, 6 workgroups per CU), 600 and 1,000 (one launch of 400-step epochs
    # and a shorter last one)
    for k in (450, 600, 1000):
        e = RaftEngine(abi.make_params(log_cap=400, steps_per_launch=k, schedule=abi.SCHED_BALANCED, **kw))
        c = e.step(600)
        info = e.kernel_info()
        assert info["balanced"] == 1 and info["steps"] == (600 % k or k)
        digests.append((e.digest(), c.tobytes()))
    # steps_per_launch changed mid-run (bench.py's streaming leg)
    e = RaftEngine(abi.make_params(log_cap=400, steps_per_launch=64, **kw))
    c1 = e.step(300)
    e.set_steps_per_launch(1)
    c2 = e.step(300)
    digests.append((e.digest(), np.concatenate([c1, c2]).tobytes()))
    assert all(d == digests[0] for d in digests)


@pytest.mark.parametrize("variant", ["ring", "general", "textbook", "partitions"])
def test_long_launch_kernel_variants(variant):
    """A forced-balanced launch of 700 steps (steps_per_launch 1,000): the ring
    and the general kernel run it as one launch of 400-step epochs; textbook
    mode and a partitions-only workload have no epochs kernel, so it is cut
    into 512 + 188.  Counters and digest equal 100-step launches, with kernel
    timing on for the long runs."""
    kw = dict(abi.CONFIGS[3], G=5000, churn_ppm=10_000)
    if variant == "ring":
        kw.update(log_window=64)
    elif variant == "textbook":
        kw.update(mode=abi.MODE_TEXTBOOK)
    elif variant == "partitions":
        kw = dict(abi.CONFIGS[5], G=3000)
    runs = []
    for k in (100, 1000):
        e = RaftEngine(abi.make_params(log_cap=2000, steps_per_launch=k, schedule=abi.SCHED_BALANCED, **kw))
        if variant == "general":
            e.set_kernel(abi.KERNEL_GENERAL)
        if k == 1000:
            e.set_kernel_timing(True)
        c = e.step(700)
        info = e.kernel_info()
        assert info["balanced"] >= 1
        if k == 1000:
            epochs = variant in ("ring", "general")
            assert info["steps"] == (700 if epochs else 188), info
            ms, launches = e.kernel_time()
            assert launches == (1 if epochs else 2) and ms > 0
        runs.append((e.digest(), c.tobytes()))
    assert runs[0] == runs[1]


def test_subrange_invariance():
    """Launch sub-ranges (raft_params.subranges: the grid split over 1-4
    streams, launches of different ranges overlapping, counter partials
    double-buffered) change nothing: per-step counters and the digest equal
    the one-range run at every launch length, also when the count changes
    mid-run and with kernel timing on."""
    kw = dict(abi.CONFIGS[3])
    kw.update(G=7000, churn_ppm=10_000)
    ref = None
    for k in (1, 37, abi.BENCH_STEPS_PER_LAUNCH):
        for n in (1, 2, 3, 4):
            e = RaftEngine(abi.make_params(log_cap=400, steps_per_launch=k, subranges=n, **kw))
            assert e.subranges == n
            e.set_kernel_timing(n == 3)
            c = e.step(600)
            if n == 3:
                ms, launches = e.kernel_time()
                assert launches == -(-600 // k) and ms > 0
            got = (e.digest(), c.tobytes())
            ref = ref or got
            assert got == ref, f"steps_per_launch {k}, {n} sub-ranges"
            e.close()
    e = RaftEngine(abi.make_params(log_cap=400, steps_per_launch=64, subranges=2, **kw))
    c1 = e.step(250)
    e.set_subranges(4)
    c2 = e.step(200)
    e.set_subranges(1)
    c3 = e.step(150)
    assert (e.digest(), np.concatenate([c1, c2, c3]).tobytes()) == ref


@pytest.fixture(scope="module")
def oracle_runs():
    """Oracle runs shared by the schedule tests: {name: (params kw, steps, counters, digest)}."""
    out = {}
    for name, kw, steps, cap in (
            ("c3", dict(abi.CONFIGS[3], G=4000, churn_ppm=10_000), 300, 200),
            ("c5", dict(abi.CONFIGS[5], G=2000), 300, 400),
            ("c2", dict(abi.CONFIGS[2], G=3000), 200, 200)):
        o = O.Oracle(abi.make_params(log_cap=cap, **kw))
        co = o.step(steps, nthreads=NTHREADS)[:, : abi.NUM_COUNTERS]
        out[name] = (dict(kw, log_cap=cap), steps, co, o.digest())
        o.close()
    return out


# (workgroups, steps per launch, sub-ranges): at G = 4000 x 5 there are 334
# chunks (64 // R groups each), so 1 workgroup takes all of them (each wave a
# quarter of 334 x K chunk-steps), 7 about 48 (heads and tails of every
# length), 83 four or five (the smallest split)
BALANCED_CASES = [(1, 20, 1), (3, 7, 1), (7, 37, 1), (7, 400, 1), (50, 20, 1), (83, 20, 1), (83, 1, 1),
                  (7, 64, 2), (40, 400, 3)]


@pytest.mark.parametrize("cfg", ["c3", "c5", "c2"])
@pytest.mark.parametrize("case", BALANCED_CASES, ids=[f"wg{a}-k{b}-sub{c}" for a, b, c in BALANCED_CASES])
def test_balanced_schedule_vs_oracle(oracle_runs, cfg, case):
    """The balanced schedule (raft_params.schedule): a
    workgroup's waves split its chunks' chunk-steps, a chunk passing from one
    wave to the next between two steps through HBM and an in-workgroup LDS
    flag.  Every per-step counter and the whole-run digest equal the oracle's
    (configs 3, 5 and 2 at reduced G: drops and churn, partitions -- redrawn at
    a piece's first step --, and R = 3)."""
    nwg, spl, nsub = case
    kw, steps, co, dg = oracle_runs[cfg]
    e = RaftEngine(abi.make_params(steps_per_launch=spl, subranges=nsub, schedule=abi.SCHED_BALANCED,
                                   schedule_workgroups=nwg, **kw))
    try:
        ce = e.step(steps)
        info = e.kernel_info()
        assert info["balanced"] == nsub and info["subranges"] == nsub
        assert info["workgroups"] <= nwg
        if not np.array_equal(ce, co):
            bad = np.argwhere(ce != co)[0]
            raise AssertionError(f"{cfg} {case}: counters differ at step {bad[0]} ({abi.COUNTER_NAMES[bad[1]]})")
        assert e.digest() == dg
    finally:
        e.close()


def test_one_per_wave_schedule_vs_oracle(oracle_runs):
    """The one-chunk-per-wave schedule, forced (RAFT_SCHED_ONE_PER_WAVE), on the same runs."""
    for cfg in ("c3", "c5", "c2"):
        kw, steps, co, dg = oracle_runs[cfg]
        e = RaftEngine(abi.make_params(steps_per_launch=37, schedule=abi.SCHED_ONE_PER_WAVE, **kw))
        ce = e.step(steps)
        assert e.kernel_info()["balanced"] == 0
        assert np.array_equal(ce, co) and e.digest() == dg, cfg
        e.close()


def test_kernel_info_names_the_launched_kernel():
    """raft_engine_kernel_info reports the NET variant the engine launched,
    which must be the one abi.step_net predicts (bench.py's launch lengths and
    occupancy assumptions rest on it), including an engine that would get the
    partitions-only kernel until write_state stores an isolation word."""
    cases = [dict(abi.CONFIGS[3], G=600), dict(abi.CONFIGS[5], G=600), dict(abi.CONFIGS[2], G=600),
             dict(abi.CONFIGS[3], G=600, partition_period=40, partition_len=10), dict(R=4, G=600, drop_ppm=1000)]
    for kw in cases:
        e = RaftEngine(abi.make_params(log_cap=64, **kw))
        e.step(1)
        assert e.kernel_info()["net"] == abi.step_net_of(kw), kw
        e.close()
    kw = dict(abi.CONFIGS[2], G=600)
    e = RaftEngine(abi.make_params(log_cap=64, **kw))
    e.step(1)
    assert e.kernel_info()["net"] == abi.NET_PART
    st = e.read_state()
    st[0, -2] = (3 << 8) | 1                              # replica 1 isolated for 3 steps
    e.write_state(st)
    e.step(1)
    assert e.kernel_info()["net"] == abi.step_net(3, iso_written=True) == abi.NET_ALL
    e.close()


@pytest.mark.parametrize("cfg", [3, 2])
def test_reset_then_general_kernel_equals_fresh_engine(cfg):
    """raft_engine_reset (a restarted node, RaftServer.kt:28-70, for every
    group) leaves the engine exactly as raft_engine_create does: an engine
    stepped N steps -- on config 2 after write_state stored an isolation
    word, which switches it to a NET_ISO kernel (step_net) -- then reset and
    switched to the general kernel (RAFT_KERNEL_GENERAL) steps N again to the
    counters, state, logs and digest of a fresh engine and of the oracle."""
    kw = dict(abi.CONFIGS[cfg], G=3000)
    if cfg == 3:
        kw["churn_ppm"] = 20_000
    steps, cap = 120, 128
    e = RaftEngine(abi.make_params(log_cap=cap, steps_per_launch=40, **kw))
    e.step(30)
    if cfg == 2:
        st = e.read_state()
        st[5, -2] = (4 << 8) | 1                          # replica 1 of group 5 isolated for 4 steps
        e.write_state(st)
        e.step(1)
        assert e.kernel_info()["net"] == abi.NET_ALL
    e.step(steps - 31)
    e.reset()
    assert e.step_index == 0
    e.set_kernel(abi.KERNEL_GENERAL)
    ce = e.step(steps)
    assert e.kernel_info()["net"] == abi.NET_ALL
    f = RaftEngine(abi.make_params(log_cap=cap, steps_per_launch=40, **kw))
    cf = f.step(steps)
    if cfg == 2:                                          # the fresh engine runs the partitions-only kernel
        assert f.kernel_info()["net"] == abi.NET_PART
    o = O.Oracle(abi.make_params(log_cap=cap, **kw))
    co = o.step(steps, nthreads=NTHREADS)[:, : abi.NUM_COUNTERS]
    assert np.array_equal(ce, cf) and np.array_equal(ce, co)
    se = e.read_state()
    assert_same_state(se, f.read_state(), kw["R"], "reset vs fresh")
    assert_same_state(se, o.read_state(), kw["R"], "reset vs oracle")
    assert_same_logs(se, e.read_log(), o.read_log(), kw["R"], "reset vs oracle")
    assert e.digest() == f.digest() == o.digest()
    e.close()
    f.close()


def test_traffic_probe_changes_nothing():
    """raft_engine_traffic_probe (the rocprofv3 calibration dispatches) moves
    exactly the bytes it reports and changes no result: the state probe writes
    every value back unchanged, the log-store probe writes only past physLen
    (never read, not in the digest); the engine then steps on to the oracle's
    counters and digest."""
    kw = dict(abi.CONFIGS[3], G=2000, churn_ppm=20_000)
    e, o = pair(log_cap=96, **kw)
    ce = e.step(40)
    co = o.step(40, nthreads=NTHREADS)[:, : abi.NUM_COUNTERS]
    assert np.array_equal(ce, co)
    d0, s0 = e.digest(), e.read_state()
    state = kw["G"] * (5 * abi.REPLICA_STATE_BYTES + abi.GROUP_STATE_BYTES)
    assert e.traffic_probe(0) == (state, state)
    phys = s0[:, [r * abi.NUM_FIELDS + abi.F_INDEX["phys"] for r in range(5)]]
    assert e.traffic_probe(1) == (4 * kw["G"] * 5, 8 * int(np.count_nonzero(phys < 96)))
    # the handler batches' scattered-access probes: 2^21 sectors of 32 B, in engine scratch
    assert e.traffic_probe(2) == (32 << 21, 0)
    assert e.traffic_probe(3) == (0, 32 << 21)
    assert e.digest() == d0 and np.array_equal(e.read_state(), s0)
    ce = e.step(40)
    co = o.step(40, nthreads=NTHREADS)[:, : abi.NUM_COUNTERS]
    assert np.array_equal(ce, co) and e.digest() == o.digest()
    w = RaftEngine(abi.make_params(log_cap=128, log_window=64, **kw))
    with pytest.raises(eng_mod.RaftError):
        w.traffic_probe(1)                                # a ring has no slot past its last entry to spare
    w.close()


def test_shard_invariance():
    """Config 4's contract: sharding by global group id does not change any group."""
    kw = dict(abi.CONFIGS[3])
    kw.update(G=4000, churn_ppm=10_000)
    full = RaftEngine(abi.make_params(log_cap=200, **kw))
    cf = full.step(200)
    parts, cs = [], []
    for g0, n in ((0, 1500), (1500, 2500)):
        e = RaftEngine(abi.make_params(log_cap=200, **dict(kw, G=n, g0=g0)))
        cs.append(e.step(200))
        parts.append(e)
    assert np.array_equal(cf, cs[0] + cs[1])
    assert full.digest() == (parts[0].digest() + parts[1].digest()) % (1 << 64)
    assert np.array_equal(full.read_state(1500, 2500), parts[1].read_state())


def test_full_size_config3_sampled():
    """10^6 x 5 groups at full size on the GPU; a random sample re-run by the oracle."""
    kw = dict(abi.CONFIGS[3])
    steps = 600
    e = RaftEngine(abi.make_params(log_cap=256, **kw))
    ce = e.step(steps)
    rng = np.random.default_rng(0)
    sample = np.sort(rng.choice(kw["G"], size=48, replace=False))
    se = e.read_state()
    for gid in sample:
        o = O.Oracle(abi.make_params(log_cap=256, **dict(kw, G=1, g0=int(gid))))
        o.step(steps)
        assert_same_state(se[gid:gid + 1], o.read_state(), 5, f"group {gid}")
        assert_same_logs(se[gid:gid + 1], e.read_log(int(gid), 1), o.read_log(), 5, f"group {gid}")
    # size-independent properties at full size
    assert ce[:, abi.C_INDEX["log_overflow"]].sum() == 0
    assert ce[-1, abi.C_INDEX["groups_with_leader"]] > 0.9 * kw["G"]
    last = se[:, [r * abi.NUM_FIELDS + abi.F_INDEX["last"] for r in range(5)]]
    phys = se[:, [r * abi.NUM_FIELDS + abi.F_INDEX["phys"] for r in range(5)]]
    assert np.all(last <= phys) and np.all(last >= 0)


# ---- RAFT_MODE_TEXTBOOK (opt-in, not the reference) ------------

@pytest.mark.parametrize("cfg", [2, 3, 5, "3w"])
def test_textbook_lockstep(cfg):
    """The textbook kernel (step_kernel<R, true>) against the oracle's textbook
    mode, bit-exact, and its committed prefixes Log-Matching clean ("3w": on a
    64-slot ring)."""
    win = 64 if cfg == "3w" else 0
    cfg = 3 if cfg == "3w" else cfg
    kw = dict(abi.CONFIGS[cfg], mode=abi.MODE_TEXTBOOK, log_window=win)
    kw.update({2: dict(G=5_000), 3: dict(G=10_000, churn_ppm=10_000), 5: dict(G=1_000)}[cfg])
    steps, cap = {2: (400, 200), 3: (1_200, 500), 5: (1_200, 1_400)}[cfg]
    e, o = pair(log_cap=cap, steps_per_launch=32, **kw)
    se, ov = run_lockstep(e, o, steps, 100, f"textbook config{cfg}", digest_every=4)
    assert ov == 0
    assert check_log_matching(e, o, f"textbook config{cfg}") == 0


@pytest.mark.parametrize("R", [1, 2, 3, 4, 5, 7, 8])
def test_textbook_other_replica_counts(R):
    e, o = pair(R=R, G=2000, seed=200 + R, log_cap=300, drop_ppm=100_000, churn_ppm=20_000, churn_steps=15,
                cmd_ppm=500_000, partition_period=40, partition_len=10, mode=abi.MODE_TEXTBOOK)
    run_lockstep(e, o, 400, 50, f"textbook R={R}")
    assert check_log_matching(e, o, f"textbook R={R}") == 0


@pytest.mark.parametrize("cfg", [2, 3, "3w", 5])
def test_textbook_multi_entry_lockstep(cfg):
    """Textbook mode with up to 8 entries per AppendEntries request
    (ae_max_entries, greeter.proto:37) against the oracle, bit-exact ("3w": on
    a 64-slot ring, window misses counted as the oracle counts them)."""
    win = 64 if cfg == "3w" else 0
    cfg = 3 if cfg == "3w" else cfg
    kw = dict(abi.CONFIGS[cfg], mode=abi.MODE_TEXTBOOK, log_window=win, ae_max_entries=8)
    kw.update({2: dict(G=5_000), 3: dict(G=10_000, churn_ppm=10_000), 5: dict(G=1_000)}[cfg])
    steps, cap = {2: (400, 200), 3: (1_200, 500), 5: (1_200, 1_400)}[cfg]
    e, o = pair(log_cap=cap, steps_per_launch=32, **kw)
    se, ov = run_lockstep(e, o, steps, 100, f"textbook x8 config{cfg}", digest_every=4)
    assert ov == 0
    assert check_log_matching(e, o, f"textbook x8 config{cfg}") == 0


@pytest.mark.parametrize("E", [2, 3, 5])
@pytest.mark.parametrize("R", [1, 2, 3, 5, 7, 8])
def test_textbook_multi_entry_replica_counts(R, E):
    e, o = pair(R=R, G=2000, seed=300 + R, log_cap=300, drop_ppm=100_000, churn_ppm=20_000, churn_steps=15,
                cmd_ppm=500_000, partition_period=40, partition_len=10, mode=abi.MODE_TEXTBOOK, ae_max_entries=E)
    run_lockstep(e, o, 400, 50, f"textbook x{E} R={R}")
    assert check_log_matching(e, o, f"textbook x{E} R={R}") == 0


def test_textbook_multi_entry_kat_on_engine():
    """tests/test_textbook_cpu.py's hand-derived multi-entry tick, replayed
    through the engine (write_state + write_log + step)."""
    import test_textbook_cpu as T
    o = T._multi_entry_group(4, [(1, 7), (2, 8), (1, 51)])
    e = RaftEngine(abi.make_params(R=3, G=1, log_cap=64, mode=abi.MODE_TEXTBOOK, ae_max_entries=4))
    e.write_state(o.read_state())
    e.write_log(*o.read_log())
    for _ in range(2):
        assert np.array_equal(e.step(1), o.step(1)[:, : abi.NUM_COUNTERS])
        assert np.array_equal(e.read_state(), o.read_state())
    assert e.digest() == o.digest()


FULL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "full_size.json")


# (config, log_window, steps_per_launch).  Config 3's bench kernel is the flat
# log (log_window 0: every slot, 130 GB at log_cap 3064), step_kernel<5, false,
# false> at 7 waves per SIMD, launched at K = 400 by default and K = 20 by the
# driver's `--steps 20` command; the 256-slot ring is step_kernel<5, false,
# true> (7 waves as well).  Config 5 is always flat; bench.py launches it at K = 400
# (the partitions-only R = 7 kernel at 7 waves per SIMD; K = 500 and 512 run
# it at 6 workgroups per CU).
# A fourth element is the launch sub-ranges (streams; default: the engine's
# automatic choice, 1 for config 3 and 3 for config 5), a fifth the schedule
# (default automatic: balanced for config 3, whose chunks outnumber the
# resident wave slots; one chunk per wave for config 5's partitions-only
# kernel).  (3, 0, 20, 1) is the driver's exact timed launch.
ONE, BAL = abi.SCHED_ONE_PER_WAVE, abi.SCHED_BALANCED
FULL_SIZE_CASES = [
    (3, 0, 1), (3, 0, 20, 1), (3, 0, 20, 1, ONE), (3, 0, abi.BENCH_STEPS_PER_LAUNCH),
    (3, 0, abi.BENCH_STEPS_PER_LAUNCH, 3), (3, 0, abi.BENCH_STEPS_PER_LAUNCH, 3, ONE),
    (3, 256, 1), (3, 256, abi.BENCH_STEPS_PER_LAUNCH), (3, 256, abi.LDS_MAX_STEPS_PER_LAUNCH),
    (5, 0, 1), (5, 0, abi.BENCH_STEPS_PER_LAUNCH), (5, 0, 500), (5, 0, abi.LDS_MAX_STEPS_PER_LAUNCH),
    (5, 0, abi.BENCH_STEPS_PER_LAUNCH, 3), (5, 0, 500, 4, ONE), (5, 0, abi.BENCH_STEPS_PER_LAUNCH, 1, BAL),
    # the bench default's one 10^4-step launch (25 epochs of 400 steps); the
    # ring the same way; config 5's sub-ranges cut it to 512-step launches
    (3, 0, abi.LONG_STEPS_PER_LAUNCH), (3, 256, abi.LONG_STEPS_PER_LAUNCH), (5, 0, abi.LONG_STEPS_PER_LAUNCH),
]


def _full_id(case):
    c, w, k = case[:3]
    return (f"{c}-{'flat' if w == 0 else f'ring{w}'}-{k}" + (f"-sub{case[3]}" if len(case) > 3 else "")
            + ("-onewave" if len(case) > 4 and case[4] == ONE else "")
            + ("-balanced" if len(case) > 4 and case[4] == BAL else ""))


@pytest.mark.parametrize("case", FULL_SIZE_CASES, ids=[_full_id(c) for c in FULL_SIZE_CASES])
def test_full_size_digest(case):
    """The north star's full-size runs, bit-exact: config 3 (10^6 x 5, 10^4
    steps) and config 5 (10^5 x 7, 10^4 steps) on the GPU against the oracle's
    whole-run digest (state, sessions and every retained log slot of every
    group) and its per-step counters, precomputed on the CPU by
    tests/golden/make_full_size.py.  For config 3 the flat-log cases are the
    exact kernel bench.py times (the digest over every physical slot,
    `digest_full_log`), at the driver's launch length (20), 400, the bench
    default (one 10^4-step launch of 400-step epochs) and one step per
    launch; the ring cases check the 256-slot window (`digest`: the retained
    slots only)."""
    import json
    cfg, window, spl = case[:3]
    nsub = case[3] if len(case) > 3 else 0
    sched = case[4] if len(case) > 4 else abi.SCHED_AUTO
    meta = json.load(open(FULL))[f"c{cfg}"]
    want = np.load(os.path.join(os.path.dirname(FULL), "full_size_counters.npz"))[f"c{cfg}_counters"]
    kw = dict(abi.CONFIGS[cfg])
    assert meta["groups"] == kw["G"] and meta["params"] == {k: v for k, v in kw.items() if k != "G"}
    e = RaftEngine(abi.make_params(log_cap=meta["log_cap"], log_window=window, steps_per_launch=spl,
                                   subranges=nsub, schedule=sched, **kw))
    try:
        ce = e.step(meta["steps"])
        one = sched == ONE or (sched == abi.SCHED_AUTO and abi.step_net_of(kw) == abi.NET_PART)
        assert e.kernel_info()["balanced"] == (0 if one else e.subranges)
        if nsub == 0:
            assert e.subranges == (3 if abi.step_net_of(kw) == abi.NET_PART else 1)
        if not np.array_equal(ce, want):
            bad = np.argwhere(ce != want)[0]
            raise AssertionError(f"config {cfg}: counters differ at step {bad[0]} ({abi.COUNTER_NAMES[bad[1]]}): "
                                 f"{ce[tuple(bad)]} vs {want[tuple(bad)]}")
        golden = meta["digest"] if window == meta["log_window"] else meta["digest_full_log"]
        if window == 0:
            assert meta["digest_full_log"] == golden
        assert f"{e.digest():016x}" == golden, f"config {cfg}: whole-run digest differs"
        assert ce[:, abi.C_INDEX["log_overflow"]].sum() == 0
        assert ce[:, abi.C_INDEX["log_window_miss"]].sum() == 0
    finally:
        e.close()


@pytest.mark.parametrize("n", [2, 4, 8])
def test_config4_strong_split_full_size(n):
    """BASELINE config 4 at full size on one GPU: config 3's 10^6 x 5 groups
    split into n contiguous global-id shards (bench.shard, "strong": the
    ranks of `bench.py --gpus n`), each its own engine at its global offset
    g0, created and closed in turn, for 10^4 steps -- at the driver's launch
    (20 steps, one sub-range), at 400 and in one 10^4-step launch (epochs).
    The summed
    per-step counter rows equal the oracle's for the whole 10^6 groups
    (full_size_counters.npz) and the digests sum (mod 2^64) to its whole-run
    digest over every physical slot (the digest is a sum over groups)."""
    import json
    import bench
    meta = json.load(open(FULL))["c3"]
    want = np.load(os.path.join(os.path.dirname(FULL), "full_size_counters.npz"))["c3_counters"]
    kw = dict(abi.CONFIGS[3])
    for spl in (20, abi.BENCH_STEPS_PER_LAUNCH, abi.LONG_STEPS_PER_LAUNCH):
        total = np.zeros_like(want)
        dsum = 0
        for rank in range(n):
            g0, G = bench.shard(kw["G"], n, rank, "strong")
            e = RaftEngine(abi.make_params(log_cap=meta["log_cap"], steps_per_launch=spl, subranges=1,
                                           **dict(kw, G=G, g0=g0)))
            try:
                total += e.step(meta["steps"])
                dsum = (dsum + e.digest()) % (1 << 64)
                assert e.kernel_info()["balanced"] == 1          # every shard outnumbers the wave slots
            finally:
                e.close()
        if not np.array_equal(total, want):
            bad = np.argwhere(total != want)[0]
            raise AssertionError(f"{n} shards, K = {spl}: counters differ at step {bad[0]} "
                                 f"({abi.COUNTER_NAMES[bad[1]]}): {total[tuple(bad)]} vs {want[tuple(bad)]}")
        assert f"{dsum:016x}" == meta["digest_full_log"], f"{n} shards, K = {spl}: digest sum differs"


def test_full_size_config3_1e5_steps_on_the_ring():
    """config 3 at 10^6 x 5 for 10^5 steps on the bench's 256-slot ring
    (log_window): 10 GB of log where a flat log would need 1.2 TB.  No access
    misses the window and no log overflows (whole engine); groups [0, 10^4)
    equal the oracle's digest (tests/golden/make_full_size.py, "c3long")."""
    import json
    meta = json.load(open(FULL))["c3long"]
    kw = dict(abi.CONFIGS[3])
    e = RaftEngine(abi.make_params(log_cap=meta["log_cap"], log_window=meta["log_window"],
                                   steps_per_launch=500, **kw))
    assert e.device_bytes < 16 * 2 ** 30
    ce = e.step(meta["steps"])
    assert ce[:, abi.C_INDEX["log_overflow"]].sum() == 0
    assert ce[:, abi.C_INDEX["log_window_miss"]].sum() == 0
    assert f"{e.digest_range(0, meta['sample_groups']):016x}" == meta["digest"]
    # (by step 10^5 only ~17 % of the groups have a leader: the reference's
    # quirks keep terms racing -- an observation the oracle sample shares)
    assert ce[-1, abi.C_INDEX["groups_with_leader"]] > 0
    e.close()


def test_window_misses_are_counted():
    """A ring too small for the run (16 slots under 10 % drops and partitions):
    the engine counts its first misses in the same step as the oracle, and
    every step before it is bit-identical (the run is invalid from there on)."""
    kw = dict(R=5, G=3000, seed=105, log_cap=300, drop_ppm=100_000, churn_ppm=20_000, churn_steps=15,
              cmd_ppm=500_000, partition_period=40, partition_len=10, log_window=16)
    e, o = pair(**kw)
    mi = abi.C_INDEX["log_window_miss"]
    for t in range(200):
        ce, co = e.step(1), o.step(1)[:, : abi.NUM_COUNTERS]
        if co[0, mi]:
            assert ce[0, mi] == co[0, mi], f"step {t}: the oracle counts {co[0, mi]} misses, the engine {ce[0, mi]}"
            assert np.array_equal(ce, co), f"step {t}: counters of the first-miss step"
            return
        assert np.array_equal(ce, co), f"step {t}"
        assert e.digest() == o.digest(), f"step {t}"
    raise AssertionError("no miss in 200 steps")


# ---- the service boundary: single handlers vs the oracle -------------------------

def random_states(rng, n, R, cap):
    w = blank_groups(n, R)
    logs_t = rng.integers(0, 4, size=(n, R, cap)).astype(np.int32)
    logs_t.sort(axis=2)
    logs_c = rng.integers(0, 1 << 32, size=(n, R, cap), dtype=np.uint64).astype(np.uint32)
    for r in range(R):
        phys = rng.integers(0, cap + 1, size=n)
        last = (phys * rng.random(n)).astype(np.int32)
        set_fld(w, R, r, "phys", phys)
        set_fld(w, R, r, "last", last)
        set_fld(w, R, r, "term", rng.integers(0, 5, size=n))
        set_fld(w, R, r, "voted", rng.integers(-1, R + 1, size=n))
        set_fld(w, R, r, "role", rng.integers(0, 3, size=n))
        set_fld(w, R, r, "commit", rng.integers(0, 6, size=n))
        set_fld(w, R, r, "flags", rng.choice([0, abi.FL_ARMED, abi.FL_ELECTING, abi.FL_ELECTING | abi.FL_PENDING_RST],
                                             size=n))
    return w, logs_t, logs_c


def random_ring_states(rng, n, R, cap, window):
    """States for a log_window ring whose handler batches stay inside the
    window: physLen up to cap (the ring wraps), lastIndex at most window / 2
    below it, so every Log.get / overwrite the requests below make reads a
    retained slot."""
    w, logs_t, logs_c = random_states(rng, n, R, cap)
    for r in range(R):
        phys = rng.integers(0, cap + 1, size=n)
        last = np.maximum(0, phys - rng.integers(0, window // 2, size=n))
        set_fld(w, R, r, "phys", phys)
        set_fld(w, R, r, "last", last)
    return w, logs_t, logs_c


def handler_messages(rng, n, G, R, cap, w=None, window=0):
    """n random (group, dst) and vote / append / command requests; on a ring
    (window > 0) the indices they read stay within window / 4 of the target's
    lastIndex (see random_ring_states)."""
    grp = rng.integers(0, G, size=n)
    dst = rng.integers(0, R, size=n).astype(np.int32)
    if window:
        last = np.array([fld(w[g], R, d, "last") for g, d in zip(grp, dst)])
        phys = np.array([fld(w[g], R, d, "phys") for g, d in zip(grp, dst)])
        li = np.maximum(0, last - rng.integers(0, 4, n))
        prev = last - 1 - rng.integers(0, window // 4, n)
        prev = np.where(prev < phys - window + window // 4, np.maximum(last - 1, -1), prev)
        prev = np.where((prev < 0) & (phys > window // 2), last - 1, np.maximum(prev, -1))
    else:
        li = rng.integers(0, cap + 1, n)
        prev = rng.integers(-1, cap, n)
    vq = np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), li, rng.integers(0, 4, n)],
                  axis=1).astype(np.int32)
    aq = np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), prev,
                   rng.integers(-1, 4, n), rng.integers(0, 2, n), rng.integers(0, 6, n),
                   rng.integers(0, 1 << 32, n, dtype=np.uint64), rng.integers(0, 8, n)], axis=1).astype(np.int64)
    cmd = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    return grp, dst, vq, aq, cmd


HANDLER_CASES = [
    # (R, mode, G, n, log_window): long per-replica runs (G = 64 groups: ~15-50
    # messages per replica), many replicas (10^5 messages), one group (runs of
    # ~800 per replica through the radix sort's passes), and the ring
    *[(R, abi.MODE_REFERENCE, 64, 10_000, 0) for R in (3, 5, 7)],
    *[(R, abi.MODE_REFERENCE, 4000, 100_000, 0) for R in (3, 5, 7)],
    (5, abi.MODE_TEXTBOOK, 64, 3000, 0), (7, abi.MODE_TEXTBOOK, 64, 3000, 0),
    (5, abi.MODE_REFERENCE, 1, 4000, 0),
    *[(R, abi.MODE_REFERENCE, 2000, 10_000, 64) for R in (3, 5, 7)],
]


@pytest.mark.parametrize("R,mode,G,n,window", HANDLER_CASES,
                         ids=[f"R{c[0]}-{'tb' if c[1] else 'ref'}-G{c[2]}-n{c[3]}-w{c[4]}" for c in HANDLER_CASES])
def test_handler_batches_vs_oracle(R, mode, G, n, window):
    """The single-handler batches (RaftServer.vote() / append() /
    appendCommand(), RaftServer.kt:228-287, :100-107) against the oracle's
    handlers message by message, at the replica counts of every BASELINE
    configuration (R = 3, 5, 7; batch_kernel takes R at run time), on a flat
    log and on a 64-slot log_window ring whose rows have wrapped."""
    rng = np.random.default_rng(7 + R + 10 * window)
    cap = 160 if window else 8
    if window:
        w, lt, lc = random_ring_states(rng, G, R, cap, window)
    else:
        w, lt, lc = random_states(rng, G, R, cap)
    grp, dst, vq, aq, cmd = handler_messages(rng, n, G, R, cap, w, window)
    se = check_handler_batches(R, G, cap, window, mode, w, lt, lc, grp, dst, vq, aq, cmd)
    if window:
        # the rows wrapped: some replica holds more physical slots than the ring
        assert int(np.max(se[:, [r * abi.NUM_FIELDS + abi.F_INDEX["phys"] for r in range(R)]])) > window


def check_handler_batches(R, G, cap, window, mode, w, lt, lc, grp, dst, vq, aq, cmd):
    """A vote, an append and a command batch of the same (group, dst) on two
    engines -- the bucketed batch path (the default) and the sorted one --
    against the oracle's handlers applied message by message in batch order;
    returns the bucketed engine's final state."""
    o = O.Oracle(abi.make_params(R=R, G=G, log_cap=cap, log_window=window, seed=3, mode=mode))
    engines = []
    for path in (abi.BATCH_PATH_BUCKETED, abi.BATCH_PATH_SORTED):
        e = RaftEngine(abi.make_params(R=R, G=G, log_cap=cap, log_window=window, seed=3, mode=mode))
        e.set_batch_path(path)
        engines.append(e)
    for x in (*engines, o):
        x.write_state(w)
        x.write_log(lt, lc)
    vo = np.array([o.vote(int(g), int(d), *map(int, q)) for g, d, q in zip(grp, dst, vq)], dtype=np.int32)
    ao = []
    for g, d, q in zip(grp, dst, aq):
        t, s, st = o.append(int(g), int(d), int(q[0]), int(q[1]), int(q[2]), int(q[3]),
                            (int(q[5]), int(q[6])) if q[4] else None, int(q[7]))
        ao.append((t, int(s), st))
    ao = np.array(ao, dtype=np.int32)
    for g, d, c in zip(grp, dst, cmd):
        o.append_command(int(g), int(d), int(c))
    so = o.read_state()
    for e, name in zip(engines, ("bucketed", "sorted")):
        ve = e.vote_batch(grp, dst, vq)
        assert np.array_equal(ve, vo), f"{name}: vote responses differ at {np.argwhere(np.any(ve != vo, axis=1))[:3].ravel()}"
        ae = e.append_batch(grp, dst, aq)
        assert np.array_equal(ae, ao), f"{name}: append responses differ at {np.argwhere(np.any(ae != ao, axis=1))[:3].ravel()}"
        e.append_command_batch(grp, dst, cmd)
        se = e.read_state()
        assert_same_state(se, so, R, f"{name} handlers")
        assert_same_logs(se, e.read_log(), o.read_log(), R, f"{name} handlers")
    return engines[0].read_state()


def test_handler_batches_skewed_vs_oracle():
    """Half of the messages to one replica (a run of ~3000 across many of the
    bucketed path's 256-message chunks, and a bucket far above the mean), the
    rest random: both batch paths against the oracle."""
    rng = np.random.default_rng(29)
    R, G, cap, n = 5, 300, 8, 6000
    w, lt, lc = random_states(rng, G, R, cap)
    grp, dst, vq, aq, cmd = handler_messages(rng, n, G, R, cap)
    hot = rng.random(n) < 0.5
    grp = np.where(hot, 7, grp)
    dst = np.where(hot, 2, dst).astype(np.int32)
    check_handler_batches(R, G, cap, 0, abi.MODE_REFERENCE, w, lt, lc, grp, dst, vq, aq, cmd)


@pytest.mark.parametrize("n", [1, 2, 63, 65, 4095, 4097])
def test_handler_batches_ragged_sizes_vs_oracle(n):
    """Batch sizes around the bucketed path's wave (64) and tile (4096)
    boundaries, a single message included: both paths against the oracle."""
    rng = np.random.default_rng(41 + n)
    R, G, cap = 5, 50, 8
    w, lt, lc = random_states(rng, G, R, cap)
    grp, dst, vq, aq, cmd = handler_messages(rng, n, G, R, cap)
    check_handler_batches(R, G, cap, 0, abi.MODE_REFERENCE, w, lt, lc, grp, dst, vq, aq, cmd)


@pytest.mark.parametrize("path", ["bucketed", "sorted"])
def test_batch_status_between_batches(path):
    """Each batch's status is its own: a batch with a message outside the
    engine fails with RAFT_ERANGE and applies nothing; the batches before and
    after it (of other sizes, which move the staging) apply exactly as the
    oracle's handlers; on a log_window ring a batch that reads below the window
    reports RAFT_EWINDOW, and the next batch reports nothing."""
    pid = abi.BATCH_PATH_BUCKETED if path == "bucketed" else abi.BATCH_PATH_SORTED
    rng = np.random.default_rng(53)
    R, G, cap = 5, 300, 8
    w, lt, lc = random_states(rng, G, R, cap)
    e, o = pair(R=R, G=G, log_cap=cap, seed=3)
    e.set_batch_path(pid)
    for x in (e, o):
        x.write_state(w)
        x.write_log(lt, lc)
    for n, bad in ((5000, False), (3000, True), (70_000, False), (40, False)):
        grp, dst, vq, _, _ = handler_messages(rng, n, G, R, cap)
        if bad:
            grp = grp.copy()
            grp[n // 3] = G
            before = e.read_state()
            with pytest.raises(RuntimeError, match="outside the engine"):
                e.vote_batch(grp, dst, vq)
            assert np.array_equal(e.read_state(), before), "a failed batch applied something"
            continue
        ve = e.vote_batch(grp, dst, vq)
        vo = np.array([o.vote(int(g), int(d), *map(int, q)) for g, d, q in zip(grp, dst, vq)], dtype=np.int32)
        assert np.array_equal(ve, vo), f"n={n}: vote responses differ"
    assert_same_state(e.read_state(), o.read_state(), R, f"{path} after a failed batch")
    # the ring: physLen = lastIndex = 100 with a 16-slot window
    W, cap2 = 16, 200
    r = RaftEngine(abi.make_params(R=R, G=4, log_cap=cap2, log_window=W, seed=3))
    r.set_batch_path(pid)
    w2 = blank_groups(4, R)
    for q in range(R):
        set_fld(w2, R, q, "phys", np.full(4, 100))
        set_fld(w2, R, q, "last", np.full(4, 100))
        set_fld(w2, R, q, "term", np.full(4, 3))
    r.write_state(w2)
    r.write_log(np.full((4, R, cap2), 3, dtype=np.int32), np.zeros((4, R, cap2), dtype=np.uint32))
    n = 4 * R
    grp, dst = np.repeat(np.arange(4), R), np.tile(np.arange(R), 4).astype(np.int32)
    aq = np.zeros((n, 8), dtype=np.int64)
    aq[:, 0], aq[:, 1], aq[:, 2], aq[:, 3] = 3, 1, 10, 3              # prevLogIndex 10: below physLen - W
    with pytest.raises(RuntimeError, match=f"{n} log accesses below the retained log_window"):
        r.append_batch(grp, dst, aq)
    vq = np.zeros((n, 4), dtype=np.int32)
    vq[:, 0], vq[:, 1], vq[:, 2], vq[:, 3] = 3, 1, 100, 3
    r.vote_batch(grp, dst, vq)                                          # inside the window: no status left over


@pytest.mark.parametrize("path", ["bucketed", "sorted"])
def test_ring_window_misses_in_a_multi_chunk_bucket(path):
    """A bucket above the bucketed path's 512-message chunk, on a log_window
    ring, whose every message reads below the window: 1,200 appends to the 8
    replicas of one bucket (three chunks, runs of ~150 per replica), each
    Log.get(prevLogIndex) a miss -- the batch reports exactly 1,200 (each chunk
    adds its own to the count), and the vote batch after it reports nothing."""
    pid = abi.BATCH_PATH_BUCKETED if path == "bucketed" else abi.BATCH_PATH_SORTED
    R, G, W, cap2 = 5, 4, 16, 200
    r = RaftEngine(abi.make_params(R=R, G=G, log_cap=cap2, log_window=W, seed=3))
    r.set_batch_path(pid)
    w2 = blank_groups(G, R)
    for q in range(R):
        set_fld(w2, R, q, "phys", np.full(G, 100))
        set_fld(w2, R, q, "last", np.full(G, 100))
        set_fld(w2, R, q, "term", np.full(G, 3))
    r.write_state(w2)
    r.write_log(np.full((G, R, cap2), 3, dtype=np.int32), np.zeros((G, R, cap2), dtype=np.uint32))
    rng = np.random.default_rng(61)
    n = 1200
    key = rng.integers(0, 8, n)                                        # keys g * R + d in [0, 8): one bucket (S = 3)
    grp, dst = (key // R).astype(np.int64), (key % R).astype(np.int32)
    aq = np.zeros((n, 8), dtype=np.int64)
    aq[:, 0], aq[:, 1], aq[:, 2], aq[:, 3] = 3, 1, 10, 3              # prevLogIndex 10 < physLen - W, no entry
    with pytest.raises(RuntimeError, match=f"{n} log accesses below the retained log_window"):
        r.append_batch(grp, dst, aq)
    vq = np.zeros((n, 4), dtype=np.int32)
    vq[:, 0], vq[:, 1], vq[:, 2], vq[:, 3] = 3, 1, 100, 3
    r.vote_batch(grp, dst, vq)                                          # inside the window: no status left over


def test_ring_multi_chunk_buckets_vs_oracle():
    """Hot replicas on a wrapped 64-slot ring: 60 % of 8,000 messages go to 3
    replicas of one bucket (a bucket of ~5,000 messages: ten 512-message
    chunks applied in order by one workgroup), every access inside the window;
    both batch paths against the oracle message by message."""
    rng = np.random.default_rng(67)
    R, G, cap, window, n = 5, 400, 160, 64, 8000
    w, lt, lc = random_ring_states(rng, G, R, cap, window)
    hot_g, hot_d = rng.integers(0, 3, n), rng.integers(0, 3, n)
    grp, dst, vq, aq, cmd = handler_messages(rng, n, G, R, cap, w, window)
    hot = rng.random(n) < 0.6
    grp = np.where(hot, hot_g, grp)
    dst = np.where(hot, hot_d, dst).astype(np.int32)
    # every message's indices drawn against its own (final) target (handler_messages' rule)
    last = np.array([fld(w[g], R, d, "last") for g, d in zip(grp, dst)])
    phys = np.array([fld(w[g], R, d, "phys") for g, d in zip(grp, dst)])
    vq[:, 2] = np.maximum(0, last - rng.integers(0, 4, n))
    prev = last - 1 - rng.integers(0, window // 4, n)
    prev = np.where(prev < phys - window + window // 4, np.maximum(last - 1, -1), prev)
    aq[:, 2] = np.where((prev < 0) & (phys > window // 2), last - 1, np.maximum(prev, -1))
    check_handler_batches(R, G, cap, window, abi.MODE_REFERENCE, w, lt, lc, grp, dst, vq, aq, cmd)


def test_non_direct_gather_on_a_ring_vs_oracle_sample():
    """The bucketed path's non-direct gather (more than 1,024 tiles: 4.2·10^6
    messages) on a 64-slot log_window ring, the device entry points: the
    responses of every message to 300 consecutive groups, and those groups' final
    state and logs, against the oracle's handlers applied in batch order."""
    import torch
    rng = np.random.default_rng(71)
    R, G, cap, window, n = 5, 50_000, 160, 64, 4_200_000
    w, lt, lc = random_ring_states(rng, G, R, cap, window)
    e = RaftEngine(abi.make_params(R=R, G=G, log_cap=cap, log_window=window, seed=3))
    e.write_state(w)
    e.write_log(lt, lc)
    grp = rng.integers(0, G, n)
    dst = rng.integers(0, R, n).astype(np.int32)
    NF = abi.NUM_FIELDS
    last = w[grp, dst * NF + abi.F_INDEX["last"]]
    phys = w[grp, dst * NF + abi.F_INDEX["phys"]]
    prev = last - 1 - rng.integers(0, window // 4, n)
    prev = np.where(prev < phys - window + window // 4, np.maximum(last - 1, -1), prev)
    prev = np.where((prev < 0) & (phys > window // 2), last - 1, np.maximum(prev, -1))
    aq = np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), prev, rng.integers(-1, 4, n),
                   rng.integers(0, 2, n), rng.integers(0, 6, n), rng.integers(0, 1 << 32, n, dtype=np.uint64),
                   rng.integers(0, 8, n)], axis=1).astype(np.int64).astype(np.uint32).view(np.int32)
    dev = torch.device("cuda:0")
    d_in = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (grp, dst, aq)]
    d_resp = torch.zeros((n, 3), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    e.append_batch_dev(*(x.data_ptr() for x in d_in), d_resp.data_ptr(), n)
    resp = d_resp.cpu().numpy()
    # the oracle on 300 consecutive groups (their global ids key the timer
    # draws): every message to them, in batch order
    s0 = int(rng.integers(0, G - 300))
    sample = np.arange(s0, s0 + 300)
    local = {int(g): i for i, g in enumerate(sample)}
    o = O.Oracle(abi.make_params(R=R, G=len(sample), g0=s0, log_cap=cap, log_window=window, seed=3))
    o.write_state(w[sample])
    o.write_log(lt[sample], lc[sample])
    idx = np.flatnonzero(np.isin(grp, sample))
    aqu = aq.view(np.uint32).astype(np.int64)
    for m in idx:
        q = aqu[m]
        t_, s_, st_ = o.append(local[int(grp[m])], int(dst[m]), int(aq[m, 0]), int(aq[m, 1]), int(aq[m, 2]),
                               int(aq[m, 3]), (int(aq[m, 5]), int(q[6])) if aq[m, 4] else None, int(aq[m, 7]))
        assert tuple(int(x) for x in resp[m]) == (int(t_), int(s_), int(st_)), f"message {m}"
    se = np.concatenate([e.read_state(int(g), 1) for g in sample])
    assert_same_state(se, o.read_state(), R, "sampled groups after the 4.2e6-message batch")
    t_e = np.concatenate([e.read_log(int(g), 1)[0] for g in sample])
    c_e = np.concatenate([e.read_log(int(g), 1)[1] for g in sample])
    assert_same_logs(se, (t_e, c_e), o.read_log(), R, "sampled groups' logs")
    assert len(idx) > 20_000                                            # ~84 messages per sampled group


def test_batch_paths_agree_at_scale():
    """4.2·10^6 votes over 10^6 groups of 5 (the bucketed path's bucket-count
    cap applies: S is raised until at most 3,072 buckets remain), then 10^6
    appends: the bucketed and the sorted path leave the same responses, state
    and logs."""
    import torch
    rng = np.random.default_rng(31)
    R, G, cap = 5, 1_000_000, 8
    dev = torch.device("cuda:0")
    engines = []
    for path in (abi.BATCH_PATH_BUCKETED, abi.BATCH_PATH_SORTED):
        e = RaftEngine(abi.make_params(R=R, G=G, log_cap=cap, seed=9))
        e.set_batch_path(path)
        e.step(3)
        engines.append(e)
    outs = []
    for kind, n in (("vote", 4_200_000), ("append", 1_000_000)):
        grp = torch.from_numpy(rng.integers(0, G, n)).to(dev)
        dst = torch.from_numpy(rng.integers(0, R, n).astype(np.int32)).to(dev)
        if kind == "vote":
            req = torch.from_numpy(np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), rng.integers(0, cap + 1, n),
                                             rng.integers(0, 4, n)], axis=1).astype(np.int32)).to(dev)
        else:
            req = torch.from_numpy(np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), rng.integers(-1, cap, n),
                                             rng.integers(-1, 4, n), rng.integers(0, 2, n), rng.integers(0, 6, n),
                                             rng.integers(0, 1 << 32, n, dtype=np.uint64), rng.integers(0, 8, n)],
                                            axis=1).astype(np.int64).astype(np.uint32).view(np.int32)).to(dev)
        torch.cuda.synchronize(dev)                  # the engine stream does not wait for torch's
        res = []
        for e in engines:
            resp = torch.zeros((n, 2 if kind == "vote" else 3), dtype=torch.int32, device=dev)
            fn = e.vote_batch_dev if kind == "vote" else e.append_batch_dev
            fn(grp.data_ptr(), dst.data_ptr(), req.data_ptr(), resp.data_ptr(), n)
            res.append(resp.cpu().numpy())
        assert np.array_equal(res[0], res[1]), f"{kind} responses differ"
    a, b = (e.read_state() for e in engines)
    assert np.array_equal(a, b)
    assert engines[0].digest() == engines[1].digest()


def test_pinned_host_batches_match_pageable():
    """Page-locked host arrays take the direct-DMA path of raft_*_batch (no
    staging copy), pageable ones the threaded copy into the engine's pinned
    staging: both leave the same responses, state and logs, at a batch large
    enough for the threaded copy (> 4 MB of requests)."""
    import torch
    rng = np.random.default_rng(12)
    R, G, cap, n = 5, 2000, 8, 300_000
    w, lt, lc = random_states(rng, G, R, cap)
    a, b = (RaftEngine(abi.make_params(R=R, G=G, log_cap=cap, seed=4)) for _ in range(2))
    for x in (a, b):
        x.write_state(w)
        x.write_log(lt, lc)
    grp = rng.integers(0, G, size=n).astype(np.int64)
    dst = rng.integers(0, R, size=n).astype(np.int32)
    vq = np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), rng.integers(0, cap + 1, n),
                   rng.integers(0, 4, n)], axis=1).astype(np.int32)
    aq = np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), rng.integers(-1, cap, n),
                   rng.integers(-1, 4, n), rng.integers(0, 2, n), rng.integers(0, 6, n),
                   rng.integers(0, 1 << 32, n, dtype=np.uint64), rng.integers(0, 8, n)],
                  axis=1).astype(np.int64).astype(np.uint32).view(np.int32)
    pin = lambda x: torch.from_numpy(np.ascontiguousarray(x)).pin_memory().numpy()   # noqa: E731
    pg = pin(grp)
    # the replica indices in the engine's own page-locked allocation (raft_host_alloc)
    lib = abi.load_library()
    raw = lib.raft_host_alloc(n * 4)
    assert raw, lib.raft_last_error()
    pd = np.ctypeslib.as_array((C.c_int32 * n).from_address(raw))
    pd[:] = dst
    ve = a.vote_batch(grp, dst, vq)
    pv = pin(np.zeros((n, 2), np.int32))
    assert b.vote_batch(pg, pd, pin(vq), out=pv) is pv
    assert np.array_equal(ve, pv)
    ae = a.append_batch(grp, dst, aq)
    pa = pin(np.zeros((n, 3), np.int32))
    b.append_batch(pg, pd, pin(aq), out=pa)
    assert np.array_equal(ae, pa)
    sa = a.read_state()
    assert np.array_equal(sa, b.read_state())
    assert_same_logs(sa, a.read_log(), b.read_log(), R, "pinned vs pageable batches")
    assert a.digest() == b.digest()
    del pd
    assert lib.raft_host_free(raw) == abi.RAFT_OK


def test_device_batches_match_host_batches():
    """raft_*_batch_dev on HBM-resident messages (torch tensors) leave the
    same responses, state and logs as the host entry points on an identical
    engine; a message outside the engine fails the whole batch with
    RAFT_ERANGE before anything is applied."""
    import torch
    rng = np.random.default_rng(11)
    R, G, cap, n = 5, 500, 8, 20_000
    w, lt, lc = random_states(rng, G, R, cap)
    a, b = (RaftEngine(abi.make_params(R=R, G=G, log_cap=cap, seed=3)) for _ in range(2))
    for x in (a, b):
        x.write_state(w)
        x.write_log(lt, lc)
    grp = rng.integers(0, G, size=n)
    dst = rng.integers(0, R, size=n).astype(np.int32)
    vq = np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), rng.integers(0, cap + 1, n),
                   rng.integers(0, 4, n)], axis=1).astype(np.int32)
    aq = np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), rng.integers(-1, cap, n),
                   rng.integers(-1, 4, n), rng.integers(0, 2, n), rng.integers(0, 6, n),
                   rng.integers(0, 1 << 32, n, dtype=np.uint64), rng.integers(0, 8, n)], axis=1).astype(np.int64)
    cmd = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    dev = torch.device("cuda", 0)
    cur = lambda: torch.cuda.current_stream(dev).cuda_stream  # noqa: E731
    tg, td = torch.from_numpy(grp.astype(np.int64)).to(dev), torch.from_numpy(dst).to(dev)
    ve = a.vote_batch(grp, dst, vq)
    tv, tvr = torch.from_numpy(vq).to(dev), torch.zeros((n, 2), dtype=torch.int32, device=dev)
    # the inputs and the zeroed responses come from torch's stream: order the batch after it
    b.vote_batch_dev(tg.data_ptr(), td.data_ptr(), tv.data_ptr(), tvr.data_ptr(), n, after_stream=cur())
    assert np.array_equal(ve, tvr.cpu().numpy())
    ae = a.append_batch(grp, dst, aq)
    ta = torch.from_numpy(aq.astype(np.uint32).view(np.int32)).to(dev)
    tar = torch.zeros((n, 3), dtype=torch.int32, device=dev)
    b.append_batch_dev(tg.data_ptr(), td.data_ptr(), ta.data_ptr(), tar.data_ptr(), n, after_stream=cur())
    assert np.array_equal(ae, tar.cpu().numpy())
    a.append_command_batch(grp, dst, cmd)
    tc = torch.from_numpy(cmd.view(np.int32)).to(dev)
    b.append_command_batch_dev(tg.data_ptr(), td.data_ptr(), tc.data_ptr(), n, after_stream=cur())
    sa = a.read_state()
    assert np.array_equal(sa, b.read_state())
    assert_same_logs(sa, a.read_log(), b.read_log(), R, "device vs host batches")
    assert a.digest() == b.digest()
    # an out-of-range message: nothing applied
    bad_g = grp.copy()
    bad_g[n // 2] = G
    with pytest.raises(RuntimeError):
        a.vote_batch(bad_g, dst, vq)
    assert np.array_equal(a.read_state(), sa) and a.digest() == b.digest()
    # the batch staging is engine memory: counted, and freed by trim_staging
    # (later batches grow it again and give the same results)
    before = b.device_bytes
    b.trim_staging()
    assert b.device_bytes < before
    assert np.array_equal(b.vote_batch(grp, dst, vq), a.vote_batch(grp, dst, vq))


def test_service_wire_path_matches_batches():
    """RaftService.vote_wire / append_wire (serialized protobufs through
    include/raft_wire.h) leave the same responses and state as the fixed-width
    batch entry points on an identical engine."""
    service_mod = importlib.import_module("raft-kotlin_amd.service")
    wire = importlib.import_module("raft-kotlin_amd.wire")
    rng = np.random.default_rng(11)
    R, G, cap, n = 5, 32, 8, 800
    w, lt, lc = random_states(rng, G, R, cap)
    a, b = (RaftEngine(abi.make_params(R=R, G=G, log_cap=cap, seed=3)) for _ in range(2))
    for x in (a, b):
        x.write_state(w)
        x.write_log(lt, lc)
    svc = service_mod.RaftService(b)
    grp = rng.integers(0, G, size=n)
    dst = rng.integers(0, R, size=n).astype(np.int32)
    vq = np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), rng.integers(0, cap + 1, n),
                   rng.integers(0, 4, n)], axis=1).astype(np.int32)
    got = wire.decode_vote_responses(svc.vote_wire(grp, dst, wire.encode_vote_requests(vq)))
    assert np.array_equal(got, a.vote_batch(grp, dst, vq))
    names = [f"cmd-{i}".encode() for i in range(7)]
    aq = np.stack([rng.integers(0, 6, n), rng.integers(1, R + 1, n), rng.integers(-2, cap, n),
                   rng.integers(-1, 4, n), rng.integers(0, 2, n), rng.integers(0, 6, n),
                   np.zeros(n), rng.integers(0, 8, n)], axis=1).astype(np.int32)
    cmds = [names[rng.integers(0, 7)] if q[4] else None for q in aq]
    resp = svc.append_wire(grp, dst, wire.encode_append_requests(aq, cmds))
    aq64 = aq.astype(np.int64)
    aq64[:, 6] = [svc.commands.intern(c.decode()) if c is not None else 0 for c in cmds]
    ref = a.append_batch(grp, dst, aq64)
    for m, r in enumerate(resp):
        if ref[m, 2]:
            assert r is None                                   # the handler threw: no response
        else:
            assert np.array_equal(wire.decode_append_responses([r])[0, :2], ref[m, :2])
    assert np.array_equal(a.read_state(), b.read_state())
    assert a.digest() == b.digest()


def test_kats_on_engine():
    """K2-K4 and K6/K7 traces replayed through the engine's C-ABI."""
    R = 3
    e = RaftEngine(abi.make_params(R=R, G=1, log_cap=64))
    w = blank_groups(1, R)
    set_fld(w, R, 0, "term", 2)
    e.write_state(w)
    q = np.array([[2, 3, 0, 0], [3, 3, 0, 0], [3, 4, 0, 0], [3, 3, 0, 0]], np.int32)
    assert e.vote_batch([0] * 4, [0] * 4, q).tolist() == [[2, 0], [3, 1], [3, 0], [3, 1]]
    # K7 via the step kernel
    a, b, cc, d = (ord(x) for x in "abcd")
    w = blank_groups(1, R)
    for r in range(R):
        set_fld(w, R, r, "term", 1)
        set_fld(w, R, r, "voted", 1)
        if r:
            set_fld(w, R, r, "flags", abi.FL_ARMED)
            set_fld(w, R, r, "election_ms", 10 ** 9)
    set_fld(w, R, 0, "role", abi.LEADER)
    set_fld(w, R, 0, "flags", abi.FL_HB_ACTIVE)
    set_fld(w, R, 0, "last", 3)
    set_fld(w, R, 0, "phys", 3)
    set_session(w, R, 0, [1] * R, [0] * R)
    e.write_state(w)
    t = np.zeros((1, R, 64), np.int32)
    c = np.zeros((1, R, 64), np.uint32)
    t[0, 0, :3] = 1
    c[0, 0, :3] = [a, b, cc]
    e.write_log(t, c)
    e.step(2)
    e.append_command_batch([0], [0], [d])
    e.step(1)
    s = e.read_state()[0]
    t, c = e.read_log()
    assert fld(s, R, 0, "commit") == 2          # tick 3: all three ack the stale slot `b`
    for r in (1, 2):
        assert fld(s, R, r, "last") == 2 and [int(c[0, r, j]) for j in range(2)] == [a, b]


def test_session_started_and_deposed_in_one_step():
    """Regression: global group 53 of this config, step 13.  The candidate in
    backoff wins its round (phase D starts its session), then the stale leader
    with the lower replica index ticks first in phase A and deposes it (Q3);
    the new session's nextIndex row must still persist (S-8)."""
    kw = dict(R=3, G=1, g0=53, seed=103, log_cap=300, drop_ppm=100_000, churn_ppm=20_000, churn_steps=15,
              cmd_ppm=500_000, partition_period=40, partition_len=10)
    o = O.Oracle(abi.make_params(**kw))
    o.step(12)
    e = RaftEngine(abi.make_params(**kw))
    e.write_state(o.read_state())
    e.write_log(*o.read_log())
    e.step_index = 12
    o.step(1)
    e.step(1)
    s = o.read_state()[0]
    assert session(s, 3, 2)[0] == [1, 1, 1] and not (fld(s, 3, 2, "flags") & abi.FL_HB_ACTIVE)
    assert_same_state(e.read_state(), o.read_state(), 3, "group 53 step 13")


def test_node_entries_term_command_dump():
    """RaftServer.entries() (RaftServer.kt:96-97, served at :84-86): the
    visible log log[0 .. lastIndex) (Commons.kt:71-72) as "term: command"
    strings.  K7's trace through RaftService: after appendCommand("d") the
    leader's physical log is [a, b, c, d] but its visible entries are [a, b]
    (ghost tail, Q1), so tick 3 ships the stale `b` and every node shows
    ["1: a", "1: b"].  Then a config-2 run: every node's dump equals the one
    formatted from the oracle's log."""
    service_mod = importlib.import_module("raft-kotlin_amd.service")
    R = 3
    e = RaftEngine(abi.make_params(R=R, G=1, log_cap=64))
    svc = service_mod.RaftService(e)
    ids = [svc.commands.intern(x) for x in "abc"]
    w = blank_groups(1, R)
    for r in range(R):
        set_fld(w, R, r, "term", 1)
        set_fld(w, R, r, "voted", 1)
        if r:
            set_fld(w, R, r, "flags", abi.FL_ARMED)
            set_fld(w, R, r, "election_ms", 10 ** 9)
    set_fld(w, R, 0, "role", abi.LEADER)
    set_fld(w, R, 0, "flags", abi.FL_HB_ACTIVE)
    set_fld(w, R, 0, "last", 3)
    set_fld(w, R, 0, "phys", 3)
    set_session(w, R, 0, [1] * R, [0] * R)
    e.write_state(w)
    t = np.zeros((1, R, 64), np.int32)
    c = np.zeros((1, R, 64), np.uint32)
    t[0, 0, :3] = 1
    c[0, 0, :3] = ids
    e.write_log(t, c)
    assert svc.node(0, 0).entries() == ["1: a", "1: b", "1: c"]
    e.step(1)
    assert svc.node(0, 0).entries() == ["1: a"]                  # self-append truncated the leader (K7)
    e.step(1)
    assert svc.node(0, 0).appendCommand("d") == "d"
    assert svc.node(0, 0).entries() == ["1: a", "1: b"]          # `d` went to the physical end
    e.step(1)
    for r in range(R):
        assert svc.node(0, r).entries() == ["1: a", "1: b"], r

    kw = dict(abi.CONFIGS[2], G=200)
    e2, o2 = pair(log_cap=200, **kw)
    e2.step(150)
    o2.step(150)
    svc2 = service_mod.RaftService(e2)
    so = o2.read_state()
    ot, oc = o2.read_log()
    for g in range(0, 200, 37):
        for r in range(3):
            last = int(fld(so[g], 3, r, "last"))
            want = [f"{int(ot[g, r, j])}: {svc2.commands.name(oc[g, r, j])}" for j in range(last)]
            assert svc2.node(g, r).entries() == want, (g, r)
            assert last == 0 or want[0].startswith(f"{int(ot[g, r, 0])}: cmd#")


# ---- K8-K14 replayed through the engine (tests/kats_election.py) -----------------
import kats_election as KE  # noqa: E402


@pytest.mark.parametrize("kat", KE.KATS, ids=lambda k: k["name"].split()[0])
def test_election_kats_on_engine(kat):
    """The hand-derived election-loop traces through the C-ABI: write_state
    (+ write_log), step, read_state; then the engine equals the oracle."""
    kw = KE.params(kat)
    e, o = pair(**kw)
    KE.run(kat, e)
    KE.run(kat, o)
    if not kat.get("window"):                  # past a window miss the engine's values are not the reference's
        assert_same_state(e.read_state(), o.read_state(), kat["R"], kat["name"])
        assert e.digest() == o.digest()
