"""bench.py's multi-GPU plumbing on CPU: `--gpus N` spawns N rank processes
itself (no torch.distributed launcher), the ranks agree on their shards over
gloo, a WORLD_SIZE that disagrees with --gpus is refused, and the shard
arithmetic covers the global group ids exactly once (config 4: 10^6 groups
split by contiguous global id)."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
spec = importlib.util.spec_from_file_location("bench", BENCH)
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
abi = bench.abi


def run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, env=e, timeout=240)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("total", [1_000_000, 999_999, 7])
def test_strong_shards_cover_every_group_once(world, total):
    spans = [bench.shard(total, world, r, "strong") for r in range(world)]
    assert sum(n for _, n in spans) == total
    nxt = 0
    for g0, n in spans:
        assert g0 == nxt and n >= total // world
        nxt = g0 + n


def test_weak_shards_are_disjoint_full_size():
    spans = [bench.shard(1000, 4, r, "weak") for r in range(4)]
    assert spans == [(0, 1000), (1000, 1000), (2000, 1000), (3000, 1000)]


@pytest.mark.parametrize("steps,spl,want", [(10_000, 512, 500), (20, 512, 20), (1024, 512, 512), (7919, 512, 512),
                                             (600, 512, 300), (5, 512, 5)])
def test_timed_launches_have_one_length(steps, spl, want):
    L = bench.launch_length(steps, spl)
    assert L == want
    if steps % L == 0:
        assert set(bench.launch_plan(steps, L)) == {L}


def test_gpus_2_spawns_two_gloo_ranks_config4_by_default():
    """Config 4 (BASELINE.json configs[3]) by default: the 10^6 groups split
    into contiguous global-id ranges over the ranks (strong scaling)."""
    r = run(["--gpus", "2", "--plan-only"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout                      # rank 0 prints the one line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["shards"] == [[0, 0, 500_000], [1, 500_000, 500_000]]


@pytest.mark.parametrize("world", [4, 8])
def test_gpus_n_strong_shards_config4(world):
    r = run(["--gpus", str(world), "--plan-only"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    per = 1_000_000 // world
    assert out["scaling"] == "strong" and out["shards"] == [[q, q * per, per] for q in range(world)]


def test_gpus_2_weak_shards_on_request():
    r = run(["--gpus", "2", "--plan-only", "--scaling", "weak"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["scaling"] == "weak"
    assert out["shards"] == [[0, 0, 1_000_000], [1, 1_000_000, 1_000_000]]


def test_rank0_weak_shard_is_the_strong_leg_groups():
    """The strong (config 4) leg splits groups 0..G-1 over the ranks; rank 0's
    weak shard (the side leg) is exactly those global groups, so rank 0's weak
    rows equal the strong leg's all-reduced rows."""
    for world in (2, 4, 8):
        g0, n = bench.shard(1_000_000, world, 0, "weak")
        strong = [bench.shard(1_000_000, world, r, "strong") for r in range(world)]
        assert (g0, n) == (0, 1_000_000) and strong[0][0] == 0 and sum(x[1] for x in strong) == n


def test_world_size_mismatch_is_refused():
    r = run(["--gpus", "4", "--plan-only"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_cpu_share_is_positive():
    assert 1 <= bench.available_cpus() <= (os.cpu_count() or 1)


def test_default_launch_length_per_kernel_variant():
    """7-waves-per-SIMD kernels (R <= 5, or R = 7 without drops) launch at most
    abi.BENCH_STEPS_PER_LAUNCH steps so 7 workgroups fit a CU's LDS; the others
    take the longest launch (raft_engine.hip RAFT_STEP_WAVES_PER_EU)."""
    assert abi.bench_steps_per_launch(5) == abi.BENCH_STEPS_PER_LAUNCH == 400
    assert abi.bench_steps_per_launch(3) == 400
    assert abi.bench_steps_per_launch(7) == abi.LDS_MAX_STEPS_PER_LAUNCH
    # epochs: the reference mode on a balanced schedule (more chunks than
    # resident wave slots) and one sub-range launches the whole default run
    net3 = abi.step_net_of(abi.CONFIGS[3])
    assert abi.bench_steps_per_launch(5, abi.MODE_REFERENCE, 0, net3, 10**6) == abi.LONG_STEPS_PER_LAUNCH
    assert abi.bench_steps_per_launch(5, abi.MODE_REFERENCE, 256, net3, 125_000) == abi.LONG_STEPS_PER_LAUNCH
    assert abi.bench_steps_per_launch(5, abi.MODE_REFERENCE, 0, net3, 10**4) == 400          # one chunk per wave
    assert abi.bench_steps_per_launch(5, abi.MODE_TEXTBOOK, 0, net3, 10**6) == 400          # no epochs kernel
    assert abi.bench_steps_per_launch(7, abi.MODE_REFERENCE, 0, abi.NET_PART, 10**6) == 400   # sub-ranges
    assert abi.LONG_STEPS_PER_LAUNCH <= abi.MAX_STEPS_PER_LAUNCH
    # config 5 (R = 7, partitions, no drops) runs the 7-wave partitions-only kernel
    net5 = abi.step_net_of(abi.CONFIGS[5])
    assert net5 == abi.NET_PART and abi.bench_steps_per_launch(7, abi.MODE_REFERENCE, 0, net5) == 400
    assert abi.step_net_of(abi.CONFIGS[3]) == abi.NET_DROP | abi.NET_ISO | abi.NET_CMDLOW
    assert abi.step_net_of(dict(abi.CONFIGS[3], cmd_mode=abi.CMD_ALL_LEADERS)) == abi.NET_ALL
    assert abi.step_net_of(abi.CONFIGS[1]) == abi.NET_PART
    assert abi.step_net_of(abi.CONFIGS[2]) == abi.NET_PART
    assert abi.step_net(5, drop_ppm=1, partition_period=50, partition_len=25) == abi.NET_ALL
    assert abi.step_net(7, partition_period=50, partition_len=25, churn_ppm=1) == abi.NET_ALL
    assert abi.step_net(7, iso_written=True) == abi.NET_ALL
    assert abi.step_net(4, drop_ppm=1) == abi.NET_ALL and abi.step_net(3) == abi.NET_PART
    assert abi.bench_steps_per_launch(5, abi.MODE_TEXTBOOK) == abi.BENCH_STEPS_PER_LAUNCH
    assert abi.bench_steps_per_launch(5, abi.MODE_REFERENCE, 256) == abi.BENCH_STEPS_PER_LAUNCH
    assert bench.launch_length(10_000, 400) == 400 and bench.launch_length(20, 400) == 20


def test_handler_requests_shapes_and_ranges():
    """bench.handler_requests: n messages over G x R replicas, vote [n, 4] and
    append [n, 8] as the structs' 32-bit words, half the appends at prev -1."""
    import numpy as np
    rng = np.random.default_rng(0)
    g, d, v, a = bench.legs().handler_requests(rng, 10_000, 50, 5, 7)
    assert g.shape == (10_000,) and d.dtype == np.int32 and v.shape == (10_000, 4) and a.shape == (10_000, 8)
    assert g.min() >= 0 and g.max() < 50 and d.min() >= 0 and d.max() < 5
    assert v.dtype == np.int32 and a.dtype == np.int32
    assert 0.45 < float(np.mean(a[:, 2] == -1)) < 0.55
    assert set(np.unique(v[:, 1])) <= set(range(1, 6))


def test_pmc_parse_launches_of_subrange_dispatches():
    """A launch of the warmup / timed legs is one dispatch per sub-range; the
    PMC parse sums them, and the trace time is the union of the intervals."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import pmc_parse
    assert pmc_parse.expand([["warmup", 5, 3], ["timed", 20, 3], ["streaming", 1, 1], ["timed", 7]]) == \
        [0, 0, 0, 1, 1, 1, 2, 3]
    assert pmc_parse.union_ms([(0, 10), (5, 20), (30, 40), (35, 38)]) == 30 / 1e6


def test_counter_allreduce_is_inside_the_timed_region_by_default():
    """The N > 1 counter all-reduce (the path's one collective, SURVEY.md
    §8(e)) is enqueued inside the timed region unless a diagnostic asks
    otherwise."""
    assert bench.parse_args([]).allreduce == "end"
    assert bench.parse_args(["--allreduce", "after"]).allreduce == "after"


def test_pmc_parse_probe_factors(tmp_path):
    """The byte factors come from the traffic probes of the same bench process:
    the state probe's known bytes over its FETCH_SIZE / WRITE_SIZE kilobytes,
    and the raw write bytes counted per 8-byte log store."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import pmc_parse
    state, stores = 312_000_000, 4_000_000
    probes = [[0, state, state]] * 3 + [[1, 20_000_000, 8 * stores]] * 3
    for i, (counter, vals) in enumerate((("FETCH_SIZE", [state / 1024 / 1.5] * 3 + [10.0] * 3),
                                         ("WRITE_SIZE", [state / 1024 / 1.25] * 3 + [stores * 64 / 1024] * 3))):
        d = tmp_path / f"pmc{i + 1}" / "host"
        d.mkdir(parents=True)
        with open(d / "run_counter_collection.csv", "w") as f:
            f.write("Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n")
            for k, v in enumerate(vals):
                f.write(f"{100 + k},traffic_probe_kernel<5>,{counter},{v}\n")
    ff, wf, info = pmc_parse.probe_factors(str(tmp_path), {"probes": probes})
    assert abs(ff - 1.5) < 1e-9 and abs(wf - 1.25) < 1e-9
    assert info["log_store_probe_stores"] == stores and abs(info["log_store_raw_bytes_per_store"] - 64) < 1e-9
