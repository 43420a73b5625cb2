"""Generate tests/golden/full_size.json + full_size_counters.npz: the oracle's
result for the north star's full-size runs, for the GPU test
tests/test_gpu_parity.py::test_full_size_digest.

  * config 3: 10^6 five-replica groups, 10^4 steps (5 % drop, churn, commands);
  * config 5: 10^5 seven-replica groups, 10^4 steps (partitions, every leader
    takes a command each step).

The oracle runs the groups in contiguous chunks (groups are independent and
every random draw is keyed by the global group id), so a chunk
holds a few GB of logs.  The digest is a sum of per-group hashes (mod 2^64)
over state, sessions and the physical logs, so the chunk digests add up to the
whole run's digest; the per-step counters add up too.  Recorded per chunk so a
mismatch on the GPU names the group range.

    python tests/golden/make_full_size.py [--configs 3 5 3long] [--threads 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as O                 # noqa: E402
from helpers import abi            # noqa: E402

CASES = {
    # config 3 runs with the bench's 256-slot ring (log_window); the digest of
    # the full log (window 0) is taken from the same run, whose state cannot
    # depend on the window while no access misses it (asserted)
    3: dict(steps=10_000, log_cap=3064, chunk=50_000, log_window=256),
    5: dict(steps=10_000, log_cap=10_064, chunk=25_000, log_window=0),
    # 10^5 steps on the 256-slot ring: the GPU runs all 10^6 groups (10 GB of
    # ring instead of 124 GB per 10^4 steps of flat log) and compares the
    # digest of groups [0, 10^4) (raft_engine_digest_range)
    "3long": dict(cfg=3, steps=100_000, log_cap=30_094, chunk=10_000, log_window=256, sample=10_000),
}
JSON = os.path.join(HERE, "full_size.json")
NPZ = os.path.join(HERE, "full_size_counters.npz")


def run_config(name, threads):
    spec = CASES[name]
    cfg = spec.get("cfg", name)
    kw = dict(abi.CONFIGS[cfg])
    G, steps, chunk, W = kw.pop("G"), spec["steps"], spec["chunk"], spec["log_window"]
    Gs = spec.get("sample", G)                       # groups the oracle runs: [0, Gs)
    total = np.zeros((steps, abi.NUM_COUNTERS), dtype=np.int64)
    chunks, digest, digest_full = [], 0, 0
    t0 = time.time()
    for g0 in range(0, Gs, chunk):
        n = min(chunk, Gs - g0)
        o = O.Oracle(abi.make_params(log_cap=spec["log_cap"], log_window=W, **dict(kw, G=n, g0=g0)))
        total += o.step(steps, nthreads=threads)[:, : abi.NUM_COUNTERS]
        d = o.digest()
        o.set_log_window(0)
        df = o.digest()
        o.close()
        digest = (digest + d) % (1 << 64)
        digest_full = (digest_full + df) % (1 << 64)
        chunks.append({"g0": g0, "n": n, "digest": f"{d:016x}", "digest_full_log": f"{df:016x}"})
        print(f"{name}: groups {g0}..{g0 + n} done, {time.time() - t0:.0f} s", flush=True)
    assert total[:, abi.C_INDEX["log_overflow"]].sum() == 0, "log_cap too small"
    assert total[:, abi.C_INDEX["log_window_miss"]].sum() == 0, "log_window too small"
    meta = {"config": cfg, "groups": G, "sample_groups": Gs, "steps": steps, "log_cap": spec["log_cap"],
            "log_window": W, "params": {k: v for k, v in kw.items()}, "digest": f"{digest:016x}",
            "digest_full_log": f"{digest_full:016x}",
            "chunks": chunks, "oracle_seconds": round(time.time() - t0, 1), "threads": threads}
    return meta, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["3", "5", "3long"])
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    a = ap.parse_args()
    meta = json.load(open(JSON)) if os.path.exists(JSON) else {}
    arrays = dict(np.load(NPZ)) if os.path.exists(NPZ) else {}
    for name in a.configs:
        name = int(name) if name.isdigit() else name
        m, total = run_config(name, a.threads)
        meta[f"c{name}"] = m
        if "sample" not in CASES[name]:              # the GPU's counters cover every group
            arrays[f"c{name}_counters"] = total
        with open(JSON, "w") as f:
            json.dump(meta, f, indent=1)
        np.savez_compressed(NPZ, **arrays)
        print(f"{name}: digest {m['digest']}", flush=True)


if __name__ == "__main__":
    main()
