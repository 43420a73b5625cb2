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

    python tests/golden/make_full_size.py [--configs 3 5] [--threads 8]
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
    3: dict(steps=10_000, log_cap=3064, chunk=50_000),
    5: dict(steps=10_000, log_cap=10_064, chunk=25_000),
}
JSON = os.path.join(HERE, "full_size.json")
NPZ = os.path.join(HERE, "full_size_counters.npz")


def run_config(cfg, threads):
    spec = CASES[cfg]
    kw = dict(abi.CONFIGS[cfg])
    G, steps, chunk = kw.pop("G"), spec["steps"], spec["chunk"]
    total = np.zeros((steps, abi.NUM_COUNTERS), dtype=np.int64)
    chunks, digest = [], 0
    t0 = time.time()
    for g0 in range(0, G, chunk):
        n = min(chunk, G - g0)
        o = O.Oracle(abi.make_params(log_cap=spec["log_cap"], **dict(kw, G=n, g0=g0)))
        total += o.step(steps, nthreads=threads)[:, : abi.NUM_COUNTERS]
        d = o.digest()
        o.close()
        digest = (digest + d) % (1 << 64)
        chunks.append({"g0": g0, "n": n, "digest": f"{d:016x}"})
        print(f"config {cfg}: groups {g0}..{g0 + n} done, {time.time() - t0:.0f} s", flush=True)
    assert total[:, abi.C_INDEX["log_overflow"]].sum() == 0, "log_cap too small"
    meta = {"config": cfg, "groups": G, "steps": steps, "log_cap": spec["log_cap"],
            "params": {k: v for k, v in kw.items()}, "digest": f"{digest:016x}",
            "chunks": chunks, "oracle_seconds": round(time.time() - t0, 1), "threads": threads}
    return meta, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", type=int, nargs="+", default=[3, 5])
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    a = ap.parse_args()
    meta = json.load(open(JSON)) if os.path.exists(JSON) else {}
    arrays = dict(np.load(NPZ)) if os.path.exists(NPZ) else {}
    for cfg in a.configs:
        m, total = run_config(cfg, a.threads)
        meta[f"c{cfg}"] = m
        arrays[f"c{cfg}_counters"] = total
        with open(JSON, "w") as f:
            json.dump(meta, f, indent=1)
        np.savez_compressed(NPZ, **arrays)
        print(f"config {cfg}: digest {m['digest']}", flush=True)


if __name__ == "__main__":
    main()
