"""Generate tests/golden/oracle_golden.npz + .json from the CPU oracle.

The reference (Kotlin/JVM) cannot run here, and ships no fixtures, so these
vectors are produced by the oracle after it passed the hand-derived KATs
K1-K7; they pin the oracle (and, on the GPU, the engine) against regressions.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as O                 # noqa: E402
from helpers import abi, masked_logs  # noqa: E402

CASES = {
    "c1": dict(steps=1100, digest_every=10, log_cap=1100, **abi.CONFIGS[1]),
    "c2s": dict(steps=300, digest_every=1, log_cap=128, **dict(abi.CONFIGS[2], G=64)),
    "c3s": dict(steps=400, digest_every=1, log_cap=160,
                **dict(abi.CONFIGS[3], G=64, churn_ppm=20_000)),
    "c5s": dict(steps=400, digest_every=1, log_cap=600, **dict(abi.CONFIGS[5], G=32)),
    # the ring-buffered log (log_window): config 2 wraps a
    # 4-slot ring ~20 times, config 3 a 64-slot one; neither misses
    "c2w": dict(steps=300, digest_every=1, log_cap=128, log_window=4, **dict(abi.CONFIGS[2], G=64)),
    "c3w": dict(steps=400, digest_every=1, log_cap=160, log_window=64,
                **dict(abi.CONFIGS[3], G=64, churn_ppm=20_000)),
}


def run_case(spec):
    spec = dict(spec)
    steps, every = spec.pop("steps"), spec.pop("digest_every")
    o = O.Oracle(abi.make_params(**spec))
    counters, digests = [], []
    for k in range(0, steps, every):
        counters.append(o.step(every)[:, : abi.NUM_COUNTERS])
        digests.append(o.digest())
    st = o.read_state()
    t, c = masked_logs(st, *o.read_log(), o.R)
    counters = np.concatenate(counters)
    assert counters[:, abi.C_INDEX["log_window_miss"]].sum() == 0
    return counters, digests, st, t, c


def main():
    arrays, meta = {}, {}
    for name, spec in CASES.items():
        counters, digests, st, t, c = run_case(spec)
        arrays[f"{name}_counters"] = counters
        arrays[f"{name}_state"] = st
        arrays[f"{name}_log_terms"] = t
        arrays[f"{name}_log_cmds"] = c
        meta[name] = {"spec": spec, "digests": [f"{d:016x}" for d in digests]}
    np.savez_compressed(os.path.join(HERE, "oracle_golden.npz"), **arrays)
    with open(os.path.join(HERE, "oracle_golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", {k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    main()
