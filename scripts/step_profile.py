"""Per-step cost profile of the step kernel: one-step launches of config 3
(or --groups G of it) from step 0, each launch's kernel time from the
engine's own events, beside the step's counters (vote rounds, sessions
ticked, appends sent, timeouts).  Shows how uneven the steps of a short
launch are (the election storm against the quiet countdown steps) -- the
input to any step-weighted split of a balanced launch.

    python scripts/step_profile.py --groups 125000 --steps 40 --also 2000:2010
Prints one JSON object.
"""
import argparse
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

abi = bench.abi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--also", default="", help="a later window a:b (steps run in between are not timed)")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    eng_mod = importlib.import_module("raft-kotlin_amd.engine")
    kw = dict(abi.CONFIGS[3], G=a.groups)
    hi = a.steps
    w0 = w1 = 0
    if a.also:
        w0, w1 = (int(x) for x in a.also.split(":"))
        hi = max(hi, w1)
    eng = eng_mod.RaftEngine(abi.make_params(log_cap=64 + hi, steps_per_launch=1, **kw))
    names = {n: abi.C_INDEX[n] for n in ("timeouts", "rounds", "votes_granted", "sessions_ticked", "append_sent",
                                          "commands")}
    prof = []
    for rep in range(a.reps):
        eng.reset()
        eng.set_kernel_timing(True)
        rows = []
        t = 0
        while t < hi:
            timed = t < a.steps or w0 <= t < w1
            if not timed:
                n = (w0 if t < w0 else hi) - t
                eng.set_kernel_timing(False)
                eng.step(n, counters=False)
                eng.set_kernel_timing(True)
                eng.kernel_time()
                t += n
                continue
            c = eng.step(1)
            ms, nl = eng.kernel_time()
            rows.append({"t": t, "ms": ms, **{k: int(c[0, v]) for k, v in names.items()}})
            t += 1
        prof.append(rows)
    out = {"groups": a.groups, "info": eng.kernel_info(), "steps": []}
    for i, r in enumerate(prof[0]):
        out["steps"].append({**r, "ms": min(p[i]["ms"] for p in prof)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
