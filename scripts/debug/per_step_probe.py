#!/usr/bin/env python3
"""Per-step cost of config 3 at 10^6 groups over the first steps of a run
(experiment; not part of the bench): one step per launch, each launch timed
by its own events, with the step's counters.  Shows which steps of the
driver's window (steps 5..24) carry the election work."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

abi = importlib.import_module("raft-kotlin_amd.abi")
RaftEngine = importlib.import_module("raft-kotlin_amd.engine").RaftEngine

N = int(os.environ.get("N", 60))
params = abi.make_params(log_cap=64 + N, log_window=0, steps_per_launch=1, subranges=1, **dict(abi.CONFIGS[3]))
eng = RaftEngine(params, device=0)
rows = []
for t in range(N):
    eng.set_kernel_timing(True)
    c = eng.step(1)
    ms, n = eng.kernel_time()
    eng.set_kernel_timing(False)
    d = {k: int(v) for k, v in zip(abi.COUNTER_NAMES, c[0])}
    rows.append({"step": t, "kernel_ms": ms / max(1, n), "leaders": d["leaders"], "timeouts": d["timeouts"],
                 "rounds": d["rounds"], "votes_granted": d["votes_granted"], "sessions_ticked": d["sessions_ticked"],
                 "append_sent": d["append_sent"], "msg_dropped": d["msg_dropped"]})
print(json.dumps(rows))
eng.close()
