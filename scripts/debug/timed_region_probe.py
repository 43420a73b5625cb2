#!/usr/bin/env python3
"""Where the driver's one-launch timed region spends its time outside the
step kernel (experiment; not part of the bench).  Config 3 at 10^6 groups,
one 20-step launch per rep, variants interleaved, median wall per variant:

  bench    : bench.py's region (torch events around the launch, kernel timing events on)
  noev     : no torch events (kernel timing events on)
  notime   : torch events, no kernel timing events
  bare     : neither
  streamsync: bare, closed by hipStreamSynchronize instead of a device sync
  empty    : the clock around a device sync alone
"""
import importlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

abi = importlib.import_module("raft-kotlin_amd.abi")
RaftEngine = importlib.import_module("raft-kotlin_amd.engine").RaftEngine

K, REPS = int(os.environ.get("K", 20)), int(os.environ.get("REPS", 25))
variants = ["bench", "noev", "notime", "bare", "streamsync", "empty"]
total = 5 + K * REPS * len(variants)
kw = dict(abi.CONFIGS[3])
params = abi.make_params(log_cap=int(64 + 0.3 * total) + 64, log_window=0, steps_per_launch=K, subranges=1, **kw)
eng = RaftEngine(params, device=0)
dev = torch.device("cuda", 0)
stream = torch.cuda.ExternalStream(eng.stream, device=dev)
counters = torch.zeros((K, abi.COUNTER_STRIDE), dtype=torch.int64, device=dev)
eng.step_async(5, None)
eng.sync()
res = {v: [] for v in variants}
kern = []
ptr = counters.data_ptr()
for rep in range(REPS):
    for v in variants:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        eng.set_kernel_timing(v in ("bench", "noev"))
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if v in ("bench", "notime"):
            ev0.record(stream)
        if v != "empty":
            eng.step_async(K, ptr)
        if v in ("bench", "notime"):
            ev1.record(stream)
        if v == "streamsync":
            eng.sync()
        else:
            torch.cuda.synchronize(dev)
        res[v].append((time.perf_counter() - t0) * 1e3)
        if v == "bench":
            ms, n = eng.kernel_time()
            kern.append(ms / max(1, n))
        elif v == "noev":
            eng.kernel_time()
        eng.set_kernel_timing(False)
out = {v: {"median_ms": statistics.median(x), "min_ms": min(x)} for v, x in res.items()}
out["kernel_ms_median"] = statistics.median(kern)
out["K"] = K
print(json.dumps(out))
eng.close()
