import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import oracle as O
from helpers import abi
RaftEngine = importlib.import_module("raft-kotlin_amd.engine").RaftEngine
before = [1, 1, 2, 0, 0, 0, 0, 8, 0, 0, 1, 1, 0, 0, 0, 0, 20259, 1, 0, 0, 1, 3, 1, 0, 0, 0, 0, 18, 713, 0,
          1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0]
w = np.array(before, np.int32)[None]
w[0, 30 + 6:30 + 9] = 77        # stale next[2][*]
w[0, 39 + 6:39 + 9] = 55        # stale match[2][*]
kw = dict(R=3, G=1, g0=328, seed=103, log_cap=300, drop_ppm=100_000, churn_ppm=20_000, churn_steps=15,
          cmd_ppm=500_000, partition_period=40, partition_len=10)
for spl in (1, 4):
    e = RaftEngine(abi.make_params(steps_per_launch=spl, **kw))
    e.write_state(w)
    o = O.Oracle(abi.make_params(**kw))
    o.write_state(w)
    # advance the step counter to 12 without touching the state: engines start at t=0
    print("spl", spl)
    ce = e.step(1); co = o.step(1)
    print(" engine", e.read_state()[0, 30:].tolist())
    print(" oracle", o.read_state()[0, 30:].tolist())
    print(" engine fields", e.read_state()[0, :30].tolist())
    print(" oracle fields", o.read_state()[0, :30].tolist())
