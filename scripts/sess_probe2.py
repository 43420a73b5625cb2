import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import oracle as O
from helpers import abi
RaftEngine = importlib.import_module("raft-kotlin_amd.engine").RaftEngine
kw = dict(R=3, G=3000, seed=103, log_cap=300, drop_ppm=100_000, churn_ppm=20_000, churn_steps=15,
          cmd_ppm=500_000, partition_period=40, partition_len=10)
o = O.Oracle(abi.make_params(**kw))
o.step(12)
S = o.read_state(); LT, LC = o.read_log()
o.step(1)
S2 = o.read_state()
for g0, n in ((53, 1), (0, 64), (0, 256), (0, 3000), (32, 64)):
    e = RaftEngine(abi.make_params(**dict(kw, G=n, g0=g0)))
    e.write_state(S[g0:g0 + n]); e.write_log(LT[g0:g0 + n], LC[g0:g0 + n]); e.step_index = 12
    e.step(1)
    se = e.read_state()
    bad = np.argwhere(se != S2[g0:g0 + n])
    print(f"g0={g0} n={n}: {len(bad)} words differ; groups {sorted(set((bad[:, 0] + g0).tolist()))[:10]}")
