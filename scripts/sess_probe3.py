import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import oracle as O
from helpers import abi, masked_logs
RaftEngine = importlib.import_module("raft-kotlin_amd.engine").RaftEngine
kw = dict(R=3, G=3000, seed=103, log_cap=300, drop_ppm=100_000, churn_ppm=20_000, churn_steps=15,
          cmd_ppm=500_000, partition_period=40, partition_len=10)
o = O.Oracle(abi.make_params(**kw)); o.step(12); S12 = o.read_state()
def diff(e, label):
    se = e.read_state()
    bad = np.argwhere(se != S12)
    print(f"{label}: {len(bad)} words differ; groups {sorted(set(bad[:, 0].tolist()))[:10]}", flush=True)
# A: straight 12 steps
e1 = RaftEngine(abi.make_params(**kw)); e1.step(12); diff(e1, "A straight")
e1b = RaftEngine(abi.make_params(**kw)); [e1b.step(1) for _ in range(12)]; diff(e1b, "A' 12x1")
# B: 11 steps, export, import into fresh engine, 1 step
e2 = RaftEngine(abi.make_params(**kw)); e2.step(11)
s11 = e2.read_state(); lt, lc = e2.read_log()
e3 = RaftEngine(abi.make_params(**kw)); e3.write_state(s11); e3.write_log(lt, lc); e3.step_index = 11; e3.step(1)
diff(e3, "B fresh import of own export")
# C: continue e2
e2.step(1); diff(e2, "C continue")
# D: zeroed logs from the start
e4 = RaftEngine(abi.make_params(**kw))
z = np.zeros((3000, 3, 300), np.int32)
e4.write_log(z, z.view(np.uint32)); e4.step(12); diff(e4, "D zeroed log")
# E: garbage log: fill with a pattern
e5 = RaftEngine(abi.make_params(**kw))
g = np.full((3000, 3, 300), 7, np.int32)
e5.write_log(g, g.view(np.uint32)); e5.step(12); diff(e5, "E log filled with 7")
