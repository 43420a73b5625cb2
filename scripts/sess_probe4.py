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
o = O.Oracle(abi.make_params(**kw)); o.step(12); S12 = o.read_state()
def diff(e, label):
    se = e.read_state()
    bad = np.argwhere(se != S12)
    print(f"{label}: {len(bad)} words differ; groups {sorted(set(bad[:, 0].tolist()))[:10]}", flush=True)
for mode in ["none", "digest", "read_state", "read_log", "digest_every_step", "all_every_step"]:
    e = RaftEngine(abi.make_params(**kw))
    for t in range(11):
        e.step(1)
        if mode == "digest_every_step": e.digest()
        if mode == "all_every_step": e.read_state(); e.read_log(); e.digest()
    if mode == "digest": e.digest()
    if mode == "read_state": e.read_state()
    if mode == "read_log": e.read_log()
    e.step(1)
    diff(e, mode)
