"""Debug aid: step the engine and the oracle together on a small workload and
dump, at the first step where the digests differ, both sides' state and logs
of the differing groups (before and after that step) to gpurun_out/.

    python scripts/debug/first_divergence.py '{"R":3,"G":64,"seed":2,...}' STEPS OUT.json
"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402

abi = importlib.import_module("raft-kotlin_amd.abi")
RaftEngine = importlib.import_module("raft-kotlin_amd.engine").RaftEngine


def main(kw, steps, out):
    e, o = RaftEngine(abi.make_params(**kw)), O.Oracle(abi.make_params(**kw))
    prev = None
    for t in range(steps):
        before = (e.read_state(), e.read_log(), o.read_state(), o.read_log())
        ce, co = e.step(1), o.step(1)[:, : abi.NUM_COUNTERS]
        se, so = e.read_state(), o.read_state()
        (te, ce_), (to, co_) = e.read_log(), o.read_log()
        bad = np.nonzero((se != so).any(1) | (te != to).any((1, 2)) | (ce_ != co_).any((1, 2)))[0]
        if len(bad) or not np.array_equal(ce, co):
            g = int(bad[0]) if len(bad) else -1
            rec = {"step": t + 1, "groups": bad.tolist()[:20], "counters_equal": bool(np.array_equal(ce, co)),
                   "engine_counters": ce[0].tolist(), "oracle_counters": co[0].tolist()}
            if g >= 0:
                rec.update({
                    "before_state": before[0][g].tolist(), "before_log_terms": before[1][0][g].tolist(),
                    "before_log_cmds": before[1][1][g].tolist(),
                    "engine_state": se[g].tolist(), "oracle_state": so[g].tolist(),
                    "engine_log_terms": te[g].tolist(), "oracle_log_terms": to[g].tolist(),
                    "engine_log_cmds": ce_[g].tolist(), "oracle_log_cmds": co_[g].tolist()})
            json.dump(rec, open(out, "w"))
            print("diverged at step", t + 1, "groups", bad[:20])
            return
    print("no divergence in", steps, "steps")


if __name__ == "__main__":
    main(json.loads(sys.argv[1]), int(sys.argv[2]), sys.argv[3])
