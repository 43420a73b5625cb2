"""The handler-batch workload for rocprofv3 (scripts/pmc_handler.sh): bench.py's
handler_batch leg without the timing loops -- a 10^6 x 5 config-3 engine after
200 steps, then REPS device-resident batches of N random vote messages and
REPS of N append messages (bench.handler_requests, seed 12345), then the
scattered-access traffic probes.  Prints the batch plan as JSON for the parser."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

abi = bench.abi
RaftEngine = importlib.import_module("raft-kotlin_amd.engine").RaftEngine
N = int(os.environ.get("HANDLER_N", "1000000"))
REPS = int(os.environ.get("HANDLER_REPS", "5"))
G = int(os.environ.get("HANDLER_G", "1000000"))
PATH = int(os.environ.get("HANDLER_PATH", "0"))        # abi.BATCH_PATH_*: 0 auto, 1 sorted, 2 bucketed


def main():
    kw = dict(abi.CONFIGS[3], G=G)
    R = kw["R"]
    e = RaftEngine(abi.make_params(log_cap=300, steps_per_launch=200, **kw))
    e.set_batch_path(PATH)
    e.step(200, counters=False)
    st = e.read_state()
    max_term = int(st[:, [r * abi.NUM_FIELDS + abi.F_INDEX["term"] for r in range(R)]].max())
    rng = np.random.default_rng(12345)
    group, dst, vote, app = bench.legs().handler_requests(rng, N, G, R, max_term)
    dev = torch.device("cuda", 0)
    d_group, d_dst = torch.from_numpy(group).to(dev), torch.from_numpy(dst).to(dev)
    plan = []
    for kind, req, w in (("vote", vote, 2), ("append", app, 3)):
        d_req = torch.from_numpy(np.ascontiguousarray(req)).to(dev)
        d_resp = torch.zeros((N, w), dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        fn = e.vote_batch_dev if kind == "vote" else e.append_batch_dev
        for _ in range(REPS):
            fn(d_group.data_ptr(), d_dst.data_ptr(), d_req.data_ptr(), d_resp.data_ptr(), N)
        plan.append([kind, REPS])
    # the scattered-access calibration (raft_engine_traffic_probe kinds 2 / 3):
    # known 32-B sectors loaded and stored one word each, in this process's own
    # --pmc pass, after the batches
    probes = [[k, *e.traffic_probe(k)] for k in (2, 2, 2, 3, 3, 3)]
    e.close()
    print(json.dumps({"n": N, "batch_path": PATH, "groups": G, "replicas": R, "kernel_src": bench.kernel_source_id(),
                      "library_src": bench.library_source_id(), "batch_src": abi.build_ids()["batch_source_id"],
                      "plan": plan, "probes": probes}))


if __name__ == "__main__":
    main()
