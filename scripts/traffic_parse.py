"""Parse scripts/traffic.sh output into per-launch HBM bytes (JSON on stdout).

rocprofv3 FETCH_SIZE / WRITE_SIZE are kilobytes (1024 B) per dispatch.  The
factors measured on the calibration engine (exact byte count known) convert
them to bytes for this kernel's access pattern."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import importlib  # noqa: E402

abi = importlib.import_module("raft-kotlin_amd.abi")
G = int(os.environ.get("TRAFFIC_GROUPS", "1000000"))
R = 5
REPLICA_BYTES = abi.REPLICA_STATE_BYTES
GROUP_BYTES = 12
NCW = (abi.NUM_COUNTERS + 1) // 2


def per_dispatch(d, counter):
    """[value in bytes] per step_kernel dispatch, in dispatch order."""
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "step_kernel" in row["Kernel_Name"] and row["Counter_Name"] == counter:
                rows.append((int(row["Dispatch_Id"]), float(row["Counter_Value"]) * 1024.0))
    return [v for _, v in sorted(rows)]


# scripts/traffic_run.py workload: 2 warmup launches + 4 launches at K=64, 2 at K=512, then 20 at K=1
SPLITS = {64: slice(2, 6), 512: slice(6, 8), 1: slice(8, 28)}


def main(d):
    state = G * (R * REPLICA_BYTES + GROUP_BYTES)
    f1 = sorted(per_dispatch(f"{d}/calib_FETCH_SIZE", "FETCH_SIZE"))
    w1 = sorted(per_dispatch(f"{d}/calib_WRITE_SIZE", "WRITE_SIZE"))
    fetch_med, write_med = f1[len(f1) // 2], w1[len(w1) // 2]
    ff, wf = state / fetch_med, state / write_med
    wfetch = per_dispatch(f"{d}/workload_FETCH_SIZE", "FETCH_SIZE")
    wwrite = per_dispatch(f"{d}/workload_WRITE_SIZE", "WRITE_SIZE")
    rows = []
    for k, sl in SPLITS.items():
        fl, wl = wfetch[sl], wwrite[sl]
        if not fl or not wl:
            continue
        fm, wm = sum(fl) / len(fl), sum(wl) / len(wl)
        rows.append({"config": 3, "groups": G, "steps_per_launch": k,
                     "bytes_per_launch": fm * ff + wm * wf,
                     "fetch_bytes_raw": fm, "write_bytes_raw": wm, "fetch_factor": ff, "write_factor": wf,
                     "calib_state_bytes": state, "calib_fetch_raw": fetch_med, "calib_write_raw": write_med,
                     "source": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes), scripts/traffic.sh"})
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
