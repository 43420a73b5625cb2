"""Per-launch PMC of the timed step-kernel launches of each traffic_attrib.sh
variant: HBM bytes (FETCH_SIZE / WRITE_SIZE, calibrated as in pmc_parse.py),
L1 read / write requests, L2 hits / misses, fabric read / write requests."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_parse import CALIB_G, CALIB_R, GROUP_BYTES, REPLICA_BYTES, dispatches  # noqa: E402

d = sys.argv[1]
state = CALIB_G * (CALIB_R * REPLICA_BYTES + GROUP_BYTES)
cf = sorted(dispatches(f"{d}/calib_FETCH_SIZE").get("FETCH_SIZE", []))
cw = sorted(dispatches(f"{d}/calib_WRITE_SIZE").get("WRITE_SIZE", []))
ff, wf = state / (cf[len(cf) // 2] * 1024.0), state / (cw[len(cw) // 2] * 1024.0)
out = {"fetch_factor": ff, "write_factor": wf, "variants": {}}
for plan in sorted(glob.glob(f"{d}/plan_*.json")):
    v = os.path.basename(plan)[5:-5]
    seq = json.load(open(plan))["launches"]
    ix = [i for i, x in enumerate(seq) if x[0] == "timed"]
    row = {"launch_steps": seq[ix[0]][1], "launches": len(ix)}
    for p in sorted(glob.glob(f"{d}/{v}_p*")):
        for c, vals in dispatches(p).items():
            row[c] = sum(vals[i] for i in ix) / len(ix)
    if "FETCH_SIZE" in row:
        row["fetch_bytes"] = row["FETCH_SIZE"] * 1024 * ff
    if "WRITE_SIZE" in row:
        row["write_bytes"] = row["WRITE_SIZE"] * 1024 * wf
    try:
        b = json.loads([ln for ln in open(f"{d}/bench_{v}.log") if ln.startswith("{")][-1])
        row["value"] = b["value"]
        row["state_bytes_per_launch"] = b["roofline"]["state_bytes_per_launch"]
        row["kernel_avg_ms"] = b["roofline"]["kernel_avg_ms"]
    except (OSError, IndexError, KeyError, ValueError):
        pass
    out["variants"][v] = row
print(json.dumps(out, indent=1))
