"""Parse scripts/pmc_bench.sh output into per-launch PMC rows of the step
kernel, written to <dir>/rows.json; `--merge` folds such files into
profiles/pmc_rows.json (bench.py attaches a row only to a run with the same
workload key and launch length).

Every step_kernel dispatch of a PMC pass is matched, in dispatch order, to
the launch sequence bench.py wrote (--plan-file: warmup, timed and streaming
launches with their step counts).  FETCH_SIZE / WRITE_SIZE are kilobytes per
dispatch.  The byte factors come from the traffic probes of the same bench
process (bench.py --traffic-probe, raft_engine_traffic_probe): kind 0 moves
exactly the state a launch moves, with the step kernel's own 4-byte-per-lane
loads and stores; kind 1 makes one 8-byte log store per replica into its own
row, the Log.add pattern.  MI355X_MICROARCH.md calibrates gfx950's factor
for 16 B/lane streams only, and a separate calibration process's factor
varied 1.30-1.86 between boxes (round 4).  The step kernel's writes are
split by the plan's log-store count: the state part at the state factor, each
log store at the 32-B sector gfx950 writes for it (profiles/r3_l)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT_FILE = os.path.join(ROOT, "profiles", "pmc_rows.json")
ID_FIELDS = ("config", "mode", "groups", "warmup", "steps", "log_window", "leg", "launch_steps", "stream_steps",
             "kernel_src", "ae_max_entries")


def dispatches(d, kernel="step_kernel"):
    """{counter: [value per `kernel` dispatch, in dispatch order]}; rows of
    one dispatch (per-XCD or per-SE instances) are summed."""
    acc = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel in row["Kernel_Name"]:
                acc[row["Counter_Name"]][int(row["Dispatch_Id"])] += float(row["Counter_Value"])
    return {c: [v for _, v in sorted(x.items())] for c, x in acc.items()}


def traced(d):
    """[(start ns, end ns) per step_kernel dispatch, in dispatch order] from
    the --kernel-trace run of the same command (empty if absent)."""
    rows = []
    for f in glob.glob(f"{d}/trace/**/*kernel_trace.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "step_kernel" in row["Kernel_Name"]:
                rows.append((int(row["Dispatch_Id"]), (int(row["Start_Timestamp"]), int(row["End_Timestamp"]))))
    return [v for _, v in sorted(rows)]


def union_ms(iv):
    """Time covered by the intervals (ns pairs), in ms: bench.py's step-kernel
    time when launch sub-ranges overlap."""
    acc, lo, hi = 0, None, None
    for a, b in sorted(iv):
        if hi is None or a > hi:
            if hi is not None:
                acc += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    return (acc + (hi - lo if hi is not None else 0)) / 1e6


def expand(seq):
    """Plan launches [leg, steps(, dispatches)] -> (launch index per dispatch)."""
    out = []
    for i, x in enumerate(seq):
        out += [i] * (x[2] if len(x) > 2 else 1)
    return out


def mean(xs):
    return sum(xs) / len(xs) if xs else None


SECTOR = 32          # bytes gfx950 writes for one lane's 8-byte store (profiles/r3_l)


def probe_factors(d, plan):
    """(fetch factor, state write factor, details) from the traffic probes'
    dispatches in the FETCH_SIZE / WRITE_SIZE passes (bench.py --traffic-probe:
    3 dispatches of kind 0, then 3 of kind 1 on a flat log)."""
    probes = plan.get("probes") or []
    f = {c: v for p in glob.glob(f"{d}/pmc*") for c, v in dispatches(p, "traffic_probe_kernel").items()
         if c in ("FETCH_SIZE", "WRITE_SIZE")}
    if not probes or len(f.get("FETCH_SIZE", [])) != len(probes) or len(f.get("WRITE_SIZE", [])) != len(probes):
        raise SystemExit(f"{d}: the traffic probes are missing (bench.py --traffic-probe)")
    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
    k0 = [i for i, p in enumerate(probes) if p[0] == 0]
    k1 = [i for i, p in enumerate(probes) if p[0] == 1]
    ff = med([probes[i][1] / (f["FETCH_SIZE"][i] * 1024.0) for i in k0])
    wf = med([probes[i][2] / (f["WRITE_SIZE"][i] * 1024.0) for i in k0])
    out = {"state_fetch_factor": ff, "state_write_factor": wf,
           "state_probe_fetch_kb_raw": [f["FETCH_SIZE"][i] for i in k0],
           "state_probe_write_kb_raw": [f["WRITE_SIZE"][i] for i in k0],
           "state_probe_bytes_each_way": probes[k0[0]][1]}
    if k1:
        stores = probes[k1[0]][2] / 8.0
        out.update({"log_store_probe_stores": stores,
                    "log_store_raw_bytes_per_store": med([f["WRITE_SIZE"][i] * 1024.0 / stores for i in k1]),
                    "log_store_probe_write_kb_raw": [f["WRITE_SIZE"][i] for i in k1]})
    return ff, wf, out


def main(d):
    plan = json.load(open(os.path.join(d, "plan.json")))
    seq = plan["launches"]
    ff, wf, probe = probe_factors(d, plan)
    owner = expand(seq)
    per = {}
    for p in sorted(glob.glob(f"{d}/pmc*")):
        for c, vals in dispatches(p).items():
            if len(vals) != len(owner):
                raise SystemExit(f"{p}: {len(vals)} step_kernel dispatches, plan has {len(owner)}")
            acc = [0.0] * len(seq)                     # a launch = the sum of its sub-range dispatches
            for k, v in zip(owner, vals):
                acc[k] += v
            per[c] = acc
    trd = traced(d)
    rows = []
    for leg in ("timed", "streaming", "general"):
        ix = [i for i, x in enumerate(seq) if x[0] == leg]
        if not ix:
            continue
        steps = {seq[i][1] for i in ix}
        trace_ms = (union_ms([iv for k, iv in zip(owner, trd) if k in set(ix)]) / len(ix)
                    if len(trd) == len(owner) else None)
        if len(steps) != 1:
            continue                                   # mixed launch lengths: no per-launch row
        m = {c: mean([v[i] for i in ix]) for c, v in per.items()}
        key = dict(plan["key"], leg=leg, launch_steps=steps.pop())
        if leg == "streaming":
            key["stream_steps"] = plan["stream_steps"]
        row = dict(key)
        # writes: the log stores (the plan's count for the timed leg) at the
        # 32-B sector each costs, the rest (state) at the probe's state factor
        ls = plan.get("log_stores_per_timed_launch", 0.0) if leg == "timed" else None
        raw_w = m["WRITE_SIZE"] * 1024.0
        per_store = probe.get("log_store_raw_bytes_per_store")
        if ls is not None and per_store:
            write_b = max(0.0, raw_w - ls * per_store) * wf + ls * SECTOR
        else:
            write_b = raw_w * wf
        row.update({
            "hbm_bytes_per_launch": m["FETCH_SIZE"] * 1024.0 * ff + write_b,
            "fetch_bytes_per_launch": m["FETCH_SIZE"] * 1024.0 * ff,
            "write_bytes_per_launch": write_b,
            "fetch_kb_raw": m["FETCH_SIZE"], "write_kb_raw": m["WRITE_SIZE"],
            "fetch_factor": ff, "write_factor": wf, "traffic_probes": probe,
            "log_stores_per_launch": ls, "state_bytes_per_launch": plan.get("state_bytes_per_launch"),
            "valu_per_launch": m.get("SQ_INSTS_VALU"), "salu_per_launch": m.get("SQ_INSTS_SALU"),
            "lds_per_launch": m.get("SQ_INSTS_LDS"), "smem_per_launch": m.get("SQ_INSTS_SMEM"),
            "waves": m.get("SQ_WAVES"), "wave_cycles": m.get("SQ_WAVE_CYCLES"),
            "busy_cycles": m.get("SQ_BUSY_CYCLES"), "active_inst_valu": m.get("SQ_ACTIVE_INST_VALU"),
            "grbm_gui_active": m.get("GRBM_GUI_ACTIVE"), "launches_averaged": len(ix),
            # every counter of every pass, per launch (the stall split:
            # SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES)
            "pmc_raw": {c: v for c, v in sorted(m.items())},
            "trace_avg_ms": trace_ms,
            "dispatches_per_launch": seq[ix[0]][2] if len(seq[ix[0]]) > 2 else 1,
            # (rocprofv3 --pmc serialises dispatches, so GRBM_GUI_ACTIVE of
            # overlapping sub-range dispatches does not time one launch)
            "effective_clock_ghz": (m["GRBM_GUI_ACTIVE"] / 8 / (trace_ms / 1e3) / 1e9
                                    if trace_ms and m.get("GRBM_GUI_ACTIVE") and
                                    (len(seq[ix[0]]) < 3 or seq[ix[0]][2] == 1) else None),
            "source": f"rocprofv3 --pmc, separate passes (scripts/pmc_bench.sh, {os.path.basename(d)})",
        })
        rows.append(row)
    json.dump(rows, open(os.path.join(d, "rows.json"), "w"), indent=1)
    print(json.dumps(rows, indent=1))


def merge(files):
    """Merge parsed rows (gpurun_out/pmc_*/rows.json, pulled back from the GPU
    box) into profiles/pmc_rows.json; a new row replaces one with the same key."""
    try:
        rows = json.load(open(OUT_FILE))
    except (OSError, ValueError):
        rows = []
    ident = lambda r: tuple(r.get(k) for k in ID_FIELDS)  # noqa: E731
    for f in files:
        new = json.load(open(f))
        keys = {ident(r) for r in new}
        rows = [r for r in rows if ident(r) not in keys] + new
    json.dump(rows, open(OUT_FILE, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--merge":
        merge(sys.argv[2:])
    else:
        main(sys.argv[1])
