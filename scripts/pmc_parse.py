"""Parse scripts/pmc_bench.sh output into per-launch PMC rows of the step
kernel, written to <dir>/rows.json; `--merge` folds such files into
profiles/pmc_rows.json (bench.py attaches a row only to a run with the same
workload key and launch length).

Every step_kernel dispatch of a PMC pass is matched, in dispatch order, to
the launch sequence bench.py wrote (--plan-file: warmup, timed and streaming
launches with their step counts).  FETCH_SIZE / WRITE_SIZE are kilobytes per
dispatch; the calibration engine, whose launches move exactly
G * (R * 60 + 12) bytes, converts them to bytes for this kernel's 4-byte
per-lane access pattern (MI355X_MICROARCH.md calibrates gfx950's factor for
16 B/lane streams only)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT_FILE = os.path.join(ROOT, "profiles", "pmc_rows.json")
CALIB_G, CALIB_R = int(os.environ.get("TRAFFIC_GROUPS", "1000000")), 5
REPLICA_BYTES, GROUP_BYTES = 4 * 13 + 8, 12
ID_FIELDS = ("config", "mode", "groups", "warmup", "steps", "log_window", "leg", "launch_steps", "stream_steps",
             "kernel_src", "ae_max_entries")


def dispatches(d):
    """{counter: [value per step_kernel dispatch, in dispatch order]}; rows of
    one dispatch (per-XCD or per-SE instances) are summed."""
    acc = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "step_kernel" in row["Kernel_Name"]:
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


def main(d):
    plan = json.load(open(os.path.join(d, "plan.json")))
    seq = plan["launches"]
    state = CALIB_G * (CALIB_R * REPLICA_BYTES + GROUP_BYTES)
    cf = sorted(dispatches(f"{d}/calib_FETCH_SIZE").get("FETCH_SIZE", []))
    cw = sorted(dispatches(f"{d}/calib_WRITE_SIZE").get("WRITE_SIZE", []))
    ff = state / (cf[len(cf) // 2] * 1024.0)
    wf = state / (cw[len(cw) // 2] * 1024.0)
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
        row.update({
            "hbm_bytes_per_launch": m["FETCH_SIZE"] * 1024.0 * ff + m["WRITE_SIZE"] * 1024.0 * wf,
            "fetch_bytes_per_launch": m["FETCH_SIZE"] * 1024.0 * ff,
            "write_bytes_per_launch": m["WRITE_SIZE"] * 1024.0 * wf,
            "fetch_kb_raw": m["FETCH_SIZE"], "write_kb_raw": m["WRITE_SIZE"],
            "fetch_factor": ff, "write_factor": wf, "calib_state_bytes": state,
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
