"""Per-phase VALU / SALU budget from scripts/phase_budget.sh: SQ_INSTS_* of the
timed step-kernel launch (the last step_kernel dispatch of the bench run) of
the product build and of each RAFT_PHASE_TWICE build; a phase's budget is the
difference (its dynamic instruction count, once), per chunk-step (one wave's
64 // R groups for one step, the unit of earlier rounds' "per wave-step")."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PHASES = {"tw_t": "T: timers, election clocks, session starts", "tw_jobs": "the step's Philox job pass",
          "tw_v": "V: RequestVote rounds", "tw_a": "A: leader ticks (AppendEntries, responses, commit rule)",
          "tw_c": "C: client commands"}


def last_dispatch(d):
    acc = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "step_kernel" in row["Kernel_Name"]:
                acc[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
    return acc[max(acc)] if acc else None


def main(d):
    line = json.loads([ln for ln in open(f"{d}/base.log") if ln.startswith("{")][-1])
    chunks, steps = line["config"]["step_waves_per_rank"], line["roofline"]["launch_steps"]
    base = last_dispatch(f"{d}/base")
    unit = chunks * steps
    out = {"command": "bench.py " + " ".join(sys.argv[2:]) if len(sys.argv) > 2 else "the driver's launch",
           "chunk_steps": unit,
           "total": {"valu": base["SQ_INSTS_VALU"] / unit, "salu": base["SQ_INSTS_SALU"] / unit,
                     "lds": base["SQ_INSTS_LDS"] / unit}, "phases": {}}
    rest_v, rest_s = out["total"]["valu"], out["total"]["salu"]
    for v, name in PHASES.items():
        if not os.path.isdir(f"{d}/{v}"):
            continue
        x = last_dispatch(f"{d}/{v}")
        dv, ds = (x["SQ_INSTS_VALU"] - base["SQ_INSTS_VALU"]) / unit, (x["SQ_INSTS_SALU"] - base["SQ_INSTS_SALU"]) / unit
        out["phases"][name] = {"valu": dv, "salu": ds, "lds": (x["SQ_INSTS_LDS"] - base["SQ_INSTS_LDS"]) / unit}
        rest_v -= dv
        rest_s -= ds
    out["phases"]["the rest: H, D, K, deferred timer draws, counter flush, piece entry/exit"] = {"valu": rest_v,
                                                                                             "salu": rest_s}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
