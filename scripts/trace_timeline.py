"""The timed region's timeline from a rocprofv3 trace of one bench.py command
(the driver's kind: one timed launch): for the last step_kernel dispatch and
every dispatch after it (the counter reduction, the row copy, the RCCL
all-reduce), start / end relative to the step kernel's start, in µs; with
--hip-runtime-trace, also the host's HIP calls from 300 µs before that start
to the end of the synchronisation that follows it, on the same clock.

    python scripts/trace_timeline.py gpurun_out/r5_d/trace_s8
"""
import csv
import glob
import os
import json
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").split("(")[0][-70:]


def main(d):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), short(row["Kernel_Name"])))
    rows.sort()
    steps = [i for i, r in enumerate(rows) if "step_kernel" in r[2]]
    if not steps:
        raise SystemExit("no step_kernel dispatch")
    # TIMELINE_STEP: which step_kernel dispatch (bench.py --kernel-timing
    # replay runs the timed launch again after the clock: -3 is the timed one)
    i0 = steps[int(os.environ.get("TIMELINE_STEP", "-1"))]
    t0 = rows[i0][0]
    gpu = [{"kernel": k, "start_us": (a - t0) / 1e3, "end_us": (b - t0) / 1e3, "dur_us": (b - a) / 1e3}
           for a, b, k in rows[i0:i0 + 8]]
    api = []
    for f in glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            a, b = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            if t0 - 300_000 <= a <= rows[min(len(rows) - 1, i0 + 8)][1] + 200_000:
                api.append((a, b, row.get("Function") or row.get("Operation") or "?", row.get("Thread_Id")))
    api.sort()
    # the host calls up to the first synchronisation that returns after the step kernel ended
    end = rows[i0][1]
    host = []
    for a, b, fn, tid in api:
        host.append({"call": fn, "start_us": (a - t0) / 1e3, "end_us": (b - t0) / 1e3, "thread": tid})
        if "Synchronize" in fn and b > end:
            break
    print(json.dumps({"dir": d, "gpu": gpu, "host": host}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
