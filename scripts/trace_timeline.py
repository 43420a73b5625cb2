"""The timed region's GPU timeline from a rocprofv3 --kernel-trace of one
bench.py command: for the last step_kernel dispatch (the timed launch of a
one-launch region, e.g. the driver's --steps 20) and every dispatch after it
(the counter reduction, copies, the RCCL all-reduce), start / end relative to
the step kernel's start, in µs.

    python scripts/trace_timeline.py gpurun_out/r4c/trace_s125000
"""
import csv
import glob
import json
import sys


def main(d):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            rows.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-70:]))
    rows.sort()
    steps = [i for i, r in enumerate(rows) if "step_kernel" in r[2]]
    if not steps:
        raise SystemExit("no step_kernel dispatch")
    i0 = steps[-1]
    t0 = rows[i0][0]
    out = [{"kernel": k, "start_us": (a - t0) / 1e3, "end_us": (b - t0) / 1e3, "dur_us": (b - a) / 1e3}
           for a, b, k in rows[i0:i0 + 8]]
    print(json.dumps({"dir": d, "timeline": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
