"""Step-kernel time from a rocprofv3 --kernel-trace CSV as bench.py's
roofline.kernel_avg_ms measures it: the union of the step-kernel dispatch
intervals (launch sub-ranges overlap), divided by the number of full-grid
K-step launches (dispatches / sub-ranges), next to the plain per-dispatch
average that rocprofv3 --stats reports.

    python scripts/trace_union.py <dir with *kernel_trace.csv> [subranges] [launches] [skip_dispatches]

launches / skip_dispatches select the timed launches of a bench run: e.g. the
default run's trace is 3 warmup dispatches, then 25 timed launches x 3, then
the streaming leg: `... 3 25 3`."""
import csv
import glob
import json
import sys


def main(d, nsub=None, first=None, skip=0):
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "step_kernel" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id"),
                             int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)))
    rows.sort()
    rows = rows[skip:]
    streams = sorted({r[2] for r in rows})
    nsub = nsub or len(streams)
    if first:
        rows = rows[: first * nsub]
    acc, lo, hi = 0, None, None
    for a, b, _, _ in rows:
        if hi is None or a > hi:
            if hi is not None:
                acc += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    if hi is not None:
        acc += hi - lo
    launches = len(rows) / nsub
    out = {"dispatches": len(rows), "streams": len(streams), "subranges": nsub, "launches": launches,
           "union_ms": acc / 1e6, "union_ms_per_launch": acc / 1e6 / launches if launches else None,
           "dispatch_avg_ms": sum(b - a for a, b, _, _ in rows) / 1e6 / len(rows) if rows else None,
           "span_ms": (rows[-1][1] - rows[0][0]) / 1e6 if rows else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None, int(sys.argv[3]) if len(sys.argv) > 3 else None,
         int(sys.argv[4]) if len(sys.argv) > 4 else 0)
