"""Per-batch kernel times of scripts/handler_probe.py runs under
`rocprofv3 --kernel-trace --stats` (one directory per run): every kernel of the
batch path with its calls and average duration, and the sum per batch.

    python scripts/htrace_summary.py gpurun_out/r5_h2b/htrace_*
"""
import csv
import glob
import json
import os
import sys

SKIP = ("step_kernel", "pack_kernel", "init_kernel", "copyBuffer", "FillFunc", "reduce_counters", "rebuild_cache")


def short(name):
    n = name.replace("rocprim::ROCPRIM_400200_NS::", "").replace("(anonymous namespace)::", "")
    for key, label in (("onesweep_iteration", "rocprim onesweep pass"), ("global_offsets", "rocprim onesweep histogram"),
                       ("scan_impl", "rocprim scan"), ("init_lookback", "rocprim init_lookback"),
                       ("fillBuffer", "memset")):
        if key in n:
            return label
    head = n.split("(")[0]
    return head.replace("void ", "")


def main(dirs):
    out = {}
    for d in dirs:
        files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if not files:
            continue
        plan = None
        log = d.rstrip("/") + ".log"
        if os.path.exists(log):
            for line in open(log):
                if line.startswith("{") and '"plan"' in line:
                    plan = json.loads(line)
        batches = sum(k for _, k in plan["plan"]) if plan else None
        rows = {}
        for r in csv.DictReader(open(files[0])):
            if any(s in r["Name"] for s in SKIP):
                continue
            name = short(r["Name"])
            c, tot = rows.get(name, (0, 0.0))
            rows[name] = (c + int(r["Calls"]), tot + float(r["TotalDurationNs"]))
        per = {k: {"calls": c, "avg_us": round(t / c / 1e3, 2),
                   "us_per_batch": round(t / batches / 1e3, 2) if batches else None} for k, (c, t) in rows.items()}
        out[os.path.basename(d.rstrip("/"))] = {
            "batches": batches, "kernels": per,
            "us_per_batch_total": round(sum(t for _, t in rows.values()) / batches / 1e3, 1) if batches else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main([a for a in sys.argv[1:] if os.path.isdir(a)])
