"""Parse scripts/pmc_handler.sh output: per handler batch (a batch_keys_kernel
or bucket_tile_kernel dispatch starts one) the HBM bytes of all its kernels
(bucketed path: the tile partition and bucket_batch_kernel; sorted path: keys,
the rocprim radix sort, batch_kernel) and of the handler kernel alone, from FETCH_SIZE / WRITE_SIZE
with the calibration engine's counter-to-bytes factors (scripts/pmc_parse.py),
and the kernels' durations from the trace.  Rows (one per batch kind) ->
<dir>/handler_rows.json; `--merge` folds them into profiles/pmc_handler.json,
which bench.py's handler_batch leg reads."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import pmc_parse  # noqa: E402

OUT_FILE = os.path.join(ROOT, "profiles", "pmc_handler.json")
# the calibration engine of scripts/traffic_run.py calib: every launch moves
# exactly CALIB_G * (CALIB_R * REPLICA_BYTES + GROUP_BYTES) bytes each way
CALIB_G, CALIB_R = int(os.environ.get("TRAFFIC_GROUPS", "1000000")), 5
REPLICA_BYTES, GROUP_BYTES = 64, 12          # abi.REPLICA_STATE_BYTES, GROUP_STATE_BYTES


def kernels(d, counter=None):
    """[(dispatch id, kernel name, value)] in dispatch order: the counter's
    value (rows of one dispatch summed) or, without a counter, the duration (ns)."""
    acc = defaultdict(float)
    name = {}
    if counter:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                if row["Counter_Name"] == counter:
                    k = int(row["Dispatch_Id"])
                    acc[k] += float(row["Counter_Value"])
                    name[k] = row["Kernel_Name"]
    else:
        for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                k = int(row["Dispatch_Id"])
                acc[k] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                name[k] = row["Kernel_Name"]
    return [(k, name[k], acc[k]) for k in sorted(acc)]


def short(nm):
    """A kernel's name without namespaces, template arguments or parameters."""
    nm = nm.replace("(anonymous namespace)::", "").split("(")[0]
    return nm.split("<")[0].split("::")[-1].replace("void ", "").strip()


def runs(names):
    """Consecutive repeats folded: ["a", "b", "b"] -> ["a", "b x2"]."""
    out = []
    for nm in names:
        if out and out[-1][0] == nm:
            out[-1][1] += 1
        else:
            out.append([nm, 1])
    return [nm if c == 1 else f"{nm} x{c}" for nm, c in out]


def batches(rows):
    """Group a dispatch list into handler batches: each starts at its first
    kernel (batch_keys_kernel on the sorted path, bucket_tile_kernel on the
    bucketed one)."""
    out, cur = [], None
    for _, n, v in rows:
        if "batch_keys_kernel" in n or "bucket_tile_kernel" in n:
            cur = []
            out.append(cur)
        elif "scatter_probe_kernel" in n:                    # the calibration probes end the batches
            cur = None
        if cur is not None:
            cur.append((n, v))
    return out


def scatter_factors(d, plan):
    """Bytes per counted byte of scattered single-word accesses: the
    scatter_probe_kernel dispatches of the same --pmc passes (kind 2 loads in
    the FETCH_SIZE pass, kind 3 stores in the WRITE_SIZE pass; each moves the
    32-B sectors the plan states), the median of each kind's dispatches."""
    probes = plan.get("probes") or []
    out = {}
    for c, kind, col in (("FETCH_SIZE", 2, 1), ("WRITE_SIZE", 3, 2)):
        known = [p[col] for p in probes if p[0] == kind]
        rows = [v for _, nm, v in kernels(f"{d}/pmc_{c}", c) if "scatter_probe_kernel" in nm]
        vals = rows[:3] if kind == 2 else rows[3:]
        if not known or not vals:
            return None
        r = sorted(known[i] / (v * 1024.0) for i, v in enumerate(vals[: len(known)]) if v)
        out[c] = {"factor": r[len(r) // 2], "probe_kb_raw": sorted(vals), "probe_bytes": known[0]}
    return out


def main(d):
    plan = json.loads([ln for ln in open(f"{d}/trace.log") if ln.startswith("{")][-1])
    state = CALIB_G * (CALIB_R * REPLICA_BYTES + GROUP_BYTES)
    cf = sorted(pmc_parse.dispatches(f"{d}/calib_FETCH_SIZE").get("FETCH_SIZE", []))
    cw = sorted(pmc_parse.dispatches(f"{d}/calib_WRITE_SIZE").get("WRITE_SIZE", []))
    # streaming factors (the calibration engine's state launches) and, when the
    # probe ran, the scattered-access factors that the handler rows use
    sff, swf = state / (cf[len(cf) // 2] * 1024.0), state / (cw[len(cw) // 2] * 1024.0)
    sc = scatter_factors(d, plan)
    ff, wf = (sc["FETCH_SIZE"]["factor"], sc["WRITE_SIZE"]["factor"]) if sc else (sff, swf)
    fb, wb, tb = (batches(kernels(f"{d}/pmc_FETCH_SIZE", "FETCH_SIZE")),
                  batches(kernels(f"{d}/pmc_WRITE_SIZE", "WRITE_SIZE")), batches(kernels(f"{d}/trace")))
    kinds = [k for k, reps in plan["plan"] for _ in range(reps)]
    if not (len(fb) == len(wb) == len(tb) == len(kinds)):
        raise SystemExit(f"batches: fetch {len(fb)} write {len(wb)} trace {len(tb)} plan {len(kinds)}")
    rows = []
    for kind in dict.fromkeys(kinds):
        ix = [i for i, k in enumerate(kinds) if k == kind][1:] or [kinds.index(kind)]   # the first is a warmup
        n = plan["n"]

        def avg(bl, sel=lambda nm: True):
            return sum(sum(v for nm, v in bl[i] if sel(nm)) for i in ix) / len(ix)
        hk = lambda nm: "batch_kernel" in nm  # noqa: E731
        fkb, wkb = avg(fb), avg(wb)                         # raw FETCH_SIZE / WRITE_SIZE, KB per batch
        fetch, write = fkb * 1024 * ff, wkb * 1024 * wf
        hfetch, hwrite = avg(fb, hk) * 1024 * ff, avg(wb, hk) * 1024 * wf
        t_all, t_h = avg(tb) / 1e6, avg(tb, hk) / 1e6
        rows.append({"kind": kind, "n": n, "groups": plan["groups"], "replicas": plan["replicas"],
                     "kernel_src": plan["kernel_src"], "library_src": plan.get("library_src"),
                     "batch_src": plan.get("batch_src"),
                     "batch_path": plan.get("batch_path", 0),
                     "batches_averaged": len(ix),
                     "hbm_bytes_per_batch": fetch + write, "hbm_bytes_per_message": (fetch + write) / n,
                     "handler_kernel_hbm_bytes_per_message": (hfetch + hwrite) / n,
                     "handler_kernel_fetch_bytes": hfetch, "handler_kernel_write_bytes": hwrite,
                     "kernels_ms_per_batch": t_all, "handler_kernel_ms": t_h,
                     "handler_kernel_hbm_gbs": (hfetch + hwrite) / (t_h / 1e3) / 1e9 if t_h else None,
                     "kernels_per_batch": runs([short(nm) for nm, _ in tb[ix[0]]]),
                     "fetch_kb_raw": fkb, "write_kb_raw": wkb,
                     "raw_bytes_per_message": (fkb + wkb) * 1024 / n,
                     "streaming_calibrated_bytes_per_message": (fkb * sff + wkb * swf) * 1024 / n,
                     "fetch_factor": ff, "write_factor": wf,
                     "calibration": "scatter" if sc else "streaming",
                     "scatter_probe": sc, "streaming_factors": {"fetch": sff, "write": swf},
                     "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes + --kernel-trace "
                               f"(scripts/pmc_handler.sh, {os.path.basename(d)})"})
    json.dump(rows, open(os.path.join(d, "handler_rows.json"), "w"), indent=1)
    print(json.dumps(rows, indent=1))


def merge(files):
    try:
        have = json.load(open(OUT_FILE))
    except (OSError, ValueError):
        have = []
    key = lambda r: (r["kind"], r["n"], r["groups"], r["replicas"], r.get("batch_path", 0),  # noqa: E731
                     r.get("batch_src") or r.get("library_src") or r["kernel_src"])
    out = {key(r): r for r in have}
    for f in files:
        for r in json.load(open(f)):
            out[key(r)] = r
    json.dump(list(out.values()), open(OUT_FILE, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "--merge":
        merge(sys.argv[2:])
    else:
        main(sys.argv[1])
