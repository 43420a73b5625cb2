"""Summarise rocprofv3 --pmc CSVs: mean per dispatch of each counter, per kernel."""
import csv, glob, sys, collections
root = sys.argv[1]
kfilter = sys.argv[2] if len(sys.argv) > 2 else "step_kernel"
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in sorted(glob.glob(f"{root}/pmc*/*counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if kfilter not in k:
            continue
        key = k.split("(")[0][-40:]
        acc[key][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[(key, row["Counter_Name"])].add(row["Dispatch_Id"])
        acc[key]["_vgpr"] = float(row.get("VGPR_Count", row.get("Arch_VGPR_Count", 0)) or 0)
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        n = len(disp[(k, c)]) or 1
        print(f"  {c:24s} {v / n:.4g}")
