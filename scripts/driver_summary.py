"""Summarise a scripts/driver_check.sh run: pytest tail, each bench line's rate
and timing split, and the traced kernels' durations."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
p = os.path.join(d, "pytest.log")
if os.path.exists(p):
    print(open(p).read().strip().splitlines()[-1])
for f in sorted(glob.glob(os.path.join(d, "*.log"))):
    for line in open(f):
        if line.startswith("{"):
            j = json.loads(line)
            t = j.get("timing", {})
            print(f"{os.path.basename(f):14s} {j['value'] / 1e10:.4f}e10 ms/step {j['ms_per_step']:.5f} "
                  f"wall {t.get('wall_ms', 0):.3f} events {t.get('stream_event_ms', 0):.3f} "
                  f"kernel {t.get('step_kernel_ms_total', 0):.3f} commits {j['counters_last_step']['commits']}")
for f in glob.glob(os.path.join(d, "prof", "**", "*kernel_trace.csv"), recursive=True):
    for k in csv.DictReader(open(f)):
        us = (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3
        print(f"  {k['Kernel_Name'][:60]:60s} {us:10.1f} us  grid {k['Grid_Size_X']}x{k['Grid_Size_Y']}")
