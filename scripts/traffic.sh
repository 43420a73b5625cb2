#!/bin/bash
# HBM traffic of the step kernel from rocprofv3 PMC counters: FETCH_SIZE and
# WRITE_SIZE in separate passes (never together, never with tracing), for a
# calibration engine and for the bench workload; then scripts/traffic_parse.py.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/traffic_${TAG:-x}; mkdir -p "$OUT"
for mode in calib workload; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/${mode}_$c" -o run --output-format csv -- \
        python scripts/traffic_run.py $mode > "$OUT/${mode}_$c.log" 2>&1
    rc=$?; echo "$mode $c rc=$rc" >> "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
  done
done
python scripts/traffic_parse.py "$OUT" > "$OUT/traffic.json"
