#!/bin/bash
# Launch length vs occupancy: a 500-step launch's LDS counter rows allow 6
# workgroups per CU, a 400-step launch's 7 (the VGPR limit at 71 registers).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-kocc}; mkdir -p "$OUT"
for g in 1000000 125000; do
  for k in 500 400 250; do
    timeout -k 10 200 python -u bench.py --groups $g --steps 10000 --steps-per-launch $k --no-cpu-baseline \
        --stream-steps 0 > "$OUT/g${g}_k$k.log" 2>&1 || exit $?
    echo "groups=$g K=$k $(grep -o '"value": [0-9.e+]*' "$OUT/g${g}_k$k.log")" >> "$OUT/status.txt"
  done
done
