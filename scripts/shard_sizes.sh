#!/bin/bash
# Per-GPU rate of config 4's strong shards on ONE MI355X: 10^6 groups split over
# N = 1, 2, 4, 8 GPUs leaves 10^6 / N groups per GPU (bench.py --groups).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-shards}; mkdir -p "$OUT"
for g in 1000000 500000 250000 125000; do
  timeout -k 10 200 python -u bench.py --groups $g --steps 10000 --no-cpu-baseline --stream-steps 0 \
      > "$OUT/g$g.log" 2>&1 || exit $?
  echo "groups=$g $(grep -o '"value": [0-9.e+]*' "$OUT/g$g.log") $(grep -o '"kernel_avg_ms": [0-9.]*' "$OUT/g$g.log" | head -1)" >> "$OUT/status.txt"
done
