#!/bin/bash
# Launch sub-ranges (streams) against the launch-boundary tail: bench.py at
# config 3's strong-shard sizes and config 5, for each sub-range count.
#   TAG=x SIZES="125000 250000 1000000" SUBS="1 2 3" scripts/subrange_sweep.sh
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-subsweep}; mkdir -p "$OUT"
for G in ${SIZES:-125000 250000 500000 1000000}; do
  for n in ${SUBS:-1 2 3 4}; do
    log="$OUT/c3_${G}_s$n.log"
    timeout -k 10 200 python -u bench.py --groups $G --subranges $n --no-cpu-baseline --stream-steps 0 ${ARGS:-} > "$log" 2>&1
    rc=$?; echo "c3 G=$G sub=$n rc=$rc $(grep -o '"value": [0-9.e+]*' "$log") $(grep -o '"kernel_avg_ms": [0-9.]*' "$log" | head -1)" >> "$OUT/status.txt"
    [ $rc -ne 0 ] && exit $rc
  done
done
for n in ${SUBS5:-1 2 3 4}; do
  log="$OUT/c5_s$n.log"
  timeout -k 10 200 python -u bench.py --config 5 --groups 100000 --subranges $n --no-cpu-baseline --stream-steps 0 ${ARGS:-} > "$log" 2>&1
  rc=$?; echo "c5 sub=$n rc=$rc $(grep -o '"value": [0-9.e+]*' "$log") $(grep -o '"kernel_avg_ms": [0-9.]*' "$log" | head -1)" >> "$OUT/status.txt"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
