#!/bin/bash
# Kernel timelines of the launch sub-ranges (do launches of different
# sub-range streams overlap?), and the sub-range sweep with more HW queues.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-subtrace}; mkdir -p "$OUT"
for n in 1 2 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace_s$n" -o run --output-format csv -- \
      python bench.py --groups 125000 --subranges $n --steps 2000 --warmup 0 --stream-steps 0 --no-cpu-baseline \
      > "$OUT/trace_s$n.log" 2>&1; rc=$?; echo "trace s$n rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
done
for q in 8 16; do
  for n in 1 2 3; do
    log="$OUT/hwq${q}_s$n.log"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --groups 125000 --subranges $n --no-cpu-baseline --stream-steps 0 > "$log" 2>&1
    rc=$?; echo "hwq=$q sub=$n rc=$rc $(grep -o '"value": [0-9.e+]*' "$log") $(grep -o '"kernel_avg_ms": [0-9.]*' "$log" | head -1)" >> "$OUT/status.txt"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
