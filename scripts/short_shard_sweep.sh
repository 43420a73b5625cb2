#!/bin/bash
# The config-4 1/8 shard (1.25e5 groups) over the driver's 20 steps: one
# 20-step launch vs shorter launches overlapped on launch sub-ranges
# (VARIANTS: "spl:subranges"), interleaved ROUNDS times.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-short_shard}; mkdir -p "$OUT"
for i in $(seq ${ROUNDS:-3}); do
  for v in ${VARIANTS:-20:1 20:3 10:1 10:2 10:3 5:3 4:3}; do
    spl=${v%%:*}; sub=${v#*:}
    timeout -k 10 120 python -u bench.py --groups ${GROUPS_:-125000} --steps 20 --warmup 5 --steps-per-launch $spl \
        --subranges $sub --no-cpu-baseline --handler-batch 0 --stream-steps 0 > "$OUT/${spl}_${sub}_$i.log" 2>&1 || exit $?
    echo "$v $i $(grep -o '"value": [0-9.e+]*' "$OUT/${spl}_${sub}_$i.log") $(grep -o '"wall_ms": [0-9.]*' "$OUT/${spl}_${sub}_$i.log")" >> "$OUT/status.txt"
  done
done
