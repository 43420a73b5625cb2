#!/bin/bash
# Round 4 probe: balanced launches with fewer workgroups than the GPU holds
# (--schedule-workgroups) at the 1/8 shard and full size, 20 steps.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4y}; mkdir -p $OUT
B="--steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 --no-general-leg --stream-steps 0"
for i in 1 2; do
  for w in 0 1536 1280; do
    timeout -k 10 200 python -u bench.py $B --groups 125000 --schedule-workgroups $w > $OUT/s8_w${w}_$i.log 2>&1 || exit $?
  done
  for w in 0 1536; do
    timeout -k 10 200 python -u bench.py $B --schedule-workgroups $w > $OUT/d20_w${w}_$i.log 2>&1 || exit $?
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1)"; done > $OUT/summary.txt
exit 0
