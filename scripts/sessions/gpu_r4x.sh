#!/bin/bash
# Round 4: config 4's per-GPU shard sizes on one MI355X at the final kernel
# (10^6 / N groups for N = 1, 2, 4, 8; the driver's 20 steps and 10^4 steps):
# the strong-scaling factor a node of N GPUs would reach, shard by shard.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4x}; mkdir -p $OUT
B="--no-cpu-baseline --handler-batch 0 --no-general-leg --stream-steps 0"
for g in 1000000 500000 250000 125000; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --groups $g $B > $OUT/d20_$g.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --groups $g $B > $OUT/def_$g.log 2>&1 || exit $?
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"ms_per_step": [0-9.e+-]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1)"; done > $OUT/summary.txt
exit 0
