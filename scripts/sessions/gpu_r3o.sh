#!/bin/bash
# The driver's 20-step command at different launch splits: one 20-step launch
# (the bench's choice) vs 2 x 10 and 4 x 5 with 3 sub-ranges.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3_o; mkdir -p $OUT
for i in 1 2 3; do
  for cfg in "20 1" "10 3" "5 3" "20 3"; do
    set -- $cfg
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --steps-per-launch $1 --subranges $2 --no-cpu-baseline --handler-batch 0 > $OUT/k$1_s$2_$i.log 2>&1 || exit $?
    echo "K=$1 sub=$2 $i $(grep -o '"value": [0-9.e+]*' $OUT/k$1_s$2_$i.log) $(grep -o '"kernel_avg_ms": [0-9.]*' $OUT/k$1_s$2_$i.log | head -1) $(grep -o '"wall_ms": [0-9.]*' $OUT/k$1_s$2_$i.log)" >> $OUT/status.txt
  done
done
