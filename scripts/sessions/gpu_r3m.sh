#!/bin/bash
# Launch length with 3 sub-ranges (config 3, 10^6 groups, 10^4 steps), and config 5.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3_m; mkdir -p $OUT
for i in 1 2; do
  for K in 400 250 200 125 433; do
    timeout -k 10 200 python -u bench.py --steps-per-launch $K --no-cpu-baseline --handler-batch 0 --stream-steps 0 > $OUT/k${K}_$i.log 2>&1 || exit $?
    echo "K=$K $i $(grep -o '"value": [0-9.e+]*' $OUT/k${K}_$i.log) $(grep -o '"steps_per_launch": [0-9]*' $OUT/k${K}_$i.log)" >> $OUT/status.txt
  done
  for K in 512 250 400; do
    timeout -k 10 200 python -u bench.py --config 5 --groups 100000 --steps-per-launch $K --no-cpu-baseline --handler-batch 0 --stream-steps 0 > $OUT/c5k${K}_$i.log 2>&1 || exit $?
    echo "c5 K=$K $i $(grep -o '"value": [0-9.e+]*' $OUT/c5k${K}_$i.log) $(grep -o '"steps_per_launch": [0-9]*' $OUT/c5k${K}_$i.log)" >> $OUT/status.txt
  done
done
