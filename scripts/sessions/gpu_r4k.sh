#!/bin/bash
# Round 4: config 5 (10^5 x 7, partitions) across schedules and launch
# sub-ranges -- the balanced schedule alone measured 5 % below round 3's three
# overlapping sub-ranges.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4k}; mkdir -p $OUT
B="--config 5 --groups 100000 --no-cpu-baseline --handler-batch 0 --no-general-leg --stream-steps 0"
for i in 1 2; do
  for v in "auto 1" "auto 2" "auto 3" "one 3" "one 1"; do
    set -- $v
    timeout -k 10 200 python -u bench.py $B --schedule $1 --subranges $2 > $OUT/c5_$1_$2_$i.log 2>&1 || exit $?
  done
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --config 5 --groups 100000 --no-cpu-baseline --handler-batch 0 --no-general-leg --stream-steps 0 > $OUT/c5d20_auto_1_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --subranges 3 --no-cpu-baseline --handler-batch 0 --no-general-leg --stream-steps 0 > $OUT/c3_auto_3_$i.log 2>&1 || exit $?
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1) $(grep -o '"steps_per_launch": [0-9]*' $f | head -1)"; done > $OUT/summary.txt
exit 0
