#!/bin/bash
# Round 4: the host side of a short timed region -- the 1/8 shard and the
# full size at 20 steps with the runtime's default wait, an active wait
# (ROC_ACTIVE_WAIT_TIMEOUT) and hipDeviceScheduleSpin.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4f}; mkdir -p $OUT
B="--steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 --stream-steps 0 --no-general-leg"
for i in 1 2; do
  for g in 125000 1000000; do
    timeout -k 10 200 python -u bench.py $B --groups $g > $OUT/def_${g}_$i.log 2>&1 || exit $?
    timeout -k 10 200 env ROC_ACTIVE_WAIT_TIMEOUT=100000 python -u bench.py $B --groups $g > $OUT/act_${g}_$i.log 2>&1 || exit $?
    timeout -k 10 200 python -u scripts/debug/spin_bench.py $B --groups $g > $OUT/spin_${g}_$i.log 2>&1 || exit $?
  done
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"wall_ms": [0-9.]*' $f | head -1) $(grep -o '"stream_event_ms": [0-9.]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1)"; done > $OUT/summary.txt
exit 0
