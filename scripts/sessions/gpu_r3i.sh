#!/bin/bash
# The 1/8 strong shard (125k groups) and the full size at the driver's 20-step
# command: timing split (wall vs stream events vs kernel), with the forced
# one-rank collective, and with spin-wait synchronisation.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3_i; mkdir -p $OUT
for i in 1 2 3; do
  for G in 125000 1000000; do
    timeout -k 10 200 python -u bench.py --groups $G --steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 > $OUT/g${G}_$i.log 2>&1 || exit $?
    RAFT_BENCH_SYNC=spin timeout -k 10 200 python -u bench.py --groups $G --steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 > $OUT/g${G}_spin_$i.log 2>&1 || exit $?
  done
  RAFT_BENCH_FORCE_COLLECTIVE=1 timeout -k 10 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 > $OUT/coll_$i.log 2>&1 || exit $?
done
echo done >> $OUT/status.txt
