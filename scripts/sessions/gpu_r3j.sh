#!/bin/bash
# The forced one-rank collective at the 1/8 shard's 20-step command, with the
# all-reduce warmed up; per-phase host timestamps (RAFT_BENCH_TRACE).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3_j; mkdir -p $OUT
for i in 1 2 3; do
  RAFT_BENCH_FORCE_COLLECTIVE=1 timeout -k 10 200 python -u bench.py --groups 125000 --steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 > $OUT/coll_$i.log 2>&1 || exit $?
  RAFT_BENCH_FORCE_COLLECTIVE=1 timeout -k 10 200 python -u bench.py --groups 1000000 --steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 > $OUT/coll1m_$i.log 2>&1 || exit $?
done
echo done >> $OUT/status.txt
