#!/bin/bash
# Round 4: priority modes (bands vs rank in the workgroup every 1, 4, 16 steps) on
# the driver's launch and the 1/8 shard, interleaved over two rounds.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4a6}; mkdir -p $OUT
B="--no-cpu-baseline --handler-batch 0 --stream-steps 0 --no-general-leg"
for i in 1 2; do
  for v in base r1 r4 r16; do
    L=$PWD/raft-kotlin_amd/lib/libraft_engine.so; [ $v != base ] && L=$PWD/raft-kotlin_amd/lib/libraft_engine_$v.so
    for g in 1000000 125000; do
      RAFT_ENGINE_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --groups $g $B > $OUT/${v}_${g}_$i.log 2>&1
      rc=$?; echo "${v}_${g}_$i rc=$rc $(grep -o '"kernel_avg_ms": [0-9.]*' $OUT/${v}_${g}_$i.log | head -1)" >> $OUT/status.txt
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
exit 0
