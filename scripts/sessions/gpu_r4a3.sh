#!/bin/bash
# Round 4 diagnostic: per-wave start / end times and hardware slots of the
# driver's launch (RAFT_WAVE_TIMES build), balanced vs one chunk per wave,
# and the 1/8 shard.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r4a3}; mkdir -p $OUT
B="--no-cpu-baseline --handler-batch 0 --stream-steps 0 --no-general-leg"
L=$PWD/raft-kotlin_amd/lib/libraft_engine_wt.so
for s in auto one; do
  RAFT_ENGINE_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --schedule $s $B > $OUT/d20_$s.log 2> $OUT/d20_$s.err
  echo "d20_$s rc=$?" >> $OUT/status.txt
  RAFT_ENGINE_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --groups 125000 --schedule $s $B > $OUT/s8_$s.log 2> $OUT/s8_$s.err
  echo "s8_$s rc=$?" >> $OUT/status.txt
done
gzip $OUT/*.err
exit 0
