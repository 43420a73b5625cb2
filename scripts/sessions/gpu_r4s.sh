#!/bin/bash
# Round 4: per-wave start / end stamps (RAFT_WAVE_TIMES build) with the
# age-shifted priority bands, at the 1/8 shard and full size (20 steps).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4s}; mkdir -p $OUT
B="--steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 --stream-steps 0 --no-general-leg"
L=$PWD/raft-kotlin_amd/lib/libraft_engine_wt.so
for g in 125000 1000000; do
  RAFT_ENGINE_LIB=$L timeout -k 10 300 python -u bench.py $B --groups $g > $OUT/wt_$g.log 2> $OUT/wt_$g.err || exit $?
done
gzip $OUT/*.err
exit 0
