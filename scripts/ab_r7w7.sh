#!/bin/bash
# A/B: config 5 (R = 7) with its step kernel allocated for 7 waves per SIMD (scratch spills) and
# 400-step launches vs the default build (6 waves, 500-step launches).  Experiment only.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-ab_r7w7}; mkdir -p $OUT
for i in 1 2; do
  for v in "base:512" "all7:400" "base:400"; do
    name=${v%%:*}; k=${v#*:}
    lib=raft-kotlin_amd/lib/libraft_engine.so; [ "$name" != base ] && lib=raft-kotlin_amd/lib/libraft_engine_$name.so
    RAFT_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --config 5 --groups 100000 --steps 10000 --steps-per-launch $k --no-cpu-baseline --stream-steps 0 > $OUT/${name}_${k}_$i.log 2>&1 || exit $?
    echo "$name K=$k $i $(grep -o '"value": [0-9.e+]*' $OUT/${name}_${k}_$i.log) $(grep -o '"kernel_avg_ms": [0-9.]*' $OUT/${name}_${k}_$i.log | head -1)" >> $OUT/status.txt
  done
done
