#!/bin/bash
# A/B: 8 waves per SIMD (scratch spills at R = 5) with 360-step launches (8 workgroups' LDS) vs the
# default build (7 waves, 400-step launches), config 3.  Experiment only.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-ab_w8}; mkdir -p $OUT
for i in 1 2; do
  for v in "base:400" "w8:360" "base:360"; do
    name=${v%%:*}; k=${v#*:}
    lib=raft-kotlin_amd/lib/libraft_engine.so; [ "$name" != base ] && lib=raft-kotlin_amd/lib/libraft_engine_$name.so
    RAFT_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 10800 --steps-per-launch $k --no-cpu-baseline --stream-steps 0 > $OUT/${name}_${k}_$i.log 2>&1 || exit $?
    echo "$name K=$k $i $(grep -o '"value": [0-9.e+]*' $OUT/${name}_${k}_$i.log) $(grep -o '"kernel_avg_ms": [0-9.]*' $OUT/${name}_${k}_$i.log | head -1)" >> $OUT/status.txt
  done
done
