cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r2ad; mkdir -p $OUT
for i in 1 2; do
  for v in "base:500" "base:400" "w7:400" "w7:500"; do
    name=${v%%:*}; k=${v#*:}
    lib=raft-kotlin_amd/lib/libraft_engine.so; [ "$name" != base ] && lib=raft-kotlin_amd/lib/libraft_engine_$name.so
    RAFT_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 10000 --steps-per-launch $k --no-cpu-baseline --stream-steps 0 > $OUT/${name}_${k}_$i.log 2>&1 || exit $?
    echo "$name K=$k $i $(grep -o '"value": [0-9.e+]*' $OUT/${name}_${k}_$i.log) $(grep -o '"kernel_avg_ms": [0-9.]*' $OUT/${name}_${k}_$i.log | head -1)" >> $OUT/status.txt
  done
done
