#!/bin/bash
# A/B timing of engine builds (RAFT_ENGINE_LIB, scripts/build_variants.sh) on
# one bench command, interleaved ROUNDS times (experiments only).
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-ab}; mkdir -p "$OUT"
for i in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    lib=raft-kotlin_amd/lib/libraft_engine.so; [ "$v" != base ] && lib=raft-kotlin_amd/lib/libraft_engine_$v.so
    RAFT_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py ${ARGS:---steps 10000} --no-cpu-baseline \
        --stream-steps 0 > "$OUT/${v}_$i.log" 2>&1
    rc=$?; echo "$v $i rc=$rc $(grep -o '"value": [0-9.e+]*' "$OUT/${v}_$i.log")" >> "$OUT/status.txt"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
