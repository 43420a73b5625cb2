#!/bin/bash
# A/B timing of engine builds on one bench command, interleaved ROUNDS times
# (experiments only).  VARIANTS lists builds as NAME or NAME:K -- NAME is
# "base" (the working tree's library) or a scripts/build_variants.sh variant,
# K an optional --steps-per-launch for that entry (e.g. "base:400 w8:360").
#   TAG=x ARGS="--steps 10000 --config 5 --groups 100000" VARIANTS="base nocnt" scripts/ab.sh
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-ab}; mkdir -p "$OUT"
for i in $(seq ${ROUNDS:-2}); do
  for spec in ${VARIANTS:-base}; do
    v=${spec%%:*}; k=""; [ "$spec" != "$v" ] && k="--steps-per-launch ${spec#*:}"
    lib=raft-kotlin_amd/lib/libraft_engine.so; [ "$v" != base ] && lib=raft-kotlin_amd/lib/libraft_engine_$v.so
    log="$OUT/${spec//:/_}_$i.log"
    RAFT_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py ${ARGS:---steps 10000} $k --no-cpu-baseline \
        --stream-steps 0 > "$log" 2>&1
    rc=$?; echo "$spec $i rc=$rc $(grep -o '"value": [0-9.e+]*' "$log") $(grep -o '"kernel_avg_ms": [0-9.]*' "$log" | head -1)" >> "$OUT/status.txt"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
