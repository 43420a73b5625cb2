#!/bin/bash
# Time alternative engine builds (RAFT_ENGINE_LIB, from scripts/build_variants.sh)
# on the default bench workload at K=64; experiments only, no parity check.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-flags}; mkdir -p "$OUT"
for v in ${VARIANTS:-base}; do
  lib=raft-kotlin_amd/lib/libraft_engine.so; [ "${v%%.*}" != base ] && lib=raft-kotlin_amd/lib/libraft_engine_${v%%.*}.so
  RAFT_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --steps ${STEPS:-2000} --warmup 100 --no-cpu-baseline \
      --stream-steps 0 ${EXTRA:-} > "$OUT/bench_$v.log" 2>&1
  rc=$?
  echo "$v rc=$rc $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_ms'])" "$OUT/bench_$v.log" 2>/dev/null)" | tee -a "$OUT/status.txt"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
