#!/bin/bash
# time alternative engine builds (RAFT_ENGINE_LIB) on the same bench workload
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-var}; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -q --timeout 200 \
   --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"; [ $rc -gt 1 ] && exit $rc
for v in ${VARIANTS:-base}; do
  lib=raft-kotlin_amd/lib/libraft_engine.so; [ "$v" != base ] && lib=raft-kotlin_amd/lib/libraft_engine_$v.so
  for k in ${KS:-1 32}; do
    RAFT_ENGINE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline \
        --steps-per-launch $k > "$OUT/bench_${v}_k$k.log" 2>&1
    rc=$?; echo "$v k=$k rc=$rc" >> "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
