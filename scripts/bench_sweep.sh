#!/bin/bash
# parity subset, then bench at several steps-per-launch values
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-sweep}; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_golden.py tests/test_gpu_parity.py::test_steps_per_launch_invariance} -m gpu -q \
   --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"; [ $rc -gt 1 ] && exit $rc
for k in ${KS:-1 8 32}; do
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline --steps-per-launch $k ${EXTRA:-} > "$OUT/bench_k$k.log" 2>&1
  rc=$?; echo "k=$k rc=$rc" >> "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
done
exit 0
