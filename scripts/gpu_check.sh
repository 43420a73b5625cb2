#!/bin/bash
# One GPU session: parity tests, then (only if no crash) smoke and a short bench.
# Every GPU step has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -m gpu -v \
    --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a "$OUT/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/smoke.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py ${BENCH_ARGS:---steps 500 --warmup 50 --no-cpu-baseline} \
    > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/bench.log"
exit $rc
