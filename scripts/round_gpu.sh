#!/bin/bash
# One GPU session: parity tests, smoke, the default bench (with CPU baseline),
# a kernel-trace profile of the bench, and the PMC traffic passes.  Every GPU
# step has its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-round}; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/bench.log"; [ $rc -ne 0 ] && exit $rc
# kernel-trace of the fused bench (K=512 launches only) and of the streaming form (K=1)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python bench.py --steps 2048 --warmup 512 --stream-steps 0 --no-cpu-baseline > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc" | tee -a "$OUT/trace.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_k1" -o run --output-format csv -- \
    python bench.py --steps 512 --warmup 64 --steps-per-launch 1 --stream-steps 0 --no-cpu-baseline \
    > "$OUT/trace_k1.log" 2>&1
rc=$?; echo "trace_k1 rc=$rc" | tee -a "$OUT/trace_k1.log"; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-round} bash scripts/traffic.sh
