#!/bin/bash
# One GPU session: parity tests, smoke, the driver's bench command, the default
# bench (with CPU baseline), the N=2 rehearsal, then rocprofv3 evidence for
# both bench commands.  Every GPU step has its own time limit; a crash, abort
# or time-out ends the script (a plain test failure, rc 1, does not).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-session}; mkdir -p "$OUT"
step() {   # step NAME LIMIT CMD...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  [ $rc -eq 0 ] || [ $rc -eq 1 -a "$name" = pytest ] || exit $rc
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest ${TEST_LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread
  step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_default 400 python -u bench.py ${BENCH_ARGS:-}
[ -n "$SKIP_C5" ] || step bench_c5 300 python -u bench.py --config 5 --groups 100000 --no-cpu-baseline
[ -n "$SKIP_DIST" ] || { TAG=${TAG:-session}/dist STEPS=512 bash scripts/dist_rehearsal.sh > "$OUT/dist.log" 2>&1; rc=$?; echo "dist rc=$rc" | tee -a "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc; }
[ -n "$SKIP_PMC" ] || {
  TAG=${TAG:-session}_d20 ARGS="--steps 20 --warmup 5" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_d20 rc=$rc" | tee -a "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
  TAG=${TAG:-session}_def ARGS="" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_def rc=$rc" | tee -a "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
}
exit 0
