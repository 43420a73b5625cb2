#!/bin/bash
# The GPU parity suite, the driver's own bench command (N runs, no CPU leg),
# one default bench, and a rocprofv3 kernel trace + stats of the driver's
# command.  Every GPU step has its own time limit; a failure ends the script.
# Summarise with: python3 scripts/driver_summary.py gpurun_out/<TAG>
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dcheck}; mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit $?
fi
for i in $(seq 1 ${N:-3}); do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/driver_$i.log" 2>&1 || exit $?
done
[ -n "$SKIP_DEFAULT" ] || { timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/default.log" 2>&1 || exit $?; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --stream-steps 0 > "$OUT/trace.log" 2>&1
