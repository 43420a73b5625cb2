#!/bin/bash
# rocprofv3 evidence for the drop-in handler batches (bench.py's handler_batch
# leg): a kernel trace and FETCH_SIZE / WRITE_SIZE passes (separate runs) of
# scripts/handler_probe.py, the calibration engine under both counters, then
# scripts/pmc_handler_parse.py -> $OUT/handler_rows.json (merge into
# profiles/pmc_handler.json back here: python scripts/pmc_handler_parse.py --merge ...).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/pmch_${TAG:-x}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python scripts/handler_probe.py > "$OUT/trace.log" 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- \
      python scripts/handler_probe.py > "$OUT/pmc_$c.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/calib_$c" -o run --output-format csv -- \
      python scripts/traffic_run.py calib > "$OUT/calib_$c.log" 2>&1 || exit $?
done
python scripts/pmc_handler_parse.py "$OUT"
