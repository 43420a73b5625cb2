#!/bin/bash
# One bench line (no CPU leg) for each of the other workloads; appended to $OUT/bench_other_configs.jsonl.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-other}; mkdir -p "$OUT"
run() {
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "$OUT/b.log" 2>&1
  rc=$?; echo "$* rc=$rc" >> "$OUT/status.txt"; [ $rc -ne 0 ] && { cat "$OUT/b.log"; exit $rc; }
  grep '^{' "$OUT/b.log" | tail -1 >> "$OUT/bench_other_configs.jsonl"
}
run --config 5 --groups 100000 --handler-batch 0
run --mode textbook --handler-batch 0
run --mode textbook --ae-max-entries 8 --handler-batch 0
run --config 5 --groups 100000 --mode textbook --handler-batch 0
run --config 2 --groups 10000 --steps 1000 --handler-batch 0
run --groups 125000 --handler-batch 0
run --groups 250000 --handler-batch 0
exit 0
