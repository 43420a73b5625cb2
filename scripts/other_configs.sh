#!/bin/bash
# One bench line (no CPU leg) for each of the other workloads; appended to $OUT/bench_other_configs.jsonl.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-other}; mkdir -p "$OUT"
run() {
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > "$OUT/b.log" 2>&1
  rc=$?; echo "$* rc=$rc" >> "$OUT/status.txt"; [ $rc -ne 0 ] && { cat "$OUT/b.log"; exit $rc; }
  grep '^{' "$OUT/b.log" | tail -1 >> "$OUT/bench_other_configs.jsonl"
}
run --config 5 --groups 100000
run --mode textbook
run --config 5 --groups 100000 --mode textbook
run --config 2 --groups 10000 --steps 1000
exit 0
