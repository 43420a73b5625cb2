#!/bin/bash
# Round 4: the handler parity cases (incl. long per-replica runs), then one
# bench line per other workload at the round-4 kernels (config 5, config 2,
# textbook config 3) with the one-chunk-per-wave schedule beside the default.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4j}; mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -x -k "handler_batches"
B="--no-cpu-baseline --handler-batch 0 --no-general-leg"
step c5 300 python -u bench.py --config 5 --groups 100000 $B
step c5_one 300 python -u bench.py --config 5 --groups 100000 --schedule one $B
step c2 300 python -u bench.py --config 2 --groups 10000 --steps 1000 --warmup 10 $B
step tb3 300 python -u bench.py --mode textbook $B
for f in $OUT/c*.log $OUT/tb*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1) $(grep -o '"frac": [0-9.]*' $f | head -1) $(grep -o '"schedule": "[a-z_]*"' $f | head -1)"; done > $OUT/summary.txt
exit 0
