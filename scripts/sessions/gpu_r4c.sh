#!/bin/bash
# Round 4 evidence, part 2: rocprofv3 kernel-trace stats and PMC rows of the
# driver's command and of the default bench (scripts/pmc_bench.sh), the
# handler batches' PMC rows (scripts/pmc_handler.sh), and kernel traces of the
# config-4 shards at 20 steps.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4c}; mkdir -p $OUT
# raw rocprofv3 csv files are compressed on the way out (gpurun copies back <= 64 MiB)
trap 'find gpurun_out -name "*.csv" -size +256k -exec gzip -q {} +' EXIT
TAG=r4c_d20 ARGS="--steps 20 --warmup 5" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_d20 rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r4c_def ARGS="--handler-batch 0" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_def rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r4c bash scripts/pmc_handler.sh > $OUT/pmch.log 2>&1; rc=$?; echo "pmch rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r4c bash scripts/phase_budget.sh; rc=$?; echo "phase rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
for g in 125000 250000 500000; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace_s$g" -o run --output-format csv -- \
      python bench.py --steps 20 --warmup 5 --groups $g --no-cpu-baseline --handler-batch 0 --stream-steps 0 \
      --no-general-leg > "$OUT/trace_s$g.log" 2>&1; rc=$?; echo "trace_s$g rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
done
exit 0
