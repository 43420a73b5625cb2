#!/bin/bash
# Round 4 final evidence at the last kernel sources (per-workload automatic
# launch shape): the GPU suite + smoke, the driver's and the default bench,
# config 5 and textbook lines, forced one-rank RCCL, the N=2 rehearsal, then
# the PMC rows (driver, default, handler batches) and the phase budget.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${TAG:-r4l}
OUT=gpurun_out/$T; mkdir -p $OUT
trap 'find gpurun_out -name "*.csv" -size +256k -exec gzip -q {} +' EXIT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc; }
step pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_default 500 python -u bench.py
B="--no-cpu-baseline --handler-batch 0 --no-general-leg"
step c5 300 python -u bench.py --config 5 --groups 100000 $B
step tb3 300 python -u bench.py --mode textbook $B
step rccl_driver 300 env RAFT_BENCH_FORCE_COLLECTIVE=1 python -u bench.py --steps 20 --warmup 5 $B
TAG=$T/dist STEPS=512 bash scripts/dist_rehearsal.sh > $OUT/dist.log 2>&1; echo "dist rc=$?" >> $OUT/status.txt
TAG=${T}_d20 ARGS="--steps 20 --warmup 5" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_d20 rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=${T}_def ARGS="--handler-batch 0" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_def rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=$T bash scripts/pmc_handler.sh > $OUT/pmch.log 2>&1; rc=$?; echo "pmch rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=$T bash scripts/phase_budget.sh; rc=$?; echo "phase rc=$rc" >> $OUT/status.txt
exit 0
