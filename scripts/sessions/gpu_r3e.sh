#!/bin/bash
# Session r3_e: slot-major layout parity and A/B timing, sub-range counts incl.
# 4, PMC rows (stall split) of the driver's command and the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r3_e; mkdir -p $OUT
RAFT_ENGINE_LIB=$PWD/raft-kotlin_amd/lib/libraft_engine_slotmaj.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x \
   --timeout 300 --timeout-method thread -k "full_size_digest or config3 or config5 or replica_counts or kats or batches" > $OUT/pytest_slotmaj.log 2>&1
rc=$?; echo "pytest slotmaj rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TAG=r3_e/ab VARIANTS="base slotmaj" ROUNDS=3 ARGS="--steps 10000 --handler-batch 0" bash scripts/ab.sh; rc=$?
echo "ab rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_e/sub SIZES="125000 1000000" SUBS="1 3 4" SUBS5="3 4" ARGS="--handler-batch 0" bash scripts/subrange_sweep.sh; rc=$?
echo "sub rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 > $OUT/driver_$i.log 2>&1 || exit $?; done
echo "driver rc=0" >> $OUT/status.txt
TAG=r3_e_d20 ARGS="--steps 20 --warmup 5 --handler-batch 0" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_d20 rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_e_def ARGS="--handler-batch 0" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_def rc=$rc" >> $OUT/status.txt
