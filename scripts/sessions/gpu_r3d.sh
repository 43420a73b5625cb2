#!/bin/bash
# Session r3_d: HBM traffic attribution (product build, slot-major layout,
# sink diagnostics), slot-major A/B timing, sub-range counts incl. 4, and the
# PMC rows (stall split) of the driver's command and the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r3_d; mkdir -p $OUT
TAG=r3_d/attrib VARIANTS="base slotmaj sinkst sinkld sinkboth" bash scripts/traffic_attrib.sh; rc=$?
echo "attrib rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_d/ab VARIANTS="base slotmaj" ROUNDS=2 ARGS="--steps 10000 --handler-batch 0" bash scripts/ab.sh; rc=$?
echo "ab rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_d/sub SIZES="125000 1000000" SUBS="3 4" SUBS5="3 4" ARGS="--handler-batch 0" bash scripts/subrange_sweep.sh; rc=$?
echo "sub rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_d_d20 ARGS="--steps 20 --warmup 5 --handler-batch 0" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_d20 rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_d_def ARGS="--handler-batch 0" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_def rc=$rc" >> $OUT/status.txt
