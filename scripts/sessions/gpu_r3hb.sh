#!/bin/bash
# Handler batches from page-locked host arrays (direct DMA) and threaded
# staging copies: the GPU suite, the driver's bench command (handler_batch
# leg), then PMC rows of both bench commands for this build.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_hb}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1
rc=$?; echo "bench_driver rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3hb_d20 ARGS="--steps 20 --warmup 5" bash scripts/pmc_bench.sh || exit $?
TAG=r3hb_def ARGS="" bash scripts/pmc_bench.sh; rc=$?
find gpurun_out -name "*counter_collection.csv" -delete
find gpurun_out -name "*kernel_trace.csv" -size +2M -delete
exit $rc
