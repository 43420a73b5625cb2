#!/bin/bash
# A kernel change: a quick parity subset on the working tree, then A/B timings
# against the HEAD build (libraft_engine_head.so) on the default bench and the
# driver's command.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-abt}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread \
   -k "${TESTS:-steps_per_launch or subrange or config3_drops or config5 or 3-flat-400 or other_replica or kats}" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=$TAG/ab VARIANTS="base head" ROUNDS=${ROUNDS:-3} ARGS="--steps 10000 --handler-batch 0" bash scripts/ab.sh || exit $?
TAG=$TAG/ab20 VARIANTS="base head" ROUNDS=${ROUNDS:-3} ARGS="--steps 20 --warmup 5 --handler-batch 0" bash scripts/ab.sh
