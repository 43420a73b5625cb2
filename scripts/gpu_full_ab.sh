#!/bin/bash
# A kernel change: the whole GPU suite on the working tree, then interleaved
# A/B against the HEAD build (libraft_engine_head.so) on the default bench, the
# driver's command and config 5.  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-.}"
T=${TAG:-fab}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=$T VARIANTS="${VARIANTS:-base head}" bash scripts/ab_multi.sh || exit $?
TAG=$T/c5 VARIANTS="${VARIANTS:-base head}" ROUNDS=2 ARGS="--steps 10000 --config 5 --groups 100000 --handler-batch 0" bash scripts/ab.sh
