#!/bin/bash
# A/B of the R = 5 job-lane change (second RequestVote sender's chunk drawn
# in the step's job pass; the working tree) against HEAD's engine, then the
# GPU parity suite on the working tree.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3_h; mkdir -p $OUT
TAG=r3_h/ab VARIANTS="base head" ROUNDS=3 ARGS="--steps 10000 --handler-batch 0" bash scripts/ab.sh; rc=$?
echo "ab rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_h/ab20 VARIANTS="base head" ROUNDS=3 ARGS="--steps 20 --warmup 5 --handler-batch 0" bash scripts/ab.sh; rc=$?
echo "ab20 rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/status.txt
