#!/bin/bash
# A/B: the round-2 kernel (rev 066f199, ISA-identical to round 2) vs the working
# tree on the driver's command (one 20-step launch) and the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3_f; mkdir -p $OUT
TAG=r3_f/d20 VARIANTS="base r2" ROUNDS=4 ARGS="--steps 20 --warmup 5 --handler-batch 0 --subranges 1" bash scripts/ab.sh; rc=$?
echo "ab d20 rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_f/def VARIANTS="base r2" ROUNDS=2 ARGS="--steps 10000 --handler-batch 0 --subranges 1" bash scripts/ab.sh; rc=$?
echo "ab def rc=$rc" >> $OUT/status.txt
