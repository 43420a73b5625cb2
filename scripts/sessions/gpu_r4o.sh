#!/bin/bash
# Round 4 experiment, third pass: age-dependent band ends (RAFT_AGE_SHIFTS: D per
# mille per slot for each band end) on the 1/8 shard, the driver's command and
# the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${TAG:-r4o}
X="--no-general-leg --handler-batch 0"
TAG=$T/s8 ROUNDS=2 ARGS="--steps 20 --warmup 5 --groups 125000 $X" VARIANTS="base a633 a6315 a8420 a10525" bash scripts/ab.sh || exit $?
TAG=$T/d20 ROUNDS=2 ARGS="--steps 20 --warmup 5 $X" VARIANTS="base a633 a6315 a8420 a10525" bash scripts/ab.sh || exit $?
TAG=$T/def ROUNDS=1 ARGS="$X" VARIANTS="base a6315 a8420 a10525" bash scripts/ab.sh || exit $?
exit 0
