#!/bin/bash
# Round 4 experiment, fifth pass: band ends (RAFT_BAND_ENDS) and age shifts (RAFT_AGE_SHIFTS, D per
# mille per slot for each band end) on the 1/8 shard, the driver's command and
# the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${TAG:-r4r}
X="--no-general-leg --handler-batch 0"
TAG=$T/s8 ROUNDS=2 ARGS="--steps 20 --warmup 5 --groups 125000 $X" VARIANTS="base e1 e2 e3 e4" bash scripts/ab.sh || exit $?
TAG=$T/d20 ROUNDS=2 ARGS="--steps 20 --warmup 5 $X" VARIANTS="base e1 e2 e3 e4" bash scripts/ab.sh || exit $?
TAG=$T/def ROUNDS=1 ARGS="$X" VARIANTS="base e1 e2 e3 e4" bash scripts/ab.sh || exit $?
exit 0
