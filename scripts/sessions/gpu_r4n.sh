#!/bin/bash
# Round 4 experiment, second pass: age-dependent band ends (first band D per
# mille per slot, second band D2) on the 1/8 shard, the driver's command and
# the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${TAG:-r4n}
X="--no-general-leg --handler-batch 0"
TAG=$T/s8 ROUNDS=2 ARGS="--steps 20 --warmup 5 --groups 125000 $X" VARIANTS="base ag40 ag60 agb40 agb60" bash scripts/ab.sh || exit $?
TAG=$T/d20 ROUNDS=2 ARGS="--steps 20 --warmup 5 $X" VARIANTS="base ag40 ag60 agb40 agb60" bash scripts/ab.sh || exit $?
TAG=$T/def ROUNDS=1 ARGS="$X" VARIANTS="base ag40 agb40" bash scripts/ab.sh || exit $?
exit 0
