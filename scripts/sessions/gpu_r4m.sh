#!/bin/bash
# Round 4 experiment: age-dependent first priority band (older workgroup
# slots step down earlier; scripts/variants/age_bands.patch, D per mille per
# slot) against the product build, on the 1/8 shard and the driver's command.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${TAG:-r4m}
X="--no-general-leg --handler-batch 0"
TAG=$T/s8 ROUNDS=2 ARGS="--steps 20 --warmup 5 --groups 125000 $X" VARIANTS="base ag40 ag80 agm40 ag0" bash scripts/ab.sh || exit $?
TAG=$T/d20 ROUNDS=2 ARGS="--steps 20 --warmup 5 $X" VARIANTS="base ag40 ag80 agm40" bash scripts/ab.sh || exit $?
exit 0
