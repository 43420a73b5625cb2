#!/bin/bash
# A/B of several engine builds (scripts/build_variants.sh) on the default bench
# and the driver's command, interleaved ROUNDS times, no parity step.
cd "${GRAFT_REPO_ROOT:-.}"
T=${TAG:-abm}
TAG=$T/ab VARIANTS="${VARIANTS:-base head}" ROUNDS=${ROUNDS:-2} ARGS="--steps 10000 --handler-batch 0" bash scripts/ab.sh || exit $?
TAG=$T/ab20 VARIANTS="${VARIANTS:-base head}" ROUNDS=${ROUNDS20:-3} ARGS="--steps 20 --warmup 5 --handler-batch 0" bash scripts/ab.sh
