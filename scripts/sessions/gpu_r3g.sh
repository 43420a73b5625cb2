#!/bin/bash
# Upper bound of removing the second-vote-round staging Philox pass (timing only).
cd "${GRAFT_REPO_ROOT:-.}"
TAG=r3_g/ab VARIANTS="base nostage" ROUNDS=2 ARGS="--steps 10000 --handler-batch 0" bash scripts/ab.sh || exit $?
TAG=r3_g/ab20 VARIANTS="base nostage" ROUNDS=3 ARGS="--steps 20 --warmup 5 --handler-batch 0" bash scripts/ab.sh
