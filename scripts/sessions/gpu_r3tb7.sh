cd "${GRAFT_REPO_ROOT:-.}"
TAG=r3_tb7/c3 VARIANTS="base tb7:400" ROUNDS=2 ARGS="--steps 10000 --mode textbook --handler-batch 0" bash scripts/ab.sh || exit $?
TAG=r3_tb7/c5 VARIANTS="base tb7:400" ROUNDS=2 ARGS="--steps 10000 --mode textbook --config 5 --groups 100000 --handler-batch 0" bash scripts/ab.sh
