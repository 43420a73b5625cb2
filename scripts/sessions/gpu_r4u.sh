#!/bin/bash
# Round 4: T phase with an empty quiet path (no register copies on it):
# parity subset, then A/B against HEAD's build.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${TAG:-r4u}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
     -k "balanced_schedule or 3-flat-20 or config4_strong or vs_oracle or kats" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
X="--no-general-leg --handler-batch 0"
TAG=$T/s8 ROUNDS=2 ARGS="--steps 20 --warmup 5 --groups 125000 $X" VARIANTS="base head" bash scripts/ab.sh || exit $?
TAG=$T/d20 ROUNDS=3 ARGS="--steps 20 --warmup 5 $X" VARIANTS="base head" bash scripts/ab.sh || exit $?
TAG=$T/def ROUNDS=1 ARGS="$X" VARIANTS="base head" bash scripts/ab.sh || exit $?
exit 0
