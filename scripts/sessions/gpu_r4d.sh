#!/bin/bash
# Round 4: VALU trims (flat-log kernels flush one counter word less, 32-bit
# coins, tail cache from t1) -- parity subset, then A/B against HEAD's build.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4d}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -x \
     -k "balanced_schedule or 3-flat-20 or config4_strong or vs_oracle or counters" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
X="--no-general-leg --handler-batch 0"
TAG=${TAG:-r4d}/d20 ROUNDS=3 ARGS="--steps 20 --warmup 5 $X" VARIANTS="base head" bash scripts/ab.sh || exit $?
TAG=${TAG:-r4d}/s8 ROUNDS=2 ARGS="--steps 20 --warmup 5 --groups 125000 $X" VARIANTS="base head" bash scripts/ab.sh || exit $?
TAG=${TAG:-r4d}/def ROUNDS=1 ARGS="$X" VARIANTS="base head" bash scripts/ab.sh || exit $?
exit 0
