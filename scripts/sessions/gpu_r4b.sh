#!/bin/bash
# Round 4 evidence, part 1: the whole GPU suite + smoke, the driver's bench
# command and the default bench (CPU baseline, general-kernel and handler
# legs), the forced one-rank RCCL path at both lengths, the N=2 rehearsal.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4b}; mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 -a "$name" = pytest ] || exit $rc; }
[ -n "$SKIP_TESTS" ] || step pytest 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_default 500 python -u bench.py
export RAFT_BENCH_FORCE_COLLECTIVE=1
step rccl_driver 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0
step rccl_default 400 python -u bench.py --no-cpu-baseline --handler-batch 0
step plain_default 400 python -u bench.py --no-cpu-baseline --handler-batch 0 --no-general-leg
unset RAFT_BENCH_FORCE_COLLECTIVE
TAG=r4b/dist STEPS=512 bash scripts/dist_rehearsal.sh > $OUT/dist.log 2>&1; echo "dist rc=$?" >> $OUT/status.txt
exit 0
