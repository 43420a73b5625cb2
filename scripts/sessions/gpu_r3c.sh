#!/bin/bash
# Session r3_c: the whole GPU suite + smoke, the driver's bench command, the
# default bench (CPU baseline included), config 5, the forced one-rank RCCL
# bench at full size.  Every GPU step has its own limit; a crash ends it.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r3_c; mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 -a "$name" = pytest ] || exit $rc; }
step pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_driver1 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_driver2 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
step bench_default 400 python -u bench.py
step bench_c5 300 python -u bench.py --config 5 --groups 100000 --no-cpu-baseline
RAFT_BENCH_FORCE_COLLECTIVE=1 step bench_forced_rccl 300 python -u bench.py --no-cpu-baseline --handler-batch 0
exit 0
