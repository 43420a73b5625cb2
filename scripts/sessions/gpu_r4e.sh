#!/bin/bash
# Round 4: the counter all-reduce in series with the launches (forced
# one-rank RCCL against the plain path), and the general-kernel leg at the
# main leg's launch length.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4e}; mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc; }
B="--no-cpu-baseline --handler-batch 0"
step general_default 400 python -u bench.py $B
step plain_default 400 python -u bench.py $B --no-general-leg
step rccl_default 400 env RAFT_BENCH_FORCE_COLLECTIVE=1 python -u bench.py $B
step rccl_driver 300 env RAFT_BENCH_FORCE_COLLECTIVE=1 python -u bench.py --steps 20 --warmup 5 $B
step general_driver 300 python -u bench.py --steps 20 --warmup 5 $B
exit 0
