#!/bin/bash
# Round 4: the counter all-reduce after the timed region (default) against
# inline (per chunk, in series): forced one-rank RCCL at the driver's command,
# the 1/8 shard and the default; the collective tests; the N=2 rehearsal.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4g}; mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc; }
step pytest 400 python -u -m pytest tests/test_gpu_bench.py -m gpu -v --timeout 300 --timeout-method thread -x
B="--no-cpu-baseline --handler-batch 0 --no-general-leg --stream-steps 0"
for i in 1 2; do
  step plain_s8_$i 200 python -u bench.py --steps 20 --warmup 5 --groups 125000 $B
  step after_s8_$i 200 env RAFT_BENCH_FORCE_COLLECTIVE=1 python -u bench.py --steps 20 --warmup 5 --groups 125000 $B
  step inline_s8_$i 200 env RAFT_BENCH_FORCE_COLLECTIVE=1 python -u bench.py --steps 20 --warmup 5 --groups 125000 --allreduce inline $B
  step plain_d20_$i 200 python -u bench.py --steps 20 --warmup 5 $B
  step after_d20_$i 200 env RAFT_BENCH_FORCE_COLLECTIVE=1 python -u bench.py --steps 20 --warmup 5 $B
done
step after_def 300 env RAFT_BENCH_FORCE_COLLECTIVE=1 python -u bench.py $B
TAG=r4g/dist STEPS=512 bash scripts/dist_rehearsal.sh > $OUT/dist.log 2>&1; echo "dist rc=$?" >> $OUT/status.txt
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"wall_ms": [0-9.]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1)"; done > $OUT/summary.txt
exit 0
