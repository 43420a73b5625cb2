#!/bin/bash
# Round 4, first session: the balanced schedule's parity (new tests), then
# A/B of the balanced vs the one-chunk-per-wave schedule on the driver's
# command, the config-4 1/8 shard (1.25e5 groups) and the default bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4a}; mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 -a "$name" = pytest ] || exit $rc; }
step pytest 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -x \
     -k "balanced_schedule or one_per_wave or kernel_info or config4_strong or 3-flat-20 or 3-flat-400 or device_batches"
B="--no-cpu-baseline --handler-batch 0 --stream-steps 0 --no-general-leg"
for s in auto one auto one; do
  step d20_$s 300 python -u bench.py --steps 20 --warmup 5 --schedule $s $B
  step s8_$s 300 python -u bench.py --steps 20 --warmup 5 --groups 125000 --schedule $s $B
done
step def_auto 400 python -u bench.py $B
step def_one3 400 python -u bench.py --schedule one --subranges 3 $B
step s8def_auto 400 python -u bench.py --groups 125000 $B
step s8def_one3 400 python -u bench.py --groups 125000 --schedule one --subranges 3 $B
TAG=r4a bash scripts/phase_budget.sh; echo "phase rc=$?" >> $OUT/status.txt
exit 0
