#!/bin/bash
# Round 4: the balanced schedule with interleaved chunks (workgroup b takes
# chunks b, b + nb, ...) against one chunk per wave, and the SQ cycle split
# of both on the driver's launch.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4a2}; mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 -a "$name" = pytest ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -x \
     -k "balanced_schedule or 3-flat-20-sub1 or config4_strong"
B="--no-cpu-baseline --handler-batch 0 --stream-steps 0 --no-general-leg"
for i in 1 2; do
  step d20_auto_$i 300 python -u bench.py --steps 20 --warmup 5 $B
  step d20_one_$i 300 python -u bench.py --steps 20 --warmup 5 --schedule one $B
  step d20_wg1536_$i 300 python -u bench.py --steps 20 --warmup 5 --schedule-workgroups 1536 $B
  step s8_auto_$i 300 python -u bench.py --steps 20 --warmup 5 --groups 125000 $B
  step s8_one_$i 300 python -u bench.py --steps 20 --warmup 5 --groups 125000 --schedule one $B
done
step def_auto 400 python -u bench.py $B
step def_one3 400 python -u bench.py --schedule one --subranges 3 $B
for s in auto one; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
      -d "$OUT/pmc_$s" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --schedule $s $B > "$OUT/pmc_$s.log" 2>&1
  echo "pmc_$s rc=$?" >> $OUT/status.txt
done
exit 0
