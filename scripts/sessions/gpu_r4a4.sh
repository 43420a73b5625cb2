#!/bin/bash
# Round 4: the balanced schedule with per-wave priority bands (s_setprio)
# against one chunk per wave; per-wave times of the balanced launches.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4a4}; mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 -a "$name" = pytest ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -x \
     -k "balanced_schedule or 3-flat-20-sub1 or config4_strong"
B="--no-cpu-baseline --handler-batch 0 --stream-steps 0 --no-general-leg"
for i in 1 2; do
  step d20_auto_$i 300 python -u bench.py --steps 20 --warmup 5 $B
  step d20_one_$i 300 python -u bench.py --steps 20 --warmup 5 --schedule one $B
  step s8_auto_$i 300 python -u bench.py --steps 20 --warmup 5 --groups 125000 $B
  step s8_one_$i 300 python -u bench.py --steps 20 --warmup 5 --groups 125000 --schedule one $B
done
step def_auto 400 python -u bench.py $B
step def_one3 400 python -u bench.py --schedule one --subranges 3 $B
L=$PWD/raft-kotlin_amd/lib/libraft_engine_wt.so
for g in 1000000 125000; do
  RAFT_ENGINE_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --groups $g $B > $OUT/wt_$g.log 2> $OUT/wt_$g.err
  echo "wt_$g rc=$?" >> $OUT/status.txt
done
gzip $OUT/*.err
exit 0
