#!/bin/bash
# Round 4: config 5 on the balanced schedule with the age-shifted bands
# against its automatic shape (one chunk per wave on 3 ranges); the default
# and the driver's bench repeated for the run-to-run spread.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4t}; mkdir -p $OUT
B="--no-cpu-baseline --handler-batch 0 --no-general-leg --stream-steps 0"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config 5 --groups 100000 $B > $OUT/c5_auto_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --config 5 --groups 100000 --schedule balanced --subranges 1 $B > $OUT/c5_bal_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py $B > $OUT/def_$i.log 2>&1 || exit $?
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 $B > $OUT/d20_$i.log 2>&1 || exit $?
done
for f in $OUT/*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1)"; done > $OUT/summary.txt
exit 0
