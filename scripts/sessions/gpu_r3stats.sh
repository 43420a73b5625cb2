#!/bin/bash
# rocprofv3 --kernel-trace --stats of both bench commands at HEAD (the PMC rows
# of the same build come from scripts/pmc_bench.sh), and the union of the
# default run's overlapping sub-range dispatches.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_stats}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_driver -o run --output-format csv -- \
     python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 > $OUT/prof_driver.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv -- \
     python3 bench.py --no-cpu-baseline --handler-batch 0 > $OUT/prof_default.log 2>&1 || exit $?
python3 scripts/trace_union.py $OUT/prof_default 3 25 3 > $OUT/prof_default_union.json 2>&1
exit 0
