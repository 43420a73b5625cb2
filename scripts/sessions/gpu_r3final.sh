#!/bin/bash
# Round-3 evidence at HEAD: the GPU suite + smoke, the driver's bench command,
# the default bench, config 5, and rocprofv3 kernel-trace stats of both bench
# commands (with the union of the overlapping sub-range dispatches).  Every
# GPU step has its own limit; a crash or time-out ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3_final}; mkdir -p $OUT
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 -a "$name" = pytest ] || exit $rc; }
step pytest 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_default 400 python -u bench.py
step bench_c5 300 python -u bench.py --config 5 --groups 100000 --no-cpu-baseline
step prof_driver 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_driver -o run --output-format csv -- \
     python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0
step prof_default 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_default -o run --output-format csv -- \
     python3 bench.py --no-cpu-baseline --handler-batch 0
python3 scripts/trace_union.py $OUT/prof_default 3 > $OUT/prof_default_union.json 2>&1
exit 0
