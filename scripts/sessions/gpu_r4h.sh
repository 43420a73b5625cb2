#!/bin/bash
# Round 4: the counter reduction folded into one-range launches
# (fold_counters) -- the GPU suite, then A/B against HEAD's build and the
# fold switched off (RAFT_FOLD_COUNTERS=0) on the 1/8 shard and the driver's command.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4h}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
B="--steps 20 --warmup 5 --no-cpu-baseline --handler-batch 0 --stream-steps 0 --no-general-leg"
H=$PWD/raft-kotlin_amd/lib/libraft_engine_head.so
for i in 1 2 3; do
  for g in 125000 1000000; do
    timeout -k 10 200 python -u bench.py $B --groups $g > $OUT/fold_${g}_$i.log 2>&1 || exit $?
    timeout -k 10 200 env RAFT_FOLD_COUNTERS=0 python -u bench.py $B --groups $g > $OUT/nofold_${g}_$i.log 2>&1 || exit $?
    timeout -k 10 200 env RAFT_ENGINE_LIB=$H python -u bench.py $B --groups $g > $OUT/head_${g}_$i.log 2>&1 || exit $?
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace_s125000 -o run --output-format csv -- \
    python bench.py $B --groups 125000 > $OUT/trace_s125000.log 2>&1 || exit $?
for f in $OUT/*_[0-9]*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.e+]*' $f | head -1) $(grep -o '"wall_ms": [0-9.]*' $f | head -1) $(grep -o '"stream_event_ms": [0-9.]*' $f | head -1) $(grep -o '"kernel_avg_ms": [0-9.]*' $f | head -1)"; done > $OUT/summary.txt
exit 0
