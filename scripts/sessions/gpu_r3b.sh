#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r3_b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -x --timeout 300 --timeout-method thread -k "subrange or batches or service or sub3 or sub2" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace_s2" -o run --output-format csv -- \
      python bench.py --groups 125000 --subranges 2 --steps 2000 --warmup 0 --stream-steps 0 --no-cpu-baseline --handler-batch 0 \
      > "$OUT/trace_s2.log" 2>&1; rc=$?; echo "trace s2 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
TAG=r3_b/sub SUBS="1 2 3" SUBS5="1 2 3" ARGS="--handler-batch 0" bash scripts/subrange_sweep.sh; rc=$?; echo "subsweep rc=$rc" >> $OUT/status.txt
