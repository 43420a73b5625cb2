#!/bin/bash
# Session r3_k: N = 2 rehearsal (two gloo ranks on cuda:0 vs one rank), the
# GPU suite's bench / sub-range / batch tests after the bench changes.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/r3_k; mkdir -p $OUT
TAG=r3_k/dist STEPS=2000 bash scripts/dist_rehearsal.sh > $OUT/dist.log 2>&1; rc=$?
echo "dist rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread \
   -k "forced or subrange or batches or shard" > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/status.txt
