cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r3_a; mkdir -p $OUT
timeout -k 5 60 rocprofv3 -L > $OUT/rocprof_counters.txt 2>&1; echo "list rc=$?" >> $OUT/status.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_parity.py -m gpu -v -x --timeout 300 --timeout-method thread -k "subrange or full_size_digest or forced_collective or window_misses or crafted or handler_batches or steps_per_launch" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TAG=r3_a/sub bash scripts/subrange_sweep.sh; rc=$?; echo "subsweep rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_a_d20 ARGS="--steps 20 --warmup 5" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_d20 rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
TAG=r3_a_def ARGS="" bash scripts/pmc_bench.sh; rc=$?; echo "pmc_def rc=$rc" >> $OUT/status.txt
