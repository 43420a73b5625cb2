#!/bin/bash
# store-merge microbenchmark under WRITE_SIZE and FETCH_SIZE (separate passes)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/r3_l; mkdir -p $OUT
timeout -k 10 120 ./scripts/ubench/store_merge > $OUT/plain.txt 2>&1 || exit $?
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/$c -o run --output-format csv -- ./scripts/ubench/store_merge > $OUT/$c.log 2>&1 || exit $?
done
echo done >> $OUT/status.txt
