#!/bin/bash
# PC sampling of the step kernel (rocprofv3, beta): where the waves' issue
# slots go, per instruction.  Lists the box's PC-sampling configurations, then
# samples a 400-step launch of the bench kernel with the stochastic (hardware)
# method; if the box does not offer it, with host_trap.  Each step has its own
# time limit; a crash or time-out ends the script.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pcs}; mkdir -p "$OUT"
ARGS=${ARGS:---steps 400 --warmup 0 --stream-steps 0 --no-cpu-baseline --handler-batch 0}
timeout -k 10 60 rocprofv3 -L > "$OUT/list.txt" 2>&1; echo "list rc=$?" >> "$OUT/status.txt"
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
    --pc-sampling-interval ${INTERVAL:-1048576} -d "$OUT/st" -o run --output-format csv -- python3 bench.py $ARGS \
    > "$OUT/st.log" 2>&1
rc=$?; echo "stochastic rc=$rc" >> "$OUT/status.txt"
if [ $rc -eq 1 ] || [ $rc -eq 2 ]; then
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
      --pc-sampling-interval ${HT_INTERVAL:-10} -d "$OUT/ht" -o run --output-format csv -- python3 bench.py $ARGS \
      > "$OUT/ht.log" 2>&1
  rc=$?; echo "host_trap rc=$rc" >> "$OUT/status.txt"
fi
# keep the merge small: compress the sample tables
find "$OUT" -name '*.csv' -size +1M -exec gzip -f {} \;
exit $rc
