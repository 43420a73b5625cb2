#!/bin/bash
# Attribute the step kernel's HBM traffic: PMC passes over
# the same bench command for the product build and diagnostic builds whose
# log stores / gated log loads go to one slot per wave
# (scripts/variants/sink_*.patch, built by scripts/build_variants.sh as
# sinkst / sinkld / sinkboth).  Then scripts/traffic_attrib.py.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-attrib}; mkdir -p "$OUT"
A="${ARGS:---steps 2000 --warmup 0} --subranges 1 --stream-steps 0 --handler-batch 0 --no-cpu-baseline"
for v in ${VARIANTS:-base sinkst sinkld sinkboth}; do
  lib=raft-kotlin_amd/lib/libraft_engine.so; [ "$v" != base ] && lib=raft-kotlin_amd/lib/libraft_engine_$v.so
  RAFT_ENGINE_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py $A --plan-file "$OUT/plan_$v.json" > "$OUT/bench_$v.log" 2>&1
  rc=$?; echo "$v bench rc=$rc $(grep -o '"value": [0-9.e+]*' "$OUT/bench_$v.log")" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
  i=0
  for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum TCC_HIT_sum TCC_MISS_sum" \
             "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_WRITEBACK_sum"; do
    i=$((i+1))
    RAFT_ENGINE_LIB=$PWD/$lib timeout -s KILL 200 rocprofv3 --pmc $pmc -d "$OUT/${v}_p$i" -o run --output-format csv -- \
        python bench.py $A > "$OUT/${v}_p$i.log" 2>&1
    rc=$?; echo "$v p$i rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/calib_$c" -o run --output-format csv -- \
      python scripts/traffic_run.py calib > "$OUT/calib_$c.log" 2>&1 || exit $?
done
python scripts/traffic_attrib.py "$OUT" > "$OUT/attrib.json"
