#!/bin/bash
# Round 4: 32-bit sort keys for the handler batches -- batch parity tests,
# the handler leg against HEAD's build, a kernel trace of the batch.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4i}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "batch or handler or wire or service or device_batches" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.txt; [ $rc -eq 0 ] || exit $rc
B="--steps 20 --warmup 5 --no-cpu-baseline --no-general-leg --stream-steps 0"
H=$PWD/raft-kotlin_amd/lib/libraft_engine_head.so
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B > $OUT/k32_$i.log 2>&1 || exit $?
  timeout -k 10 300 env RAFT_ENGINE_LIB=$H python -u bench.py $B > $OUT/head_$i.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
    python scripts/handler_probe.py > $OUT/trace.log 2>&1 || exit $?
for f in $OUT/k32_*.log $OUT/head_*.log; do python - "$f" <<'PY' >> $OUT/summary.txt
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["handler_batch"]
print(sys.argv[1].split("/")[-1], {k: (round(d[k]["ms_per_batch_device"], 4), d[k]["parity_mismatches"]) for k in ("vote", "append")})
PY
done
exit 0
