#!/bin/bash
# One A/B GPU session for a kernel change: the GPU parity suite on the current
# build, then interleaved bench timings of engine builds (scripts/ab.sh;
# VARIANTS names libraft_engine_<v>.so, "base" the current one) on config 3
# and config 5, then VALU/SALU per wave-step of each build (one SQ PMC pass,
# 2048 steps in 512-step launches).  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
T=${TAG:-abs}; OUT=gpurun_out/$T; mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
fi
TAG=$T/c3 ROUNDS=${ROUNDS:-2} bash scripts/ab.sh || exit $?
[ -n "$SKIP_C5" ] || { TAG=$T/c5 ROUNDS=${ROUNDS:-2} ARGS="--steps 10000 --config 5 --groups 100000" bash scripts/ab.sh || exit $?; }
for v in ${VARIANTS:-base}; do
  lib=raft-kotlin_amd/lib/libraft_engine.so; [ "$v" != base ] && lib=raft-kotlin_amd/lib/libraft_engine_$v.so
  RAFT_ENGINE_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      -d "$OUT/sq_$v" -o run --output-format csv -- python bench.py --steps 2048 --steps-per-launch 512 --warmup 0 --stream-steps 0 \
      --no-cpu-baseline > "$OUT/sq_$v.log" 2>&1 || exit $?
  python3 - "$OUT/sq_$v" "$v" >> "$OUT/status.txt" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "step_kernel" in row["Kernel_Name"]:
            acc[row["Counter_Name"]] += float(row["Counter_Value"])
ws = acc["SQ_WAVES"] * 512
print(f"{sys.argv[2]} per wave-step: VALU {acc['SQ_INSTS_VALU'] / ws:.1f} SALU {acc['SQ_INSTS_SALU'] / ws:.1f} "
      f"LDS {acc['SQ_INSTS_LDS'] / ws:.1f}")
PY
done
exit 0
