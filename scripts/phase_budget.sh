#!/bin/bash
# Per-phase VALU / SALU budget of the driver's launch: the
# product library and the RAFT_PHASE_TWICE builds (each runs one phase a
# second time on copies whose results are sunk; build them first, on the CPU:
#   scripts/build_variants.sh tw_t:-DRAFT_PHASE_TWICE=1 tw_jobs:-DRAFT_PHASE_TWICE=2 \
#       tw_v:-DRAFT_PHASE_TWICE=4 tw_a:-DRAFT_PHASE_TWICE=6 tw_c:-DRAFT_PHASE_TWICE=7)
# under one SQ counter pass each; scripts/phase_budget.py takes the differences.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/phase_${TAG:-x}; mkdir -p "$OUT"
A=${ARGS:-"--steps 20 --warmup 5"}
for v in base ${VARIANTS:-tw_t tw_jobs tw_v tw_a tw_c}; do
  lib=$PWD/raft-kotlin_amd/lib/libraft_engine.so; [ "$v" != base ] && lib=$PWD/raft-kotlin_amd/lib/libraft_engine_$v.so
  RAFT_ENGINE_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      -d "$OUT/$v" -o run --output-format csv -- python bench.py $A --no-cpu-baseline --handler-batch 0 \
      --stream-steps 0 --no-general-leg > "$OUT/$v.log" 2>&1
  rc=$?; echo "$v rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
done
python scripts/phase_budget.py "$OUT" > "$OUT/budget.json"
