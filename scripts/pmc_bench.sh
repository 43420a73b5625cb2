#!/bin/bash
# rocprofv3 evidence for ONE bench.py command line (the exact command whose
# JSON the numbers are attached to):
#   1. a --kernel-trace --stats run (per-kernel average durations);
#   2. PMC passes, one counter group per run and never combined with tracing:
#      FETCH_SIZE | WRITE_SIZE | SQ instruction counts + GRBM_GUI_ACTIVE;
#   3. the same passes count bench.py's traffic probes (--traffic-probe:
#      raft_engine_traffic_probe dispatches of the step kernel's own state
#      and log-store access patterns over known bytes, in the same process);
#   4. scripts/pmc_parse.py: per-launch rows keyed by the workload and launch
#      length in $OUT/rows.json; back here, `python scripts/pmc_parse.py
#      --merge gpurun_out/pmc_*/rows.json` folds them into
#      profiles/pmc_rows.json (read by bench.py).
#   TAG=r2_d20 ARGS="--steps 20 --warmup 5" scripts/pmc_bench.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-x}
mkdir -p "$OUT"
A="${ARGS:-} --no-cpu-baseline --traffic-probe --plan-file $OUT/plan.json"
echo "trace" >> "$OUT/status.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python bench.py $A > "$OUT/trace.log" 2>&1 || exit $?
i=0
# pass 4 is the disjoint cycle split of MI355X_MICROARCH.md (SQ block):
# SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (ready, not
# issued) + SQ_ACTIVE_INST_ANY (issuing) ~= SQ_WAVE_CYCLES.  Pass 5 is optional
# (names that this rocprofv3 may not list do not stop the script).
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  echo "pmc$i $pmc" >> "$OUT/status.txt"
  timeout -s KILL 300 rocprofv3 --pmc $pmc -d "$OUT/pmc$i" -o run --output-format csv -- \
      python bench.py $A > "$OUT/pmc$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pmc$i rc=$rc" >> "$OUT/status.txt"
    [ $i -le 4 ] && exit $rc
    rm -rf "$OUT/pmc$i"
    [ $rc -eq 137 ] || [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
  fi
done
python scripts/pmc_parse.py "$OUT" && echo "parsed" >> "$OUT/status.txt"
