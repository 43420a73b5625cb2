#!/bin/bash
# Counter passes for the step kernel (one pass per run, never combined with tracing).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-x}; mkdir -p "$OUT"
B=${BENCH:-"bench.py --steps 128 --warmup 64 --stream-steps 0 --no-cpu-baseline --steps-per-launch 64"}
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
i=0
IFS='|' read -ra PASSES <<< "${PMCS}"
for pmc in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -d "$OUT/pmc$i" -o run --output-format csv -- python $B > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i ($pmc) rc=$rc" >> "$OUT/status.txt"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
