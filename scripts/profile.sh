#!/bin/bash
# rocprofv3 evidence for the step kernel: kernel-trace stats, then one PMC
# pass per counter group (never combined with tracing), each under its own limit.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-x}
mkdir -p "$OUT"
B=${BENCH:-"bench.py --steps 200 --warmup 20 --no-cpu-baseline"}
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python $B > "$OUT/trace.log" 2>&1 || exit $?
i=0
# passes separated by '|', counters within a pass by spaces
IFS='|' read -ra PASSES <<< "${PMCS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY|FETCH_SIZE|WRITE_SIZE}"
for pmc in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc -d "$OUT/pmc$i" -o run --output-format csv -- python $B > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i ($pmc) rc=$rc" >> "$OUT/status.txt"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
