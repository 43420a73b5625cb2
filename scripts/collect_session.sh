#!/bin/bash
# Copy one scripts/session.sh run (gpurun_out/<TAG>, gpurun_out/pmc_<TAG>_{d20,def}) into
# profiles/<DEST>/ and fold its PMC rows into profiles/pmc_rows.json (runs here, no GPU).
#   scripts/collect_session.sh r2e r2_e
set -e
cd "$(dirname "$0")/.."
T=$1; D=profiles/$2; S=gpurun_out/$T
mkdir -p "$D"
j() { grep '^{' "$1" | tail -1 > "$2"; }
j $S/bench_default.log $D/bench_default.json
j $S/bench_driver.log $D/bench_driver_cmd.json
[ -f $S/bench_c5.log ] && j $S/bench_c5.log $D/bench_config5.json
[ -d $S/dist ] && cp $S/dist/dist_rehearsal_*.json $D/
tail -25 $S/pytest.log > $D/pytest_tail.txt
tail -1 $S/smoke.log > $D/smoke.txt
for k in d20 def; do
  P=gpurun_out/pmc_${T}_$k
  [ -d $P ] || continue
  n=$([ $k = def ] && echo default || echo driver_cmd)
  cp "$(find $P/trace -name '*kernel_stats.csv' | head -1)" $D/kernel_stats_$n.csv
  cp $P/rows.json $D/pmc_$n.json
  python3 scripts/pmc_parse.py --merge $P/rows.json
done
ls $D
