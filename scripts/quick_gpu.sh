#!/bin/bash
# Full GPU parity suite, then the bench workload (no CPU leg) for a quick A/B.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-quick}; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/pytest.log"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
STEPS=${STEPS:-4000} TAG=${TAG:-quick} VARIANTS="${VARIANTS:-base base.2}" bash scripts/flag_sweep.sh
