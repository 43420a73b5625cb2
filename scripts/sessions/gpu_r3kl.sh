#!/bin/bash
# r3_l (store-merge microbenchmark) then r3_k (N = 2 rehearsal + bench tests)
cd "${GRAFT_REPO_ROOT:-.}"
bash scripts/sessions/gpu_r3l.sh || exit $?
bash scripts/sessions/gpu_r3k.sh
