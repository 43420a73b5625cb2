#!/bin/bash
# N > 1 bench path rehearsed on ONE MI355X: 2 gloo ranks sharing cuda:0 (2 x 5e5 groups)
# against one rank with 1e6 groups; the global counters and safety flags must be equal.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-dist}; mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --steps 2048 --groups 1000000 --stream-steps 0 --no-cpu-baseline \
    > "$OUT/one_rank.log" 2>&1 || exit $?
RAFT_BENCH_BACKEND=gloo RAFT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2048 \
    --groups 500000 --stream-steps 0 --no-cpu-baseline > "$OUT/two_rank.log" 2>&1 || exit $?
grep '^{' "$OUT/one_rank.log" | tail -1 > "$OUT/dist_rehearsal_1rank.json"
grep '^{' "$OUT/two_rank.log" | tail -1 > "$OUT/dist_rehearsal_2rank_gloo_one_gpu.json"
python3 - "$OUT" <<'PY'
import json, sys
a = json.load(open(sys.argv[1] + "/dist_rehearsal_1rank.json"))
b = json.load(open(sys.argv[1] + "/dist_rehearsal_2rank_gloo_one_gpu.json"))
ok = a["safety"] == b["safety"] and a["counters_last_step"] == b["counters_last_step"]
print("rehearsal equal:", ok)
sys.exit(0 if ok else 1)
PY
