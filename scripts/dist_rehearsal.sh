#!/bin/bash
# The N > 1 bench path rehearsed on ONE MI355X: `bench.py --gpus 2` spawns its
# two ranks itself (gloo, both on cuda:0).  Config 4 (the default, 2 x 5e5
# groups) with its weak-scaling leg (2 x 1e6), whose rank-0 rows must equal
# the strong leg's all-reduced rows; against one rank with all 1e6 groups the
# global counters and the safety flags must be equal; and --scaling weak with
# its config-4 leg.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-dist}; mkdir -p "$OUT"
S=${STEPS:-2048}
timeout -k 10 300 python -u bench.py --steps $S --stream-steps 0 --no-cpu-baseline --handler-batch 0 \
    > "$OUT/one_rank.log" 2>&1 || exit $?
RAFT_BENCH_BACKEND=gloo RAFT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps $S \
    --stream-steps 0 --no-cpu-baseline > "$OUT/two_rank.log" 2>&1 || exit $?
RAFT_BENCH_BACKEND=gloo RAFT_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps $S \
    --stream-steps 0 --no-cpu-baseline --scaling weak > "$OUT/two_rank_weak.log" 2>&1 || exit $?
grep '^{' "$OUT/two_rank_weak.log" | tail -1 > "$OUT/dist_rehearsal_2rank_weak_gloo_one_gpu.json"
grep '^{' "$OUT/one_rank.log" | tail -1 > "$OUT/dist_rehearsal_1rank.json"
grep '^{' "$OUT/two_rank.log" | tail -1 > "$OUT/dist_rehearsal_2rank_gloo_one_gpu.json"
python3 - "$OUT" <<'PY'
import json, sys
a = json.load(open(sys.argv[1] + "/dist_rehearsal_1rank.json"))
b = json.load(open(sys.argv[1] + "/dist_rehearsal_2rank_gloo_one_gpu.json"))
ok = (a["safety"] == b["safety"] and a["counters_last_step"] == b["counters_last_step"] and b["n_gpus"] == 2
      and b["scaling"] == "strong" and b["config"]["groups_per_rank"] == [500000, 500000] and b["valid"]
      and b["weak_scaling"]["groups_per_rank"] == [1000000, 1000000] and b["weak_scaling"]["valid"]
      and b["weak_scaling"]["counters_equal_strong_allreduced"] is True)
w = json.load(open(sys.argv[1] + "/dist_rehearsal_2rank_weak_gloo_one_gpu.json"))
okw = (w["scaling"] == "weak" and w["config"]["groups_per_rank"] == [1000000, 1000000] and w["valid"]
       and w["config4_strong"]["groups_per_rank"] == [500000, 500000] and w["config4_strong"]["valid"]
       and w["config4_strong"]["counters_equal_rank0_weak_shard"] is True)
print("config 4 + weak leg equal to one rank:", ok, "weak + config-4 leg:", okw)
sys.exit(0 if ok and okw else 1)
PY
