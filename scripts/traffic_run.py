"""Workloads for the rocprofv3 --pmc traffic passes (scripts/traffic.sh).

    python scripts/traffic_run.py calib      # quiet engine: every launch moves exactly the group state
    python scripts/traffic_run.py workload   # bench.py's config-3 workload, K=64, K=512, then K=1 launches

The calibration engine never fires a timer, sends no message and appends
nothing, so each step-kernel launch reads and writes exactly
G * (R * REPLICA_BYTES + GROUP_BYTES) bytes: FETCH_SIZE / WRITE_SIZE of those
launches give the counter-to-bytes factors of this kernel's access pattern
(MI355X_MICROARCH.md: the gfx950 factor is only calibrated for 16 B/lane reads).
"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
abi = importlib.import_module("raft-kotlin_amd.abi")
RaftEngine = importlib.import_module("raft-kotlin_amd.engine").RaftEngine

G = int(os.environ.get("TRAFFIC_GROUPS", "1000000"))


def main(mode):
    if mode == "calib":
        p = abi.make_params(R=5, G=G, seed=3, log_cap=4, election_min_ms=1 << 30, election_max_ms=1 << 30,
                            steps_per_launch=1, subranges=1)      # one dispatch moves the whole state
        e = RaftEngine(p)
        e.step(20, counters=False)
    else:
        kw = dict(abi.CONFIGS[3], G=G)
        e = RaftEngine(abi.make_params(log_cap=640, steps_per_launch=64, subranges=1, **kw))
        e.step(128, counters=False)        # warmup (2 launches)
        e.step(256, counters=False)        # 4 launches at K=64
        e.set_steps_per_launch(512)
        e.step(1024, counters=False)       # 2 launches at K=512 (bench default)
        e.set_steps_per_launch(1)
        e.step(20, counters=False)         # 20 launches at K=1
    e.close()


if __name__ == "__main__":
    main(sys.argv[1])
