"""The Log Matching restatement (tests/helpers.log_matching_flags) on crafted
logs, CPU only: it is the checker of raft_engine_check_log_matching."""
import numpy as np

from helpers import blank_groups, log_matching_flags, set_fld


def crafted(R=3, G=6, cap=16):
    w = blank_groups(G, R)
    t = np.zeros((G, R, cap), np.int32)
    c = np.zeros((G, R, cap), np.uint32)
    for r in range(R):
        set_fld(w, R, r, "last", 8)
        set_fld(w, R, r, "phys", 8)
        set_fld(w, R, r, "commit", 6)
    t[:, :, :8] = np.arange(1, 9)
    c[:, :, :8] = 100 + np.arange(8)
    return w, t, c


def test_identical_logs_not_flagged():
    w, t, c = crafted()
    assert not log_matching_flags(w, t, c, 3).any()


def test_only_common_committed_prefix_counts():
    R = 3
    w, t, c = crafted(R)
    c[1, 2, 5] += 1                      # inside every committed prefix
    t[2, 1, 6] = 99                      # beyond every committed prefix
    set_fld(w[3:4], R, 0, "commit", 3)
    t[3, 0, 3] = 99                      # outside replica 0's shorter prefix
    set_fld(w[4:5], R, 1, "last", 5)
    t[4, 1, 5] = 77                      # commit clamps to lastIndex
    t[5, 0, 0] = 42
    assert list(np.nonzero(log_matching_flags(w, t, c, R))[0]) == [1, 5]
