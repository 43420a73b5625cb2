"""RAFT_MODE_TEXTBOOK on the CPU oracle.

Textbook mode is opt-in and NOT the reference: it replaces the quirks that
break Raft's safety properties (Q1 ghost tail, Q2 unconditional truncation,
Q3 stale-term append, Q4 commit clamp before the check, Q5/Q6/Q7 term
adoption, Q8 nextIndex from commitIndex, Q9 +1 commit without a term guard)
by the textbook rules.  These known-answer cases are hand-derived from the
Raft paper's rules (Fig. 2); the scale test shows the Log Matching checker
finds no violation in textbook mode where the reference mode has many.
"""
import numpy as np

import oracle as O
from helpers import abi, blank_groups, fld, log_matching_flags, set_fld, set_session, session
from test_oracle_kats import put

TB = abi.MODE_TEXTBOOK


def one_group(R=3, **kw):
    return O.Oracle(abi.make_params(R=R, G=1, log_cap=64, mode=TB, **kw))


def test_stale_append_refused():
    """A term-1 append reaches a term-3 LEADER: refused, nothing changes (the
    reference deposes it and truncates, K4)."""
    R = 3
    o = one_group(R)
    w = blank_groups(1, R)[0]
    set_fld(w, R, 1, "term", 3)
    set_fld(w, R, 1, "role", abi.LEADER)
    set_fld(w, R, 1, "last", 2)
    set_fld(w, R, 1, "phys", 2)
    put(o, w, {1: [(3, ord("p")), (3, ord("q"))]})
    before = o.read_state().copy()
    assert o.append(0, 1, 1, 1, -1, -1, (1, ord("z")), 0) == (3, False, 0)
    assert np.array_equal(o.read_state(), before)


def test_truncate_only_on_conflict_and_commit_after_check():
    R = 3
    o = one_group(R)
    w = blank_groups(1, R)[0]
    set_fld(w, R, 0, "term", 2)
    set_fld(w, R, 0, "last", 3)
    set_fld(w, R, 0, "phys", 3)
    set_fld(w, R, 0, "commit", 1)
    put(o, w, {0: [(1, 10), (1, 11), (2, 12)]})
    # same entry again at index 1: no truncation, lastIndex stays 3
    assert o.append(0, 0, 2, 2, 0, 1, (1, 11), 5) == (2, True, 0)
    s = o.read_state()[0]
    assert fld(s, R, 0, "last") == 3
    assert fld(s, R, 0, "commit") == 2          # min(leaderCommit 5, last new entry 2)
    # a conflicting entry at index 1: overwrite and truncate after it
    assert o.append(0, 0, 2, 2, 0, 1, (2, 99), 1) == (2, True, 0)
    s = o.read_state()[0]
    assert fld(s, R, 0, "last") == 2 and fld(s, R, 0, "phys") == 3
    assert fld(s, R, 0, "commit") == 2          # leaderCommit 1 < commit: never lowered
    # a failed consistency check leaves the commit alone (the reference clamps first, Q4)
    assert o.append(0, 0, 2, 2, 1, 7, None, 9) == (2, False, 0)
    assert fld(o.read_state()[0], R, 0, "commit") == 2


def test_array_log_no_ghost_tail():
    """After a truncation the next append lands at lastIndex (the reference
    appends at the physical end and resurrects the stale slot, K1)."""
    R = 3
    o = one_group(R)
    w = blank_groups(1, R)[0]
    set_fld(w, R, 0, "term", 2)
    set_fld(w, R, 0, "last", 3)
    set_fld(w, R, 0, "phys", 3)
    put(o, w, {0: [(1, 10), (1, 11), (1, 12)]})
    o.append(0, 0, 2, 2, 0, 1, (2, 20), 0)      # conflict at 1: last = 2
    o.append(0, 0, 2, 2, 1, 2, (2, 21), 0)      # append at 2
    t, c = o.read_log()
    s = o.read_state()[0]
    assert fld(s, R, 0, "last") == 3 and fld(s, R, 0, "phys") == 3
    assert [int(x) for x in c[0, 0, :3]] == [10, 20, 21]


def test_vote_adopts_higher_term_on_rejection():
    """The voter's log is newer: the vote is refused, but the term is adopted
    (the reference keeps its term, Q5)."""
    R = 3
    o = one_group(R)
    w = blank_groups(1, R)[0]
    set_fld(w, R, 2, "term", 1)
    set_fld(w, R, 2, "last", 2)
    set_fld(w, R, 2, "phys", 2)
    set_fld(w, R, 2, "voted", 3)
    put(o, w, {2: [(1, 1), (1, 2)]})
    assert o.vote(0, 2, 5, 1, 1, 1) == (5, False)
    s = o.read_state()[0]
    assert fld(s, R, 2, "term") == 5 and fld(s, R, 2, "voted") == -1
    # same term, free vote, up-to-date log: granted (the reference refuses, Q5)
    assert o.vote(0, 2, 5, 2, 2, 1) == (5, True)
    assert fld(o.read_state()[0], R, 2, "voted") == 2


def test_new_leader_median_commit_with_term_guard():
    """A term-2 leader holding a term-1 entry: nextIndex = lastIndex + 1, and
    the term-1 entry is committed only with the first term-2 entry (Raft §5.4.2);
    the reference commits +1 per ack with no term guard (K6)."""
    R = 3
    o = one_group(R)
    w = blank_groups(1, R)[0]
    for r in range(R):
        set_fld(w, R, r, "term", 2)
        set_fld(w, R, r, "voted", 1)
        set_fld(w, R, r, "last", 1)
        set_fld(w, R, r, "phys", 1)
        if r:
            set_fld(w, R, r, "flags", abi.FL_ARMED)
            set_fld(w, R, r, "election_ms", 10 ** 9)
    set_fld(w, R, 0, "role", abi.LEADER)
    set_fld(w, R, 0, "flags", abi.FL_HB_ACTIVE)
    set_session(w, R, 0, [2] * R, [0] * R)      # nextIndex = lastIndex + 1
    put(o, w, {r: [(1, 7)] for r in range(R)})
    o.step(1)                                   # heartbeat: matchIndex = 1, but log[0] is term 1
    s = o.read_state()[0]
    assert session(s, R, 0) == ([2, 2, 2], [1, 1, 1]) and fld(s, R, 0, "commit") == 0
    o.append_command(0, 0, 8)                   # a term-2 entry
    c = o.step(1)[0]                            # shipped and acked: median 2, log[1].term == 2
    s = o.read_state()[0]
    assert session(s, R, 0) == ([3, 3, 3], [2, 2, 2])
    assert fld(s, R, 0, "commit") == 2 and c[abi.C_INDEX["commits"]] == 1


def _multi_entry_group(E, r2_log):
    """R = 3, a term-2 LEADER r0 with log 7 | 8 9 10 (terms 1 | 2 2 2), commit 1;
    r1 holds only the committed entry, r2 holds `r2_log`; both followers sit at
    nextIndex 2 (just behind the committed prefix), the leader's own row at 5."""
    R = 3
    o = one_group(R, ae_max_entries=E)
    w = blank_groups(1, R)[0]
    logs = {0: [(1, 7), (2, 8), (2, 9), (2, 10)], 1: [(1, 7)], 2: r2_log}
    for r in range(R):
        set_fld(w, R, r, "term", 2)
        set_fld(w, R, r, "voted", 1)
        set_fld(w, R, r, "last", len(logs[r]))
        set_fld(w, R, r, "phys", len(logs[r]))
        set_fld(w, R, r, "commit", 1)
        if r:
            set_fld(w, R, r, "flags", abi.FL_ARMED)
            set_fld(w, R, r, "election_ms", 10 ** 9)
    set_fld(w, R, 0, "role", abi.LEADER)
    set_fld(w, R, 0, "flags", abi.FL_HB_ACTIVE)
    set_session(w, R, 0, [5, 2, 2], [0, 0, 0])
    put(o, w, logs)
    return o


def test_multi_entry_append_entries():
    """ae_max_entries = 4 (greeter.proto:37 `repeated LogEntry entries`; the
    reference sends one, RaftServer.kt:130-132): one tick ships the three
    entries 8 9 10 (min(4, lastIndex - nextIndex + 1)) to both followers.  r1
    appends all three; r2 keeps its matching entry 8 and overwrites from its
    first conflict (51) on (Raft Fig. 2, AppendEntries 3-4).  Each ack sets
    matchIndex = prev + 1 + 3 = 4 and nextIndex += 3, so the median commit
    reaches 4 in this one tick (log[3] is of term 2); the followers learn it
    from the next heartbeat."""
    R = 3
    o = _multi_entry_group(4, [(1, 7), (2, 8), (1, 51)])
    c = o.step(1)[0]
    s = o.read_state()[0]
    t, m = o.read_log()
    for r in range(R):
        assert [int(x) for x in t[0, r, :4]] == [1, 2, 2, 2], r
        assert [int(x) for x in m[0, r, :4]] == [7, 8, 9, 10], r
        assert fld(s, R, r, "last") == 4 and fld(s, R, r, "phys") == 4, r
    assert session(s, R, 0) == ([5, 5, 5], [4, 4, 4])
    assert fld(s, R, 0, "commit") == 4 and [int(fld(s, R, r, "commit")) for r in (1, 2)] == [1, 1]
    ix = abi.C_INDEX
    assert c[ix["append_sent"]] == 3 and c[ix["entry_reads_leader"]] == 6
    assert c[ix["entries_acked"]] == 6 and c[ix["entry_writes"]] == 3 + 2 and c[ix["commits"]] == 1
    c = o.step(1)[0]                               # heartbeats carry leaderCommit 4
    s = o.read_state()[0]
    assert [int(fld(s, R, r, "commit")) for r in range(R)] == [4, 4, 4]
    assert c[ix["entry_reads_leader"]] == 0 and c[ix["entry_writes"]] == 0


def test_single_entry_is_ae_max_entries_1():
    """ae_max_entries 0 and 1 are the one-entry request: the same tick ships
    only entry 8 (index 1), as in the reference's shape."""
    R = 3
    res = []
    for E in (0, 1):
        o = _multi_entry_group(E, [(1, 7), (2, 8), (1, 51)])
        c = o.step(1)[0]
        s = o.read_state()[0]
        res.append((s.copy(), c.copy()))
        assert session(s, R, 0) == ([5, 3, 3], [4, 2, 2])
        assert fld(s, R, 1, "last") == 2 and fld(s, R, 2, "last") == 3   # r2 keeps 8 and its tail
        assert c[abi.C_INDEX["entry_writes"]] == 1
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])


def test_ae_max_entries_validated():
    import pytest
    with pytest.raises(ValueError):
        O.Oracle(abi.make_params(ae_max_entries=2))             # reference mode: one entry
    with pytest.raises(ValueError):
        O.Oracle(abi.make_params(mode=TB, ae_max_entries=abi.MAX_AE_ENTRIES + 1))
    O.Oracle(abi.make_params(mode=TB, ae_max_entries=abi.MAX_AE_ENTRIES)).close()


def test_multi_entry_is_log_matching_safe():
    """Config 3 in textbook mode with up to 8 entries per request: committed
    prefixes still agree, no commit regresses, and no two leaders share a term."""
    kw = dict(abi.CONFIGS[3], G=300, churn_ppm=10_000)
    o = O.Oracle(abi.make_params(log_cap=500, mode=TB, ae_max_entries=8, **kw))
    c = o.step(1200, nthreads=8)
    ix = abi.C_INDEX
    assert c[:, ix["log_overflow"]].sum() == 0
    assert int(log_matching_flags(o.read_state(), *o.read_log(), kw["R"]).sum()) == 0
    assert c[:, ix["commit_regressions"]].sum() == 0 and c[:, ix["dual_leader_groups"]].sum() == 0
    assert c[:, ix["commits"]].sum() > 0


def test_textbook_mode_is_log_matching_safe():
    """At scale, committed prefixes agree in textbook mode; in the reference
    mode the same workloads violate Log Matching (Q1-Q4, Q9)."""
    for cfg, G, steps, cap in ((3, 400, 1200, 500), (5, 100, 1200, 1400)):
        flags = {}
        for mode in (abi.MODE_REFERENCE, TB):
            kw = dict(abi.CONFIGS[cfg], G=G)
            if cfg == 3:
                kw["churn_ppm"] = 10_000
            o = O.Oracle(abi.make_params(log_cap=cap, mode=mode, **kw))
            c = o.step(steps, nthreads=8)
            assert c[:, abi.C_INDEX["log_overflow"]].sum() == 0
            st = o.read_state()
            flags[mode] = int(log_matching_flags(st, *o.read_log(), kw["R"]).sum())
            if mode == TB:
                assert c[:, abi.C_INDEX["commit_regressions"]].sum() == 0
                assert c[:, abi.C_INDEX["dual_leader_groups"]].sum() == 0
                assert c[:, abi.C_INDEX["commits"]].sum() > 0
        assert flags[TB] == 0 and flags[abi.MODE_REFERENCE] > 0, (cfg, flags)


def test_mode_validated():
    import pytest
    with pytest.raises(ValueError):
        O.Oracle(abi.make_params(mode=7))
