"""The oracle against the known-answer traces K1-K7, hand-derived
from the reference source, and the Random123 Philox vectors.

These pin the CPU restatement before it is trusted as the GPU's parity oracle.
The reference ships no tests or fixtures of its own (parity is otherwise unpinned)."""
import json
import os

import numpy as np
import pytest

import oracle as O
from helpers import abi, blank_groups, fld, set_fld, set_session, session

HERE = os.path.dirname(os.path.abspath(__file__))


def test_philox_kats_oracle():
    kat = json.load(open(os.path.join(HERE, "golden", "philox_kat.json")))
    for v in kat["vectors"]:
        ctr = [int(x, 16) for x in v["ctr"]]
        key = [int(x, 16) for x in v["key"]]
        assert O.philox(ctr, key) == [int(x, 16) for x in v["out"]]


def test_k1_ghost_tail():
    """Commons.kt:53-68: add(i < lastIndex) never shrinks the ArrayList."""
    A, B, Cc, X, Y, Z, W = (ord(c) for c in "ABCXYZW")
    L = O.OracleLog()
    for i, c in enumerate([A, B, Cc]):
        assert L.add(i, 0, c) == 1
    assert L.add(1, 0, X) == 1
    assert [c for _, c in L.phys()] == [A, X, Cc] and L.last_index == 2
    assert L.add(2, 0, Y) == 1
    assert [c for _, c in L.phys()] == [A, X, Cc, Y] and L.last_index == 3
    assert [c for _, c in L.entries()] == [A, X, Cc]          # Y invisible, C resurrected
    assert L.add(3, 0, Z) == 1
    assert [c for _, c in L.phys()] == [A, X, Cc, Y, Z] and L.last_index == 4
    assert [c for _, c in L.entries()] == [A, X, Cc, Y]
    assert L.add(5, 0, W) == 0 and L.last_index == 4           # lastIndex < i -> false
    with pytest.raises(IndexError):
        L.get(4)                                               # lastIndex - 1 < i throws


def test_log_capacity_overflow_is_counted_not_wrapped():
    L = O.OracleLog(cap=2)
    assert L.add(0, 1, 1) == 1 and L.add(1, 1, 2) == 1
    assert L.add(2, 1, 3) == -1 and L.last_index == 2 and L.size == 2


def one_group(R=3, **kw):
    p = abi.make_params(R=R, G=1, log_cap=64, **kw)
    return O.Oracle(p)


def put(o, w, logs=None):
    o.write_state(w[None] if w.ndim == 1 else w)
    if logs is not None:
        t = np.zeros((1, o.R, o.cap), np.int32)
        c = np.zeros((1, o.R, o.cap), np.uint32)
        for r, ents in logs.items():
            for j, (et, ec) in enumerate(ents):
                t[0, r, j], c[0, r, j] = et, ec
        o.write_log(t, c)


def test_k2_vote():
    """RaftServer.kt:229-243: same-term grant iff votedFor == candidate."""
    R = 3
    o = one_group(R)
    w = blank_groups(1, R)[0]
    set_fld(w, R, 0, "term", 2)
    put(o, w)
    assert o.vote(0, 0, 2, 3, 0, 0) == (2, False)
    assert o.vote(0, 0, 3, 3, 0, 0) == (3, True)
    s = o.read_state()[0]
    assert fld(s, R, 0, "term") == 3 and fld(s, R, 0, "voted") == 3 and fld(s, R, 0, "role") == abi.FOLLOWER
    assert fld(s, R, 0, "flags") & abi.FL_ARMED            # send(FOLLOWER) -> reset() (RaftServer.kt:64)
    assert o.vote(0, 0, 3, 4, 0, 0) == (3, False)
    assert o.vote(0, 0, 3, 3, 0, 0) == (3, True)


def test_k3_vote_log_check():
    """RaftServer.kt:232-243, :247 (Q5: a log-check rejection does not adopt the term)."""
    R = 3
    o = one_group(R)
    w = blank_groups(1, R)[0]
    set_fld(w, R, 0, "term", 2)
    set_fld(w, R, 0, "last", 2)
    set_fld(w, R, 0, "phys", 2)
    put(o, w, {0: [(1, ord("a")), (2, ord("b"))]})
    assert o.vote(0, 0, 5, 1, 5, 1) == (2, False)
    assert o.vote(0, 0, 5, 1, 1, 2) == (2, False)
    assert o.vote(0, 0, 5, 1, 2, 2) == (5, True)


def test_k4_stale_leader_deposes():
    """RaftServer.kt:257-278 (Q3): a term-1 append deposes a term-3 leader and truncates."""
    R = 3
    o = one_group(R)
    w = blank_groups(1, R)[0]
    set_fld(w, R, 1, "term", 3)
    set_fld(w, R, 1, "role", abi.LEADER)
    set_fld(w, R, 1, "last", 2)
    set_fld(w, R, 1, "phys", 2)
    put(o, w, {1: [(3, ord("p")), (3, ord("q"))]})
    assert o.append(0, 1, 1, 1, -1, -1, (1, ord("z")), 0) == (3, True, 0)
    s = o.read_state()[0]
    assert fld(s, R, 1, "role") == abi.FOLLOWER and fld(s, R, 1, "term") == 3
    assert fld(s, R, 1, "last") == 1 and fld(s, R, 1, "phys") == 2
    t, c = o.read_log()
    assert [(t[0, 1, j], c[0, 1, j]) for j in range(2)] == [(1, ord("z")), (3, ord("q"))]


def test_k5_commit_regress():
    """RaftServer.kt:270-272 (Q4): commitIndex = min(leaderCommit, lastIndex) can decrease."""
    R = 3
    o = one_group(R)
    w = blank_groups(1, R)[0]
    set_fld(w, R, 0, "commit", 5)
    set_fld(w, R, 0, "last", 2)
    set_fld(w, R, 0, "phys", 2)
    set_fld(w, R, 0, "term", 1)
    put(o, w, {0: [(1, 1), (1, 2)]})
    o.append(0, 0, 1, 2, 1, 1, None, 6)
    assert fld(o.read_state()[0], R, 0, "commit") == 2


def leader_group(R, leader_log, follower_logs, commit=0, term=1):
    """Replica 0 LEADER with a fresh session (RaftServer.kt:112-113); followers'
    timers armed far in the future so no election interferes."""
    w = blank_groups(1, R)[0]
    for r in range(R):
        set_fld(w, R, r, "term", term)
        set_fld(w, R, r, "voted", 1)
        log = leader_log if r == 0 else follower_logs
        set_fld(w, R, r, "last", len(log))
        set_fld(w, R, r, "phys", len(log))
        if r:
            set_fld(w, R, r, "flags", abi.FL_ARMED)
            set_fld(w, R, r, "election_ms", 10 ** 9)
    set_fld(w, R, 0, "role", abi.LEADER)
    set_fld(w, R, 0, "commit", commit)
    set_fld(w, R, 0, "flags", abi.FL_HB_ACTIVE)
    set_session(w, R, 0, [commit + 1] * R, [0] * R)
    logs = {0: leader_log}
    for r in range(1, R):
        logs[r] = follower_logs
    return w, logs


def test_k6_commit_by_one():
    """RaftServer.kt:126-132, :156-165 (Q9): +1 per passing entry response, in peer order."""
    R = 3
    o = one_group(R)
    w, logs = leader_group(R, [(1, ord("a"))], [])
    put(o, w, logs)
    c = o.step(1)[0]
    s = o.read_state()[0]
    assert fld(s, R, 0, "commit") == 1 and c[abi.C_INDEX["commits"]] == 1
    assert session(s, R, 0) == ([2, 2, 2], [1, 1, 1])
    assert all(fld(s, R, r, "commit") == 0 for r in (1, 2))    # leaderCommit snapshot was 0
    o.step(1)                                                  # heartbeat: prev = 0
    s = o.read_state()[0]
    assert session(s, R, 0) == ([2, 2, 2], [1, 1, 1])
    assert all(fld(s, R, r, "commit") == 1 for r in (1, 2))


def test_k7_leader_self_truncation():
    """RaftServer.kt:100-107, :122-132, :274-278; Commons.kt:56-68 (Q8 + Q1)."""
    R = 3
    a, b, cc, d = (ord(x) for x in "abcd")
    o = one_group(R)
    w, logs = leader_group(R, [(1, a), (1, b), (1, cc)], [])
    put(o, w, logs)
    o.step(1)                                  # tick 1: everyone gets `a`; leader truncates itself
    s = o.read_state()[0]
    assert fld(s, R, 0, "last") == 1 and fld(s, R, 0, "phys") == 3 and fld(s, R, 0, "commit") == 1
    o.step(1)                                  # tick 2: heartbeat
    o.append_command(0, 0, d)                  # visible [a, b], physical [a, b, c, d]
    s = o.read_state()[0]
    assert fld(s, R, 0, "last") == 2 and fld(s, R, 0, "phys") == 4
    o.step(1)                                  # tick 3 ships the stale slot `b`, not `d`
    t, c = o.read_log()
    s = o.read_state()[0]
    for r in (1, 2):
        assert fld(s, R, r, "last") == 2
        assert [int(c[0, r, j]) for j in range(2)] == [a, b]


# ---- K8-K14: the election loop and the remaining quirks (tests/kats_election.py) ----
import kats_election as KE  # noqa: E402


@pytest.mark.parametrize("kat", KE.KATS, ids=lambda k: k["name"].split()[0])
def test_election_kats_on_oracle(kat):
    o = O.Oracle(abi.make_params(**KE.params(kat)))
    KE.run(kat, o)
