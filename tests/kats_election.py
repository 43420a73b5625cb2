"""Known-answer traces K8-K14 for the election loop, the retry/latch/backoff
clocks and the remaining quirks, derived BY HAND from the reference source
(RaftServer.kt, Commons.kt) under the lockstep schedule of DESIGN.md §3.

They pin the oracle's reading of the most intricate rules independently of
the oracle itself (tests/test_oracle_kats.py runs them on the oracle;
tests/test_gpu_parity.py replays them through the engine's C-ABI with
write_state + step).  Every scenario makes the randomness irrelevant:
election_min_ms = election_max_ms = 20000 and backoff 2000..2000, so every
timer draw is exactly the lower bound; no drops, churn or commands; message
loss only through an isolation word written into the group state (harness
word 0 = remaining steps << 8 | replica).

Timer arithmetic (S-1): one step is 2000 ms; an armed timer is decremented in
phase T and fires at <= 0; a round's clock (phase_ms) grows by 2000 per step
after the round's first step; the retry countdown of undelivered
destinations (retry{} delay 5000, Commons.kt:37-45) is set to 5000 when a
round's requests go out with some destination undelivered and counts down by
2000 while the round is open and younger than 25000 ms.

Each trace is a dict: R, a setup function filling a blank canonical state
(and optional logs), and a list of checkpoints (step number, expected field
values per replica, expected session rows, expected counters of that step).
"""
from __future__ import annotations

import numpy as np

from helpers import abi, blank_groups, set_fld, set_session

FAR = 10 ** 9                      # a timer that never fires in these traces
F, C = abi.F_INDEX, abi.C_INDEX
ARMED, ELECTING, PRST, HB, BACKOFF = (abi.FL_ARMED, abi.FL_ELECTING, abi.FL_PENDING_RST, abi.FL_HB_ACTIVE,
                                      abi.FL_BACKOFF)
L, CAND, FOL = abi.LEADER, abi.CANDIDATE, abi.FOLLOWER


def fl(*bits, pending=0, votes=0, latch=0):
    v = 0
    for b in bits:
        v |= b
    return v | (pending << 8) | (votes << 16) | (latch << 20)


def params(kat, G=1):
    return dict(R=kat["R"], G=G, log_cap=64, seed=77, election_min_ms=20000, election_max_ms=20000,
                backoff_min_ms=2000, backoff_max_ms=2000, log_window=kat.get("window", 0))


def node(w, R, r, **kv):
    for k, v in kv.items():
        set_fld(w, R, r, k, v)


def iso(w, R, replica, steps):
    w[0, R * abi.NUM_FIELDS + 2 * R * R] = (steps << 8) | replica


# ---------------------------------------------------------------------------
# K8  latch closes at majority (RaftServer.kt:196, :209, :214-215, :218-219)
#     R=3 (majority 2, :44).  Replica 0's timer fires at step 1; replica 2 is
#     isolated.  Round: term 1, self-vote (:192-193); the self response and
#     replica 1's grant are delivered, replica 2's request is lost.  Two
#     countDown()s reach the latch's count of `majority`, so await() returns
#     in this step, cancelChildren() drops the pending retry to replica 2,
#     votes 2 >= 2 -> LEADER; the consumer starts the session (next = commit
#     + 1 = 1, match 0, :112-113) and its first tick runs in the same step
#     (fixedRateTimer delay 0): heartbeats (log empty, prev = -1) to self and
#     replica 1 succeed (match = prev + 1 = 0, :164), replica 2's is lost.
# ---------------------------------------------------------------------------
def k8_setup(w, R):
    node(w, R, 0, flags=ARMED, election_ms=2000)
    for r in (1, 2):
        node(w, R, r, flags=ARMED, election_ms=FAR)
    iso(w, R, 2, 50)


K8 = dict(name="K8 latch closes at majority", R=3, setup=k8_setup, checks=[
    (1, {0: dict(role=L, term=1, voted=1, flags=HB, phase_ms=0, retry_ms=0, election_ms=0),
         1: dict(role=FOL, term=1, voted=1, flags=ARMED, election_ms=20000),   # grant -> send(FOLLOWER) -> reset
         2: dict(role=FOL, term=0, voted=-1, flags=ARMED, election_ms=FAR - 2000)},
     {0: ([1, 1, 1], [0, 0, 0])},
     dict(timeouts=1, rounds=1, votes_granted=2, leaders_elected=1, sessions_ticked=1, append_sent=3,
          msg_dropped=2, leaders=1, groups_with_leader=1)),
])

# ---------------------------------------------------------------------------
# K9  retry of undelivered destinations every 5000 ms (Commons.kt:37-45), the
#     25 s round timeout (RaftServer.kt:189, :214), the 2-3 s backoff and the
#     next round (:218-221, :191-193).  R=3; the candidate (replica 0) is
#     isolated for the whole trace, so only its self-vote is delivered.
#     step 1:  round 1 (term 1); latch 1 < 2 stays open; dsts 1, 2 pending,
#              retry countdown 5000.
#     steps 2-13: round clock 2000 .. 24000; the countdown reaches <= 0 at
#              steps 4, 7, 10, 13, each re-sending to both pending dsts (2
#              requests lost per resend) and restarting it at 5000.
#     step 14: clock 26000 >= 25000: await() times out, cancelChildren();
#              still CANDIDATE with 1 < 2 votes -> backoff delay 2000.
#     step 15: the delay has run out, state == CANDIDATE: round 2 (term 2).
# ---------------------------------------------------------------------------
def k9_setup(w, R):
    node(w, R, 0, flags=ARMED, election_ms=2000)
    for r in (1, 2):
        node(w, R, r, flags=ARMED, election_ms=FAR)
    iso(w, R, 0, 100)


_open = lambda ph, rt: dict(role=CAND, term=1, voted=1, phase_ms=ph, retry_ms=rt,   # noqa: E731
                            flags=fl(ELECTING, pending=0b110, votes=1, latch=1))
K9 = dict(name="K9 vote retry every 5000 ms, 25 s round timeout, backoff, next round", R=3, setup=k9_setup,
          checks=[
              (1, {0: _open(0, 5000)}, {}, dict(timeouts=1, rounds=1, votes_granted=1, msg_dropped=2)),
              (2, {0: _open(2000, 3000)}, {}, dict(msg_dropped=0, rounds=0)),
              (3, {0: _open(4000, 1000)}, {}, dict(msg_dropped=0)),
              (4, {0: _open(6000, 5000)}, {}, dict(msg_dropped=2, rounds=0, votes_granted=0)),
              (7, {0: _open(12000, 5000)}, {}, dict(msg_dropped=2)),
              (10, {0: _open(18000, 5000)}, {}, dict(msg_dropped=2)),
              (12, {0: _open(22000, 1000)}, {}, dict(msg_dropped=0)),
              (13, {0: _open(24000, 5000)}, {}, dict(msg_dropped=2)),
              (14, {0: dict(role=CAND, term=1, voted=1, phase_ms=2000, retry_ms=0, flags=fl(ELECTING, BACKOFF)),
                    1: dict(term=0, voted=-1, role=FOL), 2: dict(term=0, voted=-1, role=FOL)},
               {}, dict(msg_dropped=0, rounds=0, timeouts=0)),
              (15, {0: dict(role=CAND, term=2, voted=1, phase_ms=0, retry_ms=5000,
                            flags=fl(ELECTING, pending=0b110, votes=1, latch=1))},
               {}, dict(rounds=1, msg_dropped=2, votes_granted=1)),
          ])

# ---------------------------------------------------------------------------
# K10 Q6 (RaftServer.kt:210): a candidate seeing a higher-term vote response
#     becomes FOLLOWER WITHOUT adopting the term.  R=3; replica 1 is at term 5.
#     Candidate 0 (term 1) gets: self grant; replica 1 rejects (1 < 5, :229)
#     answering term 5 -> state = FOLLOWER, currentTerm stays 1; replica 2
#     grants.  Latch 3 >= 2 closes the round; state != CANDIDATE, so the loop
#     ends (:191) and `launch { send(FOLLOWER) }` (:225) re-arms the timer.
# ---------------------------------------------------------------------------
def k10_setup(w, R):
    node(w, R, 0, flags=ARMED, election_ms=2000)
    node(w, R, 1, flags=ARMED, election_ms=FAR, term=5, voted=3)
    node(w, R, 2, flags=ARMED, election_ms=FAR)


K10 = dict(name="K10 Q6 candidate steps down without the response term", R=3, setup=k10_setup, checks=[
    (1, {0: dict(role=FOL, term=1, voted=1, flags=ARMED, election_ms=20000, phase_ms=0, retry_ms=0),
         1: dict(role=FOL, term=5, voted=3, flags=ARMED, election_ms=FAR - 2000),       # rejected: no send
         2: dict(role=FOL, term=1, voted=1, flags=ARMED, election_ms=20000)},
     {}, dict(rounds=1, votes_granted=2, leaders_elected=0, leaders=0)),
])

# ---------------------------------------------------------------------------
# K11 Q7 (RaftServer.kt:146-153) and Q12/S-10 (:117).  R=3; replica 0 is LEADER
#     at term 2 (votedFor 1) with a fresh session; replica 1 is at term 5.
#     Tick: replica 1's append handler answers term 5 (no term change for it;
#     leaderId 1 != 2 -> FOLLOWER + send -> its timer re-arms, :264-266).  The
#     leader adopts term 5, becomes FOLLOWER, KEEPS votedFor 1, and its
#     offer(FOLLOWER) re-arms its timer (consumer idle).  Replica 2's
#     response (term 2, success) is still processed: match[2] = prev + 1 = 0.
#     Step 2: the session's tick finds state == FOLLOWER: cancel(), nothing sent.
# ---------------------------------------------------------------------------
def k11_setup(w, R):
    node(w, R, 0, role=L, term=2, voted=1, flags=HB)
    node(w, R, 1, term=5, voted=3, flags=ARMED, election_ms=FAR)
    node(w, R, 2, term=2, voted=1, flags=ARMED, election_ms=FAR)
    set_session(w, R, 0, [1, 1, 1], [0, 0, 0])


K11 = dict(name="K11 Q7 leader adopts a response term, keeps votedFor; S-10 cancel", R=3, setup=k11_setup, checks=[
    (1, {0: dict(role=FOL, term=5, voted=1, flags=fl(ARMED, HB), election_ms=20000),
         1: dict(role=FOL, term=5, voted=3, flags=ARMED, election_ms=20000),
         2: dict(role=FOL, term=2, voted=1, flags=ARMED, election_ms=20000)},
     {0: ([1, 1, 1], [0, 0, 0])}, dict(sessions_ticked=1, append_sent=3, leaders=0)),
    (2, {0: dict(role=FOL, term=5, voted=1, flags=ARMED, election_ms=18000)},
     {}, dict(sessions_ticked=0, append_sent=0)),
])

# ---------------------------------------------------------------------------
# K12 Q11 (RaftServer.kt:128, :170-172; Commons.kt:53-54).  R=3; leader 0 at
#     term 1 with log [(1, 0xA)] and a session whose nextIndex towards
#     replica 1 is 5: prevLogIndex 3 >= lastIndex 1, log.get(3) throws, that
#     coroutine ends in the catch -- no message, replica 1 untouched (its
#     timer is not re-armed).  Self and replica 2 get entry 0 (prev = -1):
#     after self, match [1,0,0] counts 1 < 2; after replica 2, [1,0,1] counts
#     2 >= 2 -> commitIndex 1 (+1 per acked entry, :161-162).
# ---------------------------------------------------------------------------
def k12_setup(w, R):
    node(w, R, 0, role=L, term=1, voted=1, flags=HB, last=1, phys=1)
    for r in (1, 2):
        node(w, R, r, term=1, voted=1, flags=ARMED, election_ms=FAR)
    set_session(w, R, 0, [1, 5, 1], [0, 0, 0])


K12 = dict(name="K12 Q11 leader-side Log.get throw skips that peer", R=3, setup=k12_setup,
           logs={0: [(1, 0xA)]}, checks=[
    (1, {0: dict(role=L, term=1, commit=1, last=1, phys=1),
         1: dict(flags=ARMED, election_ms=FAR - 2000, last=0, phys=0, commit=0),
         2: dict(role=FOL, flags=ARMED, election_ms=20000, last=1, phys=1, commit=0)},
     {0: ([2, 5, 2], [1, 0, 1])},
     dict(sessions_ticked=1, append_sent=2, append_skipped=1, entries_acked=2, commits=1, entry_reads_leader=2,
          prev_reads_leader=0, entry_writes=2)),
], final_logs={0: [(1, 0xA)], 2: [(1, 0xA)]})

# ---------------------------------------------------------------------------
# K13 Q12 (RaftServer.kt:117): only state == FOLLOWER stops a heartbeat tick.
#     R=3; replica 0 is LEADER (term 1, empty log) and its election timer,
#     never cancelled by leadership, fires at step 1: CANDIDATE, round term 2.
#     Replicas 1, 2 (term 1, log [(1, 0xB)]) reject: the candidate's last
#     log term 0 < 1 (:232-233), and keep term 1 (Q5).  Latch 3 closes the
#     round with 1 vote -> backoff.  The old session still ticks in phase A
#     (state is CANDIDATE, not FOLLOWER) with currentTerm 2: both followers
#     adopt term 2 with votedFor -1 (:257-262).  Step 2: the backoff ends,
#     round 2 (term 3) is rejected again, and the tick moves them to term 3.
# ---------------------------------------------------------------------------
def k13_setup(w, R):
    node(w, R, 0, role=L, term=1, voted=1, flags=fl(HB, ARMED), election_ms=2000)
    for r in (1, 2):
        node(w, R, r, term=1, voted=1, flags=ARMED, election_ms=FAR, last=1, phys=1)
    set_session(w, R, 0, [1, 1, 1], [0, 0, 0])


K13 = dict(name="K13 Q12 a CANDIDATE's heartbeat session keeps ticking", R=3, setup=k13_setup,
           logs={1: [(1, 0xB)], 2: [(1, 0xB)]}, checks=[
    (1, {0: dict(role=CAND, term=2, voted=1, flags=fl(ELECTING, BACKOFF, HB), phase_ms=2000, retry_ms=0),
         1: dict(role=FOL, term=2, voted=-1, flags=ARMED, election_ms=20000),
         2: dict(role=FOL, term=2, voted=-1, flags=ARMED, election_ms=20000)},
     {0: ([1, 1, 1], [0, 0, 0])},
     dict(timeouts=1, rounds=1, votes_granted=1, sessions_ticked=1, append_sent=3, vote_log_reads=2)),
    (2, {0: dict(role=CAND, term=3, voted=1, flags=fl(ELECTING, BACKOFF, HB), phase_ms=2000),
         1: dict(term=3, voted=-1), 2: dict(term=3, voted=-1)},
     {}, dict(rounds=1, votes_granted=1, sessions_ticked=1)),
])

# ---------------------------------------------------------------------------
# K14 the FOLLOWER send deferred while the consumer is busy (RaftServer.kt:225,
#     :241, :261-266; S-5).  R=3; replica 1 is inside leaderElection() with an
#     open round (term 3, 1 vote, dsts 0 and 2 pending, retry countdown 3000,
#     clock 2000).  Step 1: replica 0's timer fires (round term 4); replica 1
#     grants it (term 4, votedFor 1, FOLLOWER) and its `launch { send(FOLLOWER) }`
#     waits: the consumer is busy, so the timer is NOT re-armed.  Replica 0
#     wins and heartbeats; replica 1's own round stays open (latch 1 < 2,
#     clock 4000 < 25000, countdown 1000).  Step 2: replica 1's countdown
#     expires and retry{} re-sends to dsts 0 and 2 with its CURRENT term 4
#     (:204); both answer false (same term, votedFor 1 != 2, :230); the latch
#     reaches 3 >= 2, state is FOLLOWER, so leaderElection() returns and the
#     queued FOLLOWER send re-arms the timer.
# ---------------------------------------------------------------------------
def k14_setup(w, R):
    node(w, R, 0, term=3, voted=2, flags=ARMED, election_ms=2000)
    node(w, R, 1, role=CAND, term=3, voted=2, flags=fl(ELECTING, pending=0b101, votes=1, latch=1), phase_ms=2000,
         retry_ms=3000)
    node(w, R, 2, term=3, voted=2, flags=ARMED, election_ms=FAR)


K14 = dict(name="K14 FOLLOWER send deferred during an election", R=3, setup=k14_setup, checks=[
    (1, {0: dict(role=L, term=4, voted=1, flags=HB),
         1: dict(role=FOL, term=4, voted=1, election_ms=0, phase_ms=4000, retry_ms=1000,
                 flags=fl(ELECTING, PRST, pending=0b101, votes=1, latch=1)),
         2: dict(role=FOL, term=4, voted=1, flags=ARMED, election_ms=20000)},
     {}, dict(timeouts=1, rounds=1, votes_granted=3, leaders_elected=1, sessions_ticked=1)),
    (2, {0: dict(role=L, term=4, voted=1),
         1: dict(role=FOL, term=4, voted=1, flags=ARMED, election_ms=20000, phase_ms=0, retry_ms=0),
         2: dict(term=4, voted=1, election_ms=20000)},
     {}, dict(votes_granted=0, rounds=0, timeouts=0, sessions_ticked=1)),
])

# ---------------------------------------------------------------------------
# K15 the ring's window misses (raft_params.log_window).  R=3,
#     a 4-slot ring.  Every replica holds lastIndex 2 over a physical list of
#     8 (a ghost tail: 6 slots beyond lastIndex), so the retained slots are
#     [4, 8).  Leader 0's session has nextIndex 3 towards everyone: each of
#     the 3 requests does log.get(prevLogIndex = 1) (:128) -- 1 < 8 - 4, a
#     miss -- and carries no entry (lastIndex 2 < 3, :130); each destination's
#     append() does log.get(1) again (:276), another miss.  6 misses, and
#     the run is marked invalid (the values read are NOT the reference's: the
#     slots were overwritten by the ring, so no state is checked beyond it).
# ---------------------------------------------------------------------------
def k15_setup(w, R):
    node(w, R, 0, role=L, term=1, voted=1, flags=HB, last=2, phys=8)
    for r in (1, 2):
        node(w, R, r, term=1, voted=1, flags=ARMED, election_ms=FAR, last=2, phys=8)
    set_session(w, R, 0, [3, 3, 3], [0, 0, 0])


K15 = dict(name="K15 ring window misses are counted", R=3, window=4, setup=k15_setup,
           logs={r: [(1, 10 + j) for j in range(8)] for r in range(3)}, checks=[
    (1, {}, {}, dict(sessions_ticked=1, append_sent=3, prev_reads_leader=3, prev_reads_follower=3,
                     entry_reads_leader=0, log_window_miss=6)),
])

KATS = [K8, K9, K10, K11, K12, K13, K14, K15]


def initial(kat):
    R = kat["R"]
    w = blank_groups(1, R)
    kat["setup"](w, R)
    return w


def initial_logs(kat, cap=64):
    R = kat["R"]
    t = np.zeros((1, R, cap), np.int32)
    c = np.zeros((1, R, cap), np.uint32)
    for r, ents in kat.get("logs", {}).items():
        for j, (et, ec) in enumerate(ents):
            t[0, r, j], c[0, r, j] = et, ec
    return t, c


def run(kat, x):
    """Replay `kat` on x (an Oracle or a RaftEngine built from params(R));
    assert every checkpoint."""
    R = kat["R"]
    x.write_state(initial(kat))
    if kat.get("logs"):
        x.write_log(*initial_logs(kat, x.cap))
    done = 0
    for step, fields, sessions, counters in kat["checks"]:
        c = None
        if step > done + 1:
            x.step(step - done - 1)
        c = x.step(1)[0]
        done = step
        s = x.read_state()[0]
        where = f"{kat['name']} @ step {step}"
        for r, kv in fields.items():
            for k, v in kv.items():
                got = int(s[r * abi.NUM_FIELDS + F[k]])
                assert got == v, f"{where}: replica {r} {k} = {got}, expected {v}"
        for sr, (nx, mt) in sessions.items():
            got = ([int(s[R * abi.NUM_FIELDS + sr * R + d]) for d in range(R)],
                   [int(s[R * abi.NUM_FIELDS + R * R + sr * R + d]) for d in range(R)])
            assert got == (nx, mt), f"{where}: session of replica {sr} = {got}, expected {(nx, mt)}"
        for k, v in counters.items():
            assert int(c[C[k]]) == v, f"{where}: counter {k} = {int(c[C[k]])}, expected {v}"
    if "final_logs" in kat:
        t, cm = x.read_log()
        for r, ents in kat["final_logs"].items():
            assert [(int(t[0, r, j]), int(cm[0, r, j])) for j in range(len(ents))] == ents, (kat["name"], r)
