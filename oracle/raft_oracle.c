/*
 * raft_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker; see
 * raft_oracle.h).  Never linked into the product.
 *
 * One object per replica, as in the reference: each `onode_t` is one
 * `RaftServer` (RaftServer.kt:28-51) owning a `Log<LogEntry>`
 * (Commons.kt:47-74) kept as a growable array, exactly like the ArrayList it
 * restates (physical size and lastIndex tracked separately: ghost tail, Q1).
 * Every function cites the reference lines it follows.  The nondeterminism
 * of the reference (threads, coroutines, wall clock, java.util.Random) is
 * replaced by the lockstep schedule of DESIGN.md §3; the comments name the
 * schedule rule (S-x) used wherever the reference leaves a choice.
 *
 * Parity status: pinned by SURVEY.md §4 KATs K1-K7 and Random123 Philox
 * vectors only (no reference outputs exist or can be produced here).
 */
#include "raft_oracle.h"
#include "philox_ref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define MAXR RAFT_MAX_R

/* ------------------------------------------------------------------ */
/* Log<T>  (Commons.kt:47-74)                                          */
/* ------------------------------------------------------------------ */
typedef struct { int32_t term; uint32_t cmd; } entry_t;   /* LogEntry greeter.proto:29-32 */

typedef struct {
    int32_t  lastIndex;   /* Commons.kt:49  var lastIndex = 0                     */
    int32_t  size;        /* Commons.kt:51  mutableListOf<T>() physical size      */
    int32_t  alloc;
    int32_t  cap;         /* build-side physical capacity; overflow counted       */
    int32_t  textbook;    /* RAFT_MODE_TEXTBOOK: array semantics, no ghost tail   */
    int32_t  window;      /* build-side log_window W (0: every slot kept); the    *
                           * oracle keeps the whole list and counts accesses      *
                           * below size - W (RAFT_C_LOG_WINDOW_MISS)              */
    entry_t* items;
} olog_t;

/* An access of the reference (Log.get / Log.add) at physical index j that a
 * W-slot window would not hold: j < size - W.  Counted, never served
 * differently: the run is invalid, as with overflow. */
static void olog_touch(const olog_t* l, int32_t j, int64_t* c) {
    if (c && l->window && j < l->size - l->window) c[RAFT_C_LOG_WINDOW_MISS]++;
}

/* Commons.kt:53-54: get(i) = if (lastIndex - 1 < i) throw IndexOutOfBounds else log[i]
 * (log[i] itself throws for i < 0).  Returns 0 where the reference throws. */
static int olog_get(const olog_t* l, int32_t i, entry_t* out) {
    if (l->lastIndex - 1 < i) return 0;
    if (i < 0 || i >= l->size) return 0;
    *out = l->items[i];
    return 1;
}

static int olog_reserve(olog_t* l, int32_t n) {
    if (n <= l->alloc) return 1;
    int32_t a = l->alloc ? l->alloc : 8;
    while (a < n) a *= 2;
    if (a > l->cap) a = l->cap;
    entry_t* p = (entry_t*)realloc(l->items, (size_t)a * sizeof(entry_t));
    if (!p) abort();
    l->items = p;
    l->alloc = a;
    return 1;
}

/* Commons.kt:56-68.  Returns 1 (true), 0 (false), -1 (build-side overflow:
 * no physical slot left, nothing changes), -2 (ArrayList.set threw, i < 0).
 * c: the step's counters (window misses), or NULL. */
static int olog_add(olog_t* l, int32_t i, entry_t e, int64_t* c) {
    if (l->textbook && i >= 0 && i <= l->lastIndex) {
        /* textbook mode: an array log -- slot i, truncating after it (no ghost tail, Q1) */
        if (i >= l->cap) return -1;
        olog_touch(l, i, c);
        olog_reserve(l, i + 1);
        l->items[i] = e;
        l->lastIndex = i + 1;
        if (l->size < i + 1) l->size = i + 1;      /* high-water mark of written slots */
        return 1;
    }
    if (l->lastIndex == i) {                       /* :58 */
        if (l->size >= l->cap) return -1;          /* capacity exhausted: counted, never wrapped */
        olog_reserve(l, l->size + 1);
        l->lastIndex += 1;                         /* :59 */
        l->items[l->size++] = e;                   /* :60 log.add(entry): appends at the PHYSICAL end (Q1) */
        return 1;
    } else if (l->lastIndex < i) {                 /* :62 */
        return 0;
    } else {                                       /* :63-66 */
        if (i < 0) return -2;
        olog_touch(l, i, c);
        l->items[i] = e;                           /* :64 log[i] = entry (no shrink: ghost tail) */
        l->lastIndex = i + 1;                      /* :65 */
        return 1;
    }
}

/* ------------------------------------------------------------------ */
/* RaftServer node  (RaftServer.kt:28-51)                              */
/* ------------------------------------------------------------------ */
typedef struct {
    int32_t id;             /* 1-based, RaftClient(id = ...) RaftServer.kt:303-305 */
    int32_t currentTerm;    /* :35-36 */
    int32_t votedFor;       /* :38-39 */
    int32_t state;          /* :41-42 */
    int32_t commitIndex;    /* :46 */
    olog_t  log;            /* :48 */
    /* ResettableCountdownTimer (Commons.kt:10-31) */
    int32_t timerArmed, electionMs;
    /* state-change consumer (RaftServer.kt:50, :60-69) */
    int32_t electing, pendingReset;
    /* leaderElection() loop locals (RaftServer.kt:187-226) */
    int32_t backoff;        /* 0: round (latch open), 1: delay() backoff */
    int32_t phaseMs;        /* round elapsed ms, or backoff remaining ms */
    int32_t retryMs;        /* retry(delay = 5000) countdown, Commons.kt:37-45 */
    int32_t votes;          /* votesGranted :194 */
    int32_t latch;          /* responses counted on countDownLatch :196, :209 */
    uint32_t pending;       /* dsts whose retry{} has not returned yet */
    /* appendRequestAndLeaderHeartbeat() session (RaftServer.kt:109-178) */
    int32_t hbActive;
    int32_t nextIndex[MAXR], matchIndex[MAXR];
    /* per-step temporaries, not state: the vote request snapshot (S-4) */
    uint32_t sendMask;
    int32_t reqTerm, reqLastIndex, reqLastTerm;
} onode_t;

typedef struct {
    onode_t n[MAXR];
    int32_t isoRem, isoRep;   /* churn isolation (harness) */
    int32_t cmdCount;         /* commands issued (harness) */
} ogroup_t;

struct oracle {
    raft_params p;
    int32_t  R, majority;
    uint32_t key[2];
    int64_t  G;
    uint32_t t;               /* next step index */
    ogroup_t* groups;
};

/* per-(group, step) context */
typedef struct {
    const struct oracle* o;
    uint32_t t, gid;
    int64_t* c;               /* this step's counters (may be a scratch array) */
    int32_t  isoRep;          /* isolated replica this step, -1 if none */
    uint32_t partMask;        /* replicas on side B of this step's partition */
} ctx_t;

/* ------------------------------------------------------------------ */
/* harness randomness (S-9)                                            */
/* ------------------------------------------------------------------ */
static void draw4(const ctx_t* x, uint32_t c0, uint32_t purpose, uint32_t sub, uint32_t w[4]) {
    uint32_t ctr[4] = { c0, x->gid, purpose, sub };
    philox_ref(ctr, x->o->key, w);
}
/* `(lo..hi).random()` = Random().nextInt(hi - lo + 1) + lo   (Commons.kt:33-34).
 * Per-replica draws share one Philox call per 4 replicas: replica r takes
 * word (r & 3) of Philox(c0, gid, purpose, r >> 2); the word is scaled to the
 * span by a 32x32->64 multiply-shift (S-9). */
static int32_t draw_range(const ctx_t* x, uint32_t c0, uint32_t purpose, int32_t r, int32_t lo, int32_t hi) {
    uint32_t w[4];
    draw4(x, c0, purpose, (uint32_t)r >> 2, w);
    uint32_t span = (uint32_t)(hi - lo) + 1u;
    return lo + (int32_t)(((uint64_t)w[r & 3] * span) >> 32);
}
/* w / 2^32 < ppm / 10^6, exactly */
static int hit32(uint32_t w, uint32_t ppm) {
    return (uint64_t)w * 1000000ull < ((uint64_t)ppm << 32);
}
static int hit16(uint32_t u16, uint32_t ppm) {
    return (uint64_t)u16 * 1000000ull < ((uint64_t)ppm << 16);
}

/* 16-bit drop uniforms of one sender for one phase: index j = 2*dd + b where
 * dd = d < s ? d : d - 1 and b = 0 request, 1 response (S-9). */
typedef struct { uint32_t w[2][4]; } dropu_t;
static void drop_uniforms(const ctx_t* x, uint32_t purpose, int32_t s, dropu_t* u) {
    int32_t R = x->o->R;
    int32_t nj = 2 * (R - 1);
    for (int k = 0; k < 2; ++k) {
        if (k * 8 < nj) draw4(x, x->t, purpose, (uint32_t)s | ((uint32_t)k << 8), u->w[k]);
    }
}
static int lost(const ctx_t* x, const dropu_t* u, int32_t s, int32_t d, int32_t b) {
    if (s == d) return 0;                                   /* self-RPC never dropped (S-7) */
    if (x->isoRep >= 0 && (s == x->isoRep || d == x->isoRep)) return 1;
    if (((x->partMask >> s) ^ (x->partMask >> d)) & 1u) return 1;
    if (x->o->p.drop_ppm == 0) return 0;
    int32_t dd = d < s ? d : d - 1;
    int32_t j = 2 * dd + b;
    uint32_t word = u->w[j >> 3][(j & 7) >> 1];
    uint32_t u16 = (word >> (16 * (j & 1))) & 0xFFFFu;
    return hit16(u16, x->o->p.drop_ppm);
}

/* ------------------------------------------------------------------ */
/* timer and consumer                                                  */
/* ------------------------------------------------------------------ */
/* ResettableCountdownTimer.reset() (Commons.kt:16-20) -> startTimer() (:22-29):
 * a fresh (20_000..23_000).random() one-shot. */
static void reset_timer(const ctx_t* x, onode_t* n) {
    n->timerArmed = 1;
    n->electionMs = draw_range(x, x->t, RAFT_RNG_TIMER, n->id - 1,
                               x->o->p.election_min_ms, x->o->p.election_max_ms);
}

/* `launch { channel.send(state) }` with state == FOLLOWER (RaftServer.kt:241,
 * :261, :266): the consumer resets the timer (:64) when idle; while it is busy
 * in leaderElection() the send waits and is applied when the loop ends (S-5). */
static void send_follower(const ctx_t* x, onode_t* n) {
    if (n->electing) n->pendingReset = 1;
    else reset_timer(x, n);
}

/* `channel.offer(FOLLOWER)` (RaftServer.kt:152): dropped while busy (S-6). */
static void offer_follower(const ctx_t* x, onode_t* n) {
    if (!n->electing) reset_timer(x, n);
}

/* appendRequestAndLeaderHeartbeat() entry (RaftServer.kt:109-113).  A second
 * LEADER reaction re-initialises the single session (S-8). */
static void start_session(const ctx_t* x, onode_t* n) {
    n->hbActive = 1;
    for (int d = 0; d < x->o->R; ++d) {
        n->nextIndex[d] = x->o->p.mode == RAFT_MODE_TEXTBOOK
                              ? n->log.lastIndex + 1      /* textbook: the leader's next slot */
                              : n->commitIndex + 1;       /* :112 (Q8) */
        n->matchIndex[d] = 0;                      /* :113 */
    }
    x->c[RAFT_C_LEADERS_ELECTED]++;
}

/* Snapshot of the RequestVote fields built inside retry{} (RaftServer.kt:200-207). */
static void build_vote_request(const ctx_t* x, onode_t* n) {
    n->reqTerm = n->currentTerm;
    n->reqLastIndex = n->log.lastIndex;                              /* :201 */
    if (n->log.lastIndex == 0) n->reqLastTerm = 0;                   /* :202 */
    else {
        entry_t e = { 0, 0 };
        olog_get(&n->log, n->log.lastIndex - 1, &e);
        olog_touch(&n->log, n->log.lastIndex - 1, x->c);
        n->reqLastTerm = e.term;
        x->c[RAFT_C_VOTE_LOG_READS]++;
    }
}

/* One iteration head of `while (state == CANDIDATE)` (RaftServer.kt:191-199). */
static void start_round(const ctx_t* x, onode_t* n) {
    n->currentTerm += 1;                           /* :192 */
    n->votedFor = n->id;                           /* :193 */
    n->votes = 0;                                  /* :194 */
    n->latch = 0;                                  /* :196 */
    n->backoff = 0;
    n->phaseMs = 0;
    n->retryMs = 0;
    n->pending = (1u << x->o->R) - 1u;             /* one retry{} per server :198-200 */
    n->sendMask = n->pending;
    build_vote_request(x, n);
    x->c[RAFT_C_ROUNDS]++;
}

/* leaderElection() returned; `launch { channel.send(state) }` (:225) is
 * received after the FOLLOWER sends queued meanwhile (S-5). */
static void end_election(const ctx_t* x, onode_t* n) {
    n->electing = 0;
    n->backoff = 0; n->phaseMs = 0; n->retryMs = 0;
    n->votes = 0; n->latch = 0; n->pending = 0;
    if (n->pendingReset) { n->pendingReset = 0; reset_timer(x, n); }
    if (n->state == RAFT_LEADER) start_session(x, n);        /* :66 */
    else if (n->state == RAFT_FOLLOWER) reset_timer(x, n);   /* :64 */
}

/* ------------------------------------------------------------------ */
/* the two RPC handlers                                                */
/* ------------------------------------------------------------------ */
/* override suspend fun vote(request) (RaftServer.kt:228-251) */
static void vote_handler(const ctx_t* x, onode_t* n, const raft_vote_req* rq, raft_vote_resp* rs) {
    int granted;
    if (x->o->p.mode == RAFT_MODE_TEXTBOOK) {
        /* textbook: a higher term is adopted whatever the answer (the reference
         * adopts it only on a grant, Q5); grant iff votedFor is free or the
         * candidate and the candidate's log is at least as up to date */
        if (rq->term > n->currentTerm) {
            n->currentTerm = rq->term;
            n->votedFor = -1;
            if (n->state != RAFT_FOLLOWER) { n->state = RAFT_FOLLOWER; send_follower(x, n); }
        }
        granted = 0;
        if (rq->term == n->currentTerm && (n->votedFor == -1 || n->votedFor == rq->candidate_id)) {
            entry_t last = { 0, 0 };
            if (n->log.lastIndex >= 1) {
                olog_get(&n->log, n->log.lastIndex - 1, &last);
                olog_touch(&n->log, n->log.lastIndex - 1, x->c);
                x->c[RAFT_C_VOTE_LOG_READS]++;
            }
            granted = !(n->log.lastIndex >= 1 && (rq->last_log_term < last.term ||
                        (rq->last_log_term == last.term && rq->last_log_index < n->log.lastIndex)));
            if (granted) {                         /* a grant re-arms the timer (:241); the self-vote changes nothing */
                n->votedFor = rq->candidate_id;
                if (rq->candidate_id != n->id) send_follower(x, n);
            }
        }
    } else if (rq->term < n->currentTerm) granted = 0;                       /* :229 */
    else if (n->currentTerm == rq->term) granted = (n->votedFor == rq->candidate_id); /* :230 */
    else {
        entry_t last = { 0, 0 };
        if (n->log.lastIndex >= 1) {
            olog_get(&n->log, n->log.lastIndex - 1, &last);
            olog_touch(&n->log, n->log.lastIndex - 1, x->c);
            x->c[RAFT_C_VOTE_LOG_READS]++;
        }
        if (n->log.lastIndex >= 1 && rq->last_log_term < last.term) granted = 0;          /* :232-233 */
        else if (n->log.lastIndex >= 1 && rq->last_log_term == last.term &&
                 rq->last_log_index < n->log.lastIndex) granted = 0;                      /* :234-236 */
        else {
            n->currentTerm = rq->term;             /* :238 */
            n->votedFor = rq->candidate_id;        /* :239 */
            n->state = RAFT_FOLLOWER;              /* :240 */
            send_follower(x, n);                   /* :241 */
            granted = 1;
        }
    }
    if (granted) x->c[RAFT_C_VOTES_GRANTED]++;
    rs->term = n->currentTerm;                     /* :246-249 */
    rs->vote_granted = granted;
}

/* override suspend fun append(request) (RaftServer.kt:253-287).
 * Returns 0, or 1 where the reference throws (Log index < -1).
 * more / nmore: textbook mode with ae_max_entries > 1 only -- the entries the
 * request carries after its first (log indices prev + 2 ..), applied in order
 * with the first one's rule while every earlier entry is in place. */
static int append_handler(const ctx_t* x, onode_t* n, const raft_append_req* rq, raft_append_resp* rs,
                          const entry_t* more, int32_t nmore) {
    const int tb = x->o->p.mode == RAFT_MODE_TEXTBOOK;
    if (tb && rq->term < n->currentTerm) {         /* textbook: a stale leader is refused, nothing changes */
        rs->term = n->currentTerm; rs->success = 0; rs->status = 0;
        return 0;
    }
    if (rq->term > n->currentTerm) {               /* :257-262 */
        n->currentTerm = rq->term;
        n->votedFor = -1;
        n->state = RAFT_FOLLOWER;
        send_follower(x, n);
    }
    if (rq->leader_id != n->id) {                  /* :264-268 (Q3: no term check) */
        n->state = RAFT_FOLLOWER;
        send_follower(x, n);
    }
    if (!tb && rq->leader_commit > n->commitIndex) {   /* :270-272 (Q4) */
        int32_t c = rq->leader_commit < n->log.lastIndex ? rq->leader_commit : n->log.lastIndex;
        if (c < n->commitIndex) x->c[RAFT_C_COMMIT_REGRESSIONS]++;
        n->commitIndex = c;
    }
    int success;                                   /* :274-276 */
    if (rq->prev_log_index == -1) success = 1;
    else if (n->log.lastIndex > rq->prev_log_index) {
        entry_t pe;
        if (!olog_get(&n->log, rq->prev_log_index, &pe)) {   /* index < -1: ArrayList throws */
            rs->term = n->currentTerm; rs->success = 0; rs->status = 1;
            return 1;
        }
        olog_touch(&n->log, rq->prev_log_index, x->c);
        x->c[RAFT_C_PREV_READS_FOLLOWER]++;
        success = (pe.term == rq->prev_log_term);
    } else success = 0;
    int stored = 0;                                /* the entry is in the log at prev + 1 */
    if (success && rq->has_entry) {                /* :278 (Q2, Q10) */
        entry_t e = { rq->entry_term, rq->entry_cmd }, cur;
        const int32_t i = rq->prev_log_index + 1;
        const int have = tb && i < n->log.lastIndex && olog_get(&n->log, i, &cur);
        if (have) olog_touch(&n->log, i, x->c);
        if (have && cur.term == e.term) {
            stored = 1;                            /* textbook: no conflict, no truncation */
        } else {
            int r = olog_add(&n->log, i, e, x->c);
            if (r == 1) { x->c[RAFT_C_ENTRY_WRITES]++; stored = 1; }
            else if (r == -1) x->c[RAFT_C_LOG_OVERFLOW]++;
        }
        for (int32_t k = 0; tb && stored == k + 1 && k < nmore; ++k) {   /* textbook: the further entries */
            const int32_t j = i + 1 + k;
            const int hv = j < n->log.lastIndex && olog_get(&n->log, j, &cur);
            if (hv) olog_touch(&n->log, j, x->c);
            if (hv && cur.term == more[k].term) { stored++; continue; }
            int r = olog_add(&n->log, j, more[k], x->c);
            if (r == 1) { x->c[RAFT_C_ENTRY_WRITES]++; stored++; }
            else if (r == -1) x->c[RAFT_C_LOG_OVERFLOW]++;
        }
    }
    if (tb && success && rq->leader_commit > n->commitIndex) {
        /* textbook: commitIndex = min(leaderCommit, index of the last new entry), never lowered */
        const int32_t lastNew = rq->prev_log_index + 1 + stored;
        const int32_t c = rq->leader_commit < lastNew ? rq->leader_commit : lastNew;
        if (c > n->commitIndex) n->commitIndex = c;
    }
    rs->term = n->currentTerm;                     /* :282-285 */
    rs->success = success;
    rs->status = 0;
    return 0;
}

/* appendCommand(command) (RaftServer.kt:100-107) */
static void append_command(const ctx_t* x, onode_t* n, uint32_t cmd) {
    entry_t e = { n->currentTerm, cmd };           /* :101-104 */
    int r = olog_add(&n->log, n->log.lastIndex, e, x->c);   /* :105 */
    x->c[RAFT_C_COMMANDS]++;
    if (r == -1) x->c[RAFT_C_LOG_OVERFLOW]++;
}

/* ------------------------------------------------------------------ */
/* one lockstep step of one group                     */
/* ------------------------------------------------------------------ */
static void group_step(const struct oracle* o, ogroup_t* g, uint32_t gid, uint32_t t, int64_t* c) {
    const raft_params* p = &o->p;
    const int32_t R = o->R, maj = o->majority, P = p->heartbeat_ms;
    const int tb = p->mode == RAFT_MODE_TEXTBOOK;
    ctx_t x = { o, t, gid, c, -1, 0 };

    /* ---- H: harness ---- */
    uint32_t hw[4];
    draw4(&x, t, RAFT_RNG_HARNESS, 0, hw);
    if (g->isoRem > 0) { g->isoRem--; if (g->isoRem == 0) g->isoRep = 0; }
    if (p->churn_ppm && p->churn_steps > 0 && g->isoRem == 0 && hit32(hw[0], p->churn_ppm)) {
        for (int r = 0; r < R; ++r)
            if (g->n[r].state == RAFT_LEADER) { g->isoRep = r; g->isoRem = p->churn_steps; break; }
    }
    if (g->isoRem > 0) x.isoRep = g->isoRep;
    if (p->partition_period > 0 && (int64_t)(t % (uint32_t)p->partition_period) < p->partition_len) {
        uint32_t pw[4];
        draw4(&x, t - t % (uint32_t)p->partition_period, RAFT_RNG_PARTITION, 0, pw);
        x.partMask = pw[0] & ((1u << R) - 1u);
    }

    /* ---- T: timers and the election loop's clocks ---- */
    for (int r = 0; r < R; ++r) {
        onode_t* n = &g->n[r];
        int started = 0;
        if (n->timerArmed) {
            n->electionMs -= P;
            if (n->electionMs <= 0) {              /* Timer fires: Commons.kt:25-27 -> RaftServer.kt:181-185 */
                n->timerArmed = 0; n->electionMs = 0;
                c[RAFT_C_TIMEOUTS]++;
                n->state = RAFT_CANDIDATE;         /* :182 */
                if (!n->electing) {                /* :184 offer(CANDIDATE) -> :65 leaderElection() */
                    n->electing = 1;
                    start_round(&x, n);
                    started = 1;
                }
            }
        }
        if (n->electing && !started) {
            if (!n->backoff) {
                n->phaseMs += P;                   /* countDownLatch.await(25 s) clock :214 */
                if (n->pending && n->phaseMs < p->round_timeout_ms) {
                    n->retryMs -= P;               /* delay(5000) inside retry{} Commons.kt:43 */
                    if (n->retryMs <= 0) {
                        build_vote_request(&x, n);
                        n->sendMask = n->pending;
                    }
                }
            } else {
                n->phaseMs -= P;                   /* delay(backoff) :221 */
                if (n->phaseMs <= 0) {
                    if (n->state == RAFT_CANDIDATE) start_round(&x, n);   /* while (state == CANDIDATE) :191 */
                    else end_election(&x, n);
                }
            }
        }
    }

    /* ---- V: RequestVote fan-out, senders ascending, dsts ascending (S-3) ---- */
    for (int s = 0; s < R; ++s) {
        onode_t* cand = &g->n[s];
        if (!cand->sendMask) continue;
        raft_vote_req rq = { cand->reqTerm, cand->id, cand->reqLastIndex, cand->reqLastTerm };
        int32_t hiT = 0;
        dropu_t u;
        if (p->drop_ppm) drop_uniforms(&x, RAFT_RNG_VOTE_DROP, s, &u);
        for (int d = 0; d < R; ++d) {
            if (!((cand->sendMask >> d) & 1u)) continue;
            if (lost(&x, &u, s, d, 0)) { c[RAFT_C_MSG_DROPPED]++; continue; }   /* retry{} swallows, Commons.kt:41 */
            raft_vote_resp rs;
            vote_handler(&x, &g->n[d], &rq, &rs);
            if (lost(&x, &u, s, d, 1)) { c[RAFT_C_MSG_DROPPED]++; continue; }
            cand->pending &= ~(1u << d);
            cand->latch++;                                          /* :209 countDown() */
            if (cand->currentTerm < rs.term) {
                cand->state = RAFT_FOLLOWER;                        /* :210 (Q6) */
                if (rs.term > hiT) hiT = rs.term;
            }
            if (rs.vote_granted) cand->votes++;                     /* :211 */
        }
        cand->sendMask = 0;
        if (cand->pending) cand->retryMs = p->retry_ms;
        if (tb && hiT > cand->currentTerm) {       /* textbook: adopt the highest response term once the */
            cand->currentTerm = hiT;               /* round's responses are in (the reference keeps it, Q6) */
            cand->votedFor = -1;
        }
    }

    /* ---- D: latch closes -> decision (RaftServer.kt:214-222) ---- */
    for (int r = 0; r < R; ++r) {
        onode_t* n = &g->n[r];
        if (!n->electing || n->backoff) continue;
        if (n->latch < maj && n->phaseMs < p->round_timeout_ms) continue;
        n->pending = 0;                            /* cancelChildren() :215 */
        if (n->state == RAFT_CANDIDATE && n->votes >= maj) {    /* :218-219 */
            n->state = RAFT_LEADER;
            end_election(&x, n);
        } else if (n->state == RAFT_CANDIDATE) {   /* :220-221 */
            n->backoff = 1;
            n->phaseMs = draw_range(&x, t, RAFT_RNG_TIMER, r, p->backoff_min_ms, p->backoff_max_ms);   /* S-9: the replica's timer word */
            n->retryMs = 0; n->votes = 0; n->latch = 0;
        } else {
            end_election(&x, n);
        }
    }

    /* ---- A: leader ticks, senders ascending, dsts ascending (S-3, S-4) ---- */
    for (int s = 0; s < R; ++s) {
        onode_t* L = &g->n[s];
        if (!L->hbActive) continue;
        if (L->state == RAFT_FOLLOWER) { L->hbActive = 0; continue; }   /* :117 (S-10) */
        c[RAFT_C_SESSIONS_TICKED]++;
        raft_append_req rq[MAXR];
        int ok[MAXR];
        entry_t more[MAXR][RAFT_MAX_AE_ENTRIES];   /* textbook: entries after the first */
        int32_t nent[MAXR];                         /* entries each request carries */
        const int32_t E = tb && p->ae_max_entries > 1 ? p->ae_max_entries : 1;
        for (int d = 0; d < R; ++d) {              /* build every request first :122-132 */
            int32_t i = L->nextIndex[d];           /* :126 */
            int32_t prev = i - 2;                  /* :127 */
            int32_t prevTerm = -1;
            entry_t pe, ent = { 0, 0 };
            ok[d] = 1;
            if (prev >= 0) {                       /* :128 */
                if (!olog_get(&L->log, prev, &pe)) ok[d] = 0;       /* Q11: throws, caught :170 */
                else { prevTerm = pe.term; c[RAFT_C_PREV_READS_LEADER]++; olog_touch(&L->log, prev, c); }
            }
            int has = 0;
            nent[d] = 0;
            if (ok[d] && L->log.lastIndex >= L->nextIndex[d]) {     /* :130 */
                if (!olog_get(&L->log, i - 1, &ent)) ok[d] = 0;     /* :131 */
                else { has = 1; nent[d] = 1; c[RAFT_C_ENTRY_READS_LEADER]++; olog_touch(&L->log, i - 1, c); }
                /* textbook, ae_max_entries > 1: up to E entries, i - 1 .. */
                for (int32_t k = 1; has && k < E && i - 1 + k < L->log.lastIndex; ++k) {
                    if (!olog_get(&L->log, i - 1 + k, &more[d][k - 1])) break;
                    c[RAFT_C_ENTRY_READS_LEADER]++;
                    olog_touch(&L->log, i - 1 + k, c);
                    nent[d]++;
                }
            }
            if (!ok[d]) { c[RAFT_C_APPEND_SKIPPED]++; continue; }
            rq[d].term = L->currentTerm;           /* :137-143 */
            rq[d].leader_id = L->id;
            rq[d].prev_log_index = prev;
            rq[d].prev_log_term = prevTerm;
            rq[d].has_entry = has;
            rq[d].entry_term = ent.term;
            rq[d].entry_cmd = ent.cmd;
            rq[d].leader_commit = L->commitIndex;
        }
        dropu_t u;
        if (p->drop_ppm) drop_uniforms(&x, RAFT_RNG_APPEND_DROP, s, &u);
        int stepped = 0;
        int32_t T = L->currentTerm;                /* textbook: the running response term */
        for (int d = 0; d < R; ++d) {
            if (!ok[d]) continue;
            c[RAFT_C_APPEND_SENT]++;
            if (lost(&x, &u, s, d, 0)) { c[RAFT_C_MSG_DROPPED]++; continue; }   /* swallowed :170-172 */
            raft_append_resp rs;
            if (append_handler(&x, &g->n[d], &rq[d], &rs, more[d], nent[d] - 1)) continue;
            if (lost(&x, &u, s, d, 1)) { c[RAFT_C_MSG_DROPPED]++; continue; }
            if (tb && rs.term > T) {               /* textbook: adopted after the tick's responses */
                T = rs.term;
                stepped = 1;
                continue;
            }
            if (!tb && rs.term > L->currentTerm) { /* :146-154 (Q7: votedFor kept) */
                L->currentTerm = rs.term;
                L->state = RAFT_FOLLOWER;
                stepped = 1;
                offer_follower(&x, L);
                continue;                          /* return@launch: only this coroutine */
            }
            if (rs.success) {                      /* :156-165 (Q9) */
                if (rq[d].has_entry && tb) {       /* textbook: matchIndex = the last acked entry's index */
                    L->nextIndex[d] += nent[d];
                    L->matchIndex[d] = rq[d].prev_log_index + 1 + nent[d];
                    c[RAFT_C_ENTRIES_ACKED] += nent[d];
                } else if (rq[d].has_entry) {
                    L->nextIndex[d] += 1;
                    L->matchIndex[d] += 1;
                    c[RAFT_C_ENTRIES_ACKED]++;
                    int cnt = 0;
                    for (int k = 0; k < R; ++k) cnt += L->matchIndex[k] > L->commitIndex;   /* :161 */
                    if (cnt >= maj) { L->commitIndex += 1; c[RAFT_C_COMMITS]++; }           /* :162 */
                } else {
                    L->matchIndex[d] = rq[d].prev_log_index + 1;   /* :164 */
                }
            } else {
                L->nextIndex[d] -= 1;              /* :167 */
            }
        }
        if (tb && stepped) {                       /* the higher term, FOLLOWER, a new term's empty vote */
            L->currentTerm = T;
            L->state = RAFT_FOLLOWER;
            L->votedFor = -1;
            offer_follower(&x, L);
        }
        if (tb && !stepped) {
            /* textbook commit rule: N = the majority-th largest matchIndex (the
             * median of the session row); commit up to N iff log[N-1] is of the
             * leader's current term.  COMMITS counts the ticks that advanced. */
            int32_t m[MAXR];
            for (int k = 0; k < R; ++k) m[k] = L->matchIndex[k];
            for (int a = 1; a < R; ++a)            /* insertion sort, descending */
                for (int b = a; b > 0 && m[b] > m[b - 1]; --b) { int32_t v = m[b]; m[b] = m[b - 1]; m[b - 1] = v; }
            const int32_t N = m[maj - 1];
            entry_t ne;
            const int got = N > L->commitIndex && olog_get(&L->log, N - 1, &ne);
            if (got) olog_touch(&L->log, N - 1, c);
            if (got && ne.term == L->currentTerm) {
                L->commitIndex = N;
                c[RAFT_C_COMMITS]++;
            }
        }
    }

    /* ---- C: client commands (harness -> appendCommand, S-11) ---- */
    if (p->cmd_ppm && (p->cmd_limit == 0 || g->cmdCount < p->cmd_limit) && hit32(hw[1], p->cmd_ppm)) {
        int any = 0;
        for (int r = 0; r < R; ++r) {
            if (g->n[r].state != RAFT_LEADER) continue;
            append_command(&x, &g->n[r], hw[2]);
            any = 1;
            if (p->cmd_mode == RAFT_CMD_LOWEST_LEADER) break;
        }
        if (any) g->cmdCount++;
    }

    /* ---- K: end-of-step observations ---- */
    int leaders = 0, dual = 0;
    for (int r = 0; r < R; ++r) {
        if (g->n[r].state != RAFT_LEADER) continue;
        leaders++;
        for (int q = r + 1; q < R; ++q)
            if (g->n[q].state == RAFT_LEADER && g->n[q].currentTerm == g->n[r].currentTerm) dual = 1;
    }
    c[RAFT_C_LEADERS] += leaders;
    if (leaders) c[RAFT_C_GROUPS_WITH_LEADER]++;
    if (dual) c[RAFT_C_DUAL_LEADER_GROUPS]++;
}

/* ------------------------------------------------------------------ */
/* lifecycle                                                           */
/* ------------------------------------------------------------------ */
static void init_group(const struct oracle* o, ogroup_t* g, uint32_t gid) {
    memset(g, 0, sizeof(*g));
    ctx_t x = { o, RAFT_RNG_INIT_STEP, gid, NULL, -1, 0 };
    for (int r = 0; r < o->R; ++r) {
        onode_t* n = &g->n[r];
        n->id = r + 1;
        n->votedFor = -1;                          /* :39 */
        n->state = RAFT_FOLLOWER;                  /* :42 */
        n->log.cap = o->p.log_cap;
        n->log.textbook = o->p.mode == RAFT_MODE_TEXTBOOK;
        n->log.window = o->p.log_window;
        reset_timer(&x, n);                        /* init: ResettableCountdownTimer(...) starts (:58, Commons.kt:14) */
    }
}

int oracle_create(const raft_params* p, oracle_t** out) {
    if (!p || !out || p->R < 1 || p->R > MAXR || p->G < 1 || p->log_cap < 1 || p->heartbeat_ms <= 0 ||
        p->election_min_ms > p->election_max_ms || p->backoff_min_ms > p->backoff_max_ms ||
        (p->mode != RAFT_MODE_REFERENCE && p->mode != RAFT_MODE_TEXTBOOK) || p->log_window < 0 ||
        (p->log_window && ((p->log_window & (p->log_window - 1)) || p->log_window > p->log_cap)) ||
        p->ae_max_entries < 0 || p->ae_max_entries > RAFT_MAX_AE_ENTRIES ||
        (p->mode != RAFT_MODE_TEXTBOOK && p->ae_max_entries > 1))
        return RAFT_EINVAL;
    oracle_t* o = (oracle_t*)calloc(1, sizeof(*o));
    if (!o) return RAFT_ENOMEM;
    o->p = *p;
    o->R = p->R;
    o->majority = p->R / 2 + 1;                    /* RaftServer.kt:44 */
    o->key[0] = (uint32_t)p->seed;
    o->key[1] = (uint32_t)(p->seed >> 32);
    o->G = p->G;
    o->groups = (ogroup_t*)calloc((size_t)p->G, sizeof(ogroup_t));
    if (!o->groups) { free(o); return RAFT_ENOMEM; }
    for (int64_t g = 0; g < p->G; ++g) init_group(o, &o->groups[g], (uint32_t)(p->g0 + g));
    *out = o;
    return RAFT_OK;
}

void oracle_destroy(oracle_t* o) {
    if (!o) return;
    for (int64_t g = 0; g < o->G; ++g)
        for (int r = 0; r < o->R; ++r) free(o->groups[g].n[r].log.items);
    free(o->groups);
    free(o);
}

typedef struct {
    oracle_t* o; int64_t g_begin, g_end; int32_t n_steps; int64_t* counters;
} job_t;

static void* run_job(void* arg) {
    job_t* j = (job_t*)arg;
    for (int64_t g = j->g_begin; g < j->g_end; ++g) {
        for (int32_t k = 0; k < j->n_steps; ++k)
            group_step(j->o, &j->o->groups[g], (uint32_t)(j->o->p.g0 + g), j->o->t + (uint32_t)k,
                       j->counters + (size_t)k * RAFT_COUNTER_STRIDE);
    }
    return NULL;
}

int oracle_step(oracle_t* o, int32_t n_steps, int64_t* counters, int32_t nthreads) {
    if (!o || n_steps < 0) return RAFT_EINVAL;
    if (n_steps == 0) return RAFT_OK;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > o->G) nthreads = (int32_t)o->G;
    size_t cn = (size_t)n_steps * RAFT_COUNTER_STRIDE;
    int64_t* scratch = (int64_t*)calloc(cn * (size_t)nthreads, sizeof(int64_t));
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!scratch || !jobs || !th) { free(scratch); free(jobs); free(th); return RAFT_ENOMEM; }
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].o = o;
        jobs[i].g_begin = o->G * i / nthreads;
        jobs[i].g_end = o->G * (i + 1) / nthreads;
        jobs[i].n_steps = n_steps;
        jobs[i].counters = scratch + cn * (size_t)i;
        if (nthreads == 1) run_job(&jobs[i]);
        else pthread_create(&th[i], NULL, run_job, &jobs[i]);
    }
    if (nthreads > 1)
        for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    if (counters) {
        memset(counters, 0, cn * sizeof(int64_t));
        for (int i = 0; i < nthreads; ++i)
            for (size_t k = 0; k < cn; ++k) counters[k] += scratch[cn * (size_t)i + k];
    }
    o->t += (uint32_t)n_steps;
    free(scratch); free(jobs); free(th);
    return RAFT_OK;
}

int64_t oracle_step_index(const oracle_t* o) { return o ? (int64_t)o->t : -1; }
int oracle_set_step_index(oracle_t* o, int64_t t) {
    if (!o || t < 0 || t > (int64_t)0xFFFFFFFFll) return RAFT_EINVAL;
    o->t = (uint32_t)t;
    return RAFT_OK;
}

/* ------------------------------------------------------------------ */
/* canonical state export / import (include/raft_engine.h)             */
/* ------------------------------------------------------------------ */
static uint32_t node_flags(const onode_t* n) {
    return (n->timerArmed ? RAFT_FL_ARMED : 0u) | (n->electing ? RAFT_FL_ELECTING : 0u) |
           (n->pendingReset ? RAFT_FL_PENDING_RST : 0u) | (n->hbActive ? RAFT_FL_HB_ACTIVE : 0u) |
           (n->backoff ? RAFT_FL_BACKOFF : 0u) | ((n->pending & 0xFFu) << RAFT_FL_PENDING_SHIFT) |
           (((uint32_t)n->votes & 0xFu) << RAFT_FL_VOTES_SHIFT) |
           (((uint32_t)n->latch & 0xFu) << RAFT_FL_LATCH_SHIFT);
}

static void export_group(const oracle_t* o, const ogroup_t* g, int32_t* w) {
    const int R = o->R;
    for (int r = 0; r < R; ++r) {
        const onode_t* n = &g->n[r];
        int32_t* f = w + r * RAFT_NUM_FIELDS;
        f[RAFT_F_TERM] = n->currentTerm;
        f[RAFT_F_VOTED] = n->votedFor;
        f[RAFT_F_ROLE] = n->state;
        f[RAFT_F_COMMIT] = n->commitIndex;
        f[RAFT_F_LAST] = n->log.lastIndex;
        f[RAFT_F_PHYS] = n->log.size;
        f[RAFT_F_ELECTION_MS] = n->electionMs;
        f[RAFT_F_FLAGS] = (int32_t)node_flags(n);
        f[RAFT_F_PHASE_MS] = n->phaseMs;
        f[RAFT_F_RETRY_MS] = n->retryMs;
        for (int d = 0; d < R; ++d) {
            w[R * RAFT_NUM_FIELDS + r * R + d] = n->nextIndex[d];
            w[R * RAFT_NUM_FIELDS + R * R + r * R + d] = n->matchIndex[d];
        }
    }
    int32_t* ex = w + R * RAFT_NUM_FIELDS + 2 * R * R;
    ex[0] = g->isoRem > 0 ? (g->isoRem << 8) | g->isoRep : 0;
    ex[1] = g->cmdCount;
}

static void import_group(const oracle_t* o, ogroup_t* g, const int32_t* w) {
    const int R = o->R;
    for (int r = 0; r < R; ++r) {
        onode_t* n = &g->n[r];
        const int32_t* f = w + r * RAFT_NUM_FIELDS;
        uint32_t fl = (uint32_t)f[RAFT_F_FLAGS];
        n->currentTerm = f[RAFT_F_TERM];
        n->votedFor = f[RAFT_F_VOTED];
        n->state = f[RAFT_F_ROLE];
        n->commitIndex = f[RAFT_F_COMMIT];
        int32_t phys = f[RAFT_F_PHYS];
        if (phys > n->log.cap) phys = n->log.cap;
        if (phys < 0) phys = 0;
        olog_reserve(&n->log, phys > 0 ? phys : 1);
        for (int32_t j = n->log.size; j < phys; ++j) { n->log.items[j].term = 0; n->log.items[j].cmd = 0; }
        n->log.size = phys;
        n->log.lastIndex = f[RAFT_F_LAST];
        n->electionMs = f[RAFT_F_ELECTION_MS];
        n->timerArmed = (fl & RAFT_FL_ARMED) != 0;
        n->electing = (fl & RAFT_FL_ELECTING) != 0;
        n->pendingReset = (fl & RAFT_FL_PENDING_RST) != 0;
        n->hbActive = (fl & RAFT_FL_HB_ACTIVE) != 0;
        n->backoff = (fl & RAFT_FL_BACKOFF) != 0;
        n->pending = (fl >> RAFT_FL_PENDING_SHIFT) & 0xFFu;
        n->votes = (int32_t)((fl >> RAFT_FL_VOTES_SHIFT) & 0xFu);
        n->latch = (int32_t)((fl >> RAFT_FL_LATCH_SHIFT) & 0xFu);
        n->phaseMs = f[RAFT_F_PHASE_MS];
        n->retryMs = f[RAFT_F_RETRY_MS];
        n->sendMask = 0;
        for (int d = 0; d < R; ++d) {
            n->nextIndex[d] = w[R * RAFT_NUM_FIELDS + r * R + d];
            n->matchIndex[d] = w[R * RAFT_NUM_FIELDS + R * R + r * R + d];
        }
    }
    const int32_t* ex = w + R * RAFT_NUM_FIELDS + 2 * R * R;
    g->isoRem = ex[0] >> 8;
    g->isoRep = g->isoRem > 0 ? (ex[0] & 0xFF) : 0;
    g->cmdCount = ex[1];
}

static int range_ok(const oracle_t* o, int64_t g0, int64_t n) {
    return o && g0 >= 0 && n >= 0 && g0 + n <= o->G;
}

int oracle_read_state(const oracle_t* o, int64_t g0, int64_t n, int32_t* out) {
    if (!range_ok(o, g0, n) || !out) return RAFT_ERANGE;
    const int32_t W = raft_group_words(o->R);
    for (int64_t i = 0; i < n; ++i) export_group(o, &o->groups[g0 + i], out + (size_t)i * W);
    return RAFT_OK;
}

int oracle_write_state(oracle_t* o, int64_t g0, int64_t n, const int32_t* in) {
    if (!range_ok(o, g0, n) || !in) return RAFT_ERANGE;
    const int32_t W = raft_group_words(o->R);
    for (int64_t i = 0; i < n; ++i)       /* invariant 0 <= lastIndex <= physLen <= log_cap */
        for (int r = 0; r < o->R; ++r) {
            const int32_t* f = in + (size_t)i * W + r * RAFT_NUM_FIELDS;
            if (f[RAFT_F_LAST] < 0 || f[RAFT_F_LAST] > f[RAFT_F_PHYS] || f[RAFT_F_PHYS] > o->p.log_cap) return RAFT_EINVAL;
        }
    for (int64_t i = 0; i < n; ++i) import_group(o, &o->groups[g0 + i], in + (size_t)i * W);
    return RAFT_OK;
}

int oracle_read_log(const oracle_t* o, int64_t g0, int64_t n, int32_t* terms, uint32_t* cmds) {
    if (!range_ok(o, g0, n) || !terms || !cmds) return RAFT_ERANGE;
    const int64_t cap = o->p.log_cap;
    for (int64_t i = 0; i < n; ++i)
        for (int r = 0; r < o->R; ++r) {
            const olog_t* l = &o->groups[g0 + i].n[r].log;
            size_t base = ((size_t)i * o->R + r) * (size_t)cap;
            const int64_t lo = l->window && l->size > l->window ? l->size - l->window : 0;
            for (int64_t j = 0; j < cap; ++j) {       /* the retained window only, like the engine */
                const int in = j >= lo && j < l->size;
                terms[base + j] = in ? l->items[j].term : 0;
                cmds[base + j] = in ? l->items[j].cmd : 0;
            }
        }
    return RAFT_OK;
}

int oracle_write_log(oracle_t* o, int64_t g0, int64_t n, const int32_t* terms, const uint32_t* cmds) {
    if (!range_ok(o, g0, n) || !terms || !cmds) return RAFT_ERANGE;
    const int64_t cap = o->p.log_cap;
    for (int64_t i = 0; i < n; ++i)
        for (int r = 0; r < o->R; ++r) {
            olog_t* l = &o->groups[g0 + i].n[r].log;
            size_t base = ((size_t)i * o->R + r) * (size_t)cap;
            const int32_t lo = l->window && l->size > l->window ? l->size - l->window : 0;
            for (int32_t j = 0; j < l->size; ++j) {   /* below the window: 0, as the engine reads it */
                l->items[j].term = j >= lo ? terms[base + j] : 0;
                l->items[j].cmd = j >= lo ? cmds[base + j] : 0;
            }
        }
    return RAFT_OK;
}

/* ------------------------------------------------------------------ */
/* digest                                            */
/* ------------------------------------------------------------------ */
static uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}
#define FEED(h, v) do { (h) ^= (uint32_t)(v); (h) *= 0x100000001b3ull; } while (0)

uint64_t oracle_digest(const oracle_t* o) { return oracle_digest_range(o, 0, o->G); }

/* Change the log_window every replica's log is viewed through (digest,
 * read_log, miss counting); the lists themselves always hold every slot. */
int oracle_set_log_window(oracle_t* o, int32_t w) {
    if (!o || w < 0 || (w & (w - 1)) || w > o->p.log_cap) return RAFT_EINVAL;
    o->p.log_window = w;
    for (int64_t g = 0; g < o->G; ++g)
        for (int r = 0; r < o->R; ++r) o->groups[g].n[r].log.window = w;
    return RAFT_OK;
}

uint64_t oracle_digest_range(const oracle_t* o, int64_t g0, int64_t n) {
    const int R = o->R;
    const int32_t W = raft_group_words(R);
    int32_t* w = (int32_t*)malloc((size_t)W * sizeof(int32_t));
    uint64_t total = 0;
    if (g0 < 0) g0 = 0;
    if (g0 + n > o->G) n = o->G - g0;
    for (int64_t g = g0; g < g0 + n; ++g) {
        const ogroup_t* gr = &o->groups[g];
        export_group(o, gr, w);
        uint64_t gid = (uint64_t)(o->p.g0 + g);
        uint64_t h = 0xcbf29ce484222325ull ^ (gid * 0x9E3779B97F4A7C15ull);
        for (int r = 0; r < R; ++r) {
            for (int f = 0; f < RAFT_NUM_FIELDS; ++f) FEED(h, w[r * RAFT_NUM_FIELDS + f]);
            for (int d = 0; d < R; ++d) FEED(h, w[R * RAFT_NUM_FIELDS + r * R + d]);
            for (int d = 0; d < R; ++d) FEED(h, w[R * RAFT_NUM_FIELDS + R * R + r * R + d]);
            const olog_t* l = &gr->n[r].log;
            const int32_t lo = l->window && l->size > l->window ? l->size - l->window : 0;
            for (int32_t j = lo; j < l->size; ++j) { FEED(h, l->items[j].term); FEED(h, l->items[j].cmd); }
        }
        FEED(h, w[W - 2]);
        FEED(h, w[W - 1]);
        total += fmix64(h);
    }
    free(w);
    return total;
}

/* ------------------------------------------------------------------ */
/* single handlers (the service boundary)                              */
/* ------------------------------------------------------------------ */
static int64_t g_scratch_counters[RAFT_COUNTER_STRIDE];

int oracle_vote(oracle_t* o, int64_t group, int32_t dst, const raft_vote_req* req, raft_vote_resp* resp) {
    if (!o || group < 0 || group >= o->G || dst < 0 || dst >= o->R || !req || !resp) return RAFT_EINVAL;
    ctx_t x = { o, o->t, (uint32_t)(o->p.g0 + group), g_scratch_counters, -1, 0 };
    vote_handler(&x, &o->groups[group].n[dst], req, resp);
    return RAFT_OK;
}

int oracle_append(oracle_t* o, int64_t group, int32_t dst, const raft_append_req* req, raft_append_resp* resp) {
    if (!o || group < 0 || group >= o->G || dst < 0 || dst >= o->R || !req || !resp) return RAFT_EINVAL;
    ctx_t x = { o, o->t, (uint32_t)(o->p.g0 + group), g_scratch_counters, -1, 0 };
    append_handler(&x, &o->groups[group].n[dst], req, resp, NULL, 0);
    return RAFT_OK;
}

int oracle_append_command(oracle_t* o, int64_t group, int32_t replica, uint32_t cmd) {
    if (!o || group < 0 || group >= o->G || replica < 0 || replica >= o->R) return RAFT_EINVAL;
    ctx_t x = { o, o->t, (uint32_t)(o->p.g0 + group), g_scratch_counters, -1, 0 };
    append_command(&x, &o->groups[group].n[replica], cmd);
    return RAFT_OK;
}

/* ------------------------------------------------------------------ */
/* standalone Log for K1                                               */
/* ------------------------------------------------------------------ */
struct oracle_log { olog_t l; };

oracle_log_t* oracle_log_new(int32_t cap) {
    oracle_log_t* x = (oracle_log_t*)calloc(1, sizeof(*x));
    if (x) x->l.cap = cap;
    return x;
}
void oracle_log_free(oracle_log_t* x) { if (x) { free(x->l.items); free(x); } }
int32_t oracle_log_add(oracle_log_t* x, int32_t i, int32_t term, uint32_t cmd) {
    entry_t e = { term, cmd };
    return olog_add(&x->l, i, e, NULL);
}
int32_t oracle_log_get(const oracle_log_t* x, int32_t i, int32_t* term, uint32_t* cmd) {
    entry_t e;
    if (!olog_get(&x->l, i, &e)) return 0;
    *term = e.term; *cmd = e.cmd;
    return 1;
}
int32_t oracle_log_last_index(const oracle_log_t* x) { return x->l.lastIndex; }
int32_t oracle_log_size(const oracle_log_t* x) { return x->l.size; }
int32_t oracle_log_phys(const oracle_log_t* x, int32_t j, int32_t* term, uint32_t* cmd) {
    if (j < 0 || j >= x->l.size) return 0;
    *term = x->l.items[j].term; *cmd = x->l.items[j].cmd;
    return 1;
}

void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) { philox_ref(ctr, key, out); }
