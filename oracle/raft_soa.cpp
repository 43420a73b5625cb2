// raft_soa.cpp — CPU BASELINE ONLY (see raft_soa.h).  The lockstep step of
// oracle/raft_oracle.c in structure-of-arrays form, std::thread over groups.
//
// Every rule is the oracle's, which cites the reference line by line
// (RaftServer.kt, Commons.kt); the comments here name the step phase and the
// schedule rule instead of repeating them.  What differs is
// only the data layout: one array per field over all G*R replicas (the
// flag word packed exactly as the canonical export), the sessions as
// [G][R][R] rows, the logs as flat [G*R][log_cap] term and command arrays.
#include "raft_soa.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "philox_ref.h"

namespace {

constexpr uint32_t ARMED = RAFT_FL_ARMED, ELECTING = RAFT_FL_ELECTING, PRST = RAFT_FL_PENDING_RST,
                   HB = RAFT_FL_HB_ACTIVE, BACKOFF = RAFT_FL_BACKOFF;

uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

}  // namespace

struct soa {
    raft_params p;
    int32_t R, maj, cap;
    uint32_t key[2];
    int64_t G;
    uint32_t t;                                   // next step index
    // per replica, index g * R + r
    std::vector<int32_t> term, voted, role, commit, last, phys, elec, phase, retry;
    std::vector<uint32_t> fl;                     // RAFT_FL_* | pending << 8 | votes << 16 | latch << 20
    std::vector<int32_t> nx, mc;                  // session rows: [(g * R + s) * R + d]
    std::vector<int32_t> iso_rem, iso_rep, cmdc;  // per group (harness)
    std::vector<int32_t> lt;                      // logs: [(g * R + r) * cap + j]
    std::vector<uint32_t> lc;
};

namespace {

// One replica of the group being stepped: its scalars copied out of the
// arrays (registers), its log and session rows in place.
struct Node {
    int32_t id, term, voted, role, commit, last, phys, elec, phase, retry;
    bool armed, electing, prst, hb, backoff;
    uint32_t pending;
    int32_t votes, latch;
    int32_t* lt;
    uint32_t* lc;
    int32_t *nx, *mc;
    // the step's RequestVote snapshot (S-4), not state
    uint32_t send;
    int32_t qt, qli, qlt;
};

struct Step {
    const soa* s;
    uint32_t t, gid;
    int64_t* c;
    int32_t iso;        // isolated replica this step, -1 if none
    uint32_t part;      // replicas on side B of this step's partition
};

void draw4(const Step& x, uint32_t c0, uint32_t purpose, uint32_t sub, uint32_t w[4]) {
    const uint32_t ctr[4] = {c0, x.gid, purpose, sub};
    philox_ref(ctr, x.s->key, w);
}
int32_t draw_range(const Step& x, uint32_t c0, int32_t r, int32_t lo, int32_t hi) {
    uint32_t w[4];
    draw4(x, c0, RAFT_RNG_TIMER, (uint32_t)r >> 2, w);
    return lo + (int32_t)(((uint64_t)w[r & 3] * ((uint32_t)(hi - lo) + 1u)) >> 32);
}
bool hit32(uint32_t w, uint32_t ppm) { return (uint64_t)w * 1000000ull < ((uint64_t)ppm << 32); }
bool hit16(uint32_t u, uint32_t ppm) { return (uint64_t)u * 1000000ull < ((uint64_t)ppm << 16); }

struct Drops {
    uint32_t w[2][4];
};
void drop_words(const Step& x, uint32_t purpose, int32_t s, Drops& u) {
    const int32_t nj = 2 * (x.s->R - 1);
    for (int k = 0; k < 2; ++k)
        if (k * 8 < nj) draw4(x, x.t, purpose, (uint32_t)s | ((uint32_t)k << 8), u.w[k]);
}
bool lost(const Step& x, const Drops& u, int32_t s, int32_t d, int32_t b) {
    if (s == d) return false;
    if (x.iso >= 0 && (s == x.iso || d == x.iso)) return true;
    if (((x.part >> s) ^ (x.part >> d)) & 1u) return true;
    if (x.s->p.drop_ppm == 0) return false;
    const int32_t j = 2 * (d < s ? d : d - 1) + b;
    return hit16((u.w[j >> 3][(j & 7) >> 1] >> (16 * (j & 1))) & 0xFFFFu, x.s->p.drop_ppm);
}

// ---- Log<T> over a row: get / add (Q1 ghost tail; overflow counted) ----
bool log_get(const Node& n, int32_t i, int32_t& term, uint32_t& cmd) {
    if (n.last - 1 < i || i < 0 || i >= n.phys) return false;
    term = n.lt[i];
    cmd = n.lc[i];
    return true;
}
int log_add(Node& n, int32_t cap, int32_t i, int32_t term, uint32_t cmd) {
    if (n.last == i) {
        if (n.phys >= cap) return -1;
        n.last += 1;
        n.lt[n.phys] = term;
        n.lc[n.phys] = cmd;
        n.phys += 1;
        return 1;
    }
    if (n.last < i) return 0;
    if (i < 0) return -2;
    n.lt[i] = term;
    n.lc[i] = cmd;
    n.last = i + 1;
    return 1;
}

// ---- timer and consumer (S-5, S-6) ----
void reset_timer(const Step& x, Node& n) {
    n.armed = true;
    n.elec = draw_range(x, x.t, n.id - 1, x.s->p.election_min_ms, x.s->p.election_max_ms);
}
void send_follower(const Step& x, Node& n) {
    if (n.electing) n.prst = true;
    else reset_timer(x, n);
}
void start_session(const Step& x, Node& n) {
    n.hb = true;
    for (int d = 0; d < x.s->R; ++d) {
        n.nx[d] = n.commit + 1;
        n.mc[d] = 0;
    }
    x.c[RAFT_C_LEADERS_ELECTED]++;
}
void build_vote_request(const Step& x, Node& n) {
    n.qt = n.term;
    n.qli = n.last;
    n.qlt = 0;
    if (n.last != 0) {
        uint32_t cm;
        log_get(n, n.last - 1, n.qlt, cm);
        x.c[RAFT_C_VOTE_LOG_READS]++;
    }
}
void start_round(const Step& x, Node& n) {
    n.term += 1;
    n.voted = n.id;
    n.votes = n.latch = 0;
    n.backoff = false;
    n.phase = n.retry = 0;
    n.pending = (1u << x.s->R) - 1u;
    n.send = n.pending;
    build_vote_request(x, n);
    x.c[RAFT_C_ROUNDS]++;
}
void end_election(const Step& x, Node& n) {
    n.electing = n.backoff = false;
    n.phase = n.retry = n.votes = n.latch = 0;
    n.pending = 0;
    if (n.prst) {
        n.prst = false;
        reset_timer(x, n);
    }
    if (n.role == RAFT_LEADER) start_session(x, n);
    else if (n.role == RAFT_FOLLOWER) reset_timer(x, n);
}

// ---- the handlers (reference mode) ----
bool vote(const Step& x, Node& n, const raft_vote_req& q, int32_t& rterm) {
    bool granted;
    if (q.term < n.term) granted = false;
    else if (n.term == q.term) granted = n.voted == q.candidate_id;
    else {
        int32_t lterm = 0;
        if (n.last >= 1) {
            uint32_t cm;
            log_get(n, n.last - 1, lterm, cm);
            x.c[RAFT_C_VOTE_LOG_READS]++;
        }
        if (n.last >= 1 && q.last_log_term < lterm) granted = false;
        else if (n.last >= 1 && q.last_log_term == lterm && q.last_log_index < n.last) granted = false;
        else {
            n.term = q.term;
            n.voted = q.candidate_id;
            n.role = RAFT_FOLLOWER;
            send_follower(x, n);
            granted = true;
        }
    }
    if (granted) x.c[RAFT_C_VOTES_GRANTED]++;
    rterm = n.term;
    return granted;
}

// false where the reference throws (no response)
bool append(const Step& x, Node& n, const raft_append_req& q, int32_t& rterm, bool& success) {
    if (q.term > n.term) {
        n.term = q.term;
        n.voted = -1;
        n.role = RAFT_FOLLOWER;
        send_follower(x, n);
    }
    if (q.leader_id != n.id) {
        n.role = RAFT_FOLLOWER;
        send_follower(x, n);
    }
    if (q.leader_commit > n.commit) {
        const int32_t c = std::min(q.leader_commit, n.last);
        if (c < n.commit) x.c[RAFT_C_COMMIT_REGRESSIONS]++;
        n.commit = c;
    }
    if (q.prev_log_index == -1) success = true;
    else if (n.last > q.prev_log_index) {
        int32_t pt;
        uint32_t pc;
        if (!log_get(n, q.prev_log_index, pt, pc)) {
            rterm = n.term;
            success = false;
            return false;
        }
        x.c[RAFT_C_PREV_READS_FOLLOWER]++;
        success = pt == q.prev_log_term;
    } else success = false;
    if (success && q.has_entry) {
        const int r = log_add(n, x.s->cap, q.prev_log_index + 1, q.entry_term, q.entry_cmd);
        if (r == 1) x.c[RAFT_C_ENTRY_WRITES]++;
        else if (r == -1) x.c[RAFT_C_LOG_OVERFLOW]++;
    }
    rterm = n.term;
    return true;
}

// ---- one group, one step ----
void load(soa* s, int64_t g, Node* n) {
    const int R = s->R;
    for (int r = 0; r < R; ++r) {
        const int64_t i = g * R + r;
        Node& x = n[r];
        x.id = r + 1;
        x.term = s->term[i]; x.voted = s->voted[i]; x.role = s->role[i]; x.commit = s->commit[i];
        x.last = s->last[i]; x.phys = s->phys[i]; x.elec = s->elec[i]; x.phase = s->phase[i]; x.retry = s->retry[i];
        const uint32_t f = s->fl[i];
        x.armed = f & ARMED; x.electing = f & ELECTING; x.prst = f & PRST; x.hb = f & HB; x.backoff = f & BACKOFF;
        x.pending = (f >> RAFT_FL_PENDING_SHIFT) & 0xFFu;
        x.votes = (int32_t)((f >> RAFT_FL_VOTES_SHIFT) & 0xFu);
        x.latch = (int32_t)((f >> RAFT_FL_LATCH_SHIFT) & 0xFu);
        x.lt = &s->lt[(size_t)i * s->cap];
        x.lc = &s->lc[(size_t)i * s->cap];
        x.nx = &s->nx[(size_t)i * R];
        x.mc = &s->mc[(size_t)i * R];
        x.send = 0;
        x.qt = x.qli = x.qlt = 0;
    }
}

void store(soa* s, int64_t g, const Node* n) {
    const int R = s->R;
    for (int r = 0; r < R; ++r) {
        const int64_t i = g * R + r;
        const Node& x = n[r];
        s->term[i] = x.term; s->voted[i] = x.voted; s->role[i] = x.role; s->commit[i] = x.commit;
        s->last[i] = x.last; s->phys[i] = x.phys; s->elec[i] = x.elec; s->phase[i] = x.phase; s->retry[i] = x.retry;
        s->fl[i] = (x.armed ? ARMED : 0u) | (x.electing ? ELECTING : 0u) | (x.prst ? PRST : 0u) | (x.hb ? HB : 0u) |
                   (x.backoff ? BACKOFF : 0u) | ((x.pending & 0xFFu) << RAFT_FL_PENDING_SHIFT) |
                   (((uint32_t)x.votes & 0xFu) << RAFT_FL_VOTES_SHIFT) |
                   (((uint32_t)x.latch & 0xFu) << RAFT_FL_LATCH_SHIFT);
    }
}

void group_step(soa* s, int64_t g, uint32_t t, int64_t* c) {
    const raft_params& p = s->p;
    const int R = s->R, maj = s->maj, P = p.heartbeat_ms;
    Node n[RAFT_MAX_R];
    load(s, g, n);
    Step x{s, t, (uint32_t)(p.g0 + g), c, -1, 0};

    // ---- H: harness (S-11) ----
    uint32_t hw[4];
    draw4(x, t, RAFT_RNG_HARNESS, 0, hw);
    int32_t& rem = s->iso_rem[g];
    int32_t& rep = s->iso_rep[g];
    if (rem > 0 && --rem == 0) rep = 0;
    if (p.churn_ppm && p.churn_steps > 0 && rem == 0 && hit32(hw[0], p.churn_ppm))
        for (int r = 0; r < R; ++r)
            if (n[r].role == RAFT_LEADER) { rep = r; rem = p.churn_steps; break; }
    if (rem > 0) x.iso = rep;
    if (p.partition_period > 0 && (int64_t)(t % (uint32_t)p.partition_period) < p.partition_len) {
        uint32_t pw[4];
        draw4(x, t - t % (uint32_t)p.partition_period, RAFT_RNG_PARTITION, 0, pw);
        x.part = pw[0] & ((1u << R) - 1u);
    }

    // ---- T: timers and the election loop's clocks ----
    for (int r = 0; r < R; ++r) {
        Node& a = n[r];
        bool started = false;
        if (a.armed) {
            a.elec -= P;
            if (a.elec <= 0) {
                a.armed = false;
                a.elec = 0;
                c[RAFT_C_TIMEOUTS]++;
                a.role = RAFT_CANDIDATE;
                if (!a.electing) {
                    a.electing = true;
                    start_round(x, a);
                    started = true;
                }
            }
        }
        if (a.electing && !started) {
            if (!a.backoff) {
                a.phase += P;
                if (a.pending && a.phase < p.round_timeout_ms) {
                    a.retry -= P;
                    if (a.retry <= 0) {
                        build_vote_request(x, a);
                        a.send = a.pending;
                    }
                }
            } else {
                a.phase -= P;
                if (a.phase <= 0) {
                    if (a.role == RAFT_CANDIDATE) start_round(x, a);
                    else end_election(x, a);
                }
            }
        }
    }

    // ---- V: RequestVote fan-out (S-3) ----
    for (int si = 0; si < R; ++si) {
        Node& cand = n[si];
        if (!cand.send) continue;
        const raft_vote_req q{cand.qt, cand.id, cand.qli, cand.qlt};
        Drops u;
        if (p.drop_ppm) drop_words(x, RAFT_RNG_VOTE_DROP, si, u);
        for (int d = 0; d < R; ++d) {
            if (!((cand.send >> d) & 1u)) continue;
            if (lost(x, u, si, d, 0)) { c[RAFT_C_MSG_DROPPED]++; continue; }
            int32_t rt;
            const bool gr = vote(x, n[d], q, rt);
            if (lost(x, u, si, d, 1)) { c[RAFT_C_MSG_DROPPED]++; continue; }
            cand.pending &= ~(1u << d);
            cand.latch++;
            if (cand.term < rt) cand.role = RAFT_FOLLOWER;
            if (gr) cand.votes++;
        }
        cand.send = 0;
        if (cand.pending) cand.retry = p.retry_ms;
    }

    // ---- D: latch closes -> decision ----
    for (int r = 0; r < R; ++r) {
        Node& a = n[r];
        if (!a.electing || a.backoff) continue;
        if (a.latch < maj && a.phase < p.round_timeout_ms) continue;
        a.pending = 0;
        if (a.role == RAFT_CANDIDATE && a.votes >= maj) {
            a.role = RAFT_LEADER;
            end_election(x, a);
        } else if (a.role == RAFT_CANDIDATE) {
            a.backoff = true;
            a.phase = draw_range(x, t, r, p.backoff_min_ms, p.backoff_max_ms);
            a.retry = a.votes = a.latch = 0;
        } else {
            end_election(x, a);
        }
    }

    // ---- A: leader ticks (S-3, S-4, S-10) ----
    for (int si = 0; si < R; ++si) {
        Node& L = n[si];
        if (!L.hb) continue;
        if (L.role == RAFT_FOLLOWER) { L.hb = false; continue; }
        c[RAFT_C_SESSIONS_TICKED]++;
        raft_append_req rq[RAFT_MAX_R];
        bool ok[RAFT_MAX_R];
        for (int d = 0; d < R; ++d) {                    // every request from the tick-start snapshot
            const int32_t i = L.nx[d], prev = i - 2;
            int32_t pt = -1, et = 0;
            uint32_t pc, ec = 0;
            ok[d] = true;
            if (prev >= 0) {
                if (!log_get(L, prev, pt, pc)) ok[d] = false;
                else c[RAFT_C_PREV_READS_LEADER]++;
            }
            bool has = false;
            if (ok[d] && L.last >= L.nx[d]) {
                if (!log_get(L, i - 1, et, ec)) ok[d] = false;
                else { has = true; c[RAFT_C_ENTRY_READS_LEADER]++; }
            }
            if (!ok[d]) { c[RAFT_C_APPEND_SKIPPED]++; continue; }
            rq[d] = raft_append_req{L.term, L.id, prev, pt, has ? 1 : 0, et, ec, L.commit};
        }
        Drops u;
        if (p.drop_ppm) drop_words(x, RAFT_RNG_APPEND_DROP, si, u);
        for (int d = 0; d < R; ++d) {
            if (!ok[d]) continue;
            c[RAFT_C_APPEND_SENT]++;
            if (lost(x, u, si, d, 0)) { c[RAFT_C_MSG_DROPPED]++; continue; }
            int32_t rt;
            bool succ;
            if (!append(x, n[d], rq[d], rt, succ)) continue;
            if (lost(x, u, si, d, 1)) { c[RAFT_C_MSG_DROPPED]++; continue; }
            if (rt > L.term) {                          // Q7
                L.term = rt;
                L.role = RAFT_FOLLOWER;
                if (!L.electing) reset_timer(x, L);     // offer(FOLLOWER), S-6
                continue;
            }
            if (succ) {
                if (rq[d].has_entry) {                  // Q9
                    L.nx[d] += 1;
                    L.mc[d] += 1;
                    c[RAFT_C_ENTRIES_ACKED]++;
                    int cnt = 0;
                    for (int k = 0; k < R; ++k) cnt += L.mc[k] > L.commit;
                    if (cnt >= maj) { L.commit += 1; c[RAFT_C_COMMITS]++; }
                } else {
                    L.mc[d] = rq[d].prev_log_index + 1;
                }
            } else {
                L.nx[d] -= 1;
            }
        }
    }

    // ---- C: client commands (S-11) ----
    int32_t& cc = s->cmdc[g];
    if (p.cmd_ppm && (p.cmd_limit == 0 || cc < p.cmd_limit) && hit32(hw[1], p.cmd_ppm)) {
        bool any = false;
        for (int r = 0; r < R; ++r) {
            if (n[r].role != RAFT_LEADER) continue;
            const int a = log_add(n[r], s->cap, n[r].last, n[r].term, hw[2]);
            c[RAFT_C_COMMANDS]++;
            if (a == -1) c[RAFT_C_LOG_OVERFLOW]++;
            any = true;
            if (p.cmd_mode == RAFT_CMD_LOWEST_LEADER) break;
        }
        if (any) cc++;
    }

    // ---- K: end-of-step observations ----
    int leaders = 0;
    bool dual = false;
    for (int r = 0; r < R; ++r) {
        if (n[r].role != RAFT_LEADER) continue;
        leaders++;
        for (int q = r + 1; q < R; ++q)
            if (n[q].role == RAFT_LEADER && n[q].term == n[r].term) dual = true;
    }
    c[RAFT_C_LEADERS] += leaders;
    if (leaders) c[RAFT_C_GROUPS_WITH_LEADER]++;
    if (dual) c[RAFT_C_DUAL_LEADER_GROUPS]++;
    store(s, g, n);
}

void export_group(const soa* s, int64_t g, int32_t* w) {
    const int R = s->R;
    for (int r = 0; r < R; ++r) {
        const int64_t i = g * R + r;
        int32_t* f = w + r * RAFT_NUM_FIELDS;
        f[RAFT_F_TERM] = s->term[i]; f[RAFT_F_VOTED] = s->voted[i]; f[RAFT_F_ROLE] = s->role[i];
        f[RAFT_F_COMMIT] = s->commit[i]; f[RAFT_F_LAST] = s->last[i]; f[RAFT_F_PHYS] = s->phys[i];
        f[RAFT_F_ELECTION_MS] = s->elec[i]; f[RAFT_F_FLAGS] = (int32_t)s->fl[i];
        f[RAFT_F_PHASE_MS] = s->phase[i]; f[RAFT_F_RETRY_MS] = s->retry[i];
        for (int d = 0; d < R; ++d) {
            w[R * RAFT_NUM_FIELDS + r * R + d] = s->nx[(size_t)i * R + d];
            w[R * RAFT_NUM_FIELDS + R * R + r * R + d] = s->mc[(size_t)i * R + d];
        }
    }
    int32_t* ex = w + R * RAFT_NUM_FIELDS + 2 * R * R;
    ex[0] = s->iso_rem[g] > 0 ? (s->iso_rem[g] << 8) | s->iso_rep[g] : 0;
    ex[1] = s->cmdc[g];
}

void import_group(soa* s, int64_t g, const int32_t* w) {
    const int R = s->R;
    for (int r = 0; r < R; ++r) {
        const int64_t i = g * R + r;
        const int32_t* f = w + r * RAFT_NUM_FIELDS;
        s->term[i] = f[RAFT_F_TERM]; s->voted[i] = f[RAFT_F_VOTED]; s->role[i] = f[RAFT_F_ROLE];
        s->commit[i] = f[RAFT_F_COMMIT]; s->last[i] = f[RAFT_F_LAST]; s->phys[i] = f[RAFT_F_PHYS];
        s->elec[i] = f[RAFT_F_ELECTION_MS]; s->fl[i] = (uint32_t)f[RAFT_F_FLAGS];
        s->phase[i] = f[RAFT_F_PHASE_MS]; s->retry[i] = f[RAFT_F_RETRY_MS];
        for (int d = 0; d < R; ++d) {
            s->nx[(size_t)i * R + d] = w[R * RAFT_NUM_FIELDS + r * R + d];
            s->mc[(size_t)i * R + d] = w[R * RAFT_NUM_FIELDS + R * R + r * R + d];
        }
    }
    const int32_t* ex = w + R * RAFT_NUM_FIELDS + 2 * R * R;
    s->iso_rem[g] = ex[0] >> 8;
    s->iso_rep[g] = ex[0] & 0xFF;
    s->cmdc[g] = ex[1];
}

}  // namespace

extern "C" {

int soa_create(const raft_params* p, soa_t** out) {
    if (!p || !out || p->R < 1 || p->R > RAFT_MAX_R || p->G < 1 || p->log_cap < 1 || p->heartbeat_ms <= 0 ||
        p->election_min_ms > p->election_max_ms || p->backoff_min_ms > p->backoff_max_ms ||
        p->mode != RAFT_MODE_REFERENCE || p->log_window != 0)
        return RAFT_EINVAL;
    soa* s = new (std::nothrow) soa();
    if (!s) return RAFT_ENOMEM;
    try {
        s->p = *p;
        s->R = p->R;
        s->maj = p->R / 2 + 1;
        s->cap = p->log_cap;
        s->key[0] = (uint32_t)p->seed;
        s->key[1] = (uint32_t)(p->seed >> 32);
        s->G = p->G;
        s->t = 0;
        const size_t GR = (size_t)p->G * p->R;
        for (auto* v : {&s->term, &s->voted, &s->role, &s->commit, &s->last, &s->phys, &s->elec, &s->phase, &s->retry})
            v->assign(GR, 0);
        s->fl.assign(GR, ARMED);
        std::fill(s->voted.begin(), s->voted.end(), -1);
        s->nx.assign(GR * p->R, 0);
        s->mc.assign(GR * p->R, 0);
        s->iso_rem.assign(p->G, 0);
        s->iso_rep.assign(p->G, 0);
        s->cmdc.assign(p->G, 0);
        s->lt.assign(GR * (size_t)p->log_cap, 0);
        s->lc.assign(GR * (size_t)p->log_cap, 0);
    } catch (...) {
        delete s;
        return RAFT_ENOMEM;
    }
    for (int64_t g = 0; g < p->G; ++g) {              // the initial timers (RaftServer.kt:58, Commons.kt:14)
        Step x{s, RAFT_RNG_INIT_STEP, (uint32_t)(p->g0 + g), nullptr, -1, 0};
        for (int r = 0; r < p->R; ++r)
            s->elec[g * p->R + r] = draw_range(x, RAFT_RNG_INIT_STEP, r, p->election_min_ms, p->election_max_ms);
    }
    *out = s;
    return RAFT_OK;
}

void soa_destroy(soa_t* s) { delete s; }

int soa_step(soa_t* s, int32_t n_steps, int64_t* counters, int32_t nthreads) {
    if (!s || n_steps < 0) return RAFT_EINVAL;
    if (n_steps == 0) return RAFT_OK;
    nthreads = std::max(1, std::min<int32_t>(nthreads, (int32_t)std::min<int64_t>(s->G, 1 << 16)));
    const size_t cn = (size_t)n_steps * RAFT_COUNTER_STRIDE;
    std::vector<std::vector<int64_t>> part(nthreads, std::vector<int64_t>(cn, 0));
    auto run = [&](int k) {
        const int64_t g0 = s->G * k / nthreads, g1 = s->G * (k + 1) / nthreads;
        for (int64_t g = g0; g < g1; ++g)             // groups are independent: each runs all its steps
            for (int32_t q = 0; q < n_steps; ++q)
                group_step(s, g, s->t + (uint32_t)q, part[k].data() + (size_t)q * RAFT_COUNTER_STRIDE);
    };
    std::vector<std::thread> th;
    for (int k = 1; k < nthreads; ++k) th.emplace_back(run, k);
    run(0);
    for (auto& x : th) x.join();
    if (counters) {
        std::memset(counters, 0, cn * sizeof(int64_t));
        for (int k = 0; k < nthreads; ++k)
            for (size_t q = 0; q < cn; ++q) counters[q] += part[k][q];
    }
    s->t += (uint32_t)n_steps;
    return RAFT_OK;
}

int soa_read_state(const soa_t* s, int64_t g0, int64_t n, int32_t* out) {
    if (!s || g0 < 0 || n < 0 || g0 + n > s->G || !out) return RAFT_ERANGE;
    const int32_t W = raft_group_words(s->R);
    for (int64_t i = 0; i < n; ++i) export_group(s, g0 + i, out + (size_t)i * W);
    return RAFT_OK;
}

int soa_read_log(const soa_t* s, int64_t g0, int64_t n, int32_t* terms, uint32_t* cmds) {
    if (!s || g0 < 0 || n < 0 || g0 + n > s->G || !terms || !cmds) return RAFT_ERANGE;
    const size_t row = (size_t)s->cap;
    for (int64_t i = 0; i < n * s->R; ++i) {
        const size_t src = ((size_t)g0 * s->R + i) * row;
        const int32_t ph = s->phys[(size_t)g0 * s->R + i];
        for (size_t j = 0; j < row; ++j) {
            terms[i * row + j] = (int32_t)j < ph ? s->lt[src + j] : 0;
            cmds[i * row + j] = (int32_t)j < ph ? s->lc[src + j] : 0;
        }
    }
    return RAFT_OK;
}

int soa_write_state(soa_t* s, int64_t g0, int64_t n, const int32_t* in) {
    if (!s || g0 < 0 || n < 0 || g0 + n > s->G || !in) return RAFT_ERANGE;
    const int32_t W = raft_group_words(s->R);
    for (int64_t i = 0; i < n; ++i) import_group(s, g0 + i, in + (size_t)i * W);
    return RAFT_OK;
}

int soa_write_log(soa_t* s, int64_t g0, int64_t n, const int32_t* terms, const uint32_t* cmds) {
    if (!s || g0 < 0 || n < 0 || g0 + n > s->G || !terms || !cmds) return RAFT_ERANGE;
    const size_t cells = (size_t)n * s->R * s->cap, at = (size_t)g0 * s->R * s->cap;
    std::memcpy(s->lt.data() + at, terms, cells * sizeof(int32_t));
    std::memcpy(s->lc.data() + at, cmds, cells * sizeof(uint32_t));
    return RAFT_OK;
}

int soa_set_step_index(soa_t* s, int64_t t) {
    if (!s || t < 0 || t > 0xFFFFFFFFll) return RAFT_EINVAL;
    s->t = (uint32_t)t;
    return RAFT_OK;
}

uint64_t soa_digest(const soa_t* s) {
    const int R = s->R;
    const int32_t W = raft_group_words(R);
    std::vector<int32_t> w(W);
    uint64_t total = 0;
    for (int64_t g = 0; g < s->G; ++g) {
        export_group(s, g, w.data());
        uint64_t h = 0xcbf29ce484222325ull ^ ((uint64_t)(s->p.g0 + g) * 0x9E3779B97F4A7C15ull);
        auto feed = [&](int32_t v) { h ^= (uint32_t)v; h *= 0x100000001b3ull; };
        for (int r = 0; r < R; ++r) {
            for (int f = 0; f < RAFT_NUM_FIELDS; ++f) feed(w[r * RAFT_NUM_FIELDS + f]);
            for (int d = 0; d < R; ++d) feed(w[R * RAFT_NUM_FIELDS + r * R + d]);
            for (int d = 0; d < R; ++d) feed(w[R * RAFT_NUM_FIELDS + R * R + r * R + d]);
            const size_t i = (size_t)g * R + r;
            for (int32_t j = 0; j < s->phys[i]; ++j) {
                feed(s->lt[i * s->cap + j]);
                feed((int32_t)s->lc[i * s->cap + j]);
            }
        }
        feed(w[W - 2]);
        feed(w[W - 1]);
        total += fmix64(h);
    }
    return total;
}

}  // extern "C"
