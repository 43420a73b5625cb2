// raft_step.h — the per-node consensus step of arodionov/raft-kotlin as
// register-resident SIMT code for gfx950.
//
// One lane owns one Raft group: all R replicas' scalar state, the group's
// primary leader session (nextIndex/matchIndex of one leader) and the step's
// message temporaries live in VGPRs; replica loops are unrolled against the
// compile-time R, so the R x R request/response "message tensor" of a phase
// never exists in memory: a message is a handler call whose arguments are
// registers of the sender and whose effects land in registers of the
// receiver.  The logs (the reference's ArrayList, Commons.kt:51) stay in HBM
// and are touched only at the slots the handlers read or write.
//
// Leader ticks (phase A) iterate only the lane's *active* sessions (one, in
// steady state) with the leader index as a per-lane runtime value; the
// leader's scalars are picked with select chains and the destination loop
// stays unrolled.  Sessions other than the primary live in their canonical
// HBM rows and are swapped in when they tick (partitions, stale leaders).
//
// The phase order and every tie-break follow DESIGN.md §3 (the same schedule
// the CPU oracle in oracle/raft_oracle.c restates object by object).
#pragma once
#include <hip/hip_runtime.h>
#include "philox.h"
#include "../../include/raft_engine.h"

extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);

namespace raft {

constexpr int NC = RAFT_NUM_COUNTERS;
constexpr int NCW = (NC + 1) / 2;          // counters packed as 16-bit pairs per lane

// exported flag bits (include/raft_engine.h) and engine-internal ones
constexpr uint32_t FL_ARMED = RAFT_FL_ARMED;
constexpr uint32_t FL_ELECTING = RAFT_FL_ELECTING;
constexpr uint32_t FL_PRST = RAFT_FL_PENDING_RST;
constexpr uint32_t FL_HB = RAFT_FL_HB_ACTIVE;
constexpr uint32_t FL_BACKOFF = RAFT_FL_BACKOFF;
constexpr uint32_t FL_DRAW = 1u << 5;      // internal: timer re-armed this step, draw pending
constexpr uint32_t FL_EXPORT_MASK = ~FL_DRAW;
constexpr int PEND_SH = RAFT_FL_PENDING_SHIFT, VOTES_SH = RAFT_FL_VOTES_SHIFT, LATCH_SH = RAFT_FL_LATCH_SHIFT;

struct DevParams {
    uint2* log;                                // [G][R][cap] (term, cmd)
    int32_t* nx;                               // [R][R][G] session rows (canonical home)
    int32_t* mt;                               // [R][R][G]
    int64_t G, g0;
    int32_t R, cap;
    uint32_t key0, key1;
    int32_t P, emin, emax, bmin, bmax, round_to, retry;
    uint32_t drop_ppm, drop_thr16;             // hit16(u) == (u < drop_thr16)
    uint64_t churn_thr32, cmd_thr32;           // hit32(w) == (w < thr)
    int32_t churn_steps, part_period, part_len;
    int32_t cmd_mode, cmd_limit;
};

struct Entry { int32_t term; uint32_t cmd; };

// Per-lane step counters, two 16-bit counters per register (a lane's count in
// one step is far below 2^16 / 64, so a wave sum of a packed word cannot
// carry between halves).
struct Counters {
    uint32_t w[NCW];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < NCW; ++i) w[i] = 0;
    }
    __device__ __forceinline__ void add(int c, uint32_t v = 1) { w[c >> 1] += v << (16 * (c & 1)); }
};

__device__ __forceinline__ u32x4 draw(const DevParams& p, uint32_t c0, uint32_t gid, uint32_t purpose, uint32_t sub) {
    return philox4x32_10(c0, gid, purpose, sub, p.key0, p.key1);
}

// Per-(group, step) context.
struct Ctx {
    uint32_t t, gid;
    int64_t i;            // engine-local group index (lane)
    int32_t iso;          // isolated replica this step, -1 if none
    uint32_t part;        // replicas on side B of this step's partition
    uint2* lg;            // this group's log, [R][cap] entries (term, cmd)
    int cap;
    Counters* cnt;        // this lane's counters for the step
};

// One replica's scalar state, by reference into the owning lane's registers.
struct Rep {
    int32_t &term, &voted, &role, &commit, &last, &phys, &elec, &phase, &retry;
    uint32_t& fl;
    int32_t &t1, &t2;          // log-tail cache: term of log[last-1], log[last-2]
    uint32_t& c1;              //                 cmd  of log[last-1]
};

// Pick / replace element s of a register array for a per-lane runtime s,
// given as the one-hot mask 1 << s.  Written as masked OR / blend so the
// optimiser cannot turn it into a dynamically indexed load or store (which
// would demote the whole register array to scratch memory).
template <int R>
__device__ __forceinline__ uint32_t pick(const uint32_t (&a)[R], uint32_t onehot) {
    uint32_t v = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) v |= a[r] & (0u - ((onehot >> r) & 1u));
    return v;
}
template <int R>
__device__ __forceinline__ int32_t pick(const int32_t (&a)[R], uint32_t onehot) {
    int32_t v = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) v |= a[r] & -(int32_t)((onehot >> r) & 1u);
    return v;
}
template <int R>
__device__ __forceinline__ void place(int32_t (&a)[R], uint32_t onehot, int32_t v) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int32_t m = -(int32_t)((onehot >> r) & 1u);
        a[r] = (a[r] & ~m) | (v & m);
    }
}

// ---- timer / consumer (Commons.kt:10-31, RaftServer.kt:50-69) -------------
// reset(): re-arm with a fresh draw.  The draw is a pure function of
// (step, group, replica), so it is resolved once at the end of the step
// (resolve_timer_draws) no matter how many resets the step performed.
__device__ __forceinline__ void reset_timer(Rep n) { n.fl |= FL_ARMED | FL_DRAW; }
// launch { channel.send(FOLLOWER) } (RaftServer.kt:241, :261, :266), S-5
__device__ __forceinline__ void send_follower(Rep n) {
    if (n.fl & FL_ELECTING) n.fl |= FL_PRST; else reset_timer(n);
}

// ---- Log<T> (Commons.kt:47-74) over one replica's HBM slots ---------------
// The engine keeps a 2-deep tail cache per replica (t1 = log[last-1].term,
// t2 = log[last-2].term, c1 = log[last-1].cmd; derived state, never
// exported).  In steady state every read the handlers make (prev checks,
// the newest entry, vote last-terms) hits it; HBM is read only for older
// slots and when the ghost tail resurfaces a stale slot.
__device__ __forceinline__ int32_t term_at(const uint2* lr, int32_t last, int32_t t1, int32_t t2, int32_t j) {
    return j == last - 1 ? t1 : j == last - 2 ? t2 : (int32_t)lr[j].x;
}

// Log.add(i, e): 1 true, 0 false, -1 capacity overflow (counted), -2 threw
__device__ __forceinline__ int log_add(uint2* lr, int cap, Rep n, int32_t i, Entry e) {
    if (n.last == i) {                                 // :58-61 append at the PHYSICAL end (Q1)
        if (n.phys >= cap) return -1;
        lr[n.phys] = make_uint2((uint32_t)e.term, e.cmd);
        if (n.phys == n.last) {                        // no ghost: the new last entry is e
            n.t2 = n.t1; n.t1 = e.term; n.c1 = e.cmd;
        } else {                                       // ghost: stale slot log[last] resurfaces
            const uint2 gs = lr[n.last];
            n.t2 = n.t1; n.t1 = (int32_t)gs.x; n.c1 = gs.y;
        }
        n.phys += 1;
        n.last += 1;
        return 1;
    }
    if (n.last < i) return 0;                          // :62
    if (i < 0) return -2;
    lr[i] = make_uint2((uint32_t)e.term, e.cmd);       // :63-66 overwrite, no shrink
    // new last = i + 1; log[i-1] is unchanged
    n.t2 = i == 0 ? 0 : (i == n.last - 1 ? n.t2 : (int32_t)lr[i - 1].x);
    n.t1 = e.term;
    n.c1 = e.cmd;
    n.last = i + 1;
    return 1;
}

// ---- vote() (RaftServer.kt:228-251) ---------------------------------------
__device__ __forceinline__ void vote_handler(Rep n, const uint2* lr, int32_t rt, int32_t rc, int32_t rli,
                                             int32_t rlt, Counters& cnt, int32_t& resp_term, bool& granted) {
    granted = false;
    if (rt < n.term) {
    } else if (n.term == rt) {
        granted = n.voted == rc;
    } else {
        int32_t lt = 0;
        if (n.last >= 1) { lt = n.t1; cnt.add(RAFT_C_VOTE_LOG_READS); }
        if (n.last >= 1 && rlt < lt) {
        } else if (n.last >= 1 && rlt == lt && rli < n.last) {
        } else {
            n.term = rt; n.voted = rc; n.role = RAFT_FOLLOWER;
            send_follower(n);
            granted = true;
        }
    }
    if (granted) cnt.add(RAFT_C_VOTES_GRANTED);
    resp_term = n.term;
}

// ---- append() (RaftServer.kt:253-287); returns false where it throws -------
// dprev = term of this replica's log[prev], read by the caller ahead of time
// (valid whenever 0 <= prev < lastIndex, the only case it is used).
__device__ __forceinline__ bool append_handler(Rep n, int32_t id, uint2* lr, int cap, int32_t rt, int32_t rlead,
                                               int32_t prev, int32_t prevTerm, bool has, Entry e,
                                               int32_t lcommit, int32_t dprev, Counters& cnt, int32_t& resp_term,
                                               bool& success) {
    if (rt > n.term) {                                  // :257-262
        n.term = rt; n.voted = -1; n.role = RAFT_FOLLOWER;
        send_follower(n);
    }
    if (rlead != id) {                                  // :264-268 (Q3)
        n.role = RAFT_FOLLOWER;
        send_follower(n);
    }
    if (lcommit > n.commit) {                           // :270-272 (Q4)
        const int32_t c = min(lcommit, n.last);
        if (c < n.commit) cnt.add(RAFT_C_COMMIT_REGRESSIONS);
        n.commit = c;
    }
    if (prev == -1) success = true;                     // :274-276
    else if (n.last > prev) {
        if (prev < 0) { resp_term = n.term; success = false; return false; }
        cnt.add(RAFT_C_PREV_READS_FOLLOWER);
        success = dprev == prevTerm;
    } else success = false;
    if (success && has) {                               // :278 (Q2, Q10)
        const int r = log_add(lr, cap, n, prev + 1, e);
        if (r == 1) cnt.add(RAFT_C_ENTRY_WRITES);
        else if (r == -1) cnt.add(RAFT_C_LOG_OVERFLOW);
    }
    resp_term = n.term;
    return true;
}

// ---- appendCommand() (RaftServer.kt:100-107) ------------------------------
__device__ __forceinline__ void append_command(Rep n, uint2* lr, int cap, uint32_t cmd, Counters& cnt) {
    const int r = log_add(lr, cap, n, n.last, Entry{n.term, (uint32_t)cmd});
    cnt.add(RAFT_C_COMMANDS);
    if (r == -1) cnt.add(RAFT_C_LOG_OVERFLOW);
}

// ---------------------------------------------------------------------------
// The register-resident group.
// ---------------------------------------------------------------------------
template <int R>
struct Group {
    int32_t term[R], voted[R], role[R], commit[R], last[R], phys[R], elec[R], phase[R], retry[R];
    uint32_t fl[R];
    int32_t t1[R], t2[R];           // log-tail cache (terms of log[last-1], log[last-2])
    uint32_t c1[R];                 //                (cmd of log[last-1])
    int32_t s0;                     // owner of the primary session in registers, -1 none
    int32_t nx0[R], mc0[R];         // its nextIndex / matchIndex (RaftServer.kt:112-113)
    int32_t iso, cmdc;              // harness: isolation word, commands issued

    __device__ __forceinline__ Rep rep(int r) {
        return Rep{term[r], voted[r], role[r], commit[r], last[r], phys[r], elec[r], phase[r], retry[r], fl[r],
                   t1[r], t2[r], c1[r]};
    }
};

// primary-session spill / fill (canonical HBM rows nx/mt[s][d][G])
template <int R>
__device__ __forceinline__ void session_store(const Group<R>& g, const DevParams& p, int64_t i) {
#pragma unroll
    for (int d = 0; d < R; ++d) {
        p.nx[((int64_t)g.s0 * R + d) * p.G + i] = g.nx0[d];
        p.mt[((int64_t)g.s0 * R + d) * p.G + i] = g.mc0[d];
    }
}
template <int R>
__device__ __forceinline__ void session_load(Group<R>& g, const DevParams& p, int64_t i, int s) {
    g.s0 = s;
#pragma unroll
    for (int d = 0; d < R; ++d) {
        g.nx0[d] = p.nx[((int64_t)s * R + d) * p.G + i];
        g.mc0[d] = p.mt[((int64_t)s * R + d) * p.G + i];
    }
}

template <int R>
struct Stepper {
    static constexpr int MAJ = R / 2 + 1;              // RaftServer.kt:44
    static constexpr uint32_t ALL = (1u << R) - 1u;

    // vote request snapshot of sender s (S-4); send mask per sender
    int32_t qt[R], qli[R], qlt[R];
    uint32_t send[R];

    // 16-bit drop uniform j = 2*dd + b of sender s (S-9); s may be a runtime value
    __device__ __forceinline__ static bool lost(const DevParams& p, const Ctx& c, const u32x4* du, int s, int d, int b) {
        if (s == d) return false;                                      // S-7
        if (c.iso >= 0 && (s == c.iso || d == c.iso)) return true;
        if (((c.part >> s) ^ (c.part >> d)) & 1u) return true;
        if (p.drop_thr16 == 0) return false;
        const int dd = d < s ? d : d - 1;
        const int j = 2 * dd + b;                   // 0 .. 2R-3 < 16
        // word j >> 1 of the 8-word (du[0], du[1]) pair, by one-hot masks (no
        // dynamic indexing: it would demote du to scratch)
        const uint32_t oh = 1u << (j >> 1);
        const uint32_t w8[8] = {du[0].x, du[0].y, du[0].z, du[0].w, du[1].x, du[1].y, du[1].z, du[1].w};
        uint32_t word = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) word |= w8[k] & (0u - ((oh >> k) & 1u));
        return ((word >> (16 * (j & 1))) & 0xFFFFu) < p.drop_thr16;
    }

    __device__ __forceinline__ static void drop_uniforms(const DevParams& p, const Ctx& c, uint32_t purpose, int s, u32x4* du) {
        du[0] = draw(p, c.t, c.gid, purpose, (uint32_t)s);
        if (2 * (R - 1) > 8) du[1] = draw(p, c.t, c.gid, purpose, (uint32_t)s | (1u << 8));
        else du[1] = du[0];
    }

    // RequestVote snapshot built inside retry{} (RaftServer.kt:200-207)
    __device__ __forceinline__ void build_vote_request(Group<R>& g, const Ctx& c, int r) {
        qt[r] = g.term[r];
        qli[r] = g.last[r];
        if (g.last[r] == 0) qlt[r] = 0;
        else {
            qlt[r] = g.t1[r];                                  // log.get(lastIndex - 1).term
            c.cnt->add(RAFT_C_VOTE_LOG_READS);
        }
    }

    // while (state == CANDIDATE) iteration head (RaftServer.kt:191-199)
    __device__ __forceinline__ void start_round(Group<R>& g, const Ctx& c, int r) {
        g.term[r] += 1;
        g.voted[r] = r + 1;
        g.fl[r] = (g.fl[r] & ~(FL_BACKOFF | (0xFFu << PEND_SH) | (0xFu << VOTES_SH) | (0xFu << LATCH_SH))) |
                  (ALL << PEND_SH);
        g.phase[r] = 0;
        g.retry[r] = 0;
        send[r] = ALL;
        build_vote_request(g, c, r);
        c.cnt->add(RAFT_C_ROUNDS);
    }

    // appendRequestAndLeaderHeartbeat() entry (RaftServer.kt:109-113), S-8.
    // The primary slot is taken over; the previous owner's row goes home.
    __device__ __forceinline__ static void start_session(Group<R>& g, const DevParams& p, const Ctx& c, int r) {
        g.fl[r] |= FL_HB;
        if (g.s0 >= 0 && g.s0 != r) session_store<R>(g, p, c.i);
        g.s0 = r;
#pragma unroll
        for (int d = 0; d < R; ++d) { g.nx0[d] = g.commit[r] + 1; g.mc0[d] = 0; }
        c.cnt->add(RAFT_C_LEADERS_ELECTED);
    }

    // leaderElection() returns; queued sends then the final state (S-5)
    __device__ __forceinline__ static void end_election(Group<R>& g, const DevParams& p, const Ctx& c, int r) {
        uint32_t f = g.fl[r];
        const bool prst = f & FL_PRST;
        f &= ~(FL_ELECTING | FL_PRST | FL_BACKOFF | (0xFFu << PEND_SH) | (0xFu << VOTES_SH) | (0xFu << LATCH_SH));
        if (prst) f |= FL_ARMED | FL_DRAW;
        g.fl[r] = f;
        g.phase[r] = 0;
        g.retry[r] = 0;
        if (g.role[r] == RAFT_LEADER) start_session(g, p, c, r);             // :66
        else if (g.role[r] == RAFT_FOLLOWER) g.fl[r] |= FL_ARMED | FL_DRAW;  // :64
    }

    // One fixedRateTimer tick of leader s (RaftServer.kt:115-176); s is a
    // per-lane runtime index.  Requests are all built before any handler runs
    // (S-4); responses are processed in dst order on a working copy of the
    // leader's scalars, written back at the end.  The self-handler (d == s)
    // only ever touches s's log, lastIndex and physLen (its request carries
    // leaderId == id and the tick-start term and commit), so the copy and the
    // registers never disagree on anything a handler reads.
    __device__ __forceinline__ static void tick(Group<R>& g, const DevParams& p, Ctx& c, int s) {
        Counters& cnt = *c.cnt;
        const uint32_t oh = 1u << s;
        if (pick(g.role, oh) == RAFT_FOLLOWER) {                      // :117 cancel() (S-10)
#pragma unroll
            for (int r = 0; r < R; ++r) g.fl[r] &= ~(((oh >> r) & 1u) * FL_HB);
            return;
        }
        cnt.add(RAFT_C_SESSIONS_TICKED);
        if (s != g.s0) {                                               // swap the session in
            if (g.s0 >= 0) session_store<R>(g, p, c.i);
            session_load<R>(g, p, c.i, s);
        }
        const int32_t Lterm = pick(g.term, oh), Lcommit = pick(g.commit, oh), Llast = pick(g.last, oh);
        const int32_t Lt1 = pick(g.t1, oh), Lt2 = pick(g.t2, oh), Lc1 = (int32_t)pick(g.c1, oh);
        const uint2* ls = c.lg + s * c.cap;
        // Every log slot this tick reads is resolved up front: the leader's
        // log[prev] and log[i-1] for each request (built before any handler
        // runs, RaftServer.kt:122-132) and each follower's own log[prev]
        // (append() :274-276).  The tail cache answers the steady-state ones;
        // the rest are loaded in one batch.  A handler only writes its own
        // replica's log, so no earlier handler of the tick can change a slot a
        // later one reads.
        int32_t lpt[R], dpt[R];
        uint2 lent[R];
#pragma unroll
        for (int d = 0; d < R; ++d) {
            const int32_t i = g.nx0[d], prev = i - 2;
            lpt[d] = (prev >= 0 && prev <= Llast - 1) ? term_at(ls, Llast, Lt1, Lt2, prev) : -1;
            lent[d] = (i >= 1 && i <= Llast) ? (i == Llast ? make_uint2((uint32_t)Lt1, (uint32_t)Lc1) : ls[i - 1])
                                             : make_uint2(0u, 0u);
            const uint2* lr = c.lg + d * c.cap;
            dpt[d] = (prev >= 0 && prev < g.last[d]) ? term_at(lr, g.last[d], g.t1[d], g.t2[d], prev) : 0;
        }
        // build every request (RaftServer.kt:122-132)
        uint32_t okm = 0, hasm = 0;
#pragma unroll
        for (int d = 0; d < R; ++d) {
            const int32_t i = g.nx0[d], prev = i - 2;
            bool ok = true;
            if (prev >= 0) {                                           // :128 (Q11)
                if (prev > Llast - 1) ok = false;
                else cnt.add(RAFT_C_PREV_READS_LEADER);
            }
            if (ok && Llast >= i) {                                    // :130-131
                if (i - 1 < 0) ok = false;
                else { hasm |= 1u << d; cnt.add(RAFT_C_ENTRY_READS_LEADER); }
            }
            if (ok) okm |= 1u << d;
            else cnt.add(RAFT_C_APPEND_SKIPPED);
        }
        u32x4 du[2];
        if (p.drop_thr16) drop_uniforms(p, c, RAFT_RNG_APPEND_DROP, s, du);
        int32_t T = Lterm, C = Lcommit;
        bool stepdown = false;
#pragma unroll
        for (int d = 0; d < R; ++d) {
            if (!((okm >> d) & 1u)) continue;
            cnt.add(RAFT_C_APPEND_SENT);
            if (lost(p, c, du, s, d, 0)) { cnt.add(RAFT_C_MSG_DROPPED); continue; }   // :170-172
            const int32_t prev = g.nx0[d] - 2;
            const bool has = (hasm >> d) & 1u;
            int32_t rterm; bool succ;
            if (!append_handler(g.rep(d), d + 1, c.lg + d * c.cap, c.cap, Lterm, s + 1, prev, lpt[d], has,
                                Entry{(int32_t)lent[d].x, lent[d].y}, Lcommit, dpt[d], cnt, rterm, succ))
                continue;
            if (lost(p, c, du, s, d, 1)) { cnt.add(RAFT_C_MSG_DROPPED); continue; }
            if (rterm > T) { T = rterm; stepdown = true; continue; }  // :146-154 (Q7)
            if (succ) {                                                // :156-165 (Q9)
                if (has) {
                    g.nx0[d] += 1;
                    g.mc0[d] += 1;
                    cnt.add(RAFT_C_ENTRIES_ACKED);
                    int k = 0;
#pragma unroll
                    for (int q = 0; q < R; ++q) k += g.mc0[q] > C;     // :161
                    if (k >= MAJ) { C += 1; cnt.add(RAFT_C_COMMITS); } // :162
                } else {
                    g.mc0[d] = prev + 1;                               // :164
                }
            } else {
                g.nx0[d] -= 1;                                         // :167
            }
        }
        place(g.term, oh, T);
        place(g.commit, oh, C);
        if (stepdown) {                                                // :148 + offer(FOLLOWER) :152 (S-6)
            place(g.role, stepdown ? oh : 0u, RAFT_FOLLOWER);
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (((oh >> r) & 1u) && !(g.fl[r] & FL_ELECTING)) g.fl[r] |= FL_ARMED | FL_DRAW;
        }
    }

    __device__ __forceinline__ void step(Group<R>& g, const DevParams& p, Ctx& c) {
        Counters& cnt = *c.cnt;
        // ---------------- H: harness ----------------
        u32x4 hw = u32x4{0u, 0u, 0u, 0u};
        if (p.churn_thr32 | p.cmd_thr32) hw = draw(p, c.t, c.gid, RAFT_RNG_HARNESS, 0);
        {
            int32_t rem = g.iso >> 8, rep = g.iso & 0xFF;
            if (rem > 0) { rem--; if (rem == 0) rep = 0; }
            if (p.churn_thr32 && p.churn_steps > 0 && rem == 0 && hw.x < p.churn_thr32) {
                int L = -1;
#pragma unroll
                for (int r = R - 1; r >= 0; --r) if (g.role[r] == RAFT_LEADER) L = r;
                if (L >= 0) { rep = L; rem = p.churn_steps; }
            }
            g.iso = rem > 0 ? (rem << 8) | rep : 0;
            c.iso = rem > 0 ? rep : -1;
        }
        c.part = 0;
        if (p.part_period > 0) {
            const uint32_t ph = c.t % (uint32_t)p.part_period;
            if ((int64_t)ph < p.part_len) c.part = draw(p, c.t - ph, c.gid, RAFT_RNG_PARTITION, 0).x & ALL;
        }

        // ---------------- T: timers and election clocks ----------------
#pragma unroll
        for (int r = 0; r < R; ++r) {
            send[r] = 0;
            bool started = false;
            if (g.fl[r] & FL_ARMED) {
                g.elec[r] -= p.P;
                if (g.elec[r] <= 0) {                                   // Commons.kt:25-27
                    g.fl[r] &= ~FL_ARMED;
                    g.elec[r] = 0;
                    cnt.add(RAFT_C_TIMEOUTS);
                    g.role[r] = RAFT_CANDIDATE;                         // RaftServer.kt:182
                    if (!(g.fl[r] & FL_ELECTING)) {                     // :184 -> :65
                        g.fl[r] |= FL_ELECTING;
                        start_round(g, c, r);
                        started = true;
                    }
                }
            }
            if ((g.fl[r] & FL_ELECTING) && !started) {
                if (!(g.fl[r] & FL_BACKOFF)) {
                    g.phase[r] += p.P;                                  // latch clock :214
                    const uint32_t pend = (g.fl[r] >> PEND_SH) & 0xFFu;
                    if (pend && g.phase[r] < p.round_to) {
                        g.retry[r] -= p.P;                              // Commons.kt:43
                        if (g.retry[r] <= 0) { build_vote_request(g, c, r); send[r] = pend; }
                    }
                } else {
                    g.phase[r] -= p.P;                                  // delay(backoff) :221
                    if (g.phase[r] <= 0) {
                        if (g.role[r] == RAFT_CANDIDATE) start_round(g, c, r);   // :191
                        else end_election(g, p, c, r);
                    }
                }
            }
        }

        // ---------------- V: RequestVote fan-out (S-3) ----------------
        bool anysend = false;
#pragma unroll
        for (int s = 0; s < R; ++s) anysend |= send[s] != 0;
        if (__any(anysend)) {
#pragma unroll
            for (int s = 0; s < R; ++s) {
                if (!__any(send[s] != 0)) continue;
                u32x4 du[2];
                if (p.drop_thr16 && send[s]) drop_uniforms(p, c, RAFT_RNG_VOTE_DROP, s, du);
                if (send[s]) {
#pragma unroll
                    for (int d = 0; d < R; ++d) {
                        if (!((send[s] >> d) & 1u)) continue;
                        if (lost(p, c, du, s, d, 0)) { cnt.add(RAFT_C_MSG_DROPPED); continue; }
                        int32_t rterm; bool granted;
                        vote_handler(g.rep(d), c.lg + d * c.cap, qt[s], s + 1, qli[s], qlt[s], cnt, rterm, granted);
                        if (lost(p, c, du, s, d, 1)) { cnt.add(RAFT_C_MSG_DROPPED); continue; }
                        uint32_t f = g.fl[s];
                        f &= ~(1u << (PEND_SH + d));
                        f += 1u << LATCH_SH;                              // :209
                        if (granted) f += 1u << VOTES_SH;                 // :211
                        g.fl[s] = f;
                        if (g.term[s] < rterm) g.role[s] = RAFT_FOLLOWER; // :210 (Q6)
                    }
                    send[s] = 0;
                    if ((g.fl[s] >> PEND_SH) & 0xFFu) g.retry[s] = p.retry;
                }
            }
        }

        // ---------------- D: latch closes -> decision (RaftServer.kt:214-222) ----------------
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t f = g.fl[r];
            if (!(f & FL_ELECTING) || (f & FL_BACKOFF)) continue;
            const int latch = (f >> LATCH_SH) & 0xF, votes = (f >> VOTES_SH) & 0xF;
            if (latch < MAJ && g.phase[r] < p.round_to) continue;
            g.fl[r] = f & ~(0xFFu << PEND_SH);                          // cancelChildren() :215
            if (g.role[r] == RAFT_CANDIDATE && votes >= MAJ) {          // :218-219
                g.role[r] = RAFT_LEADER;
                end_election(g, p, c, r);
            } else if (g.role[r] == RAFT_CANDIDATE) {                   // :220-221
                g.fl[r] = (g.fl[r] & ~((0xFu << VOTES_SH) | (0xFu << LATCH_SH))) | FL_BACKOFF;
                const u32x4 w = draw(p, c.t, c.gid, RAFT_RNG_BACKOFF, (uint32_t)(r >> 2));
                g.phase[r] = scale_range(word_of(w, r & 3), p.bmin, p.bmax);
                g.retry[r] = 0;
            } else {
                end_election(g, p, c, r);
            }
        }

        // ---------------- A: leader ticks, senders ascending (S-3, S-4) ----------------
        uint32_t todo = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) todo |= (g.fl[r] & FL_HB) ? (1u << r) : 0u;
        while (__any(todo != 0)) {
            if (todo != 0) {
                const int s = __builtin_ctz(todo);
                todo &= todo - 1u;
                tick(g, p, c, s);
            }
        }

        // ---------------- C: client commands (S-11) ----------------
        if (p.cmd_thr32 && (p.cmd_limit == 0 || g.cmdc < p.cmd_limit) && hw.y < p.cmd_thr32) {
            bool any = false;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (g.role[r] == RAFT_LEADER && !(any && p.cmd_mode == RAFT_CMD_LOWEST_LEADER)) {
                    append_command(g.rep(r), c.lg + r * c.cap, c.cap, hw.z, cnt);
                    any = true;
                }
            }
            if (any) g.cmdc++;
        }

        // ---------------- K: end-of-step observations ----------------
        int leaders = 0;
        bool dual = false;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (g.role[r] != RAFT_LEADER) continue;
            leaders++;
#pragma unroll
            for (int q = r + 1; q < R; ++q)
                dual |= g.role[q] == RAFT_LEADER && g.term[q] == g.term[r];
        }
        cnt.add(RAFT_C_LEADERS, (uint32_t)leaders);
        if (leaders > 0) cnt.add(RAFT_C_GROUPS_WITH_LEADER);
        if (dual) cnt.add(RAFT_C_DUAL_LEADER_GROUPS);

        resolve_timer_draws(g, p, c);
    }

    // the deferred ResettableCountdownTimer draws of this step (S-9)
    __device__ __forceinline__ static void resolve_timer_draws(Group<R>& g, const DevParams& p, const Ctx& c) {
#pragma unroll
        for (int q = 0; q < (R + 3) / 4; ++q) {
            bool need = false;
#pragma unroll
            for (int r = 4 * q; r < R && r < 4 * q + 4; ++r) need |= (g.fl[r] & FL_DRAW) != 0;
            if (!__any(need)) continue;
            if (need) {
                const u32x4 w = draw(p, c.t, c.gid, RAFT_RNG_TIMER, (uint32_t)q);
#pragma unroll
                for (int r = 4 * q; r < R && r < 4 * q + 4; ++r) {
                    if (g.fl[r] & FL_DRAW) {
                        g.elec[r] = scale_range(word_of(w, r & 3), p.emin, p.emax);
                        g.fl[r] &= ~FL_DRAW;
                    }
                }
            }
        }
    }
};

}  // namespace raft
