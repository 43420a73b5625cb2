// raft_step.h — the per-node consensus step of arodionov/raft-kotlin as
// register-resident SIMT code for gfx950.
//
// One lane owns one Raft group: all R replicas' scalar state, their leader
// sessions (nextIndex/matchIndex) and the step's message temporaries live in
// VGPRs.  Every loop over replicas is unrolled against the compile-time R, so
// the R x R request/response "message tensor" of a phase never exists in
// memory: a message is a handler call whose arguments are registers of the
// sender and whose effects land in registers of the receiver.  Only the logs
// (the reference's ArrayList, Commons.kt:51) stay in HBM, touched at the
// slots the handlers read or write.
//
// The phase order and every tie-break follow DESIGN.md §3 (the same schedule
// the CPU oracle in oracle/raft_oracle.c restates object by object).
#pragma once
#include <hip/hip_runtime.h>
#include "philox.h"
#include "../../include/raft_engine.h"

namespace raft {

constexpr int NC = RAFT_NUM_COUNTERS;

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

__device__ __forceinline__ u32x4 draw(const DevParams& p, uint32_t c0, uint32_t gid, uint32_t purpose, uint32_t sub) {
    return philox4x32_10(c0, gid, purpose, sub, p.key0, p.key1);
}

// Per-(group, step) context.
struct Ctx {
    uint32_t t, gid;
    int32_t iso;          // isolated replica this step, -1 if none
    uint32_t part;        // replicas on side B of this step's partition
    uint2* lg;            // this group's log, [R][cap] entries (term, cmd)
    int cap;
    int* cnt;             // this lane's counters for the step
};

// One replica's scalar state, by reference into the owning lane's registers.
struct Rep {
    int32_t &term, &voted, &role, &commit, &last, &phys, &elec, &phase, &retry;
    uint32_t& fl;
};

// ---- timer / consumer (Commons.kt:10-31, RaftServer.kt:50-69) -------------
// reset(): re-arm with a fresh draw.  The draw is a pure function of
// (step, group, replica), so it is resolved once at the end of the step
// (resolve_timer_draws) no matter how many resets the step performed.
__device__ __forceinline__ void reset_timer(Rep n) { n.fl |= FL_ARMED | FL_DRAW; }
// launch { channel.send(FOLLOWER) } (RaftServer.kt:241, :261, :266), S-5
__device__ __forceinline__ void send_follower(Rep n) {
    if (n.fl & FL_ELECTING) n.fl |= FL_PRST; else reset_timer(n);
}
// channel.offer(FOLLOWER) (RaftServer.kt:152), S-6
__device__ __forceinline__ void offer_follower(Rep n) {
    if (!(n.fl & FL_ELECTING)) reset_timer(n);
}

// ---- Log<T> (Commons.kt:47-74) over one replica's HBM slots ---------------
// Log.add(i, e): 1 true, 0 false, -1 capacity overflow (counted), -2 threw
__device__ __forceinline__ int log_add(uint2* lr, int cap, int32_t& last, int32_t& phys, int32_t i, Entry e) {
    if (last == i) {                                   // :58-61 append at the PHYSICAL end (Q1)
        if (phys >= cap) return -1;
        lr[phys] = make_uint2((uint32_t)e.term, e.cmd);
        phys += 1;
        last += 1;
        return 1;
    }
    if (last < i) return 0;                            // :62
    if (i < 0) return -2;
    lr[i] = make_uint2((uint32_t)e.term, e.cmd);       // :63-66 overwrite, no shrink
    last = i + 1;
    return 1;
}

// ---- vote() (RaftServer.kt:228-251) ---------------------------------------
__device__ __forceinline__ void vote_handler(Rep n, const uint2* lr, int32_t rt, int32_t rc, int32_t rli,
                                             int32_t rlt, int* cnt, int32_t& resp_term, bool& granted) {
    granted = false;
    if (rt < n.term) {
    } else if (n.term == rt) {
        granted = n.voted == rc;
    } else {
        int32_t lt = 0;
        if (n.last >= 1) { lt = (int32_t)lr[n.last - 1].x; cnt[RAFT_C_VOTE_LOG_READS]++; }
        if (n.last >= 1 && rlt < lt) {
        } else if (n.last >= 1 && rlt == lt && rli < n.last) {
        } else {
            n.term = rt; n.voted = rc; n.role = RAFT_FOLLOWER;
            send_follower(n);
            granted = true;
        }
    }
    if (granted) cnt[RAFT_C_VOTES_GRANTED]++;
    resp_term = n.term;
}

// ---- append() (RaftServer.kt:253-287); returns false where it throws -------
__device__ __forceinline__ bool append_handler(Rep n, int32_t id, uint2* lr, int cap, int32_t rt, int32_t rlead,
                                               int32_t prev, int32_t prevTerm, bool has, Entry e,
                                               int32_t lcommit, int* cnt, int32_t& resp_term, bool& success) {
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
        if (c < n.commit) cnt[RAFT_C_COMMIT_REGRESSIONS]++;
        n.commit = c;
    }
    if (prev == -1) success = true;                     // :274-276
    else if (n.last > prev) {
        if (prev < 0) { resp_term = n.term; success = false; return false; }
        cnt[RAFT_C_PREV_READS_FOLLOWER]++;
        success = (int32_t)lr[prev].x == prevTerm;
    } else success = false;
    if (success && has) {                               // :278 (Q2, Q10)
        const int r = log_add(lr, cap, n.last, n.phys, prev + 1, e);
        if (r == 1) cnt[RAFT_C_ENTRY_WRITES]++;
        else if (r == -1) cnt[RAFT_C_LOG_OVERFLOW]++;
    }
    resp_term = n.term;
    return true;
}

// ---- appendCommand() (RaftServer.kt:100-107) ------------------------------
__device__ __forceinline__ void append_command(Rep n, uint2* lr, int cap, uint32_t cmd, int* cnt) {
    const int r = log_add(lr, cap, n.last, n.phys, n.last, Entry{n.term, cmd});
    cnt[RAFT_C_COMMANDS]++;
    if (r == -1) cnt[RAFT_C_LOG_OVERFLOW]++;
}

// ---------------------------------------------------------------------------
// The register-resident group.
// ---------------------------------------------------------------------------
template <int R>
struct Group {
    int32_t term[R], voted[R], role[R], commit[R], last[R], phys[R], elec[R], phase[R], retry[R];
    uint32_t fl[R];
    int32_t nx[R][R], mc[R][R];     // leader session of replica s: [s][d]
    int32_t iso, cmdc;              // harness: isolation word, commands issued
    uint32_t sdirty;                // sessions to write back: active at load or started since

    __device__ __forceinline__ Rep rep(int r) {
        return Rep{term[r], voted[r], role[r], commit[r], last[r], phys[r], elec[r], phase[r], retry[r], fl[r]};
    }
};

template <int R>
struct Stepper {
    static constexpr int MAJ = R / 2 + 1;              // RaftServer.kt:44
    static constexpr uint32_t ALL = (1u << R) - 1u;

    // vote request snapshot of sender s (S-4); send mask per sender
    int32_t qt[R], qli[R], qlt[R];
    uint32_t send[R];

    __device__ __forceinline__ static bool lost(const DevParams& p, const Ctx& c, const u32x4* du, int s, int d, int b) {
        if (s == d) return false;                                      // S-7
        if (c.iso >= 0 && (s == c.iso || d == c.iso)) return true;
        if (((c.part >> s) ^ (c.part >> d)) & 1u) return true;
        if (p.drop_thr16 == 0) return false;
        const int dd = d < s ? d : d - 1;
        const int j = 2 * dd + b;
        const uint32_t word = word_of(du[j >> 3], (j & 7) >> 1);
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
            const uint2* lr = c.lg + r * c.cap;
            qlt[r] = (int32_t)lr[g.last[r] - 1].x;
            c.cnt[RAFT_C_VOTE_LOG_READS]++;
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
        c.cnt[RAFT_C_ROUNDS]++;
    }

    // appendRequestAndLeaderHeartbeat() entry (RaftServer.kt:109-113), S-8
    // (a session can start and end in one step: a stale leader ticking earlier
    //  in phase A deposes the new one, Q3; its arrays still persist, S-8)
    __device__ __forceinline__ static void start_session(Group<R>& g, const Ctx& c, int r) {
        g.fl[r] |= FL_HB;
        g.sdirty |= 1u << r;
#pragma unroll
        for (int d = 0; d < R; ++d) { g.nx[r][d] = g.commit[r] + 1; g.mc[r][d] = 0; }
        c.cnt[RAFT_C_LEADERS_ELECTED]++;
    }

    // leaderElection() returns; queued sends then the final state (S-5)
    __device__ __forceinline__ static void end_election(Group<R>& g, const Ctx& c, int r) {
        uint32_t f = g.fl[r];
        const bool prst = f & FL_PRST;
        f &= ~(FL_ELECTING | FL_PRST | FL_BACKOFF | (0xFFu << PEND_SH) | (0xFu << VOTES_SH) | (0xFu << LATCH_SH));
        if (prst) f |= FL_ARMED | FL_DRAW;
        g.fl[r] = f;
        g.phase[r] = 0;
        g.retry[r] = 0;
        if (g.role[r] == RAFT_LEADER) start_session(g, c, r);                 // :66
        else if (g.role[r] == RAFT_FOLLOWER) g.fl[r] |= FL_ARMED | FL_DRAW;   // :64
    }

    __device__ __forceinline__ void step(Group<R>& g, const DevParams& p, Ctx& c) {
        int* cnt = c.cnt;
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
                    cnt[RAFT_C_TIMEOUTS]++;
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
                        else end_election(g, c, r);
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
                        if (lost(p, c, du, s, d, 0)) { cnt[RAFT_C_MSG_DROPPED]++; continue; }
                        int32_t rterm; bool granted;
                        vote_handler(g.rep(d), c.lg + d * c.cap, qt[s], s + 1, qli[s], qlt[s], cnt, rterm, granted);
                        if (lost(p, c, du, s, d, 1)) { cnt[RAFT_C_MSG_DROPPED]++; continue; }
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
                end_election(g, c, r);
            } else if (g.role[r] == RAFT_CANDIDATE) {                   // :220-221
                g.fl[r] = (g.fl[r] & ~((0xFu << VOTES_SH) | (0xFu << LATCH_SH))) | FL_BACKOFF;
                const u32x4 w = draw(p, c.t, c.gid, RAFT_RNG_BACKOFF, (uint32_t)(r >> 2));
                g.phase[r] = scale_range(word_of(w, r & 3), p.bmin, p.bmax);
                g.retry[r] = 0;
            } else {
                end_election(g, c, r);
            }
        }

        // ---------------- A: leader ticks (S-3, S-4) ----------------
#pragma unroll
        for (int s = 0; s < R; ++s) {
            bool active = (g.fl[s] & FL_HB) != 0;
            if (active && g.role[s] == RAFT_FOLLOWER) { g.fl[s] &= ~FL_HB; active = false; }   // :117 (S-10)
            if (!__any(active)) continue;
            if (active) {
                cnt[RAFT_C_SESSIONS_TICKED]++;
                // build every request first (RaftServer.kt:122-132)
                const uint2* ls = c.lg + s * c.cap;
                const int32_t sterm = g.term[s], scommit = g.commit[s], slast = g.last[s];
                bool ok[R], has[R];
                int32_t pv[R], pvt[R];
                Entry ent[R];
#pragma unroll
                for (int d = 0; d < R; ++d) {
                    const int32_t i = g.nx[s][d];
                    pv[d] = i - 2;
                    pvt[d] = -1;
                    ok[d] = true;
                    has[d] = false;
                    ent[d] = Entry{0, 0u};
                    if (pv[d] >= 0) {                                  // :128 (Q11)
                        if (pv[d] > slast - 1) ok[d] = false;
                        else { pvt[d] = (int32_t)ls[pv[d]].x; cnt[RAFT_C_PREV_READS_LEADER]++; }
                    }
                    if (ok[d] && slast >= i) {                          // :130-131
                        if (i - 1 < 0) ok[d] = false;
                        else {
                            const uint2 e = ls[i - 1];
                            ent[d] = Entry{(int32_t)e.x, e.y};
                            has[d] = true;
                            cnt[RAFT_C_ENTRY_READS_LEADER]++;
                        }
                    }
                    if (!ok[d]) cnt[RAFT_C_APPEND_SKIPPED]++;
                }
                u32x4 du[2];
                if (p.drop_thr16) drop_uniforms(p, c, RAFT_RNG_APPEND_DROP, s, du);
#pragma unroll
                for (int d = 0; d < R; ++d) {
                    if (!ok[d]) continue;
                    cnt[RAFT_C_APPEND_SENT]++;
                    if (lost(p, c, du, s, d, 0)) { cnt[RAFT_C_MSG_DROPPED]++; continue; }   // :170-172
                    int32_t rterm; bool succ;
                    if (!append_handler(g.rep(d), d + 1, c.lg + d * c.cap, c.cap, sterm, s + 1, pv[d], pvt[d],
                                        has[d], ent[d], scommit, cnt, rterm, succ))
                        continue;
                    if (lost(p, c, du, s, d, 1)) { cnt[RAFT_C_MSG_DROPPED]++; continue; }
                    if (rterm > g.term[s]) {                            // :146-154 (Q7)
                        g.term[s] = rterm;
                        g.role[s] = RAFT_FOLLOWER;
                        offer_follower(g.rep(s));
                        continue;
                    }
                    if (succ) {                                         // :156-165 (Q9)
                        if (has[d]) {
                            g.nx[s][d] += 1;
                            g.mc[s][d] += 1;
                            cnt[RAFT_C_ENTRIES_ACKED]++;
                            int k = 0;
#pragma unroll
                            for (int q = 0; q < R; ++q) k += g.mc[s][q] > g.commit[s];   // :161
                            if (k >= MAJ) { g.commit[s] += 1; cnt[RAFT_C_COMMITS]++; }    // :162
                        } else {
                            g.mc[s][d] = pv[d] + 1;                     // :164
                        }
                    } else {
                        g.nx[s][d] -= 1;                                // :167
                    }
                }
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
        cnt[RAFT_C_LEADERS] += leaders;
        cnt[RAFT_C_GROUPS_WITH_LEADER] += leaders > 0;
        cnt[RAFT_C_DUAL_LEADER_GROUPS] += dual;

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
