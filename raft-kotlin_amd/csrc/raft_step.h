// raft_step.h — the per-node consensus step of arodionov/raft-kotlin as
// lane-per-replica SIMT code for gfx950.
//
// Lane mapping.  A wave64 holds GPW = 64 / R whole groups: lane L serves
// replica r = L % R of group j = L / R (lanes >= GPW * R idle).  Every lane
// keeps ONE replica's scalar state in VGPRs (RaftServer.kt:35-48: term,
// votedFor, state, commitIndex, the Log's lastIndex and physical size, the
// timer and election-loop clocks) plus its column of the group's primary
// leader session (nextIndex / matchIndex towards this replica,
// RaftServer.kt:112-113).  The reference's RPC fan-out becomes cross-lane
// traffic inside the wave:
//   * a request is a ds_bpermute broadcast of the sender lane's fields to the
//     group's lanes, and every destination runs its handler IN PARALLEL on its
//     own registers (one handler per lane instead of R x R unrolled calls);
//   * responses come back as __ballot bitmasks: the candidate's vote tally is
//     popcount(ballot(delivered & granted)) (RaftServer.kt:209-211) and the
//     leader's commit rule (RaftServer.kt:161-162) is a popcount of
//     ballot(matchIndex > commitIndex) re-evaluated after every acknowledged
//     entry in destination order.
// The logs (the reference's ArrayList, Commons.kt:51) stay in HBM; a lane
// touches only its own replica's slots, plus the leader's slots it is shipped.
//
// Every step follows the lockstep schedule of DESIGN.md §3 (the same schedule
// the CPU oracle in oracle/raft_oracle.c restates object by object).  The
// parallel form is exact because (a) a handler only writes its own
// replica, (b) a sender's self-message never changes the sender's state
// (its request carries its own snapshot term, which can only be <= its
// current term), and (c) the sender-side response processing that IS
// order-dependent (Q6/Q7 term adoption, the +1 commit rule) is replayed in
// destination order with ballots.
//
// Cross-lane rule: every ds_bpermute / ballot that reads another lane runs in
// control flow that is uniform across a whole group (whole groups are either
// active or not), so a source lane is never masked off.
#pragma once
#include <hip/hip_runtime.h>
#include "philox.h"
#include "../../include/raft_engine.h"

extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);
// v_writelane_b32: one SGPR value into one lane of a VGPR
extern "C" __device__ int32_t raft_writelane(int32_t val, int32_t lane, int32_t old) __asm("llvm.amdgcn.writelane.i32");

namespace raft {

constexpr int NC = RAFT_NUM_COUNTERS;
constexpr int NCW = (NC + 1) / 2;          // counters packed as 16-bit pairs per lane
// Half-word slot of each counter in the packed rows (slot >> 1: word, slot & 1:
// half).  The counters added most often per wave-step take the low halves, which
// need no shift before the add (one SALU fewer per event mask; SALU issue is a
// bottleneck of the step kernel).  The reduction decodes with counter_of_slot.
constexpr int COUNTER_SLOT[RAFT_NUM_COUNTERS] = {
    /* LEADERS            */ 7,  /* GROUPS_WITH_LEADER */ 9,  /* TIMEOUTS           */ 11,
    /* ROUNDS             */ 13, /* VOTES_GRANTED      */ 6,  /* LEADERS_ELECTED    */ 15,
    /* SESSIONS_TICKED    */ 8,  /* APPEND_SENT        */ 10, /* APPEND_SKIPPED     */ 21,
    /* ENTRIES_ACKED      */ 20, /* COMMITS            */ 1,  /* MSG_DROPPED        */ 0,
    /* COMMANDS           */ 5,  /* COMMIT_REGRESSIONS */ 3,  /* DUAL_LEADER_GROUPS */ 17,
    /* LOG_OVERFLOW       */ 4,  /* PREV_READS_LEADER  */ 12, /* ENTRY_READS_LEADER */ 14,
    /* PREV_READS_FOLLOWER*/ 16, /* ENTRY_WRITES       */ 18, /* VOTE_LOG_READS     */ 2,
    /* LOG_WINDOW_MISS    */ 19,
};
static_assert(RAFT_NUM_COUNTERS == 22, "COUNTER_SLOT lists every counter");
__host__ __device__ constexpr int counter_of_slot(int slot) {
    for (int c = 0; c < RAFT_NUM_COUNTERS; ++c)
        if (COUNTER_SLOT[c] == slot) return c;
    return -1;
}
constexpr bool counter_slots_are_a_permutation() {
    for (int q = 0; q < 2 * NCW; ++q)
        if (q < RAFT_NUM_COUNTERS && counter_of_slot(q) < 0) return false;
    return true;
}
static_assert(counter_slots_are_a_permutation(), "every counter has its own half-word slot");

// exported flag bits (include/raft_engine.h) and engine-internal ones
constexpr uint32_t FL_ARMED = RAFT_FL_ARMED;
constexpr uint32_t FL_ELECTING = RAFT_FL_ELECTING;
constexpr uint32_t FL_PRST = RAFT_FL_PENDING_RST;
constexpr uint32_t FL_HB = RAFT_FL_HB_ACTIVE;
constexpr uint32_t FL_BACKOFF = RAFT_FL_BACKOFF;
constexpr uint32_t FL_DRAW = 1u << 5;      // internal: timer re-armed this step, draw pending
constexpr uint32_t FL_EXPORT_MASK = ~FL_DRAW;
constexpr int PEND_SH = RAFT_FL_PENDING_SHIFT, VOTES_SH = RAFT_FL_VOTES_SHIFT, LATCH_SH = RAFT_FL_LATCH_SHIFT;

// engine-internal per-replica fields after the canonical ones: the log-tail
// cache (term of log[last-1], log[last-2]; cmd of log[last-1]) and the
// group's primary leader session towards this replica (nextIndex, matchIndex)
constexpr int F_T1 = RAFT_NUM_FIELDS, F_T2 = RAFT_NUM_FIELDS + 1, F_C1 = RAFT_NUM_FIELDS + 2;
constexpr int F_NX = RAFT_NUM_FIELDS + 3, F_MC = RAFT_NUM_FIELDS + 4;
constexpr int F_DEV = RAFT_NUM_FIELDS + 5;
// The 15 fields live in 4 quads of 4 int32 per replica (st, below): a piece
// entry / exit moves a replica with 4 dwordx4 accesses, and a handler of the
// batch path touches only the quads it needs, one 32-B sector each (vote():
// quads 0 and 1, append(): 0-2).  Slot 4q + k of a field = word k of quad q.
//   quad 0: term, votedFor, state, flags       (every handler reads and writes)
//   quad 1: lastIndex, physLen, t1, electionMs (vote() reads, the timer re-arm writes)
//   quad 2: commitIndex, t2, c1, phaseMs       (append() and appendCommand)
//   quad 3: retryMs, nextIndex, matchIndex, -  (the step kernel only)
constexpr int ST_QUADS = 4;
constexpr int FIELD_SLOT[F_DEV] = {
    /* TERM */ 0, /* VOTED */ 1, /* ROLE */ 2, /* COMMIT */ 8, /* LAST */ 4, /* PHYS */ 5,
    /* ELECTION_MS */ 7, /* FLAGS */ 3, /* PHASE_MS */ 11, /* RETRY_MS */ 12,
    /* T1 */ 6, /* T2 */ 9, /* C1 */ 10, /* NX */ 13, /* MC */ 14,
};
static_assert(RAFT_NUM_FIELDS == 10 && RAFT_F_RETRY_MS == 9, "FIELD_SLOT lists the canonical fields in order");
// group words gx[GX_*][G]
constexpr int GX_ISO = 0, GX_CMDS = 1, GX_S0 = 2, GX_WORDS = 3;

// HBM layout (all per-replica arrays indexed by idx = g * R + r, so the lanes
// of a wave read one contiguous run per quad):
//   st    int4  [ST_QUADS][G*R]     replica scalars, tail cache and the primary session of group g
//                                   (nextIndex / matchIndex towards replica r), FIELD_SLOT
//   spill int32 [2][G*R][R]         every other session row: [(g*R + d) * R + s]
//   gx    int32 [GX_WORDS][G]       isolation word, commands issued, primary-session owner s0 (-1 none)
//   log   uint2 [waves][64][NW]     (term, cmd) physical slots, one contiguous block per step-kernel
//                                   wave (GPW = 64 / R groups): physical index j of the replica in
//                                   lane l of wave w at [w][l][j & wmask]; NW = log_window (a ring
//                                   of the newest NW slots) or log_cap (every slot, no wrap)
struct DevParams {
    int32_t* st;
    int32_t* spill;
    int32_t* gx;
    uint2* log;
    int64_t G, g0, GR;
    int32_t R, cap;
    uint32_t wmask;                            // slot of physical index j: j & wmask
    int32_t W;                                 // window: accesses below physLen - W are misses (FLAT_W if none)
    int32_t nslots;                            // NW: slots per replica (< 2^23: 32-bit offsets in a block)
    uint32_t key0, key1;
    int32_t P, emin, emax, bmin, bmax, round_to, retry;
    uint32_t drop_ppm, drop_thr16;             // hit16(u) == (u < drop_thr16)
    uint64_t churn_thr32, cmd_thr32;           // hit32(w) == (w < thr)
    int32_t churn_steps, part_period, part_len;
    int32_t cmd_mode, cmd_limit;
    int32_t ae_max;                            // entries per AppendEntries request (textbook mode; else 1)
    uint32_t rk[20];                           // Philox round keys (k0, k1) of rounds 0..9 (kdraw)
    // step_kernel launches only: this launch's sub-range of the waves (chunks
    // of GPW groups, one log block each), its columns of the counter partials
    // [k][NCW][part_stride], and its schedule: bal_chunks == 0, one chunk per
    // wave (wave0 + blockIdx.x * STEP_WAVES + wave); else the balanced
    // schedule over bal_chunks chunks (raft_engine.hip piece_of)
    uint32_t* part;
    int32_t wave0, part_col0, part_stride;
    int32_t bal_chunks, bal_q, bal_rem;        // (bal_q, bal_rem) = bal_chunks / and % the workgroups
    int32_t epoch;                             // balanced: steps per epoch of a longer launch (0: one epoch)
    uint32_t* status;                          // engine status word (page-locked host): RAFT_DEV_* bits
};
constexpr uint32_t RAFT_DEV_WAIT_TIMEOUT = 1u;  // a balanced-schedule wave gave up waiting for its head piece

constexpr int32_t FLAT_W = 1 << 30;            // DevParams::W of a flat log (log_window 0): nothing is ever below it

struct Entry { int32_t term; uint32_t cmd; };

// One replica's log in HBM (the reference's ArrayList, Commons.kt:51): its
// row of its wave's block [64][NW] of DevParams::log.  A wave's slots are one
// contiguous region, and a replica's consecutive physical slots are adjacent,
// so its appends over successive steps fill the same cache lines.
struct LogView {
    uint2* lr;                // slot 0 of this replica's row
    uint32_t ns, wmask;       // NW slots per replica (the row stride); slot of physical index j: j & wmask
    int32_t cap, W;
    template <bool RING = true>
    __device__ __forceinline__ uint2* at(int32_t j) const { return lr + (RING ? ((uint32_t)j & wmask) : (uint32_t)j); }
    // the view of the replica `d` lanes (replica indices) away in the same group
    __device__ __forceinline__ LogView lane(int d) const { return LogView{lr + (int64_t)d * ns, ns, wmask, cap, W}; }
    // a reference access of physical index j is below the retained window
    __device__ __forceinline__ uint64_t miss(int32_t j, int32_t phys) const { return __ballot(j < phys - W); }
};

// The step kernel's DevParams as seen through the kernarg segment (constant
// address space, so every field read is one scalar load).  Rarely used
// fields are re-read through an opaque pointer where they are needed: kept
// live across the step loop they would pin SGPRs, which the kernel would
// spill into VGPR lanes and reload with v_readlane at every use.
// Valid only inside step_kernel, whose first kernel argument is the DevParams.
typedef const __attribute__((address_space(4))) DevParams* KernArgs;
__device__ __forceinline__ KernArgs kernargs() {
    KernArgs kp = (KernArgs)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return kp;
}

// The step kernel's draws (S-9): Philox4x32-10 (philox.h) with the 20 round
// keys read from the kernarg segment (DevParams::rk, made at create), a few
// scalar loads per pass instead of 20 s_add (SALU issue is a bottleneck of the
// step kernel).  The key pointer is opaque per call (kernargs()), so the loads
// are not hoisted out of the step loop.  Valid only inside step_kernel.
__device__ __forceinline__ u32x4 kdraw(const DevParams& p, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    const KernArgs kp = kernargs();
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, kp->rk[2 * i], 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, kp->rk[2 * i + 1], 0x96);
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    return u32x4{c0, c1, c2, c3};
}

// Lane masks.  The step's predicates are built as 64-bit lane masks (SGPR
// pairs): lm() of a single comparison is that comparison's own v_cmp result,
// masks combine with scalar &, |, &~, and ib() turns a mask back into this
// lane's bool for a select at no cost.  (__ballot of a composite bool such as
// a && b would make the compiler materialise the bool in a VGPR and compare
// it again: two VALU per ballot.)  Negations are only ever taken inside a
// positive mask, so dead lanes (inert nodes) never satisfy a predicate.
__device__ __forceinline__ uint64_t lm(bool cmp) { return __ballot(cmp); }
// Branch hints for the wave-uniform rare paths: the common path falls through
// (a taken s_cbranch restarts the wave's instruction fetch).
#define RARE(x) __builtin_expect(!!(x), 0)
#define LIKELY(x) __builtin_expect(!!(x), 1)
__device__ __forceinline__ bool ib(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
// x + 1 on the lanes of m: one v_addc_co_u32 with the mask as carry-in (the
// compiler would emit a v_cndmask and a v_add)
__device__ __forceinline__ int32_t inc_if(int32_t x, uint64_t m) {
    int32_t y;
    uint64_t carry;
    asm("v_addc_co_u32_e64 %0, %1, 0, %2, %3" : "=v"(y), "=s"(carry) : "v"(x), "s"(m));
    return y;
}
// x - 1 on the lanes of m: one v_subbrev_co_u32 (x - 0 - borrow) with the mask as borrow-in
__device__ __forceinline__ int32_t dec_if(int32_t x, uint64_t m) {
    int32_t y;
    uint64_t borrow;
    asm("v_subbrev_co_u32_e64 %0, %1, 0, %2, %3" : "=v"(y), "=s"(borrow) : "v"(x), "s"(m));
    return y;
}

// Step counters of a wave.  add(m, c) adds popcount(m) -- the lanes where
// counter c's event happened -- into the wave-uniform (SGPR) total of counter
// c, two 16-bit counters per word (a wave's count per step is < 2^16).  Called
// in wave-uniform control flow, where a lane mask covers the whole wave.
struct Counters {
    uint32_t s[NCW];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < NCW; ++i) s[i] = 0;
    }
    __device__ __forceinline__ void add(uint64_t m, int c) {
        s[COUNTER_SLOT[c] >> 1] += (uint32_t)__popcll(m) << (16 * (COUNTER_SLOT[c] & 1));
    }
};
// The per-message handlers of batch_kernel run in divergent control flow and
// report no counters.
struct NoCounters {
    __device__ __forceinline__ void add(uint64_t, int) {}
};

// drop_ppm == 0 (no drop draws at all), tested per use on an opaque copy of
// the threshold: made once, the compiler keeps it as a lane mask live across
// the step loop, spilled into a VGPR lane and reloaded in every phase
__device__ __forceinline__ bool no_drops(const DevParams& p) {
    uint32_t thr = p.drop_thr16;
    asm("" : "+s"(thr));
    return thr == 0;
}

// The network faults a step kernel is built for (its NET template argument):
// NET_DROP, seeded message drops (drop_ppm > 0); NET_PART, partitions
// (partition_period > 0); NET_ISO, leader isolation (churn_ppm > 0, or an
// isolation word written into the state).  A kernel without one of them
// compiles its checks out (per vote / tick round: the drop compares of both
// directions, the partition-side extract and compare, or the isolated-sender
// compare; per step: H's isolation bookkeeping); NET_ALL decides drops at run
// time.  NET_CMDLOW: the harness's commands go to the lowest-id LEADER with
// no per-group limit (cmd_mode LOWEST_LEADER, cmd_limit 0), fixed at compile
// time instead of two run-time selects per step.  The host picks the kernel
// from the engine's raft_params (raft_engine.hip step_fn).
constexpr int NET_DROP = 1, NET_PART = 2, NET_ISO = 4, NET_CMDLOW = 8;
constexpr int NET_ALL = NET_DROP | NET_PART | NET_ISO;
// no drop can happen: compile-time in a kernel built without NET_DROP, and
// at run time (drop_ppm == 0) in a NET_ALL kernel
template <int NET>
__device__ __forceinline__ bool drops_off(const DevParams& p) {
    if constexpr (!(NET & NET_DROP)) return true;
    else if constexpr (NET == NET_ALL) return no_drops(p);
    else return false;
}

__device__ __forceinline__ u32x4 draw(const DevParams& p, uint32_t c0, uint32_t gid, uint32_t purpose, uint32_t sub) {
    return philox4x32_10(c0, gid, purpose, sub, p.key0, p.key1);
}

// Phase timing (diagnostic builds only, -DRAFT_PROFILE_PHASES): s_memtime
// deltas per step phase, summed per wave in SGPRs and added to a global
// array at the end of the launch.  Never compiled into the product build.
enum { PH_T = 0, PH_JOBS, PH_H, PH_V, PH_D, PH_A, PH_C, PH_K, PH_TDRAW, PH_CNT, PH_N };
struct PhaseClock {
#ifdef RAFT_PROFILE_PHASES
    uint64_t last, acc[PH_N];
    __device__ __forceinline__ void start() {
        last = __builtin_amdgcn_s_memtime();
        for (int k = 0; k < PH_N; ++k) acc[k] = 0;
    }
    __device__ __forceinline__ void mark(int k) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        acc[k] += now - last;
        last = now;
    }
#elif defined(RAFT_PHASE_MARKS)
    // ISA inspection builds: an assembly comment at each phase end
    __device__ __forceinline__ void start() {}
    template <class I>
    __device__ __forceinline__ void mark(I k) { asm volatile(";@PHASE_END %0" ::"i"((int)k)); }
#else
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void mark(int) {}
#endif
};

// Branch statistics (diagnostic builds only, -DRAFT_BRANCH_STATS): how often
// each wave-uniform branch of the step runs, per wave, added into a global
// array at the end of the launch (raft_engine.hip prints it at destroy).
// Never compiled into the product build.
enum { BS_STEPS = 0, BS_T_BUSY, BS_V_PHASE, BS_V_ROUNDS, BS_V_STAGE, BS_D_DEC, BS_D_BACKOFF, BS_D_START,
       BS_A_PHASE, BS_A_ROUNDS, BS_A_STAGE, BS_A_SWAP, BS_A_LOADS, BS_A_HIB, BS_A_SLOW, BS_A_COMMIT,
       BS_H_BUSY, BS_K_DUAL, BS_DRAW, BS_DIRECT_DROP, BS_N };
#ifdef RAFT_BRANCH_STATS
#define BSTAT(c, i) ((c).bs[i] += 1u)
#else
#define BSTAT(c, i) ((void)0)
#endif

// Phase budget (diagnostic builds only, -DRAFT_PHASE_TWICE=1 + PH_x): phase
// x runs a second time first, on copies of the node, context and counters
// whose results are sunk, so SQ_INSTS_VALU / SALU of that build minus the
// product build's is the phase's dynamic instruction count (DESIGN.md §4.5,
// scripts/phase_budget.sh).  Never compiled into the product build.
#ifndef RAFT_PHASE_TWICE
#define RAFT_PHASE_TWICE 0
#endif
#define RAFT_TWICE(PH, CALL)                                                        \
    if constexpr (RAFT_PHASE_TWICE == (PH) + 1) {                                  \
        auto c2 = c;                                                               \
        auto n2 = n;                                                               \
        auto k2 = cnt;                                                             \
        CALL;                                                                      \
        sink_copy(n2, k2);                                                         \
    }

// One replica's scalar state, by reference.
struct Rep {
    int32_t &term, &voted, &role, &commit, &last, &phys, &elec, &phase, &retry;
    uint32_t& fl;
    int32_t &t1, &t2;          // log-tail cache: term of log[last-1], log[last-2]
    uint32_t& c1;              //                 cmd  of log[last-1]
};

// ---- timer / consumer (Commons.kt:10-31, RaftServer.kt:50-69) -------------
// `launch { channel.send(FOLLOWER) }` (RaftServer.kt:241, :261, :266), S-5: an
// idle consumer re-arms the timer (reset() with a fresh draw, resolved once
// at the end of the step because the draw is a pure function of (step, group,
// replica), S-9); a consumer busy in leaderElection() queues the reset.
__device__ __forceinline__ uint32_t follower_sent(uint32_t fl) {
    return (fl & FL_ELECTING) ? FL_PRST : (FL_ARMED | FL_DRAW);
}

// The handlers below are written as predicated selects (applied on the lanes
// of the mask `act`) with at most one optional load and one optional store,
// not as nested ifs: in SIMT every branch side costs the whole wave, and
// branch merges cost register copies.  Their predicates are lane masks (see
// lm()), which also work in the divergent per-message loops of batch_kernel
// (inactive lanes are simply absent from every mask).  Semantics are exactly
// the reference's (cited per line).

// ---- Log<T> (Commons.kt:47-74) over one replica's HBM slots ---------------
// The 2-deep tail cache answers every steady-state read (prev checks, the
// newest entry, vote last-terms); HBM is read for older slots and when the
// ghost tail resurfaces a stale slot.
__device__ __forceinline__ int32_t cached_term(int32_t last, int32_t t1, int32_t t2, int32_t j) {
    return j == last - 1 ? t1 : t2;                    // valid for j in {last-1, last-2}
}

// Log.add(i, e) for 0 <= i <= lastIndex, the only indices its callers pass:
// appendCommand adds at lastIndex, and append() adds at prevLogIndex + 1 only
// after the consistency check passed (prevLogIndex == -1 or < lastIndex).
//   i == lastIndex: :58-61, log.add(entry) appends at the PHYSICAL end (Q1);
//   i <  lastIndex: :63-66, log[i] = entry, lastIndex = i + 1, no shrink.
// The build refuses an append beyond log_cap (counted, never wrapped).
//
// TB (RAFT_MODE_TEXTBOOK): an array log instead -- slot i is written and
// everything after it dropped (no ghost tail); physLen is the high-water mark.
//
// miss: the lanes whose write is a reference access below the window (the
// overwrite branch, or any textbook write, at i < physLen - W); an append at
// physLen never is.
// CHK: count window misses (the log is a log_window ring; a flat log never misses).
// RNG: the log is a ring, so slots are masked (a flat log's never wrap).
// The caller passes app = lm(i == lastIndex) and ige1 = lm(i >= 1): it has
// made (or can fold) those comparisons already, and a comparison re-used in
// another basic block would be re-materialised through a VGPR (lm()).
// AT_END: i == lastIndex on every lane (appendCommand).
template <bool TB, bool CHK, bool RNG, bool AT_END = false>
__device__ __forceinline__ void log_add(const LogView& lv, Rep n, int32_t i, Entry e, uint64_t act, uint64_t app,
                                        uint64_t ige1, uint64_t& wrote, uint64_t& overflow, uint64_t& miss) {
    const int32_t last = n.last, phys = n.phys;
    if constexpr (AT_END) app = ~0ull;
    const uint64_t ghost = TB ? 0ull : app & lm(phys != last);   // the stale slot log[last] becomes the last entry
    overflow = TB ? act & lm(i >= lv.cap) : act & app & lm(phys >= lv.cap);
    wrote = act & ~overflow;
    miss = CHK ? (TB ? wrote : wrote & ~app) & lv.miss(i, phys) : 0ull;
    // the one slot the new tail cache needs from HBM
    const uint64_t ld = wrote & (ghost | (AT_END ? 0ull : ~app & ige1 & lm(i != last - 1)));
    const bool ap = ib(app);
    // the new tail cache without HBM (every value but the loaded slot's)
    int32_t t1 = e.term;
    uint32_t c1 = e.cmd;
    int32_t t2 = ap ? n.t1 : (i == 0 ? 0 : n.t2);
    // rare: the slot is read only if some lane of the wave needs it, and its
    // value is consumed inside the branch, so the wave waits (vmcnt, which
    // also counts its earlier log stores) only when a load was issued
    if (ld) {
        if (ib(ld)) {
            const uint2 g = *lv.template at<RNG>(AT_END ? last : (ap ? last : i - 1));
            t1 = ap ? (int32_t)g.x : t1;                    // ghost: log[last] is the new last entry
            c1 = ap ? g.y : c1;
            t2 = ap ? t2 : (int32_t)g.x;                    // overwrite: log[i-1] becomes second-to-last
        }
    }
    const bool w = ib(wrote);
    if (w) *lv.template at<RNG>((ap && !TB) ? phys : i) = make_uint2((uint32_t)e.term, e.cmd);
    n.t1 = w ? t1 : n.t1;
    n.c1 = w ? c1 : n.c1;
    n.t2 = w ? t2 : n.t2;
    if constexpr (TB) n.phys = w ? max(phys, i + 1) : phys;
    else n.phys = inc_if(phys, wrote & app);
    n.last = AT_END ? inc_if(last, wrote) : (w ? i + 1 : last);
}

// ---- vote() (RaftServer.kt:228-251), applied on the lanes of act ----------
// gapw: the lanes whose log.get(lastIndex - 1) is below the log_window
// (physLen - lastIndex >= W), for the window-miss count (CHK).
// hasl: the lanes with lastIndex >= 1 (the caller's mask; no handler of a
// RequestVote phase changes a log).  fsent = follower_sent(fl): made once per
// phase by the caller (only T and D change FL_ELECTING).
template <bool TB, bool CHK, class CNT>
__device__ __forceinline__ void vote_handler(Rep n, uint64_t act, int32_t id, int32_t rt, int32_t rc, int32_t rli,
                                             int32_t rlt, uint64_t gapw, uint64_t hasl, uint32_t fsent, CNT& cnt,
                                             int32_t& resp_term, uint64_t& granted) {
    if constexpr (TB) {
        // textbook: a higher term is adopted whatever the answer (Q5 adopts it
        // only on a grant); grant iff votedFor is free or the candidate and the
        // candidate's log is at least as up to date; the self-vote changes nothing
        const uint64_t higher = act & lm(rt > n.term);
        const bool h = ib(higher);
        n.fl |= ib(higher & lm(n.role != RAFT_FOLLOWER)) ? fsent : 0u;
        n.term = h ? rt : n.term;
        n.voted = h ? -1 : n.voted;
        n.role = h ? (int32_t)RAFT_FOLLOWER : n.role;
        const uint64_t elig = act & lm(rt == n.term) & (lm(n.voted == -1) | lm(n.voted == rc));
        const uint64_t logrej = hasl & (lm(rlt < n.t1) | (lm(rlt == n.t1) & lm(rli < n.last)));
        granted = elig & ~logrej;
        cnt.add(elig & hasl, RAFT_C_VOTE_LOG_READS);
        if constexpr (CHK) cnt.add(elig & hasl & gapw, RAFT_C_LOG_WINDOW_MISS);     // log.get(lastIndex - 1)
        cnt.add(granted, RAFT_C_VOTES_GRANTED);
        n.voted = ib(granted) ? rc : n.voted;
        n.fl |= ib(granted & lm(rc != id)) ? fsent : 0u;
        resp_term = n.term;
        return;
    }
    const uint64_t higher = lm(rt > n.term);                                    // :229-231
    const uint64_t logrej = hasl & (lm(rlt < n.t1) | (lm(rlt == n.t1) & lm(rli < n.last)));   // :232-236 (Q5)
    const uint64_t up = act & higher & ~logrej;                                 // :237-242
    granted = up | (act & lm(rt == n.term) & lm(n.voted == rc));                // :230
    cnt.add(act & higher & hasl, RAFT_C_VOTE_LOG_READS);
    if constexpr (CHK) cnt.add(act & higher & hasl & gapw, RAFT_C_LOG_WINDOW_MISS);   // :233 log.get
    cnt.add(granted, RAFT_C_VOTES_GRANTED);
    const bool u = ib(up);
    n.fl |= u ? fsent : 0u;                                                     // :241
    n.term = u ? rt : n.term;
    n.voted = u ? rc : n.voted;
    n.role = u ? (int32_t)RAFT_FOLLOWER : n.role;
    resp_term = n.term;                                                         // :246-249
}

// ---- append() (RaftServer.kt:253-287), applied on the lanes of act --------
// Returns the lanes where the reference throws (Log.get with prevLogIndex <
// -1): those calls have no response.  dprev = term of this replica's
// log[prev], read by the caller ahead of time (valid whenever 0 <= prev <
// lastIndex).
//
// TB: a request with a stale term is refused with no state change; the entry
// is written only if the slot is absent or holds another term (dnext = term of
// this replica's log[prev+1], valid whenever 0 <= prev+1 < lastIndex); the
// commit follows leaderCommit only after the consistency check, up to the last
// entry the request vouches for, and never goes down.
//
// CHK: the log is a log_window ring: mask slots, count window misses.
// at_last = lm(prev + 1 == lastIndex), p0 = lm(prev >= 0), other = lm(rlead != id):
// the caller's masks (see log_add); fsent = follower_sent(fl), made once per
// phase (see vote_handler).
template <bool TB, bool CHK, class CNT>
__device__ __forceinline__ uint64_t append_handler(Rep n, uint64_t act, int32_t id, const LogView& lv, int32_t rt,
                                                   int32_t rlead, int32_t prev, int32_t prevTerm, uint64_t has,
                                                   Entry e, int32_t lcommit, int32_t dprev, int32_t dnext,
                                                   uint64_t at_last, uint64_t p0, uint64_t other, uint32_t fsent,
                                                   CNT& cnt, int32_t& resp_term, uint64_t& success,
                                                   uint64_t& stored) {
    if constexpr (TB) act &= ~lm(rt < n.term);
    const uint64_t up = act & lm(rt > n.term);                                  // :257-262
    const uint64_t fol = up | (act & other);                                    // :264-268 (Q3): rlead != id
    const bool u = ib(up), f = ib(fol);
    n.fl |= f ? fsent : 0u;
    n.term = u ? rt : n.term;
    n.voted = u ? -1 : n.voted;
    n.role = f ? (int32_t)RAFT_FOLLOWER : n.role;
    if constexpr (!TB) {
        const uint64_t cu = act & lm(lcommit > n.commit);                       // :270-272 (Q4)
        const int32_t cc = min(lcommit, n.last);
        const uint64_t regr = cu & lm(cc < n.commit);
        if (RARE(regr)) cnt.add(regr, RAFT_C_COMMIT_REGRESSIONS);
        n.commit = ib(cu) ? cc : n.commit;
    }
    const uint64_t lgt = lm(n.last > prev);                                     // :274-276
    const uint64_t rd = p0 & lgt;                                               // log.get(prev) is read
    const uint64_t thrown = lm(prev < -1) & lgt;                                // ... and throws (prev < -1)
    cnt.add(act & rd, RAFT_C_PREV_READS_FOLLOWER);
    if constexpr (CHK) cnt.add(act & rd & lv.miss(prev, n.phys), RAFT_C_LOG_WINDOW_MISS);   // :276
    success = act & (lm(prev == -1) | (rd & lm(dprev == prevTerm)));
    uint64_t wrote, ovf, wmiss;
    uint64_t same = 0;                                                          // TB: entry already there
    if constexpr (TB) {
        const uint64_t rd = success & has & lm(prev + 1 < n.last);              // TB: reads log[prev + 1]
        if constexpr (CHK) cnt.add(rd & lv.miss(prev + 1, n.phys), RAFT_C_LOG_WINDOW_MISS);
        same = rd & lm(dnext == e.term);
    }
    log_add<TB, CHK, CHK>(lv, n, prev + 1, e, success & has & ~same, at_last, p0, wrote, ovf, wmiss);   // :278 (Q2, Q10)
    cnt.add(wrote, RAFT_C_ENTRY_WRITES);
    cnt.add(ovf, RAFT_C_LOG_OVERFLOW);
    if constexpr (CHK) cnt.add(wmiss, RAFT_C_LOG_WINDOW_MISS);                 // the write
    stored = wrote | same;                                                      // TB: the entry is in place
    if constexpr (TB) {
        const int32_t lastNew = prev + 1 + (ib(wrote | same) ? 1 : 0);
        const int32_t cc = max(n.commit, min(lcommit, lastNew));
        n.commit = ib(success & lm(lcommit > n.commit)) ? cc : n.commit;
    }
    resp_term = n.term;                                                         // :282-285
    return thrown;
}

// ---- appendCommand() (RaftServer.kt:100-107), applied on the lanes of act -
template <bool TB, bool CHK, class CNT>
__device__ __forceinline__ void append_command(Rep n, uint64_t act, const LogView& lv, uint32_t cmd, CNT& cnt) {
    uint64_t wrote, ovf, wmiss;
    log_add<TB, CHK && TB, CHK, true>(lv, n, n.last, Entry{n.term, cmd}, act, ~0ull, 0ull, wrote, ovf, wmiss);   // the reference
    cnt.add(act, RAFT_C_COMMANDS);                                              // appends at physLen: no miss;
    cnt.add(ovf, RAFT_C_LOG_OVERFLOW);                                          // TB writes slot lastIndex
    if constexpr (CHK && TB) cnt.add(wmiss, RAFT_C_LOG_WINDOW_MISS);
}

// ---------------------------------------------------------------------------
// Lane-per-replica machinery
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t bcast(int32_t v, int src_lane) {
    return __builtin_amdgcn_ds_bpermute(src_lane << 2, v);
}
__device__ __forceinline__ uint32_t bcastu(uint32_t v, int src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int32_t)v);
}

// One lane's replica plus the group words every lane of the group replicates.
struct Node {
    int32_t term, voted, role, commit, last, phys, elec, phase, retry;
    uint32_t fl;
    int32_t t1, t2;
    uint32_t c1;
    int32_t nx, mc;           // primary session (owner s0) towards this replica
    int32_t iso, cmdc, s0;    // group words
    __device__ __forceinline__ Rep rep() {
        return Rep{term, voted, role, commit, last, phys, elec, phase, retry, fl, t1, t2, c1};
    }
};

// keeps a phase copy's results alive (RAFT_PHASE_TWICE builds)
template <class NODE, class CNT>
__device__ __forceinline__ void sink_copy(const NODE& n, const CNT& k) {
    asm volatile("" ::"v"(n.term), "v"(n.voted), "v"(n.role), "v"(n.commit), "v"(n.last), "v"(n.phys));
    asm volatile("" ::"v"(n.elec), "v"(n.phase), "v"(n.retry), "v"(n.fl), "v"(n.t1), "v"(n.t2), "v"(n.c1));
    asm volatile("" ::"v"(n.nx), "v"(n.mc), "v"(n.iso), "v"(n.cmdc), "v"(n.s0));
#pragma unroll
    for (int i = 0; i < NCW; ++i) asm volatile("" ::"s"(k.s[i]));
}

template <int R>
struct Lanes {
    static constexpr int GPW = 64 / R;                 // groups per wave
    static constexpr uint32_t ALL = (1u << R) - 1u;
    static constexpr int MAJ = R / 2 + 1;              // RaftServer.kt:44
    // Per-step Philox jobs (S-9), one per lane of the group, all evaluated in
    // ONE Philox pass of the wave: J_HARNESS, then the NQ timer quads (the
    // per-replica draw word, used by the election timer and the backoff), then
    // the NCH drop-word chunks of the first leader to tick and of the first
    // RequestVote sender.  Jobs that do not fit in R lanes are drawn on demand.
    static constexpr int NQ = (R + 3) / 4;             // Philox calls per 4-replica quad
    static constexpr int NCH = (R + 2) / 4;            // drop-word chunks per sender: ceil((R - 1) / 4)
    static constexpr int J_TIMER = 1, J_TICK = 1 + NQ, J_VOTE = 1 + NQ + NCH;
    static constexpr bool JOBS = 1 + NQ <= R;          // harness + timer quads fit
    static constexpr bool TICK_JOB = JOBS && J_TICK + NCH <= R;
    static constexpr bool VOTE_JOB = JOBS && J_VOTE + NCH <= R;
    // one chunk per sender: a pass of the group's R lanes covers every sender
    static constexpr bool SENDERS_STAGED = NCH == 1;

    // lanes whose replica index is s (compile-time masks)
    // lanes whose replica index is <= s
    static constexpr uint64_t lanes_upto(int s) {
        uint64_t m = 0;
        for (int q = 0; q <= s; ++q) m |= lanes_of(q);
        return m;
    }
    static constexpr uint64_t lanes_of(int s) {
        uint64_t m = 0;
        for (int j = 0; j < GPW; ++j) m |= 1ull << (j * R + s);
        return m;
    }
    // lanes whose replica index is in [a, b) (compile-time masks)
    static constexpr uint64_t lanes_in(int a, int b) {
        uint64_t m = 0;
        for (int q = a; q < b && q < R; ++q) m |= lanes_of(q);
        return m;
    }
    // the job lanes of the step's Philox pass, and those holding a sender's
    // second drop-word chunk (R > 5)
    static constexpr uint64_t TIMER_LANES = lanes_in(J_TIMER, J_TICK);
    static constexpr uint64_t TICK_LANES = lanes_in(J_TICK, J_VOTE);
    static constexpr uint64_t VOTE_LANES = lanes_in(J_VOTE, R);
    static constexpr uint64_t CHUNK1_LANES = lanes_in(J_TICK + 1, J_VOTE) | lanes_in(J_VOTE + 1, R);
};

// Per-lane, per-step context.
template <int R>
struct Ctx {
    uint32_t t;
    uint32_t wg0, gg0;        // wave-uniform: engine-local / global id of the wave's first group
    int r, base;              // replica index, first lane of the group
    bool live;                // lane holds a real replica (whole groups are live or not)
    int iso;                  // isolated replica this step, -1 if none
    uint64_t iso_me;          // lanes whose replica is the isolated one (lm(r == iso), made once per step)
    uint32_t part;            // replicas on side B of this step's partition
    uint64_t part_me;         // lanes whose replica is on side B (lm(part >> r & 1), made once per step)

    u32x4 job;                // this lane's Philox job of the step (Lanes::JOBS), dead after the fetch
    uint32_t* jl;             // the wave's LDS staging of the job words, [64 lanes][4]
    uint32_t* tl;             // the wave's vote-tally words, [16] (one per group at base >> 2, R >= 4)
    uint32_t lead;            // the group's LEADER bits at the end of the last step (loop-carried)
    uint32_t tw, dwt, dwv;    // this lane's timer word and prefetched tick / vote drop words
    PhaseClock clk;
#ifdef RAFT_BRANCH_STATS
    uint32_t bs[BS_N];
#endif
    int s_tick, s_vote;       // senders whose drop words the jobs hold (-1 none)
    uint2* lr;                // this replica's log row: slot 0 (its wave's block, its lane)

    // opaque result: tested against 0, (b >> base) & ALL would be rewritten as
    // b & (ALL << base) != 0 with the mask ANDs moved from SALU to VALU
    __device__ __forceinline__ uint32_t gbits(uint64_t b) const {
        uint32_t g = (uint32_t)(b >> base) & Lanes<R>::ALL;
        asm("" : "+v"(g));
        return g;
    }
    __device__ __forceinline__ int src(int s) const { return base + s; }
    // derived on demand instead of held in VGPRs (register pressure)
    __device__ __forceinline__ uint32_t j() const {                 // group within the wave: base / R
        return ((uint32_t)base * ((65536u + R - 1) / R)) >> 16;
    }
    __device__ __forceinline__ uint32_t gid() const { return gg0 + j(); }          // global group id
    __device__ __forceinline__ int64_t idx() const { return (int64_t)wg0 * R + base + r; }   // g * R + r
    // This replica's log.  The wave's block and the ring's geometry are
    // re-derived from the kernarg segment where they are used (kept live
    // across the step loop they would pin SGPRs, see kernargs()).
    // RING = false: a flat log's row stride is log_cap itself (one SGPR fewer)
    template <bool RING = true>
    __device__ __forceinline__ LogView log(const DevParams& p) const {
        return LogView{lr, (uint32_t)(RING ? p.nslots : p.cap), p.wmask, p.cap, p.W};
    }
};

// The lanes whose message s -> d is lost (S-7): churn isolation, partition
// sides, or the drop uniform j = 2*dd + b (word dd, half b); self never lost.
// d is this lane's replica (c.iso_me, c.part_me are its isolation and
// partition-side masks).
// mself: the lanes where d == s (the caller's lm(r == s)).
// lost_net: the network part (isolation, partition) of sender s's messages,
// made once per round for both directions.  (Skipping its compares in waves
// with no isolation or partition measured slower: the branches cost more
// SALU issue than the VALU they save.)
template <int R, int NET>
__device__ __forceinline__ uint64_t lost_net(const Ctx<R>& c, int s) {
    uint64_t net = 0;
    if constexpr ((NET & NET_ISO) != 0) net = lm(s == c.iso) | c.iso_me;        // iso = -1: nobody isolated
    if constexpr ((NET & NET_PART) != 0)
        net |= c.part_me ^ lm(__builtin_amdgcn_ubfe(c.part, (uint32_t)s, 1u));    // s, d on two sides
    return net;
}
template <int NET>
__device__ __forceinline__ uint64_t lost(const DevParams& p, uint64_t net, uint64_t mself, uint32_t dw, int b) {
    if constexpr (!(NET & NET_DROP)) return ~mself & net;
    else return ~mself & (net | lm(((dw >> (16 * b)) & 0xFFFFu) < p.drop_thr16));
}

// 16-bit drop uniforms of sender s for this lane as destination d (S-9):
// word dd = (d < s ? d : d - 1) of Philox(t, gid, purpose, s | (dd >> 2) << 8).
// drop_word_direct evaluates it in this lane (one Philox pass serves every
// destination of the wave); drop_word takes it from the step's jobs when they
// hold sender s (first_job = J_TICK / J_VOTE), else draws it directly.
// drop_word draws only for groups with `act`, and MUST be called in
// group-uniform control flow.
template <int R>
__device__ __forceinline__ uint32_t drop_word_direct(const DevParams& p, const Ctx<R>& c, uint32_t purpose, int s) {
    const int dd = c.r < s ? c.r : c.r - 1;
    const int q = dd < 0 ? 0 : dd;
    const u32x4 w = kdraw(p, c.t, c.gid(), purpose, (uint32_t)s | ((uint32_t)(q >> 2) << 8));
    return word_of(w, q & 3);
}

// Word q of the jobs that this lane's group drew from its job lane first_job
// on, read from the wave's LDS staging (one ds_read_b32 instead of four
// ds_bpermute and a select).  The staging is [64 lanes][4 words], so word
// q & 3 of the job of lane first_job + (q >> 2) is word 4 * first_job + q of
// the group's rows: no split into lane and word.  Dead lanes may address past
// their wave's rows; their words are never used.
template <int R>
__device__ __forceinline__ uint32_t job_word(const Ctx<R>& c, int first_job, int q) {
    return c.jl[((c.base + first_job) << 2) + q];
}

template <int R, bool HAVE_JOB, int NET>
__device__ __forceinline__ uint32_t drop_word(const DevParams& p, Ctx<R>& c, uint32_t purpose, uint64_t act,
                                              int s, uint32_t prefetched, int s_job) {
    if (drops_off<NET>(p)) return 0u;
    uint32_t w = 0;
    uint64_t need = act;
    if constexpr (HAVE_JOB) {
        w = prefetched;
        need = act & lm(s != s_job);
    }
    if (RARE(need)) {
        BSTAT(c, BS_DIRECT_DROP);
        if (ib(need)) w = drop_word_direct(p, c, purpose, s);
    }
    return w;
}

// This lane's word of the drop-word chunks the step's jobs drew for sender s
// (first_job = J_TICK / J_VOTE).  MUST be called in group-uniform control flow.
// Word dd = (d < s ? d : d - 1) for destination d = this lane; the sender's
// own lane (d == s, never lost) reads word d, a valid word it ignores.
template <int R>
__device__ __forceinline__ uint32_t job_drop_word(const Ctx<R>& c, int first_job, int s) {
    return job_word(c, first_job, dec_if(c.r, lm(c.r > s)));
}

// The step's per-replica draw word, word r & 3 of Philox(t, gid, TIMER, r >> 2)
// (S-9): the election timeout and the candidate backoff both scale it (a
// replica never needs both in one step).  MUST be called in group-uniform
// control flow.
template <int R>
__device__ __forceinline__ uint32_t timer_word(const DevParams& p, const Ctx<R>& c) {
    if constexpr (Lanes<R>::JOBS) {
        return c.tw;
    } else {
        return word_of(kdraw(p, c.t, c.gid(), RAFT_RNG_TIMER, (uint32_t)(c.r >> 2)), c.r & 3);
    }
}

// TB: RAFT_MODE_TEXTBOOK (include/raft_engine.h), compiled as its own kernel
// so the reference-parity kernel carries none of it.
// RING: the log is a log_window ring, so every reference access is checked
// against the window (a flat log keeps every slot: no access can miss).
template <int R, bool TB, bool RING, int NET>
struct Stepper {
    using L = Lanes<R>;
    static constexpr int MAJ = L::MAJ;
    static constexpr uint32_t ALL = L::ALL;

    // ---- session rows (S-8): the primary lives in n.nx / n.mc, the others in spill
    // (rare: a session other than the primary starts or ticks; the spill
    // base is re-read from the kernarg segment, see kernargs())
    __device__ __forceinline__ static void spill_store(const DevParams&, const Ctx<R>& c, const Node& n, int s) {
        const KernArgs kp = kernargs();
        int32_t* sp = kp->spill;
        sp[c.idx() * R + s] = n.nx;
        sp[kp->GR * R + c.idx() * R + s] = n.mc;
    }
    __device__ __forceinline__ static void spill_load(const DevParams&, const Ctx<R>& c, Node& n, int s) {
        const KernArgs kp = kernargs();
        const int32_t* sp = kp->spill;
        n.nx = sp[c.idx() * R + s];
        n.mc = sp[kp->GR * R + c.idx() * R + s];
    }

    // The flags after leaderElection() returns (S-5): the queued FOLLOWER
    // send first, then the final state -- LEADER starts the heartbeat session
    // (RaftServer.kt:66), FOLLOWER re-arms the timer (:64).
    __device__ __forceinline__ static uint32_t end_flags(uint32_t f, int32_t role) {
        const bool prst = f & FL_PRST;
        f &= ~(FL_ELECTING | FL_PRST | FL_BACKOFF | (0xFFu << PEND_SH) | (0xFu << VOTES_SH) | (0xFu << LATCH_SH));
        f |= prst ? (FL_ARMED | FL_DRAW) : 0u;
        f |= role == RAFT_LEADER ? FL_HB : (role == RAFT_FOLLOWER ? (FL_ARMED | FL_DRAW) : 0u);
        return f;
    }

    // appendRequestAndLeaderHeartbeat() entry (RaftServer.kt:109-113) for every
    // lane of `starting`, in ascending replica order within a group: each
    // start takes over the primary slot, the previous owner's row goes to spill.
    // Called in wave-uniform control flow.
    __device__ __forceinline__ static void start_sessions(const DevParams& p, const Ctx<R>& c, Node& n, uint64_t starting,
                                                          Counters& cnt) {
        if (starting == 0) return;
        cnt.add(starting, RAFT_C_LEADERS_ELECTED);
        const uint32_t sb = c.gbits(starting);
#pragma unroll
        for (int s = 0; s < R; ++s) {
            if (!(starting & L::lanes_of(s))) continue;                   // wave-uniform
            const int32_t cs = bcast(TB ? n.last : n.commit, c.src(s));  // TB: nextIndex = lastIndex + 1
            const uint64_t mst = lm((sb >> s) & 1u);
            const uint64_t msp = mst & lm(n.s0 >= 0) & lm(n.s0 != s);
            if (RARE(msp)) {
                if (ib(msp)) spill_store(p, c, n, n.s0);
            }
            const bool st = ib(mst);
            n.s0 = st ? s : n.s0;
            n.nx = st ? cs + 1 : n.nx;                                    // :112 (Q8)
            n.mc = st ? 0 : n.mc;                                         // :113
        }
    }

    // One fixedRateTimer tick of leader s (RaftServer.kt:115-176) in every
    // group with `tk` (group-uniform s, runtime; s = 0 where !tk).  Requests
    // are built from the leader's tick-start snapshot (S-4) and delivered to
    // all destinations at once; responses are replayed in destination order.
    // Predicated, called in wave-uniform control flow.
    template <bool STAGED = false>
    __device__ __forceinline__ static void tick(const DevParams& p, Ctx<R>& c, Node& n, uint64_t mtk, int s,
                                                uint32_t fs, Counters& cnt) {
        const int sl = c.src(s);
        BSTAT(c, BS_A_ROUNDS);
        // the leader's tick-start snapshot and this destination's drop word,
        // all cross-lane reads issued together (one LDS round trip)
        const int32_t role_s = bcast(n.role, sl);
        const int32_t Lterm = bcast(n.term, sl), Lcommit = bcast(n.commit, sl), Llast = bcast(n.last, sl);
        const int32_t Lt1 = bcast(n.t1, sl), Lt2 = bcast(n.t2, sl);
        const uint32_t Lc1 = bcastu(n.c1, sl);
        const uint64_t mme = lm(c.r == s);
        const uint64_t run = mtk & lm(role_s != RAFT_FOLLOWER);
        uint32_t dw;
        if constexpr (STAGED) dw = drops_off<NET>(p) ? 0u : job_drop_word(c, s, s);   // stage_sender_chunks
        else dw = drop_word<R, L::TICK_JOB, NET>(p, c, RAFT_RNG_APPEND_DROP, run, s, c.dwt, c.s_tick);
        const uint64_t cancel = mtk & ~run & mme;                         // :117 cancel() (S-10)
        if (RARE(cancel)) n.fl &= ib(cancel) ? ~FL_HB : ~0u;
        cnt.add(run & mme, RAFT_C_SESSIONS_TICKED);
        const uint64_t swap = run & lm(n.s0 != s);                        // swap the session in (rare)
        if (RARE(swap)) {
            BSTAT(c, BS_A_SWAP);
            if (ib(swap)) {
                if (n.s0 >= 0) spill_store(p, c, n, n.s0);
                spill_load(p, c, n, s);
                // wait for the loads here: consumed after the branch, they
                // would put a vmcnt wait (which also counts this tick's log
                // store) on the common path
                asm volatile("" :: "v"(n.nx), "v"(n.mc));
            }
        }
        n.s0 = ib(swap) ? s : n.s0;
        // build this destination's request (RaftServer.kt:122-132).  With
        // prev = i - 2: Log.get(prev) throws for prev > lastIndex - 1 (:128,
        // Q11) and log[i-1] for i < 1 (:131), so the request goes out iff
        // -1 <= prev < lastIndex, and carries an entry iff also i <= lastIndex.
        const int32_t i = n.nx, prev = i - 2;
        const uint64_t pge = lm(prev >= -1), plt = lm(prev < Llast), p0 = lm(prev >= 0);
        const uint64_t at_last = lm(prev + 1 == n.last);                  // own log[prev] is the tail (log_add: i == lastIndex)
        const uint64_t ok = run & pge & plt;
        const uint64_t has = pge & lm(i <= Llast);
        cnt.add(ok & p0, RAFT_C_PREV_READS_LEADER);                      // ok = run & pge & plt, p0 within pge
        cnt.add(run & has, RAFT_C_ENTRY_READS_LEADER);
        // RAFT_C_APPEND_SKIPPED (run & ~ok) is not counted here: run covers
        // whole groups, so it is R * SESSIONS_TICKED - APPEND_SENT, which the
        // counter reduction derives (reduce_counters_kernel)
        cnt.add(ok, RAFT_C_APPEND_SENT);
        // every log slot of the tick, resolved up front: the leader's log[prev]
        // and log[i-1], and this replica's own log[prev] (append() :274-276);
        // a handler only writes its own replica's log, so no handler of the
        // tick can change a slot another one reads.  The tail caches answer
        // all but: leader log[prev] below its last two slots, an entry other
        // than the leader's newest, own log[prev] below the last two slots.
        const LogView lv = c.template log<RING>(p);
        const LogView ls = lv.lane(s - c.r);                              // the leader's log
        int32_t lpt = cached_term(Llast, Lt1, Lt2, prev);
        int32_t dpt = ib(at_last) ? n.t1 : n.t2;                          // cached_term(n.last, .., prev)
        int32_t dnt = TB ? cached_term(n.last, n.t1, n.t2, prev + 1) : 0;  // TB: own log[prev+1]
        uint2 lent = make_uint2((uint32_t)Lt1, Lc1);
        const uint64_t ld1 = ok & p0 & lm(prev < Llast - 2);
        const uint64_t ld2 = run & has & lm(i < Llast);
        const uint64_t ld3 = ok & p0 & lm(prev < n.last - 2);
        const uint64_t ld4 = TB ? ok & has & lm(prev + 1 < n.last - 2) : 0ull;
        if (ld1 | ld2 | ld3 | ld4) {                                      // rare: tail-cache misses
            BSTAT(c, BS_A_LOADS);
            if (ib(ld1)) lpt = (int32_t)ls.template at<RING>(prev)->x;
            if (ib(ld2)) lent = *ls.template at<RING>(i - 1);
            if (ib(ld3)) dpt = (int32_t)lv.template at<RING>(prev)->x;
            if (TB && ib(ld4)) dnt = (int32_t)lv.template at<RING>(prev + 1)->x;
            asm volatile("" :: "v"(lpt), "v"(lent.x), "v"(lent.y), "v"(dpt), "v"(dnt));   // wait inside the branch
        }
        int32_t Llo = 0;                                                  // RING: the leader's window floor
        if constexpr (RING) {                                             // window misses (every access counted)
            Llo = bcast(n.phys, sl) - p.W;
            cnt.add(run & p0 & plt & lm(prev < Llo), RAFT_C_LOG_WINDOW_MISS);  // :128 log.get(prevLogIndex)
            cnt.add(run & has & lm(i - 1 < Llo), RAFT_C_LOG_WINDOW_MISS);     // :131 log.get(i - 1)
        }

        // both directions' losses resolved here: a lane mask of comparisons made
        // in an earlier basic block (before the handler's log store) would be
        // re-materialised through a VGPR
        const uint64_t net = lost_net<R, NET>(c, s);
        const uint64_t lreq = ok & lost<NET>(p, net, mme, dw, 0);         // :170-172
        const uint64_t act = ok & ~lreq;
        const uint64_t lresp = act & lost<NET>(p, net, mme, dw, 1);
        int32_t rterm;
        uint64_t succ, stored;
        // no lane of act throws: ok implies prev >= -1
        append_handler<TB, RING>(n.rep(), act, c.r + 1, lv, Lterm, s + 1, prev, lpt, has,
                           Entry{(int32_t)lent.x, lent.y}, Lcommit, dpt, dnt, at_last, p0, ~mme, fs, cnt, rterm, succ,
                           stored);
        // TB, ae_max_entries > 1: the request carries kq = min(E, Llast - i + 1)
        // entries (greeter.proto:37); the first went through append_handler, the
        // rest follow with its rule while every earlier one is in place
        int32_t kq = 1;
        if constexpr (TB) {
            const int32_t E = p.ae_max;
            if (E > 1) {
                kq = min(E, Llast - i + 1);
                int32_t nst = ib(stored) ? 1 : 0;                          // entries in place
                uint64_t in = stored;
                for (int e = 1; e < E; ++e) {
                    const uint64_t req = run & has & lm(e < kq);              // entries the leader reads
                    if (!req) break;                                          // wave-uniform
                    const int32_t j = prev + 1 + e;
                    cnt.add(req, RAFT_C_ENTRY_READS_LEADER);
                    if constexpr (RING) cnt.add(req & lm(j < Llo), RAFT_C_LOG_WINDOW_MISS);
                    const uint64_t m = in & lm(e < kq);
                    // the leader's log[j] (its tail cache for its newest entry)
                    // and this replica's own log[j] term (its tail cache for its
                    // last two)
                    uint2 ent = make_uint2((uint32_t)Lt1, Lc1);
                    int32_t dj = cached_term(n.last, n.t1, n.t2, j);
                    const uint64_t lde = m & lm(j < Llast - 1);
                    const uint64_t rd = m & lm(j < n.last);
                    const uint64_t ldo = rd & lm(j < n.last - 2);
                    if (lde | ldo) {                                          // rare outside catch-up
                        if (ib(lde)) ent = *ls.template at<RING>(j);
                        if (ib(ldo)) dj = (int32_t)lv.template at<RING>(j)->x;
                        asm volatile("" :: "v"(ent.x), "v"(ent.y), "v"(dj));
                    }
                    if constexpr (RING) cnt.add(rd & lv.miss(j, n.phys), RAFT_C_LOG_WINDOW_MISS);
                    const uint64_t same = rd & lm(dj == (int32_t)ent.x);
                    uint64_t wrote, ovf, wmiss;
                    log_add<true, RING, RING>(lv, n.rep(), j, Entry{(int32_t)ent.x, ent.y}, m & ~same,
                                              lm(j == n.last), lm(j >= 1), wrote, ovf, wmiss);
                    cnt.add(wrote, RAFT_C_ENTRY_WRITES);
                    cnt.add(ovf, RAFT_C_LOG_OVERFLOW);
                    if constexpr (RING) cnt.add(wmiss, RAFT_C_LOG_WINDOW_MISS);
                    in = same | wrote;
                    nst = inc_if(nst, in);
                }
                // the follower's commit with every entry in place (the handler
                // applied it for the first; max/min make this idempotent)
                const int32_t cc = max(n.commit, min(Lcommit, prev + 1 + nst));
                n.commit = ib(succ & lm(Lcommit > n.commit)) ? cc : n.commit;
            }
        }
        const uint64_t delivered = act & ~lresp;
        cnt.add(lreq | lresp, RAFT_C_MSG_DROPPED);

        // responses in destination order (S-4).  :146-154 (Q7): a response
        // with a term above the running term adopts it and skips the rest of
        // that response; the running term is the prefix max.
        int32_t T = Lterm;
        uint64_t sdb = 0;                                                 // responses that stepped down
        const uint64_t hib = delivered & lm(rterm > Lterm);
        bool stepdown = false;
        if (RARE(hib)) {                                                  // wave-uniform, rare
            BSTAT(c, BS_A_HIB);
            stepdown = c.gbits(hib) != 0;
            const uint32_t dl = c.gbits(delivered);
#pragma unroll
            for (int q = 0; q < R; ++q) {
                const int32_t rq = bcast(rterm, c.src(q));
                const uint64_t up = lm((dl >> q) & 1u) & lm(rq > T);
                T = ib(up) ? rq : T;
                sdb |= up & L::lanes_of(q);                               // response q stepped down
            }
        }
        const int32_t mc_old = n.mc;
        const uint64_t nd = delivered & ~sdb;
        const uint64_t chk = nd & succ & has;                             // :156-162 (Q9)
        const uint64_t hbk = nd & succ & ~has;                            // :163-164
        const uint64_t nak = nd & ~succ;                                  // :166-167
        if constexpr (TB) {
            // TB: nextIndex += the entries acked, matchIndex = the last one's index
            n.nx = ib(chk) ? n.nx + kq : dec_if(n.nx, nak);
            n.mc = ib(chk) ? prev + 1 + kq : (ib(hbk) ? prev + 1 : mc_old);
            cnt.add(chk, RAFT_C_ENTRIES_ACKED);
            for (int e = 1; e < p.ae_max; ++e) {
                const uint64_t more = chk & lm(e < kq);
                if (!more) break;                                         // wave-uniform
                cnt.add(more, RAFT_C_ENTRIES_ACKED);
            }
        } else {
            n.nx = dec_if(inc_if(n.nx, chk), nak);                       // chk and nak are disjoint
            n.mc = ib(hbk) ? prev + 1 : inc_if(mc_old, chk);
            cnt.add(chk, RAFT_C_ENTRIES_ACKED);
        }
        // commit rule, after each acknowledged entry in destination order:
        // count(matchIndex > commitIndex) >= majority => commitIndex += 1
        int32_t C = Lcommit;
        if (!TB && chk) {                                                 // wave-uniform
            BSTAT(c, BS_A_COMMIT);
            const uint32_t ck = c.gbits(chk);                             // the group's acked responses
            // Closed form (common case).  While no row went down (monotone:
            // an ack raises matchIndex, a nak keeps it), the count of rows
            // above a fixed C after response q never falls as q grows, so
            // "some acked q reaches a majority at C = Lcommit" is the test at
            // the group's LAST acked response q*: rows up to q* as they are
            // after the tick, the rest as before it.  If fewer than a majority
            // of rows ends above Lcommit + 1, a second increment is impossible.
            // Otherwise (a row went down, or a majority ends above Lcommit + 1:
            // a lagging commitIndex, Q9) the replay below runs.
            const uint64_t hi2 = run & lm(n.mc > C + 1);                 // (the ticking groups' rows)
            uint64_t slow = run & lm(n.mc < mc_old);
            if (RARE(hi2)) slow |= lm(__popc(c.gbits(hi2)) >= MAJ);             // wave-uniform, rare
            if (LIKELY(!slow)) {
                const uint64_t upto = lm((ck >> c.r) != 0u);              // rows at or before q*
                const int32_t cur = ib(upto) ? n.mc : mc_old;
                const uint64_t inc = lm(__popc(c.gbits(lm(cur > C))) >= MAJ) & lm(ck != 0u);   // :161-162
                C = inc_if(C, inc);
                cnt.add(inc & L::lanes_of(0), RAFT_C_COMMITS);            // one lane per group
            } else {
                BSTAT(c, BS_A_SLOW);
                // the replay in destination order.  Bit q of the group's acks,
                // pre-shifted so that one v_bcnt adds it (as 16 << q) to the
                // popcount: pc >= (16 << q) + MAJ tests "response q acked and
                // count >= majority" in one compare
                const uint32_t ck16 = ck << 4;
                uint64_t commits = 0;                                     // one lane per increment
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    if (!(chk & L::lanes_of(q))) continue;                // wave-uniform
                    const int32_t cur = ib(L::lanes_upto(q)) ? n.mc : mc_old;   // rows after / before response q
                    const uint32_t gt = c.gbits(lm(cur > C));             // :161
                    const uint32_t pc = __popc(gt) + (ck16 & (16u << q));
                    const uint64_t inc = lm(pc >= (16u << q) + MAJ);      // :162 (whole groups)
                    C = inc_if(C, inc);
                    commits |= inc & L::lanes_of(q);                      // disjoint lanes per q
                }
                cnt.add(commits, RAFT_C_COMMITS);
            }
        }
        if constexpr (TB) {
            // textbook commit rule: N = the majority-th largest matchIndex of the
            // session row (a sorting network over the group's R lanes); commit up
            // to N iff the leader's log[N-1] is of its current term and it did
            // not step down this tick.  COMMITS counts the ticks that advance.
            if (run) {                                                    // wave-uniform
                int32_t v[R];
#pragma unroll
                for (int q = 0; q < R; ++q) v[q] = bcast(n.mc, c.src(q));
#pragma unroll
                for (int a = 0; a < R; ++a)                               // descending
#pragma unroll
                    for (int b = R - 1; b > a; --b) {
                        const int32_t hi = max(v[b - 1], v[b]), lo = min(v[b - 1], v[b]);
                        v[b - 1] = hi; v[b] = lo;
                    }
                const int32_t N = v[MAJ - 1];
                const uint64_t cand = run & lm(!stepdown) & lm(N > C) & lm(N <= Llast);
                int32_t NT = N - 1 == Llast - 1 ? Lt1 : Lt2;
                const uint64_t ldn = cand & lm(N - 1 < Llast - 2);
                if constexpr (RING) cnt.add(cand & mme & lm(N - 1 < bcast(n.phys, sl) - p.W), RAFT_C_LOG_WINDOW_MISS);
                if (ldn) {
                    if (ib(ldn)) NT = (int32_t)ls.template at<RING>(N - 1)->x;
                    asm volatile("" :: "v"(NT));
                }
                const uint64_t adv = cand & lm(NT == Lterm);
                C = ib(adv) ? N : C;
                cnt.add(adv & mme, RAFT_C_COMMITS);
            }
        }
        const bool wb = ib(run & mme);
        const bool sd = wb && stepdown;                                   // :148 + offer(FOLLOWER) :152 (S-6)
        n.term = wb ? T : n.term;
        n.commit = wb ? C : n.commit;
        n.role = sd ? (int32_t)RAFT_FOLLOWER : n.role;
        if constexpr (TB) n.voted = sd ? -1 : n.voted;                    // TB: a new term has no vote yet
        n.fl |= sd ? (fs & (FL_ARMED | FL_DRAW)) : 0u;                    // no reset while electing (S-5)
    }

    // The drop-word chunk of EVERY sender of the group in one Philox pass of
    // the wave (lane r: sender r, the chunk drop_word_direct would draw),
    // staged over the job rows, whose words are all fetched by now.  The
    // second and later vote / tick rounds of a step read their words from LDS
    // (job_drop_word(c, s, s)) instead of one direct pass each.  Called in
    // wave-uniform control flow.
    __device__ __forceinline__ static void stage_sender_chunks(const DevParams& p, Ctx<R>& c, uint32_t purpose) {
        if (drops_off<NET>(p)) return;
        BSTAT(c, purpose == RAFT_RNG_VOTE_DROP ? BS_V_STAGE : BS_A_STAGE);
        const u32x4 w = kdraw(p, c.t, c.gid(), purpose, (uint32_t)c.r);
        *(uint4*)&c.jl[(c.base + c.r) << 2] = make_uint4(w.x, w.y, w.z, w.w);
        asm volatile("" ::: "memory");
    }

    // One RequestVote round: every group with a pending sender delivers the
    // requests of its lowest remaining sender s to all destinations at once.
    // Predicated, called in wave-uniform control flow.
    // mvr: the lanes of groups with a pending sender (the caller's ballot of
    // vtodo != 0); hasl: lanes with lastIndex >= 1 (constant over the phase).
    template <bool STAGED = false>
    __device__ __forceinline__ static void vote_round(const DevParams& p, Ctx<R>& c, Node& n, Counters& cnt,
                                                      uint32_t& vtodo, uint64_t mvr, uint32_t send, int32_t qt,
                                                      int32_t qli, int32_t qlt, uint64_t gapw, uint64_t hasl,
                                                      uint32_t fs) {
        const int r = c.r;
        const int s = ib(mvr) ? __builtin_ctz(vtodo) : 0;
        vtodo &= vtodo - 1u;
        BSTAT(c, BS_V_ROUNDS);
        const int sl = c.src(s);
        const uint32_t ms = bcastu(send, sl);                       // sender s's pending dsts
        const int32_t rt = bcast(qt, sl), rli = bcast(qli, sl), rlt = bcast(qlt, sl);
        const int32_t st = bcast(n.term, sl);
        uint32_t dw;
        if constexpr (STAGED) dw = drops_off<NET>(p) ? 0u : job_drop_word(c, s, s);   // stage_sender_chunks
        else dw = drop_word<R, L::VOTE_JOB, NET>(p, c, RAFT_RNG_VOTE_DROP, mvr, s, c.dwv, c.s_vote);
        const uint64_t mine = mvr & lm((ms >> r) & 1u);
        const uint64_t mme = lm(r == s);
        const uint64_t net = lost_net<R, NET>(c, s);
        const uint64_t lreq = mine & lost<NET>(p, net, mme, dw, 0); // retry{} swallows, Commons.kt:41
        const uint64_t act = mine & ~lreq;
        int32_t rterm;
        uint64_t granted;
        vote_handler<TB, RING>(n.rep(), act, r + 1, rt, s + 1, rli, rlt, gapw, hasl, fs, cnt, rterm, granted);
        const uint64_t lresp = act & lost<NET>(p, net, mme, dw, 1);
        const uint64_t delivered = act & ~lresp;
        cnt.add(lreq | lresp, RAFT_C_MSG_DROPPED);
        const uint64_t him = delivered & lm(rterm > st);
        uint32_t hi = 0;
        if (RARE(him)) hi = c.gbits(him);                                 // wave-uniform, rare
        const bool me = ib(mvr & mme);
        constexpr bool LDS_TALLY = R >= 4;                          // a word per group at base >> 2
        uint32_t f;
        if constexpr (LDS_TALLY) {
            // the sender's tally through LDS (RaftServer.kt:208-212): each
            // delivered destination d adds one response (:209 countDown()),
            // its grant (:211) and minus its pending bit (set in the sender's
            // flags: it was sent to) into its group's word; the sender reads
            // the sum.  A wave's LDS operations complete in order.
            // Every lane of a group zeroes its word and adds (0 unless
            // delivered): no exec-mask changes.
            uint32_t* const tw = c.tl + (c.base >> 2);                 // one word per group (R >= 4)
            *tw = 0u;
            const uint32_t add = (1u << LATCH_SH) + (ib(granted) ? (1u << VOTES_SH) : 0u) - (1u << (PEND_SH + c.r));
            __hip_atomic_fetch_add(tw, ib(delivered) ? add : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            asm volatile("" ::: "memory");
            f = n.fl + *tw;
        } else {
            // the sender's tally: ballot + popcount (RaftServer.kt:208-212)
            const uint32_t dl = c.gbits(delivered);
            const uint32_t gr = c.gbits(delivered & granted);
            f = n.fl & ~(dl << PEND_SH);
            f += (uint32_t)__popc(dl) << LATCH_SH;                  // :209 countDown()
            f += (uint32_t)__popc(gr) << VOTES_SH;                  // :211
        }
        n.fl = me ? f : n.fl;
        n.role = (me && hi) ? (int32_t)RAFT_FOLLOWER : n.role;     // :210 (Q6)
        if constexpr (TB) {
            // textbook: the candidate adopts the highest response term once its
            // round's responses are in (the reference keeps its term, Q6)
            if (RARE(lm(hi != 0))) {                                      // wave-uniform, rare
                int32_t T = st;
                const uint32_t dl = c.gbits(delivered);
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    const int32_t tq = bcast(rterm, c.src(q));
                    T = ((dl >> q) & 1u) ? max(T, tq) : T;
                }
                n.term = (me && hi) ? T : n.term;
                n.voted = (me && hi) ? -1 : n.voted;
            }
        }
        n.retry = (me && ((f >> PEND_SH) & 0xFFu)) ? p.retry : n.retry;
    }

    // One lockstep step of every group of the wave.
    // Called by all 64 lanes (converged); `n` of a dead lane is inert.
    __device__ __forceinline__ static void step(const DevParams& p, Ctx<R>& c, Node& n, Counters& cnt) {
        const int r = c.r;
        BSTAT(c, BS_STEPS);
        // H needs the roles at step start (the lowest-id LEADER to isolate);
        // T draws no randomness, so it runs before the step's Philox pass and
        // that pass already knows the first RequestVote sender.
        // the group's LEADER bits at step start: K's of the previous step (no
        // role changes between K and the next T), made at launch start
        const uint32_t lead0 = c.lead;

        uint32_t send;
        int32_t qt, qli, qlt;
        uint64_t sstart;
        auto phase_t = [&](Ctx<R>& c, Node& n, Counters& cnt, uint32_t& send, int32_t& qt, int32_t& qli, int32_t& qlt,
                           uint64_t& sstart) {
            // ---------------- T: timers and election clocks ----------------
            // a wave where no timer fires and no replica is electing only counts
            // its armed timers down (most waves in steady state)
            const int32_t P = p.P;
            const uint64_t t_armed = lm(n.fl & FL_ARMED);
            const int32_t t_el = n.elec - P;
            const uint64_t t_fire = t_armed & lm(t_el <= 0);                    // Commons.kt:25-27
            const uint64_t electing = lm(n.fl & FL_ELECTING);                   // T does not change it before use
            // the quiet wave's whole update first, so that its path through
            // the branch is empty (an else-side that redefines the outputs
            // made the register allocator copy a dozen values on it)
            n.elec = ib(t_armed) ? t_el : n.elec;
            send = 0u; sstart = 0; qt = qli = qlt = 0;
            if (t_fire | electing) {
                BSTAT(c, BS_T_BUSY);
                uint32_t f = n.fl;
                const bool fire = ib(t_fire);
                n.elec = fire ? 0 : n.elec;                                     // fire is within t_armed
                f &= fire ? ~FL_ARMED : ~0u;
                n.role = fire ? (int32_t)RAFT_CANDIDATE : n.role;               // RaftServer.kt:182
                cnt.add(t_fire, RAFT_C_TIMEOUTS);
                const uint64_t backoff = lm(f & FL_BACKOFF);
                const uint64_t start_fire = t_fire & ~electing;                 // offer(CANDIDATE) :184 -> :65
                const uint64_t in_round = electing & ~backoff, in_bo = electing & backoff;
                const int32_t ph = n.phase + (ib(in_round) ? P : (ib(in_bo) ? -P : 0));   // latch clock :214 / delay :221
                const uint32_t pend = (f >> PEND_SH) & 0xFFu;
                const uint64_t rtick = in_round & lm(pend != 0) & lm(ph < p.round_to);
                const int32_t rty = n.retry - (ib(rtick) ? P : 0);             // retry delay, Commons.kt:43
                const uint64_t resend = rtick & lm(rty <= 0);
                const uint64_t bo_end = in_bo & lm(ph <= 0);
                const uint64_t restart = bo_end & lm(n.role == RAFT_CANDIDATE); // while (state == CANDIDATE) :191
                const uint64_t endel = bo_end & ~restart;
                const uint64_t sr = start_fire | restart;                       // round head :191-199
                const bool bsr = ib(sr), bend = ib(endel);
                n.term = inc_if(n.term, sr);                                    // :192
                n.voted = bsr ? r + 1 : n.voted;                                // :193
                const uint32_t fr = (f & ~(FL_BACKOFF | (0xFFu << PEND_SH) | (0xFu << VOTES_SH) | (0xFu << LATCH_SH))) |
                                    (ALL << PEND_SH) | (ib(start_fire) ? FL_ELECTING : 0u);
                uint32_t fe = f;                                                // the flags of an election that ends
                if (RARE(endel)) fe = end_flags(f, n.role);                     // (rare: ~9 VALU skipped)
                n.fl = bsr ? fr : (bend ? fe : f);
                n.phase = (bsr || bend) ? 0 : ph;
                n.retry = (bsr || bend) ? 0 : rty;
                sstart = endel & lm(n.role == RAFT_LEADER);
                send = bsr ? ALL : (ib(resend) ? pend : 0u);
                // the RequestVote snapshot, built inside retry{} (:200-207)
                qt = n.term;
                qli = n.last;
                qlt = n.last != 0 ? n.t1 : 0;
                cnt.add((sr | resend) & lm(n.last != 0), RAFT_C_VOTE_LOG_READS);
                if constexpr (RING) cnt.add((sr | resend) & lm(n.last != 0) & lm(n.phys - n.last >= p.W), RAFT_C_LOG_WINDOW_MISS);
                cnt.add(sr, RAFT_C_ROUNDS);
            }
            start_sessions(p, c, n, sstart, cnt);
        };
        RAFT_TWICE(PH_T, ({ uint32_t s_; int32_t a_, b_, d_; uint64_t e_;
                            phase_t(c2, n2, k2, s_, a_, b_, d_, e_);
                            asm volatile("" ::"v"(s_), "v"(a_), "v"(b_), "v"(d_), "s"(e_)); }));
        phase_t(c, n, cnt, send, qt, qli, qlt, sstart);
        c.clk.mark(PH_T);

        // ---------------- the step's Philox pass (S-9) ----------------
        // lane J_HARNESS of a group: harness words; lanes J_TIMER..: timer
        // quads; lanes J_TICK.. / J_VOTE..: drop-word chunks of the first
        // leader to tick (lowest heartbeat session now) and of the first
        // RequestVote sender.  One Philox evaluation of the wave.
        uint32_t hw0, hw1, hw2;
        uint32_t vtodo = c.gbits(__ballot(send != 0));                     // the group's RequestVote senders
        // the group's heartbeat sessions: only D's new leaders add to them
        // before A (A re-reads them only in a wave where one started)
        const uint32_t hb = c.gbits(__ballot((n.fl & FL_HB) != 0));
        c.s_tick = hb ? __builtin_ctz(hb) : -1;
        c.s_vote = vtodo ? __builtin_ctz(vtodo) : -1;
        if constexpr (L::JOBS) {
            uint32_t purpose = RAFT_RNG_HARNESS, sub = 0;
            if constexpr (L::CHUNK1_LANES != 0) {
                // R > 5 (two drop-word chunks per sender): each lane's job by
                // compile-time lane masks (selects, no compares or exec-mask
                // branches): timer quad r - J_TIMER; chunk r - J_TICK / r - J_VOTE
                // of the first leader to tick / RequestVote sender.  Measured
                // +1.3 % at R = 7 and -0.25 % at R = 5 (profiles/r2_jobsel)
                const bool jt = ib(L::TIMER_LANES), jk = ib(L::TICK_LANES), jv = ib(L::VOTE_LANES);
                purpose = jt ? RAFT_RNG_TIMER : (jk ? RAFT_RNG_APPEND_DROP : (jv ? RAFT_RNG_VOTE_DROP : RAFT_RNG_HARNESS));
                sub = jt ? (uint32_t)(r - L::J_TIMER) : (jk ? (uint32_t)c.s_tick : (jv ? (uint32_t)c.s_vote : 0u));
                sub = (sub & 0xFFu) | (ib(L::CHUNK1_LANES) ? 0x100u : 0u);
            } else if (r >= L::J_TIMER && r < L::J_TICK) {
                purpose = RAFT_RNG_TIMER; sub = (uint32_t)(r - L::J_TIMER);
            } else if (r >= L::J_TICK && r < L::J_VOTE) {
                purpose = RAFT_RNG_APPEND_DROP; sub = (uint32_t)(c.s_tick & 0xFF) | ((uint32_t)(r - L::J_TICK) << 8);
            } else if (r >= L::J_VOTE) {
                purpose = RAFT_RNG_VOTE_DROP; sub = (uint32_t)(c.s_vote & 0xFF) | ((uint32_t)(r - L::J_VOTE) << 8);
            }
            // opaque: otherwise the compiler folds the first Philox round for
            // every lane's constant purpose and keeps those products in VGPRs
            // across the step loop (R = 7 spilled them to scratch)
            asm volatile("" : "+v"(purpose));
            RAFT_TWICE(PH_JOBS, ({ uint32_t z = 0; asm volatile("" : "+v"(z));
                                   const u32x4 w = kdraw(p, c.t, c.gid(), purpose ^ z, sub);
                                   asm volatile("" ::"v"(w.x), "v"(w.y), "v"(w.z), "v"(w.w)); }));
            c.job = kdraw(p, c.t, c.gid(), purpose, sub);
            // stage the wave's jobs in LDS (one ds_write_b128 per lane); a
            // wave's LDS accesses complete in order, so its reads below see
            // them, and the previous step's reads were issued before this write
            *(uint4*)&c.jl[(c.base + c.r) << 2] = make_uint4(c.job.x, c.job.y, c.job.z, c.job.w);
            asm volatile("" ::: "memory");
            const uint4 h = *(const uint4*)&c.jl[c.base << 2];
            hw0 = h.x;
            hw1 = h.y;
            hw2 = h.z;
            // every word this lane needs from the jobs, fetched in one batch
            c.tw = job_word(c, L::J_TIMER, r);                              // word r & 3 of timer quad r >> 2
            if constexpr (L::TICK_JOB) c.dwt = job_drop_word(c, L::J_TICK, c.s_tick);
            if constexpr (L::VOTE_JOB) c.dwv = job_drop_word(c, L::J_VOTE, c.s_vote);
        } else {
            const u32x4 h = kdraw(p, c.t, c.gid(), RAFT_RNG_HARNESS, 0);
            hw0 = h.x; hw1 = h.y; hw2 = h.z;
        }

        c.clk.mark(PH_JOBS);
        // ---------------- H: harness ----------------
        {
            // harness parameters re-read where used (kernargs()): held across
            // the step they would be spilled into VGPR lanes
            const KernArgs kp = kernargs();
            const uint64_t churn_thr = kp->churn_thr32;
            c.iso = -1;
            c.iso_me = 0;
            // only waves where an isolation runs or may start (~1/5) do the rest
            // (none in a kernel built without NET_ISO: no churn, no isolation word)
            if ((NET & NET_ISO) != 0 && RARE(lm(n.iso != 0) | lm((uint64_t)hw0 < churn_thr))) {
                BSTAT(c, BS_H_BUSY);
                const int32_t churn_steps = kp->churn_steps;
                int32_t rem = n.iso >> 8, rep = n.iso & 0xFF;
                if (rem > 0) { rem--; if (rem == 0) rep = 0; }
                if (churn_thr && churn_steps > 0 && rem == 0 && hw0 < churn_thr && lead0) {
                    rep = __builtin_ctz(lead0);                             // lowest-id LEADER
                    rem = churn_steps;
                }
                n.iso = rem > 0 ? (rem << 8) | rep : 0;
                c.iso = rem > 0 ? rep : -1;
                c.iso_me = lm(r == c.iso);
            }
        }

        c.clk.mark(PH_H);
        // ---------------- V: RequestVote fan-out (S-3) ----------------
        // Each group walks its own senders in ascending order (group-uniform,
        // runtime s), so the wave runs as many rounds as its busiest group has
        // senders -- usually one -- with one handler per destination lane.
        // the lanes of groups with a pending sender: each round's predicate
        // and the loop condition (one ballot per round)
        auto phase_v = [&](Ctx<R>& c, Node& n, Counters& cnt, uint32_t vtodo, uint64_t mv) {
            if (mv) {
                BSTAT(c, BS_V_PHASE);
                // RING: the replicas whose log.get(lastIndex - 1) is below the
                // window; hasl: lastIndex >= 1 (the vote handlers do not touch the
                // logs, so both hold for the whole phase)
                const uint64_t gapw = RING ? lm(n.phys - n.last >= p.W) : 0ull;
                const uint64_t hasl = lm(n.last >= 1);
                const uint32_t fs = follower_sent(n.fl);                        // FL_ELECTING is fixed during V
                if constexpr (L::SENDERS_STAGED && !L::VOTE_JOB) {
                    // the job lanes do not hold the first sender's chunk (R < 4):
                    // one staging pass serves every round, the first included
                    stage_sender_chunks(p, c, RAFT_RNG_VOTE_DROP);
                    do {
                        vote_round<true>(p, c, n, cnt, vtodo, mv, send, qt, qli, qlt, gapw, hasl, fs);
                        mv = lm(vtodo != 0);
                    } while (mv);
                } else {
                    vote_round(p, c, n, cnt, vtodo, mv, send, qt, qli, qlt, gapw, hasl, fs);
                    mv = lm(vtodo != 0);
                    if (mv) {                                                   // groups with 2+ senders
                        if constexpr (L::SENDERS_STAGED) stage_sender_chunks(p, c, RAFT_RNG_VOTE_DROP);
                        do {
                            vote_round<L::SENDERS_STAGED>(p, c, n, cnt, vtodo, mv, send, qt, qli, qlt, gapw, hasl, fs);
                            mv = lm(vtodo != 0);
                        } while (mv);
                    }
                }
            }
        };
        RAFT_TWICE(PH_V, phase_v(c2, n2, k2, vtodo, lm(vtodo != 0)));
        // the senders' ballot made here, after H's branch (hoisted above it,
        // it came back through a VGPR: v_cndmask + v_cmp)
        asm volatile("" : "+v"(vtodo));
        phase_v(c, n, cnt, vtodo, lm(vtodo != 0));

        c.clk.mark(PH_V);
        // ---------------- D: latch closes -> decision (RaftServer.kt:214-222) ----------------
        // only waves where some round closes this step do any of it
        uint64_t dstart = 0, need_bo = 0;
        {
            const uint32_t f = n.fl;
            const uint64_t inr = lm(f & FL_ELECTING) & ~lm(f & FL_BACKOFF);     // in a vote round
            uint64_t dec = 0;
            if (inr) {                                                      // wave-uniform
                const int latch = (f >> LATCH_SH) & 0xF;
                dec = inr & (lm(latch >= MAJ) | lm(n.phase >= p.round_to));
            }
            if (dec) {                                                      // wave-uniform
                BSTAT(c, BS_D_DEC);
                const int votes = (f >> VOTES_SH) & 0xF;
                const uint64_t cand = dec & lm(n.role == RAFT_CANDIDATE);
                const uint64_t win = cand & lm(votes >= MAJ);               // :218-219
                need_bo = cand & ~win;                                      // :220-221
                const uint64_t endel = dec & ~need_bo;
                const uint32_t fc = f & ~(0xFFu << PEND_SH);                // cancelChildren() :215
                n.role = ib(win) ? (int32_t)RAFT_LEADER : n.role;
                const uint32_t fb = (fc & ~((0xFu << VOTES_SH) | (0xFu << LATCH_SH))) | FL_BACKOFF;
                uint32_t fe = f;
                if (endel) fe = end_flags(fc, n.role);                      // wave-uniform
                n.fl = ib(endel) ? fe : (ib(need_bo) ? fb : f);
                n.phase = ib(endel) ? 0 : n.phase;
                n.retry = ib(dec) ? 0 : n.retry;
                dstart = endel & lm(n.role == RAFT_LEADER);
            }
        }
        if (need_bo) {
            BSTAT(c, BS_D_BACKOFF);
            const uint32_t w = timer_word(p, c);
            const KernArgs kp = kernargs();
            if (ib(need_bo)) n.phase = scale_range(w, kp->bmin, kp->bmax);
        }
        if (dstart) BSTAT(c, BS_D_START);
        start_sessions(p, c, n, dstart, cnt);
        c.clk.mark(PH_D);

        // ---------------- A: leader ticks, senders ascending (S-3, S-4) ----------------
        uint32_t todo = hb;
        if (RARE(dstart)) todo = c.gbits(__ballot((n.fl & FL_HB) != 0));   // D started a session
        // the first round peeled: the common case runs no loop (a loop makes
        // the compiler carry the counters in VGPRs and copy the node per round).
        // mt: the lanes of groups with a session left to tick (each round's
        // predicate and the loop condition, one ballot per round)
        auto phase_a = [&](Ctx<R>& c, Node& n, Counters& cnt, uint32_t todo, uint64_t mt) {
            if (LIKELY(mt)) {
                BSTAT(c, BS_A_PHASE);
                const uint32_t fs = follower_sent(n.fl);                        // FL_ELECTING is fixed during A
                {
                    // R = 2: the job lanes do not hold the first leader's chunk,
                    // so one staging pass serves every round, the first included
                    constexpr bool FIRST_STAGED = L::SENDERS_STAGED && !L::TICK_JOB;
                    if constexpr (FIRST_STAGED) stage_sender_chunks(p, c, RAFT_RNG_APPEND_DROP);
                    const int s = ib(mt) ? __builtin_ctz(todo) : 0;
                    todo &= todo - 1u;
                    tick<FIRST_STAGED>(p, c, n, mt, s, fs, cnt);
                }
                mt = lm(todo != 0);
                if (RARE(mt)) {                                                 // 2+ sessions (rare)
                    constexpr bool ALL = L::SENDERS_STAGED;
                    if constexpr (ALL && L::TICK_JOB) stage_sender_chunks(p, c, RAFT_RNG_APPEND_DROP);
                    do {
                        const int s = ib(mt) ? __builtin_ctz(todo) : 0;
                        todo &= todo - 1u;
                        tick<ALL>(p, c, n, mt, s, fs, cnt);
                        mt = lm(todo != 0);
                    } while (mt);
                }
            }
        };
        RAFT_TWICE(PH_A, phase_a(c2, n2, k2, todo, lm(todo != 0)));
        phase_a(c, n, cnt, todo, lm(todo != 0));

        c.clk.mark(PH_A);
        // ---------------- C: client commands (S-11) ----------------
        // the leaders after A: appendCommand changes no role, so C and K share them
        const uint64_t isl = lm(n.role == RAFT_LEADER);
        const uint32_t lead = c.gbits(isl);
        const KernArgs kp = kernargs();
        const uint64_t cmd_thr = kp->cmd_thr32;
        auto phase_c = [&](Ctx<R>& c, Node& n, Counters& cnt) {
            if (cmd_thr) {
                const int32_t cmd_limit = kp->cmd_limit, cmd_mode = kp->cmd_mode;
                constexpr bool CL = (NET & NET_CMDLOW) != 0;                   // lowest LEADER, no limit
                const uint64_t cm = (CL || cmd_limit == 0 ? ~0ull : lm(n.cmdc < cmd_limit)) &
                                    lm((uint64_t)hw1 < cmd_thr) & lm(lead != 0);
                const uint64_t tgt = cm & (CL || cmd_mode == RAFT_CMD_LOWEST_LEADER ? lm(r == __builtin_ctz(lead)) : isl);
                append_command<TB, RING>(n.rep(), tgt, c.template log<RING>(p), hw2, cnt);
                n.cmdc = inc_if(n.cmdc, cm);
            }
        };
        RAFT_TWICE(PH_C, phase_c(c2, n2, k2));
        phase_c(c, n, cnt);

        c.clk.mark(PH_C);
        // ---------------- K: end-of-step observations ----------------
        {
            c.lead = lead;                                                  // the next step's lead0
            const uint64_t glead = lm(lead != 0) & L::lanes_of(0);         // one lane per group with a leader
            cnt.add(isl, RAFT_C_LEADERS);
            cnt.add(glead, RAFT_C_GROUPS_WITH_LEADER);
            if (RARE(__popcll(isl) != __popcll(glead))) {                   // some group has 2+ leaders (rare)
                BSTAT(c, BS_K_DUAL);
                bool dual = false;
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    const int32_t tq = bcast(n.term, c.src(q));
                    if (ib(isl) && r < q && ((lead >> q) & 1u) && tq == n.term) dual = true;
                }
                const uint32_t db = c.gbits(lm(dual));
                cnt.add(lm(db != 0) & L::lanes_of(0), RAFT_C_DUAL_LEADER_GROUPS);
            }
        }

        c.clk.mark(PH_K);
        // the deferred ResettableCountdownTimer draws of this step (S-9)
        const uint64_t dm = lm(n.fl & FL_DRAW);
        if (dm) {
            BSTAT(c, BS_DRAW);
            const uint32_t w = timer_word(p, c);
            if (ib(dm)) {
                const KernArgs kp = kernargs();
                n.elec = scale_range(w, kp->emin, kp->emax);
                n.fl &= ~FL_DRAW;
            }
        }
    }
};

}  // namespace raft
