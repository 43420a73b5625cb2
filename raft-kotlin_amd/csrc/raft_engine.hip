// raft_engine.hip — HIP kernels (gfx950) and the C-ABI of include/raft_engine.h.
//
// HBM layout: see raft_step.h (DevParams).  Per-replica arrays are indexed by
// g * R + r, so one wave (GPW = 64 / R whole groups, one lane per replica)
// reads or writes one contiguous run per field.  The step kernel keeps every
// replica in VGPRs for a whole launch (1..K fused lockstep steps) and touches
// HBM only for the state load/store at the launch edges, the log slots the
// handlers read or write, and (rarely) non-primary session rows.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "raft_engine_impl.h"

using namespace raft;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return fail(RAFT_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#ifdef RAFT_PROFILE_PHASES
__device__ unsigned long long g_phase_cycles[PH_N];   // diagnostic builds only
#endif
#ifdef RAFT_BRANCH_STATS
__device__ unsigned long long g_branch_stats[BS_N];   // diagnostic builds only (raft_step.h BSTAT)
#endif
#ifdef RAFT_WAVE_TIMES
// diagnostic builds only: per wave of the last step launch, its start and end
// (s_memrealtime, 100 MHz, chip-wide) and its HW_ID / XCC_ID registers
constexpr int WT_MAX = 1 << 17;
__device__ unsigned long long g_wave_times[WT_MAX][3];
#endif
// step_kernel's workgroup: its LDS holds one counter row per step for the
// whole workgroup, so larger workgroups leave room for longer launches
#ifndef RAFT_STEP_BLOCK
#define RAFT_STEP_BLOCK 256
#endif
constexpr int STEP_BLOCK = RAFT_STEP_BLOCK;
constexpr int STEP_WAVES = STEP_BLOCK / 64;
constexpr int JOB_LDS_WORDS = STEP_WAVES * 64 * 4;        // step_kernel's per-wave job-word staging
constexpr int TALLY_LDS_WORDS = STEP_WAVES * 16;          // per-wave vote-tally words (Ctx::tl, R >= 4)
constexpr int FLAG_LDS_WORDS = STEP_WAVES;                // balanced schedule: a wave's head piece is stored
constexpr int PLAN_LDS_WORDS = STEP_WAVES * 16;           // each wave's plans (plan_of) and priority band
constexpr int PRE_CNT_LDS_WORDS = JOB_LDS_WORDS + TALLY_LDS_WORDS + FLAG_LDS_WORDS + PLAN_LDS_WORDS;
// the longest launch whose LDS (job rows, tally words, K counter rows) still
// lets 7 step workgroups share a CU's 160 KB
constexpr int STEP_K_7WG = (160 * 1024 / 7 / 4 - PRE_CNT_LDS_WORDS) / NCW;
static_assert(STEP_K_7WG >= 400, "a 400-step launch (or epoch) keeps 7 workgroups per CU");
// the longest launch without epochs (its counter rows in LDS; 6 workgroups per
// CU beyond STEP_K_7WG); a longer balanced launch on one sub-range runs as
// epochs of EPOCH_STEPS, any other is cut into launches of LDS_MAX_STEPS
constexpr int LDS_MAX_STEPS = 512;
constexpr int EPOCH_STEPS = 400;
constexpr uint32_t PART_STALE = 0x80000000u;   // Ctx::part of a piece's entry: its first step draws the window's mask


// ---------------------------------------------------------------------------
// replica state <-> registers
// ---------------------------------------------------------------------------
// (the quads' word order: raft_step.h FIELD_SLOT).  One dword access per
// field: merged into dwordx4 per quad, the accesses need 4 consecutive VGPRs
// each, and the step kernel's register allocation spilled 60 B to scratch to
// find them (the compiler barriers keep the loads in flight together)
#define NOMERGE asm volatile("" ::: "memory")
__device__ __forceinline__ void load_node(Node& n, const DevParams& p, int64_t g, int64_t idx) {
    const int32_t* st = p.st;
    NOMERGE; n.term = st[fidx(p, RAFT_F_TERM, idx)];
    NOMERGE; n.voted = st[fidx(p, RAFT_F_VOTED, idx)];
    NOMERGE; n.role = st[fidx(p, RAFT_F_ROLE, idx)];
    NOMERGE; n.commit = st[fidx(p, RAFT_F_COMMIT, idx)];
    NOMERGE; n.last = st[fidx(p, RAFT_F_LAST, idx)];
    NOMERGE; n.phys = st[fidx(p, RAFT_F_PHYS, idx)];
    NOMERGE; n.elec = st[fidx(p, RAFT_F_ELECTION_MS, idx)];
    NOMERGE; n.fl = (uint32_t)st[fidx(p, RAFT_F_FLAGS, idx)];
    NOMERGE; n.phase = st[fidx(p, RAFT_F_PHASE_MS, idx)];
    NOMERGE; n.retry = st[fidx(p, RAFT_F_RETRY_MS, idx)];
    NOMERGE; n.t1 = st[fidx(p, F_T1, idx)];
    NOMERGE; n.t2 = st[fidx(p, F_T2, idx)];
    NOMERGE; n.c1 = (uint32_t)st[fidx(p, F_C1, idx)];
    NOMERGE; n.nx = st[fidx(p, F_NX, idx)];
    NOMERGE; n.mc = st[fidx(p, F_MC, idx)];
    NOMERGE; n.iso = p.gx[GX_ISO * p.G + g];
    NOMERGE; n.cmdc = p.gx[GX_CMDS * p.G + g];
    NOMERGE; n.s0 = p.gx[GX_S0 * p.G + g];
}

__device__ __forceinline__ void inert_node(Node& n) {
    n.term = n.commit = n.last = n.phys = n.elec = n.phase = n.retry = 0;
    n.voted = -1;
    n.role = RAFT_FOLLOWER;
    n.fl = 0;
    n.t1 = n.t2 = 0;
    n.c1 = 0;
    n.nx = n.mc = 0;
    n.iso = n.cmdc = 0;
    n.s0 = -1;
}

__device__ __forceinline__ void store_node(const Node& n, const DevParams& p, int64_t g, int64_t idx, bool group_lead) {
    int32_t* st = p.st;
    NOMERGE; st[fidx(p, RAFT_F_TERM, idx)] = n.term;
    NOMERGE; st[fidx(p, RAFT_F_VOTED, idx)] = n.voted;
    NOMERGE; st[fidx(p, RAFT_F_ROLE, idx)] = n.role;
    NOMERGE; st[fidx(p, RAFT_F_COMMIT, idx)] = n.commit;
    NOMERGE; st[fidx(p, RAFT_F_LAST, idx)] = n.last;
    NOMERGE; st[fidx(p, RAFT_F_PHYS, idx)] = n.phys;
    NOMERGE; st[fidx(p, RAFT_F_ELECTION_MS, idx)] = n.elec;
    NOMERGE; st[fidx(p, RAFT_F_FLAGS, idx)] = (int32_t)(n.fl & FL_EXPORT_MASK);
    NOMERGE; st[fidx(p, RAFT_F_PHASE_MS, idx)] = n.phase;
    NOMERGE; st[fidx(p, RAFT_F_RETRY_MS, idx)] = n.retry;
    NOMERGE; st[fidx(p, F_T1, idx)] = n.t1;
    NOMERGE; st[fidx(p, F_T2, idx)] = n.t2;
    NOMERGE; st[fidx(p, F_C1, idx)] = (int32_t)n.c1;
    NOMERGE; st[fidx(p, F_NX, idx)] = n.nx;
    NOMERGE; st[fidx(p, F_MC, idx)] = n.mc;
    if (group_lead) {
        p.gx[GX_ISO * p.G + g] = n.iso;
        p.gx[GX_CMDS * p.G + g] = n.cmdc;
        p.gx[GX_S0 * p.G + g] = n.s0;
    }
}

// canonical session rows: the primary (owner s0) lives in the state quads
// (F_NX / F_MC), the rest in spill
__device__ __forceinline__ int32_t canon_next(const DevParams& p, int R, int64_t g, int s0, int s, int d) {
    const int64_t idx = g * R + d;
    return s == s0 ? p.st[fidx(p, F_NX, idx)] : p.spill[idx * R + s];
}
__device__ __forceinline__ int32_t canon_match(const DevParams& p, int R, int64_t g, int s0, int s, int d) {
    const int64_t idx = g * R + d;
    return s == s0 ? p.st[fidx(p, F_MC, idx)] : p.spill[p.GR * R + idx * R + s];
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
// one thread per replica: the reference's initial node (RaftServer.kt:35-48)
// with the election timer started by init (RaftServer.kt:58, Commons.kt:14)
template <int R>
__global__ __launch_bounds__(BLOCK) void init_kernel(DevParams p) {
    const int64_t idx = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (idx >= p.GR) return;
    const int64_t g = idx / R;
    const int r = (int)(idx - g * R);
    const uint32_t gid = (uint32_t)(p.g0 + g);
    for (int q = 0; q < ST_QUADS; ++q) *quad(p, q, idx) = make_int4(0, 0, 0, 0);   // sessions and tail cache too
    p.st[fidx(p, RAFT_F_VOTED, idx)] = -1;                               // RaftServer.kt:39
    const u32x4 w = draw(p, RAFT_RNG_INIT_STEP, gid, RAFT_RNG_TIMER, (uint32_t)(r >> 2));
    p.st[fidx(p, RAFT_F_ELECTION_MS, idx)] = scale_range(word_of(w, r & 3), p.emin, p.emax);
    p.st[fidx(p, RAFT_F_FLAGS, idx)] = (int32_t)FL_ARMED;
    for (int s = 0; s < R; ++s) {
        p.spill[idx * R + s] = 0;
        p.spill[p.GR * R + idx * R + s] = 0;
    }
    if (r == 0) {
        p.gx[GX_ISO * p.G + g] = 0;
        p.gx[GX_CMDS * p.G + g] = 0;
        p.gx[GX_S0 * p.G + g] = -1;
    }
}

// K lockstep steps of every group.  A wave holds GPW whole groups, one lane
// per replica.  Counters: a wave's totals of a step (SGPRs) are added into the
// workgroup's LDS row [k][NCW] with one return-less ds_add (no wait in the
// step loop), and after the loop the workgroup copies its rows into column
// part_col0 + blockIdx.x of the partials [k][NCW][part_stride = all step
// workgroups of the engine].  A launch may cover a sub-range of the waves
// (wave0 on): the engine's sub-range streams, raft_engine_step_async.  One row per workgroup (not per wave) keeps the
// LDS footprint at K * NCW words, so K can reach RAFT_MAX_STEPS_PER_LAUNCH
// without costing occupancy; the launch's two barriers (zeroing, final copy)
// sit outside the step loop.
// Waves per SIMD the register allocation targets: 7 (72 VGPRs, 94 SGPRs)
// where the kernel fits them (every kernel at R <= 5, and at R = 7 without
// drop checks), else 6 (80 VGPRs, 106 SGPRs).  Seven
// workgroups per CU also need the LDS of a launch of at most STEP_K_7WG steps,
// which bench.py's default launch length respects.
// (round 3: also R = 7 built for partitions only, config 5's kernel, which
// the dropped drop checks brought to 72 VGPRs with 12 B of spills: +4.3 %,
// profiles/r3_w7; and the textbook-mode flat kernels, 72 VGPRs with 12-20 B
// of spills: +4.4 % on config 3, +4 % on config 5, profiles/r3_tb7; and the
// ring kernels, 72 VGPRs with 16 B of spills at R = 5: +3.8 %, profiles/r3_all7)
#ifndef RAFT_STEP_WAVES_PER_EU
#define RAFT_STEP_WAVES_PER_EU(R, TB, RING, NET) (((R) <= 5 || ((R) == 7 && (NET) == NET_PART)) ? 7 : 6)
#endif
// NET: the network faults the kernel is built for (raft_step.h NET_DROP /
// NET_PART; the host's step_fn picks it from raft_params).
//
// The launch's schedule.  A chunk is one wave's worth of groups (GPW, one log
// block); a piece is (chunk, steps [k0, k1)): load the chunk's replicas, run
// those steps, store them back -- exactly a launch boundary, which results
// never depend on.
//  * One chunk per wave (bal_chunks == 0): chunk wave0 + blockIdx.x *
//    STEP_WAVES + wave, all steps; the grid has a wave per chunk.  When the
//    chunks outnumber the chip's resident wave slots, the last round of waves
//    runs on a part-empty chip (1.25e5 groups: 10,417 waves = 1.45 rounds of
//    the 7,168 slots).
//  * Balanced (bal_chunks > 0): the grid is the workgroups the chip holds at
//    once; workgroup b takes the interleaved chunks b, b + nb, b + 2 nb, ...
//    (n = bal_chunks, nb = gridDim.x; m = n / nb or one more, at least
//    STEP_WAVES of them; piece_chunk) and its waves
//    split the m chunks' m * K chunk-steps into equal quarters (McNaughton's
//    wrap-around rule).  A quarter [u0, u1) is a head piece (the first e steps
//    of the chunk it ends in), whole chunks, and a tail piece (the last K - s
//    steps of the chunk it starts in, whose first s steps are the previous
//    wave's head).  A wave runs its head FIRST and its tail LAST, so the tail
//    starts (at >= K chunk-steps into the wave's quarter, which is >= K long)
//    after the previous wave's head ended (at <= K): the one dependency, wave
//    w's tail on wave w - 1's head, is an in-workgroup hand-off through an
//    LDS flag (both waves on one CU, always co-resident; no other workgroup
//    is involved, so dispatch order and XCD placement do not matter).  Every
//    wave then ends within one chunk-step of the others.
struct Piece {
    int32_t chunk, k0, k1;
    bool wait;                    // tail: wait until the previous wave has stored its head
    bool signal;                  // head: tell the next wave it is stored
};
// A wave's plan, 4 words (made once per launch by plan_of, kept in LDS and
// read back at each piece boundary, so the step loop carries no schedule
// arithmetic): the head's steps e (0: none), the first whole chunk f, the
// whole chunks nf, the tail's first step s (0: none).  The head is chunk
// f + nf, the tail chunk f - 1.
__device__ __forceinline__ uint4 plan_of(int wib, int K) {
    const KernArgs kp = kernargs();
    if (kp->bal_chunks == 0)
        return make_uint4(0u, (uint32_t)(kp->wave0 + (int32_t)blockIdx.x * STEP_WAVES + wib), 1u, 0u);
    // workgroup b: its i-th chunk is wave0 + b + i * nb (piece_chunk), i < m,
    // m = q or q + 1 (q = n / nb, the first n % nb workgroups take one more):
    // the chunks running at one time are neighbours, as in the one-chunk-per-
    // wave schedule; the plan holds indices i; 32-bit throughout (launch_geo
    // refuses a launch with STEP_WAVES * m * K >= 2^32)
    const uint32_t b = blockIdx.x, q = (uint32_t)kp->bal_q, rem = (uint32_t)kp->bal_rem, k = (uint32_t)K;
    const uint32_t U = (q + (b < rem ? 1u : 0u)) * k;
    const uint32_t u0 = (uint32_t)wib * U / STEP_WAVES, u1 = (uint32_t)(wib + 1) * U / STEP_WAVES;
    const uint32_t a = u0 / k, s = u0 - a * k, z = u1 / k, e = u1 - z * k;
    const uint32_t f = a + (s != 0);
    return make_uint4(e, f, z - f, s);
}
__device__ __forceinline__ int n_pieces(uint4 pl) { return (pl.x != 0) + (int)pl.z + (pl.w != 0); }
// the chunk of a piece: the one-chunk-per-wave plan holds it, a balanced
// plan the workgroup's chunk index i (plan_of)
__device__ __forceinline__ int piece_chunk(int32_t i) {
    const KernArgs kp = kernargs();
    return kp->bal_chunks == 0 ? i : kp->wave0 + (int32_t)blockIdx.x + i * (int32_t)gridDim.x;
}
__device__ __forceinline__ Piece piece_of(uint4 pl, int q, int K) {
    const int32_t e = (int32_t)pl.x, f = (int32_t)pl.y, nf = (int32_t)pl.z, s = (int32_t)pl.w;
    if (e != 0) {
        if (q == 0) return Piece{f + nf, 0, e, false, true};                       // head
        --q;
    }
    if (q < nf) return Piece{f + q, 0, K, false, false};                           // whole chunks
    return Piece{f - 1, s, K, true, false};                                        // tail
}
// Issue priority of a wave of the balanced schedule (s_setprio, 3 = the
// highest).  A SIMD's arbiter issues from the oldest ready wave of the
// highest priority, so among long-lived waves of equal work the oldest race
// ahead and the youngest starve until they are left alone at low occupancy
// (measured: waves of equal work ended between 560 and 1,278 us of a 1.28 ms
// launch, profiles/r4_a3).  Each wave therefore starts at 3 and steps down as
// its own work runs out (band_end: at about 1/2, 3/4 and 9/10 of it, earlier
// for older workgroups), so a wave that got ahead yields to the ones behind it.
__device__ __forceinline__ void set_priority(int band) {
    if (band >= 3) __builtin_amdgcn_s_setprio(3);
    else if (band == 2) __builtin_amdgcn_s_setprio(2);
    else if (band == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}
// a wave's chunk-steps from its plan (balanced schedule)
__device__ __forceinline__ uint32_t plan_units(uint4 pl, int K) {
    return pl.x + pl.z * (uint32_t)K + (pl.w != 0 ? (uint32_t)K - pl.w : 0u);
}
// chunk-steps from the start of the wave's quarter to the end of band b (b =
// 3, 2, 1): E per mille of its work, shifted by D per mille for each
// dispatch round of the workgroup from the middle one (slot 0..W-1 of the W
// workgroups a CU holds; the oldest has slot 0).  The oldest still win every
// tie on their SIMD, so they step down earlier: slot 0 of 7 at 26 / 63 / 84 %
// of its work, slot 6 at 74 / 87 / 96 % (-3 to -4 % launch time against
// unshifted 50 / 75 / 90 %, profiles/r4_o, r4_p).  Tuning builds set others.
#ifndef RAFT_BAND_ENDS
#define RAFT_BAND_ENDS 500, 750, 900
#endif
#ifndef RAFT_AGE_SHIFTS
#define RAFT_AGE_SHIFTS 80, 40, 20
#endif
template <int W>
__device__ __forceinline__ uint32_t band_end(uint32_t Q, int b) {
    constexpr int E[3] = {RAFT_BAND_ENDS};
    constexpr int D[3] = {RAFT_AGE_SHIFTS};
    const int slot = (int)((blockIdx.x * (uint32_t)W) / gridDim.x);    // wave-uniform
    return (uint32_t)(((uint64_t)Q * (uint32_t)(E[3 - b] + (2 * slot - (W - 1)) * D[3 - b] / 2)) / 1000u);
}

// Bounded wait for the previous wave's head piece (never reached by a correct
// schedule without the flag set; the bound keeps a broken one from hanging the
// GPU).  A wave that gives up sets RAFT_DEV_WAIT_TIMEOUT in the engine's
// status word (page-locked host memory, a vector atomic), and the engine's
// next sync, step or kernel_time returns RAFT_EDEVICE: the launch's results
// are not the reference's.  The flag is set after the producer's stores
// completed (vmcnt(0)); the producer is on this CU, whose vector L1 is
// invalidated here before the chunk's state is read.
__device__ __forceinline__ void wait_head(const uint32_t* flag) {
    bool set = false;
    for (uint32_t spins = 0; spins < (1u << 24); ++spins) {
        if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u) {
            set = true;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    if (!set) {
        const KernArgs kp = kernargs();
        if ((threadIdx.x & 63) == 0)
            __hip_atomic_fetch_or(kp->status, RAFT_DEV_WAIT_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    asm volatile("buffer_inv sc0\n\ts_waitcnt vmcnt(0)" ::: "memory");
}

// Enter a piece: chunk `wid`'s replicas into VGPRs.  The lane geometry comes
// from the context (lane = base + r, group j = base / R) and the parameters
// from the kernarg segment: kept live across the step loop for the next
// piece's entry, they would pin registers (kernargs()).
template <int R, bool RING>
__device__ __forceinline__ void enter_piece(Ctx<R>& c, Node& n, int wid) {
    using L = Lanes<R>;
    const KernArgs kp = kernargs();
    DevParams p;
    p.st = kp->st; p.gx = kp->gx; p.GR = kp->GR; p.G = kp->G;
    const int j = (int)c.j();
    const int64_t g = (int64_t)wid * L::GPW + j;
    c.live = j < L::GPW && g < p.G;
    c.wg0 = (uint32_t)__builtin_amdgcn_readfirstlane(wid * L::GPW);
    c.gg0 = (uint32_t)(kp->g0 + c.wg0);
    c.lr = kp->log + ((int64_t)wid * 64 + c.base + c.r) * (RING ? kp->nslots : kp->cap);   // its chunk's block, its row
    if (c.live) load_node(n, p, g, g * R + c.r);
    else inert_node(n);
    c.lead = c.gbits(__ballot(n.role == RAFT_LEADER));                  // Stepper::step's lead0 of the first step
    // Drain the state loads here: left pending into the loop, they make the
    // loop header wait on vmcnt(0) every step -- and vmcnt also counts the
    // previous step's log stores, so each step would start by waiting for them.
    __builtin_amdgcn_s_waitcnt(0x0F70);                                   // vmcnt(0)
}

// EPOCHS: the kernel of a launch run as epochs (a separate instantiation, so
// that the others carry none of its code: its epoch boundary in the step loop
// costs the register allocation 2 VGPRs)
template <int R, bool TB, bool RING, int NET, bool EPOCHS = false>
__global__ __launch_bounds__(STEP_BLOCK) __attribute__((amdgpu_waves_per_eu(RAFT_STEP_WAVES_PER_EU(R, TB, RING, NET))))
void step_kernel(DevParams p, uint32_t t0, int nsteps) {
    using L = Lanes<R>;
    constexpr int SLOTS = RAFT_STEP_WAVES_PER_EU(R, TB, RING, NET);   // workgroups a CU holds (band_end)
    // LDS: [STEP_WAVES][64][4] the step's Philox job words (Ctx::jl), the
    // tally words, the head-piece flags, then the counter rows [nsteps][NCW]
    extern __shared__ uint32_t lds[];
    uint32_t* const lds_cnt = lds + PRE_CNT_LDS_WORDS;
    uint32_t* const lds_flag = lds + JOB_LDS_WORDS + TALLY_LDS_WORDS;
    uint32_t* const lds_plan = lds_flag + FLAG_LDS_WORDS;
    const int lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: the schedule's loop is uniform
    const int j = lane / R;
    const int r = lane - j * R;

#ifdef RAFT_WAVE_TIMES
    const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
    // A balanced launch longer than the LDS rows hold runs as epochs of
    // `epoch` steps: each epoch is the schedule of a launch of that length
    // (the same chunks, McNaughton split, hand-off and priority bands), and
    // at its end the workgroup's waves meet at a barrier, copy the epoch's
    // counter rows to the partials and zero them.  Only the workgroup's four
    // waves wait for each other there (their SIMDs issue other workgroups'
    // waves meanwhile), where a launch boundary waits for every wave of the
    // chip.
    const int elen = EPOCHS && p.epoch > 0 && p.epoch < nsteps ? p.epoch : nsteps;
    for (int q = threadIdx.x; q < elen * NCW; q += STEP_BLOCK) lds_cnt[q] = 0u;
    if (threadIdx.x < FLAG_LDS_WORDS) lds_flag[threadIdx.x] = 0u;
    __syncthreads();                                                      // counter rows and flags zeroed

    Ctx<R> c;
    c.r = r;
    c.base = j * R;
    c.iso = -1;
    c.iso_me = 0;
    c.part = 0;
    c.part_me = 0;
    c.job = u32x4{0u, 0u, 0u, 0u};
    c.tw = c.dwt = c.dwv = 0u;
    c.jl = lds + wib * 256;
    c.tl = lds + JOB_LDS_WORDS + wib * 16;
    c.clk.start();
#ifdef RAFT_BRANCH_STATS
    for (int q = 0; q < BS_N; ++q) c.bs[q] = 0;
#endif
    Node n;
    // One loop over the wave's chunk-steps; a piece boundary (the launch's
    // end in the one-chunk-per-wave schedule) is a rare branch in it that
    // stores the chunk and loads the next.  (A loop over pieces around the
    // step loop made the compiler hoist and duplicate: 76 B of scratch and
    // +600 static VALU at R = 5.)
    int pc = 0;                                    // this wave's current piece
    int k, k1;                                     // its step, the step it ends before
    int band_left;                                 // chunk-steps to the next priority band (balanced)
    // steps are counted from the epoch's start (k, the pieces' k0 / k1, the
    // counter rows); the epoch's first step is tb - t0, its first step index
    // tb, and its length and first step sit in the wave's plan words [5], [7]
    uint32_t tb = t0;
    {   // (a wave's first piece is never a tail: a wave runs its head first)
        const uint4 pl = plan_of(wib, elen);
        *(uint4*)(lds_plan + wib * 16) = pl;
        // [8..11]: the plan of a whole epoch, [12..15]: of the last one (the
        // epoch boundary only reads them: plan_of's divisions in the step
        // loop made the register allocation spill)
        *(uint4*)(lds_plan + wib * 16 + 8) = pl;
        if (EPOCHS && elen < nsteps)
            *(uint4*)(lds_plan + wib * 16 + 12) = plan_of(wib, nsteps - (nsteps - 1) / elen * elen);
        const bool bal = kernargs()->bal_chunks != 0;
        const uint32_t Q = plan_units(pl, elen);
        // [4]: the band now, [5]: the epoch's length, [6]: Q, [7]: its first step
        *(uint4*)(lds_plan + wib * 16 + 4) = make_uint4(3u, (uint32_t)elen, Q, 0u);
        band_left = bal ? (int)band_end<SLOTS>(Q, 3) : 0x7FFFFFFF;
        if (bal) set_priority(3);
        const Piece pz = piece_of(pl, 0, elen);
        enter_piece<R, RING>(c, n, piece_chunk(pz.chunk));
        k = pz.k0;
        c.part = PART_STALE;
        k1 = pz.k1;
    }
    for (;;) {
        const uint32_t t = tb + (uint32_t)k;
        c.t = t;
        // The lane geometry (r, base) is carried across steps behind an opaque
        // copy: otherwise the optimiser hoists dozens of loop-invariant lane
        // masks (r == 1, r < 2, ...) out of the step loop, and each one pins an
        // SGPR pair for the whole kernel (spilled to VGPR lanes and reloaded at
        // every use).  (Round 1 re-derived both from the lane id each step:
        // 6 VALU more per wave-step and 6 VGPRs more at R = 5, profiles/r2_geom.)
        {
            int cb = c.base, cr = c.r;
            asm volatile("" : "+v"(cb), "+v"(cr));
            c.base = cb;
            c.r = cr;
        }
        c.part_me = 0;                                                    // made each step: not loop-carried
        if constexpr ((NET & NET_PART) != 0) {
            const KernArgs kp = kernargs();
            const int32_t pperiod = kp->part_period;
            if (pperiod > 0) {                                            // S-11 partitions
                const uint32_t ph = t % (uint32_t)pperiod;
                if ((int64_t)ph < kp->part_len) {
                    // (a piece enters with c.part = PART_STALE: its first step in a window draws)
                    if ((int32_t)c.part < 0 || ph == 0) c.part = kdraw(p, t - ph, c.gid(), RAFT_RNG_PARTITION, 0).x & L::ALL;
                } else {
                    c.part = 0;
                }
                c.part_me = lm((c.part >> c.r) & 1u);
            }
        }
        Counters cnt;
        cnt.clear();
        Stepper<R, TB, RING, NET>::step(p, c, n, cnt);
        c.clk.mark(PH_TDRAW);
        uint32_t v = 0;                                                     // lane cw <- wave total cw
#pragma unroll
        for (int cw = 0; cw < NCW; ++cw) v = (uint32_t)raft_writelane((int32_t)cnt.s[cw], cw, (int32_t)v);
        // < 2^16 per half per workgroup: a wave counts < 2^13 events of a kind per step
        // lanes 0 .. NCW-1 as a constant lane mask (lane < NCW would be a compare
        // hoisted out of the loop and spilled)
        if (ib((1ull << NCW) - 1))
            __hip_atomic_fetch_add(&lds_cnt[k * NCW + lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        c.clk.mark(PH_CNT);
        if (RARE(--band_left == 0)) {              // this wave's next priority band (balanced)
            const int wb = __builtin_amdgcn_readfirstlane((int)((c.jl - lds) >> 8));
            uint4 bs = *(const uint4*)(lds_plan + wb * 16 + 4);
            const int b = __builtin_amdgcn_readfirstlane((int)bs.x) - 1;
            const uint32_t Q = __builtin_amdgcn_readfirstlane(bs.z);
            set_priority(b);
            band_left = b > 0 ? (int)(band_end<SLOTS>(Q, b) - band_end<SLOTS>(Q, b + 1)) : 0x7FFFFFFF;
            *(lds_plan + wb * 16 + 4) = (uint32_t)b;
        }
        if (++k == k1) {                           // the piece ends: store its chunk (rare)
            if (c.live) {
                const KernArgs kp = kernargs();    // state pointers re-read, not kept live across the loop
                DevParams q;
                q.st = kp->st; q.gx = kp->gx; q.GR = kp->GR; q.G = kp->G;
                store_node(n, q, (int64_t)c.wg0 + j, c.idx(), r == 0);
            }
            // this wave's index from its job rows' address (kept live across
            // the loop, the index would pin a register)
            const int wb = __builtin_amdgcn_readfirstlane((int)((c.jl - lds) >> 8));
            uint4 pl = *(const uint4*)(lds_plan + wb * 16);
            pl.x = __builtin_amdgcn_readfirstlane(pl.x);        // one word for the whole wave
            pl.y = __builtin_amdgcn_readfirstlane(pl.y);
            pl.z = __builtin_amdgcn_readfirstlane(pl.z);
            pl.w = __builtin_amdgcn_readfirstlane(pl.w);
            if (pc == 0 && pl.x != 0) {            // a head stored: the next wave's tail may load it
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(lds_flag + wb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (++pc == n_pieces(pl)) {
                if constexpr (!EPOCHS) break;
                const uint32_t ke = __builtin_amdgcn_readfirstlane(lds_plan[wb * 16 + 5]);
                const uint32_t kb = __builtin_amdgcn_readfirstlane(lds_plan[wb * 16 + 7]);
                if (kb + ke >= (uint32_t)nsteps) break;
                // the epoch ends: its rows to the partials (rows [kb, kb + ke)
                // of the launch), zeroed for the next; the chunks' states of
                // every wave stored (vmcnt(0) before the barrier) and this
                // CU's vector L1 invalidated before the next epoch loads them
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                {
                    // (the thread index behind an opaque copy: hoisted out of
                    // the step loop, its products would pin registers there)
                    int tid = (int)threadIdx.x;
                    asm volatile("" : "+v"(tid));
                    const KernArgs kp = kernargs();
                    uint32_t* const part = kp->part + kp->part_col0 + blockIdx.x;
                    const uint32_t stride = (uint32_t)kp->part_stride;          // partials < 2^32 words
                    for (int q = tid; q < (int)ke * NCW; q += STEP_BLOCK) {
                        part[(kb * NCW + (uint32_t)q) * stride] = lds_cnt[q];
                        lds_cnt[q] = 0u;
                    }
                    if (tid < FLAG_LDS_WORDS) lds_flag[tid] = 0u;
                }
                __syncthreads();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                asm volatile("buffer_inv sc0\n\ts_waitcnt vmcnt(0)" ::: "memory");
                const uint32_t kb2 = kb + ke;
                const int ke2 = min(kernargs()->epoch, nsteps - (int)kb2);
                tb += ke;
                pl = *(const uint4*)(lds_plan + wb * 16 + (ke2 == kernargs()->epoch ? 8 : 12));
                pl.x = __builtin_amdgcn_readfirstlane(pl.x);
                pl.y = __builtin_amdgcn_readfirstlane(pl.y);
                pl.z = __builtin_amdgcn_readfirstlane(pl.z);
                pl.w = __builtin_amdgcn_readfirstlane(pl.w);
                *(uint4*)(lds_plan + wb * 16) = pl;
                const uint32_t Q = plan_units(pl, ke2);
                *(uint4*)(lds_plan + wb * 16 + 4) = make_uint4(3u, (uint32_t)ke2, Q, kb2);
                band_left = (int)band_end<SLOTS>(Q, 3);
                set_priority(3);
                pc = 0;
            }
            const int kel = EPOCHS ? (int)__builtin_amdgcn_readfirstlane(lds_plan[wb * 16 + 5]) : nsteps;
            const Piece pz = piece_of(pl, pc, kel);
            if (pz.wait) wait_head(lds_flag + wb - 1);
            enter_piece<R, RING>(c, n, piece_chunk(pz.chunk));
            k = pz.k0;
            c.part = PART_STALE;
            k1 = pz.k1;
        }
    }
#ifdef RAFT_PROFILE_PHASES
    if (lane == 0)
        for (int q = 0; q < PH_N; ++q) atomicAdd(&g_phase_cycles[q], (unsigned long long)c.clk.acc[q]);
#endif
#ifdef RAFT_BRANCH_STATS
    if (lane == 0)
        for (int q = 0; q < BS_N; ++q) atomicAdd(&g_branch_stats[q], (unsigned long long)c.bs[q]);
#endif
#ifdef RAFT_WAVE_TIMES
    {
        const unsigned long long wt1 = __builtin_amdgcn_s_memrealtime();
        const int w = blockIdx.x * STEP_WAVES + wib;
        if (lane == 0 && w < WT_MAX) {
            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);        // HW_REG_HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);      // HW_REG_XCC_ID
            g_wave_times[w][0] = wt0;
            g_wave_times[w][1] = wt1;
            g_wave_times[w][2] = ((unsigned long long)xcc << 32) | hw;
        }
    }
#endif
    __syncthreads();
    {   // workgroup partials; the launch's partials geometry re-read from the
        // kernarg segment (held across the step loop it would pin SGPRs)
        const KernArgs kp = kernargs();
        uint32_t* const part = kp->part + kp->part_col0 + blockIdx.x;
        const int64_t stride = kp->part_stride;
        const int ke = EPOCHS ? (int)lds_plan[5] : nsteps, kb = EPOCHS ? (int)lds_plan[7] : 0;   // (the last epoch)
        for (int q = threadIdx.x; q < ke * NCW; q += STEP_BLOCK) part[((int64_t)kb * NCW + q) * stride] = lds_cnt[q];
    }
}

// Traffic probes (rocprofv3 calibration of FETCH_SIZE / WRITE_SIZE; never on
// the step path): the step kernel's own HBM access patterns over a known
// byte count, in the same process and on the same box as the launches they
// calibrate.  One wave per chunk, the step kernel's lane geometry.
//  kind 0: each chunk's state into VGPRs and back, exactly as a piece's entry
//          and exit (load_node / store_node): G * (R * 64 + 12) bytes read and
//          the same written, values unchanged.
//  kind 1: one 8-byte store per replica into its own log row at slot physLen
//          (a flat log's slot past the last entry, never read), the pattern of
//          Log.add (Commons.kt:56-68): 8 bytes per store, counted in *stores.
template <int R>
__global__ __launch_bounds__(BLOCK) void traffic_probe_kernel(DevParams p, int kind, int nwaves,
                                                              unsigned long long* stores) {
    constexpr int GPW = 64 / R;
    const int w = blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
    if (w >= nwaves) return;                                            // wave-uniform
    const int lane = threadIdx.x & 63, j = lane / R, r = lane - j * R;
    const int64_t g = (int64_t)w * GPW + j;
    const bool live = j < GPW && g < p.G;
    const int64_t idx = g * R + r;
    if (kind == 0) {
        Node n;
        if (live) load_node(n, p, g, idx);
        else inert_node(n);
        asm volatile("" : "+v"(n.term), "+v"(n.voted), "+v"(n.role), "+v"(n.commit), "+v"(n.last), "+v"(n.phys));
        asm volatile("" : "+v"(n.elec), "+v"(n.fl), "+v"(n.phase), "+v"(n.retry), "+v"(n.t1), "+v"(n.t2), "+v"(n.c1));
        asm volatile("" : "+v"(n.nx), "+v"(n.mc), "+v"(n.iso), "+v"(n.cmdc), "+v"(n.s0));
        if (live) store_node(n, p, g, idx, r == 0);
    } else {
        const int32_t phys = live ? p.st[fidx(p, RAFT_F_PHYS, idx)] : p.cap;
        const bool st = phys < p.cap;
        if (st) p.log[((int64_t)w * 64 + lane) * p.nslots + phys] = make_uint2(0u, 0u);
        const uint64_t b = __ballot(st);
        if (lane == 0 && b) atomicAdd(stores, (unsigned long long)__popcll(b));
    }
}

// Scattered-access probes (the handler batches' calibration, include/raft_engine.h
// RAFT_PROBE_SCATTER_*): thread i touches one 4-byte word at the start of
// sector s(i) = (i * 2654435761) mod 2^SCATTER_LOG2 of a scratch buffer of
// 32-byte sectors -- an odd multiplier, so the n < 2^SCATTER_LOG2 sectors are
// distinct and spread over the whole buffer like a random replica's fields.
// kind 2 loads (sunk), kind 3 stores; the known traffic is n sectors of 32 B.
constexpr int SCATTER_LOG2 = 24;                          // 2^24 sectors: a 512 MB scratch
constexpr int SCATTER_N = 1 << 21;                        // sectors touched per probe
__global__ __launch_bounds__(BLOCK) void scatter_probe_kernel(uint32_t* scratch, int kind) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t s = (i * 2654435761u) & ((1u << SCATTER_LOG2) - 1u);
    uint32_t* w = scratch + (size_t)s * 8;
    if (kind == 2) {
        const uint32_t v = *w;                                // a plain load, as the handlers' field reads
        asm volatile("" ::"v"(v));                            // kept: nothing else consumes it
    } else {
        *w = i;
    }
}

// the retained physical slots of a replica: [max(0, physLen - W), physLen)
__device__ __forceinline__ int32_t window_lo(const DevParams& p, int32_t phys) { return max(0, phys - p.W); }

// (re)derive the log-tail cache from lastIndex and the log (after host writes)
__global__ __launch_bounds__(BLOCK) void rebuild_cache_kernel(DevParams p) {
    const int64_t idx = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (idx >= p.GR) return;
    const int32_t last = p.st[fidx(p, RAFT_F_LAST, idx)];
    const LogView lv = log_of(p, idx);
    const uint2 a = last >= 1 ? *lv.at(last - 1) : make_uint2(0u, 0u);
    const uint2 b = last >= 2 ? *lv.at(last - 2) : make_uint2(0u, 0u);
    p.st[fidx(p, F_T1, idx)] = (int32_t)a.x;
    p.st[fidx(p, F_C1, idx)] = (int32_t)a.y;
    p.st[fidx(p, F_T2, idx)] = (int32_t)b.x;
}

// counters[k][c] = sum over the step workgroups b of the 16-bit half of
// partials[k][][b] at COUNTER_SLOT[c] (raft_step.h), in ONE dispatch with no memset (a memset, an
// atomic-add reduction and their two dependent dispatch gaps were ~6 % of a
// 20-step run).  Grid chunks x nsteps * NCW: each workgroup sums both halves
// of one packed counter word over a chunk of REDUCE_CHUNK partials (each word
// is read once) and adds each half, with a ticket of 1 << 48, into that
// counter's 64-bit accumulator (one returning atomic, no fence: a
// device-scope fence writes back the L2 and cost more than the whole
// reduction).  The workgroup that draws a counter's last ticket stores its
// total outright and resets the accumulator for the next launch.  The first
// chunk of word 0 zeroes the row's padding.  A step's count is far below 2^48.
constexpr int REDUCE_CHUNK = 16 * BLOCK;
constexpr int ACC_TICKET_SH = 48;
__device__ __forceinline__ uint32_t part_word(const uint32_t* part, int64_t k, int w, int64_t nparts, int b) {
    return part[(k * NCW + w) * nparts + b];
}
// counter c's half of a partial word of its slot
__device__ __forceinline__ uint32_t half_of(uint32_t x, int c) { return (x >> (16 * (COUNTER_SLOT[c] & 1))) & 0xFFFFu; }
// One counter's total: a direct store for a one-chunk grid, else the ticketed accumulator.
__device__ __forceinline__ void reduce_emit(int64_t* row, int c, unsigned long long s, unsigned long long nch,
                                            unsigned long long* acc) {
    if (nch == 1) {
        row[c] = (int64_t)s;
        return;
    }
    const unsigned long long old = atomicAdd(acc, s + (1ull << ACC_TICKET_SH));
    if ((old >> ACC_TICKET_SH) != nch - 1) return;
    row[c] = (int64_t)((old + s) & ((1ull << ACC_TICKET_SH) - 1));
    atomicExch(acc, 0ull);                                 // ready for the next launch (stream-ordered)
}
// APPEND_SKIPPED is derived per workgroup partial as R * SESSIONS_TICKED -
// APPEND_SENT (the step kernel does not count it, see Stepper::tick).
// Grid: nch chunks x (K * NCW) words, flattened (a launch of 10^4 steps has
// more words than a grid dimension of 2^16).
__global__ __launch_bounds__(BLOCK) void reduce_counters_kernel(const uint32_t* __restrict__ partials, int nparts,
                                                                int nch_, int R, int64_t* __restrict__ counters,
                                                                unsigned long long* __restrict__ accum) {
    __shared__ uint32_t acc[2][WAVES_PER_BLOCK];
    const int kw = (int)(blockIdx.x / (unsigned)nch_), chunk = (int)(blockIdx.x - (unsigned)kw * (unsigned)nch_);
    const int k = kw / NCW, w = kw % NCW;
    const int c0 = counter_of_slot(2 * w), c1 = counter_of_slot(2 * w + 1);   // -1: an unused slot
    const int b0 = chunk * REDUCE_CHUNK;
    constexpr int SK = RAFT_C_APPEND_SKIPPED;
    constexpr int TK = RAFT_C_SESSIONS_TICKED, SN = RAFT_C_APPEND_SENT;
    uint32_t lo = 0, hi = 0;        // < 2^19 * 16 per thread
#pragma unroll
    for (int i = 0; i < REDUCE_CHUNK / BLOCK; ++i) {      // independent loads
        const int b = b0 + i * BLOCK + threadIdx.x;
        if (b < nparts) {
            const uint32_t x = part_word(partials, k, w, nparts, b);
            uint32_t d = 0;
            if (w == COUNTER_SLOT[SK] >> 1)
                d = (uint32_t)R * half_of(part_word(partials, k, COUNTER_SLOT[TK] >> 1, nparts, b), TK) -
                    half_of(part_word(partials, k, COUNTER_SLOT[SN] >> 1, nparts, b), SN);
            lo += c0 == SK ? d : x & 0xFFFFu;
            hi += c1 == SK ? d : x >> 16;
        }
    }
    const uint32_t wl = __ockl_wfred_add_u32(lo), wh = __ockl_wfred_add_u32(hi);   // < 2^19 * 1024 = 2^29
    if ((threadIdx.x & 63) == 0) {
        acc[0][threadIdx.x >> 6] = wl;
        acc[1][threadIdx.x >> 6] = wh;
    }
    __syncthreads();
    int64_t* row = counters + (int64_t)k * RAFT_COUNTER_STRIDE;
    if (w == 0 && chunk == 0 && threadIdx.x >= NC && threadIdx.x < RAFT_COUNTER_STRIDE) row[threadIdx.x] = 0;
    if (threadIdx.x != 0) return;
    unsigned long long sl = 0, sh = 0;
    for (int q = 0; q < WAVES_PER_BLOCK; ++q) {
        sl += acc[0][q];
        sh += acc[1][q];
    }
    const unsigned long long nch = (unsigned long long)nch_;
    if (c0 >= 0) reduce_emit(row, c0, sl, nch, &accum[(int64_t)k * NC + c0]);
    if (c1 >= 0) reduce_emit(row, c1, sh, nch, &accum[(int64_t)k * NC + c1]);
}

// canonical export [n][W] of groups [g0, g0+n): one thread per group
template <int R>
__global__ __launch_bounds__(BLOCK) void pack_kernel(DevParams p, int64_t g0, int64_t n, int32_t* out) {
    const int64_t jx = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (jx >= n) return;
    const int64_t g = g0 + jx;
    constexpr int W = R * RAFT_NUM_FIELDS + 2 * R * R + RAFT_GROUP_EXTRA;
    int32_t* w = out + jx * W;
    for (int r = 0; r < R; ++r)
        for (int f = 0; f < RAFT_NUM_FIELDS; ++f) {
            const int32_t v = p.st[fidx(p, f, g * R + r)];
            w[r * RAFT_NUM_FIELDS + f] = f == RAFT_F_FLAGS ? (int32_t)((uint32_t)v & FL_EXPORT_MASK) : v;
        }
    const int s0 = p.gx[GX_S0 * p.G + g];
    for (int s = 0; s < R; ++s)
        for (int d = 0; d < R; ++d) {
            w[R * RAFT_NUM_FIELDS + s * R + d] = canon_next(p, R, g, s0, s, d);
            w[R * RAFT_NUM_FIELDS + R * R + s * R + d] = canon_match(p, R, g, s0, s, d);
        }
    w[W - 2] = p.gx[GX_ISO * p.G + g];
    w[W - 1] = p.gx[GX_CMDS * p.G + g];
}

template <int R>
__global__ __launch_bounds__(BLOCK) void unpack_kernel(DevParams p, int64_t g0, int64_t n, const int32_t* in) {
    const int64_t jx = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (jx >= n) return;
    const int64_t g = g0 + jx;
    constexpr int W = R * RAFT_NUM_FIELDS + 2 * R * R + RAFT_GROUP_EXTRA;
    const int32_t* w = in + jx * W;
    for (int r = 0; r < R; ++r)
        for (int f = 0; f < RAFT_NUM_FIELDS; ++f) p.st[fidx(p, f, g * R + r)] = w[r * RAFT_NUM_FIELDS + f];
    // every session row goes to spill; no primary until a session ticks
    for (int s = 0; s < R; ++s)
        for (int d = 0; d < R; ++d) {
            const int64_t idx = g * R + d;
            p.spill[idx * R + s] = w[R * RAFT_NUM_FIELDS + s * R + d];
            p.spill[p.GR * R + idx * R + s] = w[R * RAFT_NUM_FIELDS + R * R + s * R + d];
        }
    p.gx[GX_ISO * p.G + g] = w[W - 2];
    p.gx[GX_CMDS * p.G + g] = w[W - 1];
    p.gx[GX_S0 * p.G + g] = -1;
}

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// order-independent state digest: sum of per-group FNV-1a/fmix64
template <int R>
__global__ __launch_bounds__(BLOCK) void log_match_kernel(DevParams p, int64_t g0, int64_t n, uint8_t* flags,
                                                         unsigned long long* count) {
    // one wave per group; the lanes stride the log indices, so each replica's
    // committed prefix is read as coalesced 512-B runs
    const int lane = threadIdx.x & 63;
    const int64_t k = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6);
    if (k >= n) return;                                                   // wave-uniform
    const int64_t g = g0 + k;
    int32_t c[R], lo[R];
    int32_t cmax = 0, lmin = 0x7FFFFFFF;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t idx = g * R + r;
        const int32_t cm = min(p.st[fidx(p, RAFT_F_COMMIT, idx)], p.st[fidx(p, RAFT_F_LAST, idx)]);
        c[r] = max(0, min(cm, p.cap));
        lo[r] = window_lo(p, p.st[fidx(p, RAFT_F_PHYS, idx)]);     // retained slots only
        cmax = max(cmax, c[r]);
        lmin = min(lmin, lo[r]);
    }
    bool bad = false;
    for (int32_t i = lmin + lane; i < cmax; i += 64) {
        bool have = false;
        uint2 ref = make_uint2(0u, 0u);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (i < c[r] && i >= lo[r]) {
                const uint2 v = *log_of(p, g * R + r).at(i);
                bad |= have && (v.x != ref.x || v.y != ref.y);
                ref = have ? ref : v;
                have = true;
            }
        }
    }
    const bool any = __ballot(bad) != 0;
    if (lane == 0) {
        if (flags) flags[k] = any ? 1 : 0;
        if (any) atomicAdd(count, 1ull);
    }
}

template <int R>
__global__ __launch_bounds__(BLOCK) void digest_kernel(DevParams p, int64_t g0, int64_t n, unsigned long long* out) {
    __shared__ unsigned long long part[WAVES_PER_BLOCK];
    const int64_t g = g0 + (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint64_t hv = 0;
    if (g < g0 + n) {
        uint64_t h = 0xcbf29ce484222325ull ^ ((uint64_t)(p.g0 + g) * 0x9E3779B97F4A7C15ull);
        auto feed = [&](int32_t v) { h ^= (uint32_t)v; h *= 0x100000001b3ull; };
        const int s0 = p.gx[GX_S0 * p.G + g];
        for (int r = 0; r < R; ++r) {
            const int64_t idx = g * R + r;
            for (int f = 0; f < RAFT_NUM_FIELDS; ++f) {
                const int32_t v = p.st[fidx(p, f, idx)];
                feed(f == RAFT_F_FLAGS ? (int32_t)((uint32_t)v & FL_EXPORT_MASK) : v);
            }
            for (int d = 0; d < R; ++d) feed(canon_next(p, R, g, s0, r, d));
            for (int d = 0; d < R; ++d) feed(canon_match(p, R, g, s0, r, d));
            const int32_t phys = p.st[fidx(p, RAFT_F_PHYS, idx)];
            const LogView lv = log_of(p, idx);
            for (int32_t q = window_lo(p, phys); q < phys; ++q) {
                const uint2 e = *lv.at(q);
                feed((int32_t)e.x);
                feed((int32_t)e.y);
            }
        }
        feed(p.gx[GX_ISO * p.G + g]);
        feed(p.gx[GX_CMDS * p.G + g]);
        hv = fmix64(h);
    }
    // wave sum of 64-bit values
    uint32_t lo = (uint32_t)hv, hi = (uint32_t)(hv >> 32);
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t olo = __shfl_xor(lo, o, 64), ohi = __shfl_xor(hi, o, 64);
        const uint64_t s = ((uint64_t)hi << 32 | lo) + ((uint64_t)ohi << 32 | olo);
        lo = (uint32_t)s; hi = (uint32_t)(s >> 32);
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = (uint64_t)hi << 32 | lo;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int w = 0; w < WAVES_PER_BLOCK; ++w) s += part[w];
        atomicAdd(out, s);
    }
}

// read_log / write_log: the host's [n][R][log_cap] image of groups [g0, g0+n)
// <-> the engine's log rows.  A read copies the retained slots [max(0,
// physLen - W), physLen) (the rest reads as 0).  A write to a flat log
// (log_window 0) stores every slot below log_cap, so it does not depend on
// the physLen in the engine at the time; a write to a ring stores the slots
// the current physLen retains (write_state first, include/raft_engine.h).
__global__ __launch_bounds__(BLOCK) void log_image_kernel(DevParams p, int64_t g0, int64_t n, uint2* img, int to_ring) {
    const int64_t total = n * p.R * (int64_t)p.cap;
    for (int64_t k = (int64_t)blockIdx.x * BLOCK + threadIdx.x; k < total; k += (int64_t)gridDim.x * BLOCK) {
        const int64_t rr = k / p.cap;                                     // (group - g0) * R + r
        const int32_t j = (int32_t)(k - rr * p.cap);
        const int64_t idx = g0 * p.R + rr;
        const int32_t phys = p.st[fidx(p, RAFT_F_PHYS, idx)];
        const bool in = j >= window_lo(p, phys) && j < phys;
        uint2* slot = log_of(p, idx).at(j);
        if (to_ring) {
            if (in || p.W == FLAT_W) *slot = img[k];
        } else {
            img[k] = in ? *slot : make_uint2(0u, 0u);
        }
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

template <template <int> class Fn, typename... A>
static void dispatch_R(int R, A&&... a) {
#ifdef RAFT_ISA_ONLY_R              // ISA inspection builds (scripts/isa_stats.sh): one R only
    if (R == RAFT_ISA_ONLY_R) Fn<RAFT_ISA_ONLY_R>::run(a...);
#else
    switch (R) {
        case 1: Fn<1>::run(a...); break;
        case 2: Fn<2>::run(a...); break;
        case 3: Fn<3>::run(a...); break;
        case 4: Fn<4>::run(a...); break;
        case 5: Fn<5>::run(a...); break;
        case 6: Fn<6>::run(a...); break;
        case 7: Fn<7>::run(a...); break;
        case 8: Fn<8>::run(a...); break;
        default: break;
    }
#endif
}

template <int R> struct InitL {
    static void run(raft_engine* e) {
        const unsigned nb = (unsigned)((e->dp.GR + BLOCK - 1) / BLOCK);
        init_kernel<R><<<nb, BLOCK, 0, e->stream>>>(e->dp);
    }
};
// The step kernel for the engine's network faults: at the replica counts of
// BASELINE.json's configurations (3, 5, 7) a kernel built for drops and
// isolation churn without partitions, with config 3's command harness (the
// lowest LEADER, no limit), or for partitions alone (config 5, and no faults
// at all: configs 1 and 2), so the other checks are compiled out; otherwise
// the NET_ALL kernel.  `iso`: churn is configured or an isolation word was
// written into the state (raft_engine_write_state).
typedef void (*StepKernel)(DevParams, uint32_t, int);
static int step_net(const DevParams& d, const raft_params& p, int R, bool iso) {
    if (R == 3 || R == 5 || R == 7) {
        const bool drops = d.drop_thr16 != 0, parts = p.partition_period > 0 && p.partition_len > 0;
        const bool cmdlow = p.cmd_mode == RAFT_CMD_LOWEST_LEADER && p.cmd_limit == 0;
        if (drops && !parts && cmdlow) return NET_DROP | NET_ISO | NET_CMDLOW;
        if (!drops && !iso) return NET_PART;
    }
    return NET_ALL;
}
template <int R, bool TB, bool RING>
static StepKernel step_fn(const DevParams& d, const raft_params& p, bool iso) {
    if (p.kernel == RAFT_KERNEL_GENERAL) return step_kernel<R, TB, RING, NET_ALL>;
    if constexpr (R == 3 || R == 5 || R == 7) {
        const int net = step_net(d, p, R, iso);
        if (net == (NET_DROP | NET_ISO | NET_CMDLOW)) return step_kernel<R, TB, RING, NET_DROP | NET_ISO | NET_CMDLOW>;
        if (net == NET_PART) return step_kernel<R, TB, RING, NET_PART>;
    }
    return step_kernel<R, TB, RING, NET_ALL>;
}
// the epochs kernels: the reference mode's drops + churn kernel (config 3 and
// its shards) and the general kernel; a launch of another is cut (nullptr)
template <int R, bool RING>
static StepKernel step_fn_epochs(const DevParams& d, const raft_params& p, bool iso) {
    if (p.kernel == RAFT_KERNEL_GENERAL) return step_kernel<R, false, RING, NET_ALL, true>;
    if constexpr (R == 3 || R == 5 || R == 7) {
        const int net = step_net(d, p, R, iso);
        if (net == (NET_DROP | NET_ISO | NET_CMDLOW)) return step_kernel<R, false, RING, NET_DROP | NET_ISO | NET_CMDLOW, true>;
        if (net == NET_PART) return nullptr;
    }
    return step_kernel<R, false, RING, NET_ALL, true>;
}
template <int R> struct KernL {
    static void run(raft_engine* e, bool epochs, StepKernel* out) {
        // a flat log (log_window 0) keeps every slot: the kernel without window checks
        const bool iso = e->dp.churn_thr32 != 0 || e->iso_written;
        if (epochs)
            *out = e->p.mode == RAFT_MODE_TEXTBOOK ? nullptr
                   : (e->p.log_window ? step_fn_epochs<R, true>(e->dp, e->p, iso)
                                      : step_fn_epochs<R, false>(e->dp, e->p, iso));
        else
            *out = e->p.mode == RAFT_MODE_TEXTBOOK
                       ? (e->p.log_window ? step_fn<R, true, true>(e->dp, e->p, iso)
                                          : step_fn<R, true, false>(e->dp, e->p, iso))
                       : (e->p.log_window ? step_fn<R, false, true>(e->dp, e->p, iso)
                                          : step_fn<R, false, false>(e->dp, e->p, iso));
    }
};
static StepKernel step_kernel_of(raft_engine* e, bool epochs = false) {
    StepKernel k = nullptr;
    dispatch_R<KernL>(e->p.R, e, epochs, &k);
    return k;
}
static size_t step_lds_bytes(int k) { return (size_t)(PRE_CNT_LDS_WORDS + k * NCW) * 4; }

// One launch's geometry over the sub-ranges: sub-range q covers the chunks
// [w0[q], w0[q + 1]) with nb[q] workgroups, balanced (bal[q] = its chunks) or
// one chunk per wave (bal[q] = 0), and writes partial columns [col0[q],
// col0[q] + nb[q]) of a launch with `stride` columns.
struct LaunchGeo {
    int w0[RAFT_MAX_SUBRANGES + 1], nb[RAFT_MAX_SUBRANGES], col0[RAFT_MAX_SUBRANGES], bal[RAFT_MAX_SUBRANGES];
    int stride, resident, balanced;
    int epoch;                    // steps per epoch (0: one epoch)
};
static int launch_geo(raft_engine* e, StepKernel kern, int k, int epoch, LaunchGeo& geo) {
    const size_t lds = step_lds_bytes(epoch > 0 ? std::min(k, epoch) : k);
    // workgroups per CU, cached per (kernel, LDS bytes): a run alternates a
    // few launch lengths (warmup, timed, a remainder), and the query costs
    // ~1 us of host time ahead of the launch
    int slot = -1;
    for (int q = 0; q < raft_engine::OCC_SLOTS; ++q)
        if (e->occ_kern[q] == (const void*)kern && e->occ_lds[q] == lds) slot = q;
    if (slot < 0) {
        int wg = 0;
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&wg, (const void*)kern, STEP_BLOCK, lds));
        slot = (int)(e->occ_next++ % raft_engine::OCC_SLOTS);
        e->occ_kern[slot] = (const void*)kern;
        e->occ_lds[slot] = lds;
        e->occ_wg[slot] = std::max(1, wg);
    }
    geo.epoch = epoch;
    geo.resident = e->occ_wg[slot] * e->ncu;
    const int cap = std::max(1, (e->sched_wg > 0 ? std::min(e->sched_wg, geo.resident) : geo.resident) / e->nsub);
    geo.stride = 0;
    geo.balanced = 0;
    for (int q = 0; q < e->nsub; ++q) {
        const int a = e->sub_b0[q] * STEP_WAVES, b = std::min(e->sub_b0[q + 1] * STEP_WAVES, e->nwaves);
        const int n = b - a;
        // AUTO: when the chunks outnumber the resident wave slots (of this
        // sub-range's share); BALANCED: whenever a workgroup gets 4 chunks
        const bool bal = e->schedule == RAFT_SCHED_BALANCED
                             ? n >= STEP_WAVES
                             : e->schedule == RAFT_SCHED_AUTO && !e->part_only && n > STEP_WAVES * cap;
        geo.w0[q] = a;
        geo.w0[q + 1] = b;
        geo.bal[q] = bal ? n : 0;
        geo.nb[q] = bal ? std::min(cap, n / STEP_WAVES) : e->sub_b0[q + 1] - e->sub_b0[q];
        // plan_of's 32-bit arithmetic: (wave + 1) * m * K < 2^32 for a
        // workgroup's m = ceil(n / nb) chunks
        const int kp_ = epoch > 0 ? std::min(k, epoch) : k;                // a plan spans one epoch
        if (bal && (uint64_t)STEP_WAVES * (uint64_t)((n + geo.nb[q] - 1) / geo.nb[q]) * (uint64_t)kp_ >= (1ull << 32))
            return fail(RAFT_EINVAL, "balanced launch too long for its workgroups (4 * chunks per workgroup * "
                                     "steps_per_launch >= 2^32): raise schedule_workgroups or lower steps_per_launch");
        geo.col0[q] = geo.stride;
        geo.stride += geo.nb[q];
        geo.balanced += bal;
    }
    return RAFT_OK;
}

template <int R> struct StepL {
    static void run(raft_engine* e, StepKernel kern, uint32_t t0, int k, hipEvent_t ev0, hipEvent_t ev1,
                    hipStream_t st, const LaunchGeo& geo, int q, uint32_t* partials) {
        // the launch's own start / stop timestamps (ev0, ev1 nullable): no
        // marker packets around the dispatch
        DevParams d = e->dp;
        d.part = partials;
        d.wave0 = geo.w0[q];
        d.bal_chunks = geo.bal[q];
        d.bal_q = geo.bal[q] / geo.nb[q];
        d.bal_rem = geo.bal[q] % geo.nb[q];
        d.part_col0 = geo.col0[q];
        d.part_stride = geo.stride;
        d.epoch = geo.epoch;
        hipExtLaunchKernelGGL(kern, dim3(geo.nb[q]), dim3(STEP_BLOCK),
                              (uint32_t)step_lds_bytes(geo.epoch > 0 ? std::min(k, geo.epoch) : k), st, ev0, ev1, 0u,
                              d, t0, k);
    }
};
template <int R> struct PackL {
    static void run(raft_engine* e, int64_t g0, int64_t n, int32_t* buf) {
        pack_kernel<R><<<(unsigned)((n + BLOCK - 1) / BLOCK), BLOCK, 0, e->stream>>>(e->dp, g0, n, buf);
    }
};
template <int R> struct UnpackL {
    static void run(raft_engine* e, int64_t g0, int64_t n, const int32_t* buf) {
        unpack_kernel<R><<<(unsigned)((n + BLOCK - 1) / BLOCK), BLOCK, 0, e->stream>>>(e->dp, g0, n, buf);
    }
};
template <int R> struct ProbeL {
    static void run(raft_engine* e, int kind, unsigned long long* stores) {
        const unsigned grid = (unsigned)((e->nwaves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
        traffic_probe_kernel<R><<<grid, BLOCK, 0, e->stream>>>(e->dp, kind, e->nwaves, stores);
    }
};
template <int R> struct LogMatchL {
    static void run(raft_engine* e, int64_t g0, int64_t n, uint8_t* flags, unsigned long long* count) {
        const unsigned grid = (unsigned)((n + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
        log_match_kernel<R><<<grid, BLOCK, 0, e->stream>>>(e->dp, g0, n, flags, count);
    }
};
template <int R> struct DigestL {
    static void run(raft_engine* e, int64_t g0, int64_t n, unsigned long long* out) {
        digest_kernel<R><<<(unsigned)((n + BLOCK - 1) / BLOCK), BLOCK, 0, e->stream>>>(e->dp, g0, n, out);
    }
};

// raft_wire.cpp reports its errors through raft_last_error() too
int raft_internal_fail(int code, const std::string& msg) { return fail(code, msg); }
void raft_internal_ensure_cache(raft_engine* e) {
    if (e->cache_valid) return;
    rebuild_cache_kernel<<<(unsigned)((e->dp.GR + BLOCK - 1) / BLOCK), BLOCK, 0, e->stream>>>(e->dp);
    e->cache_valid = true;
    e->fork_needed = true;
}
// raft_comm.cpp: the engine's GPU (a communicator must be on it)
extern "C" int raft_internal_device(const raft_engine* e) { return e ? e->device : -1; }

static uint64_t ppm_thr(uint32_t ppm, int bits) {
    // smallest u with u * 1e6 >= ppm << bits  ==  ceil(ppm * 2^bits / 1e6)
    const unsigned __int128 num = (unsigned __int128)ppm << bits;
    return (uint64_t)((num + 999999u) / 1000000u);
}

extern "C" {

void raft_params_default(raft_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->R = 5;
    p->log_cap = 1024;
    p->G = 1;
    p->g0 = 0;
    p->seed = 1;
    p->heartbeat_ms = 2000;
    p->election_min_ms = 20000;
    p->election_max_ms = 23000;
    p->backoff_min_ms = 2000;
    p->backoff_max_ms = 3000;
    p->round_timeout_ms = 25000;
    p->retry_ms = 5000;
    p->cmd_mode = RAFT_CMD_LOWEST_LEADER;
}

const char* raft_last_error(void) { return g_err.c_str(); }
int raft_abi_version(void) { return RAFT_ABI_VERSION; }
#ifndef RAFT_BUILD_SOURCE_ID
#define RAFT_BUILD_SOURCE_ID "unknown"
#endif
#ifndef RAFT_BUILD_KERNEL_ID
#define RAFT_BUILD_KERNEL_ID "unknown"
#endif
const char* raft_build_source_id(void) { return RAFT_BUILD_SOURCE_ID; }
const char* raft_build_kernel_source_id(void) { return RAFT_BUILD_KERNEL_ID; }

void raft_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    const u32x4 v = philox4x32_10(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1]);
    out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
}

int raft_engine_create(const raft_params* p, int device, raft_engine** out) {
    if (!p || !out) return fail(RAFT_EINVAL, "null argument");
    *out = nullptr;
    if (p->R < 1 || p->R > RAFT_MAX_R) return fail(RAFT_EINVAL, "R must be in 1..8");
    if (p->G < 1 || p->G > (int64_t)0x7FFFFFFF) return fail(RAFT_EINVAL, "G out of range");
    if (p->g0 < 0 || p->g0 + p->G > (int64_t)0x100000000ll) return fail(RAFT_EINVAL, "g0 + G exceeds 2^32");
    if (p->log_cap < 1) return fail(RAFT_EINVAL, "log_cap must be >= 1");
    if (p->steps_per_launch < 0 || p->steps_per_launch > RAFT_MAX_STEPS_PER_LAUNCH)
        return fail(RAFT_EINVAL, "steps_per_launch must be in 0..RAFT_MAX_STEPS_PER_LAUNCH");
    if (p->heartbeat_ms <= 0 || p->election_min_ms > p->election_max_ms || p->backoff_min_ms > p->backoff_max_ms)
        return fail(RAFT_EINVAL, "bad timer constants");
    if (p->mode != RAFT_MODE_REFERENCE && p->mode != RAFT_MODE_TEXTBOOK)
        return fail(RAFT_EINVAL, "mode must be RAFT_MODE_REFERENCE or RAFT_MODE_TEXTBOOK");
    if (p->log_window < 0 || (p->log_window & (p->log_window - 1)) || p->log_window > p->log_cap)
        return fail(RAFT_EINVAL, "log_window must be 0 or a power of two <= log_cap");
    if (p->ae_max_entries < 0 || p->ae_max_entries > RAFT_MAX_AE_ENTRIES ||
        (p->mode != RAFT_MODE_TEXTBOOK && p->ae_max_entries > 1))
        return fail(RAFT_EINVAL, "ae_max_entries must be 0..RAFT_MAX_AE_ENTRIES, and 0 or 1 in reference mode");
    if (p->subranges < 0 || p->subranges > RAFT_MAX_SUBRANGES)
        return fail(RAFT_EINVAL, "subranges must be 0..RAFT_MAX_SUBRANGES");
    if (p->schedule < RAFT_SCHED_AUTO || p->schedule > RAFT_SCHED_BALANCED || p->schedule_workgroups < 0)
        return fail(RAFT_EINVAL, "schedule must be a RAFT_SCHED_* value and schedule_workgroups >= 0");
    if (p->kernel != RAFT_KERNEL_AUTO && p->kernel != RAFT_KERNEL_GENERAL)
        return fail(RAFT_EINVAL, "kernel must be RAFT_KERNEL_AUTO or RAFT_KERNEL_GENERAL");
    if ((p->log_window ? p->log_window : p->log_cap) >= (1 << 23))
        return fail(RAFT_EINVAL, "log slots per replica (log_window, else log_cap) must be < 2^23");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RAFT_ENODEV, "no HIP device");
    if (device < 0 || device >= ndev) return fail(RAFT_EINVAL, "bad device index");
    HIP_TRY(hipSetDevice(device));

    raft_engine* e = new raft_engine();
    e->p = *p;
    e->timing = false;
    e->cache_valid = true;
    e->ev_used = 0;
    e->timed_launches = 0;
    e->nsub = 1;
    e->launches_issued = 0;
    e->fork_needed = true;
    e->ev_fork = nullptr;
    e->ev_wait = nullptr;
    for (int q = 0; q < RAFT_MAX_SUBRANGES; ++q) { e->sub_stream[q] = nullptr; e->ev_sub_done[q] = nullptr; }
    e->ev_red_done[0] = e->ev_red_done[1] = nullptr;
    e->bst = e->bio = e->hst = nullptr;
    e->bst_bytes = e->bio_bytes = e->hst_bytes = 0;
    e->bflags_host = nullptr;
    e->aux = nullptr;
    e->aux_bytes = 0;
    e->hpart = nullptr;
    e->hpart_bytes = 0;
    e->device = device;
    e->t = 0;
    const int64_t G = p->G, R = p->R;
    DevParams& d = e->dp;
    d.G = G; d.g0 = p->g0; d.R = p->R; d.cap = p->log_cap;
    // the ring: log_window slots per replica (mask j & (W - 1)), or every
    // physical slot (no wrap: j < log_cap, and no access is ever a miss)
    const int64_t nslots = p->log_window ? p->log_window : p->log_cap;
    d.wmask = p->log_window ? (uint32_t)(p->log_window - 1) : 0xFFFFFFFFu;
    d.W = p->log_window ? p->log_window : FLAT_W;
    d.nslots = (int32_t)nslots;
    const int64_t log_waves = (G + 64 / R - 1) / (64 / R);           // step-kernel waves: one log block each
    d.key0 = (uint32_t)p->seed; d.key1 = (uint32_t)(p->seed >> 32);
    for (int i = 0; i < 10; ++i) {                                    // Philox round keys (kdraw)
        d.rk[2 * i] = d.key0 + (uint32_t)i * 0x9E3779B9u;
        d.rk[2 * i + 1] = d.key1 + (uint32_t)i * 0xBB67AE85u;
    }
    d.P = p->heartbeat_ms; d.emin = p->election_min_ms; d.emax = p->election_max_ms;
    d.bmin = p->backoff_min_ms; d.bmax = p->backoff_max_ms; d.round_to = p->round_timeout_ms; d.retry = p->retry_ms;
    d.drop_ppm = p->drop_ppm; d.drop_thr16 = (uint32_t)ppm_thr(p->drop_ppm, 16);
    d.churn_thr32 = ppm_thr(p->churn_ppm, 32); d.cmd_thr32 = ppm_thr(p->cmd_ppm, 32);
    d.churn_steps = p->churn_steps; d.part_period = p->partition_period; d.part_len = p->partition_len;
    d.cmd_mode = p->cmd_mode; d.cmd_limit = p->cmd_limit;
    d.ae_max = p->mode == RAFT_MODE_TEXTBOOK && p->ae_max_entries > 1 ? p->ae_max_entries : 1;
    e->nwaves = (int)log_waves;
    e->nblocks = (e->nwaves + STEP_WAVES - 1) / STEP_WAVES;
    e->schedule = p->schedule;
    e->sched_wg = p->schedule_workgroups;
    for (int q = 0; q < raft_engine::OCC_SLOTS; ++q) {
        e->occ_kern[q] = nullptr;
        e->occ_lds[q] = 0;
        e->occ_wg[q] = 1;
    }
    e->occ_next = 0;
    e->last = raft_kernel_info{};
    e->ncu = 0;
    if (hipDeviceGetAttribute(&e->ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || e->ncu < 1)
        e->ncu = 1;
    d.GR = G * R;
    e->K = p->steps_per_launch > 0 ? p->steps_per_launch : 1;

    const size_t st_b = (size_t)ST_QUADS * 16 * R * G;
    const size_t spill_b = (size_t)2 * R * R * G * 4;
    const size_t gx_b = (size_t)GX_WORDS * G * 4;
    const size_t log_b = (size_t)log_waves * nslots * 64 * 8;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    // sized for the largest launch, so steps_per_launch can change later
    const size_t part_b = (size_t)LDS_MAX_STEPS * NCW * e->nblocks * 4;
    const size_t cnt_b = (size_t)RAFT_MAX_STEPS_PER_LAUNCH * RAFT_COUNTER_STRIDE * 8;
    const size_t acc_b = (size_t)RAFT_MAX_STEPS_PER_LAUNCH * NC * 8;
    e->bytes = al(st_b) + al(spill_b) + al(gx_b) + 2 * al(part_b) + al(cnt_b) + al(acc_b) + al(log_b);
    hipError_t err = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (err != hipSuccess) { delete e; return fail(RAFT_EDEVICE, "hipStreamCreate failed"); }
    err = hipMalloc(&e->base, e->bytes);
    if (err != hipSuccess) {
        (void)hipStreamDestroy(e->stream);
        delete e;
        return fail(RAFT_ENOMEM, "hipMalloc of " + std::to_string(e->bytes) + " bytes failed");
    }
    char* b = (char*)e->base;
    d.st = (int32_t*)b; b += al(st_b);
    d.spill = (int32_t*)b; b += al(spill_b);
    d.gx = (int32_t*)b; b += al(gx_b);
    e->partials = (uint32_t*)b; b += al(part_b);
    e->partials2 = (uint32_t*)b; b += al(part_b);
    e->counters_dev = (int64_t*)b; b += al(cnt_b);
    e->accum = (unsigned long long*)b; b += al(acc_b);
    d.log = (uint2*)b;
    *out = e;
    err = hipHostMalloc((void**)&e->bflags_host, 64, hipHostMallocDefault);
    if (err == hipSuccess) {
        // word 8: the step kernel's status word (RAFT_DEV_*), written by the
        // device and read by the host after a synchronisation
        e->bflags_host[8] = 0u;
        err = hipHostGetDevicePointer((void**)&d.status, e->bflags_host + 8, 0);
    }
    if (err != hipSuccess) {
        raft_engine_destroy(e);
        *out = nullptr;
        return fail(RAFT_ENOMEM, "hipHostMalloc of the batch status flags failed");
    }
    e->part_only = step_net(d, *p, p->R, d.churn_thr32 != 0) == NET_PART;
    if (int rc = raft_engine_set_subranges(e, p->subranges)) {
        raft_engine_destroy(e);
        *out = nullptr;
        return rc;
    }
    dispatch_R<InitL>(p->R, e);
    err = hipMemsetAsync(e->accum, 0, acc_b, e->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) {
        (void)hipFree(e->base);
        (void)hipStreamDestroy(e->stream);
        delete e;
        *out = nullptr;
        return fail(RAFT_EDEVICE, std::string("init kernel: ") + hipGetErrorString(err));
    }
    return RAFT_OK;
}

int raft_engine_destroy(raft_engine* e) {
    if (!e) return RAFT_OK;
#ifdef RAFT_PROFILE_PHASES
    {
        unsigned long long v[PH_N] = {0};
        (void)hipSetDevice(e->device);
        (void)hipStreamSynchronize(e->stream);
        if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_phase_cycles), sizeof(v)) == hipSuccess) {
            const char* names[PH_N] = {"T", "JOBS", "H", "V", "D", "A", "C", "K", "TDRAW", "CNT"};
            unsigned long long tot = 0;
            for (int q = 0; q < PH_N; ++q) tot += v[q];
            fprintf(stderr, "[phase-cycles]");
            for (int q = 0; q < PH_N; ++q) fprintf(stderr, " %s=%.1f%%", names[q], tot ? 100.0 * v[q] / tot : 0.0);
            fprintf(stderr, " total=%llu\n", tot);
        }
    }
#endif
#ifdef RAFT_BRANCH_STATS
    {   // per wave-step frequency of each branch over the engine's step launches, to stderr
        unsigned long long v[BS_N] = {0};
        (void)hipSetDevice(e->device);
        (void)hipStreamSynchronize(e->stream);
        if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_branch_stats), sizeof(v)) == hipSuccess) {
            const char* names[BS_N] = {"steps", "T_busy", "V_phase", "V_rounds", "V_stage", "D_dec", "D_backoff",
                                       "D_start", "A_phase", "A_rounds", "A_stage", "A_swap", "A_loads", "A_hib",
                                       "A_slow", "A_commit", "H_busy", "K_dual", "draw", "direct_drop"};
            fprintf(stderr, "[branch-stats] wave_steps=%llu", v[0]);
            for (int q = 1; q < BS_N; ++q) fprintf(stderr, " %s=%.4f", names[q], v[0] ? (double)v[q] / v[0] : 0.0);
            fprintf(stderr, "\n");
            unsigned long long z[BS_N] = {0};
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_branch_stats), z, sizeof(z));
        }
    }
#endif
#ifdef RAFT_WAVE_TIMES
    {   // the last step launch's waves: start / end offsets and slots, to stderr
        (void)hipSetDevice(e->device);
        (void)hipStreamSynchronize(e->stream);
        const int nw = std::min(WT_MAX, e->last.workgroups * STEP_WAVES);
        std::vector<unsigned long long> v((size_t)nw * 3);
        if (nw > 0 && hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_wave_times), v.size() * 8) == hipSuccess) {
            unsigned long long t0 = ~0ull;
            for (int w = 0; w < nw; ++w) t0 = std::min(t0, v[3 * w]);
            fprintf(stderr, "[wave-times] waves=%d workgroups=%d\n", nw, e->last.workgroups);
            for (int w = 0; w < nw; ++w)
                fprintf(stderr, "[wt] %d %llu %llu %llx\n", w, v[3 * w] - t0, v[3 * w + 1] - t0, v[3 * w + 2]);
        }
    }
#endif
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->stream);
    for (hipEvent_t x : e->ev) (void)hipEventDestroy(x);
    for (int q = 0; q < RAFT_MAX_SUBRANGES; ++q) {
        if (e->sub_stream[q]) (void)hipStreamDestroy(e->sub_stream[q]);
        if (e->ev_sub_done[q]) (void)hipEventDestroy(e->ev_sub_done[q]);
    }
    for (hipEvent_t x : {e->ev_fork, e->ev_red_done[0], e->ev_red_done[1], e->ev_wait})
        if (x) (void)hipEventDestroy(x);
    if (e->bst) (void)hipFree(e->bst);
    if (e->bio) (void)hipFree(e->bio);
    if (e->hst) (void)hipHostFree(e->hst);
    if (e->bflags_host) (void)hipHostFree(e->bflags_host);
    if (e->aux) (void)hipFree(e->aux);
    if (e->hpart) (void)hipFree(e->hpart);
    (void)hipFree(e->base);
    (void)hipStreamDestroy(e->stream);
    delete e;
    return RAFT_OK;
}

// Grow the timing-event pool to hold `pairs` more launches.  Called when
// timing is switched on, so a timed region never creates events (64
// hipEventCreate calls cost ~0.1 ms of host time, 7 % of a 20-step run).
static int grow_dev(raft_engine* e, char** buf, size_t* have, size_t need);
static int reserve_events(raft_engine* e, size_t pairs) {
    while (e->ev_used + 2 * pairs > e->ev.size()) {
        hipEvent_t x;
        HIP_TRY(hipEventCreate(&x));
        e->ev.push_back(x);
    }
    return RAFT_OK;
}

int raft_engine_step_async(raft_engine* e, int32_t n_steps, int64_t* counters_dev) {
    if (!e || n_steps < 0) return fail(RAFT_EINVAL, "bad argument");
    HIP_TRY(hipSetDevice(e->device));
    if (n_steps > 0) raft_internal_ensure_cache(e);
    // One sub-range: every launch and its counter reduction on the engine
    // stream.  nsub > 1: launch k of sub-range q runs on sub_stream[q] and
    // writes its workgroups' columns of partials buffer k & 1; the engine
    // stream waits for launch k of every sub-range, reduces that buffer and
    // marks it free (ev_red_done), which launch k + 2 of each sub-range
    // waits for.  A sub-range thus runs up to a launch ahead of another, and
    // its launches follow each other without waiting for the other ranges'
    // tails.  Work enqueued on the engine stream after this call sees every
    // launch finished (the last reductions wait for all of them).  The
    // sub-range streams wait for the engine stream only when an engine call
    // other than a step enqueued work there since (fork_needed): waiting for
    // the previous call's reductions would re-join the ranges at every call,
    // and bench.py calls once per launch.  Callers must not change the
    // engine's device state on the engine stream themselves (it is engine
    // memory; the API calls that do, set fork_needed).
    const bool split = e->nsub > 1;
    if (split && n_steps > 0 && e->fork_needed) {
        HIP_TRY(hipEventRecord(e->ev_fork, e->stream));
        for (int q = 0; q < e->nsub; ++q) HIP_TRY(hipStreamWaitEvent(e->sub_stream[q], e->ev_fork, 0));
        e->fork_needed = false;
    }
    const StepKernel kern = n_steps > 0 ? step_kernel_of(e) : nullptr;
    const StepKernel kern_ep = n_steps > 0 && !split && e->K > LDS_MAX_STEPS ? step_kernel_of(e, true) : nullptr;
    for (int32_t done = 0; done < n_steps;) {
        int k = std::min<int32_t>(e->K, n_steps - done);
        const int buf = split ? (int)(e->launches_issued & 1) : 0;
        uint32_t* part = buf ? e->partials2 : e->partials;
        LaunchGeo geo;
        // a launch beyond LDS_MAX_STEPS: epochs when balanced on one
        // sub-range (its partials [k][NCW][workgroups] in a grow-only
        // buffer), else cut to LDS_MAX_STEPS
        bool epochs = false;
        if (k > LDS_MAX_STEPS && kern_ep) {
            if (int rc = launch_geo(e, kern_ep, k, EPOCH_STEPS, geo)) return rc;
            epochs = geo.balanced == 1;
        }
        if (epochs) {
            const size_t need = (size_t)k * NCW * (size_t)geo.stride * 4;
            if (int rc = grow_dev(e, (char**)&e->hpart, &e->hpart_bytes, need)) return rc;
            part = e->hpart;
        } else {
            k = std::min(k, LDS_MAX_STEPS);
            if (int rc = launch_geo(e, kern, k, 0, geo)) return rc;
        }
        if (e->timing && e->ev_used + 2 * e->nsub > e->ev.size())
            if (int rc = reserve_events(e, 64 + e->nsub)) return rc;
        for (int q = 0; q < e->nsub; ++q) {
            hipEvent_t ev0 = nullptr, ev1 = nullptr;
            if (e->timing) {
                ev0 = e->ev[e->ev_used];
                ev1 = e->ev[e->ev_used + 1];
                e->ev_used += 2;
            }
            hipStream_t st = split ? e->sub_stream[q] : e->stream;
            if (split && e->launches_issued >= 2) HIP_TRY(hipStreamWaitEvent(st, e->ev_red_done[buf], 0));
            dispatch_R<StepL>(e->p.R, e, epochs ? kern_ep : kern, (uint32_t)(e->t + done), k, ev0, ev1, st, geo, q,
                              part);
            if (split) {
                HIP_TRY(hipEventRecord(e->ev_sub_done[q], st));
                HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_sub_done[q], 0));
            }
        }
        if (e->timing) ++e->timed_launches;
        e->last = raft_kernel_info{};
        e->last.net = e->p.kernel == RAFT_KERNEL_GENERAL
                          ? NET_ALL : step_net(e->dp, e->p, e->p.R, e->dp.churn_thr32 != 0 || e->iso_written);
        e->last.textbook = e->p.mode == RAFT_MODE_TEXTBOOK;
        e->last.ring = e->p.log_window != 0;
        e->last.steps = k;
        e->last.workgroups = geo.stride;
        e->last.resident_workgroups = geo.resident;
        e->last.balanced = geo.balanced;
        e->last.subranges = e->nsub;
        int64_t* dst = counters_dev ? counters_dev + (int64_t)done * RAFT_COUNTER_STRIDE : e->counters_dev;
        const int nch = (geo.stride + REDUCE_CHUNK - 1) / REDUCE_CHUNK;
        reduce_counters_kernel<<<(unsigned)(nch * k * NCW), BLOCK, 0, e->stream>>>(part, geo.stride, nch, e->p.R, dst,
                                                                                  e->accum);
        if (split) HIP_TRY(hipEventRecord(e->ev_red_done[buf], e->stream));
        ++e->launches_issued;
        done += k;
    }
    HIP_TRY(hipGetLastError());
    e->t += (uint64_t)n_steps;
    return RAFT_OK;
}

// The step kernel's status word, read after a synchronisation of the engine
// stream (every step launch has finished): nonzero means a launch's results
// are not the reference's.
static int check_device_status(raft_engine* e) {
    const uint32_t s = __atomic_load_n(&e->bflags_host[8], __ATOMIC_ACQUIRE);
    if (s & RAFT_DEV_WAIT_TIMEOUT)
        return fail(RAFT_EDEVICE, "a balanced-schedule wave timed out waiting for the previous wave's head piece: "
                                  "the engine's state is not the reference's (raft_engine_reset clears this)");
    return RAFT_OK;
}

int raft_engine_sync(raft_engine* e) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    HIP_TRY(hipStreamSynchronize(e->stream));
    return check_device_status(e);
}

int raft_engine_step(raft_engine* e, int32_t n_steps, int64_t* counters_host) {
    if (!e || n_steps < 0) return fail(RAFT_EINVAL, "bad argument");
    HIP_TRY(hipSetDevice(e->device));
    for (int32_t done = 0; done < n_steps;) {
        const int k = std::min<int32_t>(e->K, n_steps - done);
        const int rc = raft_engine_step_async(e, k, e->counters_dev);
        if (rc) return rc;
        if (counters_host)
            HIP_TRY(hipMemcpyAsync(counters_host + (int64_t)done * RAFT_COUNTER_STRIDE, e->counters_dev,
                                   (size_t)k * RAFT_COUNTER_STRIDE * 8, hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        if (int rc = check_device_status(e)) return rc;
        done += k;
    }
    return RAFT_OK;
}

void* raft_engine_stream(raft_engine* e) { return e ? (void*)e->stream : nullptr; }

int raft_engine_set_kernel_timing(raft_engine* e, int enable) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    e->timing = enable != 0;
    if (e->timing) {
        HIP_TRY(hipSetDevice(e->device));
        return reserve_events(e, 256);
    }
    return RAFT_OK;
}

int raft_engine_kernel_time(raft_engine* e, double* total_ms, int64_t* launches) {
    if (!e || !total_ms || !launches) return fail(RAFT_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    // intervals relative to the first launch's start, merged: the time during
    // which at least one step kernel ran (sub-range launches overlap)
    std::vector<std::pair<double, double>> iv;
    for (size_t q = 0; q + 1 < e->ev_used; q += 2) {
        float a = 0.f, b = 0.f;
        if (q) HIP_TRY(hipEventElapsedTime(&a, e->ev[0], e->ev[q]));
        HIP_TRY(hipEventElapsedTime(&b, e->ev[0], e->ev[q + 1]));
        iv.emplace_back(a, b);
    }
    // (an interval may start before ev[0]: a sub-range can run a launch ahead
    // of sub-range 0, so the merge starts from the earliest interval)
    std::sort(iv.begin(), iv.end());
    double acc = 0.0;
    if (!iv.empty()) {
        double lo = iv[0].first, hi = iv[0].second;
        for (size_t q = 1; q < iv.size(); ++q) {
            if (iv[q].first > hi) {
                acc += hi - lo;
                lo = iv[q].first;
                hi = iv[q].second;
            } else {
                hi = std::max(hi, iv[q].second);
            }
        }
        acc += hi - lo;
    }
    *total_ms = acc;
    *launches = e->timed_launches;
    e->ev_used = 0;
    e->timed_launches = 0;
    return check_device_status(e);
}
int raft_engine_timed_span(raft_engine* e, void* end_event, double* ms) {
    if (!e || !end_event || !ms) return fail(RAFT_EINVAL, "null argument");
    if (e->ev_used < 2) return fail(RAFT_EINVAL, "no timed launch since kernel timing was switched on");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipEventSynchronize((hipEvent_t)end_event));
    // from the earliest launch start (a sub-range can start a launch ahead of
    // sub-range 0, see raft_engine_kernel_time) to the caller's event
    float lo = 0.f, end = 0.f;
    for (size_t q = 2; q + 1 < e->ev_used; q += 2) {
        float a = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, e->ev[0], e->ev[q]));
        lo = std::min(lo, a);
    }
    HIP_TRY(hipEventElapsedTime(&end, e->ev[0], (hipEvent_t)end_event));
    *ms = (double)end - (double)lo;
    return RAFT_OK;
}
int64_t raft_engine_step_index(raft_engine* e) { return e ? (int64_t)e->t : -1; }
int raft_engine_set_steps_per_launch(raft_engine* e, int32_t k) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    if (k < 0 || k > RAFT_MAX_STEPS_PER_LAUNCH) return fail(RAFT_EINVAL, "steps_per_launch out of range");
    e->K = k > 0 ? k : 1;
    return RAFT_OK;
}
// Sub-ranges: contiguous workgroup ranges of (nearly) equal size.  Automatic
// (n = 0): one.  (ABI 1 chose three, which overlapped one range's last waves
// with another's next launch: 1.25e5 groups 1.36 -> 1.73e10, 1e6 groups 1.78
// -> 1.86e10 group-steps/s; the balanced schedule ends a launch's waves
// together instead, with no side streams)
// The automatic launch shape.  Drops and churn (config 3 and its shards):
// one range on the balanced schedule.  Partitions alone (configs 5, 2, 1: the
// partitions-only kernel): one chunk per wave over three overlapping ranges,
// which measured 3.6 % above the balanced schedule on config 5 (whose
// partitions make a chunk's work uneven, which equal chunk-steps per wave do
// not balance) and 23 % above one range (profiles/r4_k).
static int auto_subranges(const raft_engine* e) { return e->part_only ? 3 : 1; }
int raft_engine_wait_stream(raft_engine* e, void* stream) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    HIP_TRY(hipSetDevice(e->device));
    if (!e->ev_wait) HIP_TRY(hipEventCreateWithFlags(&e->ev_wait, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(e->ev_wait, (hipStream_t)stream));
    HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_wait, 0));
    e->fork_needed = true;                 // the sub-range streams must see it too
    return RAFT_OK;
}
int raft_engine_set_kernel(raft_engine* e, int32_t kernel) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    if (kernel != RAFT_KERNEL_AUTO && kernel != RAFT_KERNEL_GENERAL)
        return fail(RAFT_EINVAL, "kernel must be RAFT_KERNEL_AUTO or RAFT_KERNEL_GENERAL");
    e->p.kernel = kernel;
    return RAFT_OK;
}
int raft_engine_reset(raft_engine* e) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (int q = 0; q < e->nsub && e->nsub > 1; ++q) HIP_TRY(hipStreamSynchronize(e->sub_stream[q]));
    dispatch_R<InitL>(e->p.R, e);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->bflags_host[8] = 0u;                // the step kernel's status word
    e->t = 0;
    e->cache_valid = true;                 // init zeroes the tail cache with the logs' lastIndex
    e->iso_written = false;
    e->fork_needed = true;
    return RAFT_OK;
}
int raft_engine_kernel_info(raft_engine* e, raft_kernel_info* out) {
    if (!e || !out) return fail(RAFT_EINVAL, "null argument");
    *out = e->last;
    return RAFT_OK;
}
int raft_engine_set_subranges(raft_engine* e, int32_t n) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    if (n < 0 || n > RAFT_MAX_SUBRANGES) return fail(RAFT_EINVAL, "subranges must be 0..RAFT_MAX_SUBRANGES");
    if (n == 0) n = auto_subranges(e);
    n = std::min(n, e->nblocks);
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (n > 1 && !e->ev_fork) {
        HIP_TRY(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
        for (int b = 0; b < 2; ++b) HIP_TRY(hipEventCreateWithFlags(&e->ev_red_done[b], hipEventDisableTiming));
    }
    for (int q = 0; q < n && n > 1; ++q) {
        if (!e->sub_stream[q]) HIP_TRY(hipStreamCreateWithFlags(&e->sub_stream[q], hipStreamNonBlocking));
        if (!e->ev_sub_done[q]) HIP_TRY(hipEventCreateWithFlags(&e->ev_sub_done[q], hipEventDisableTiming));
    }
    e->nsub = n;
    for (int q = 0; q <= n; ++q) e->sub_b0[q] = (int)((int64_t)e->nblocks * q / n);
    e->launches_issued = 0;              // both partials buffers are free (the engine stream is idle)
    return RAFT_OK;
}
int32_t raft_engine_subranges(raft_engine* e) { return e ? e->nsub : -1; }
int raft_engine_set_step_index(raft_engine* e, int64_t t) {
    if (!e || t < 0 || t > (int64_t)0xFFFFFFFFll) return fail(RAFT_EINVAL, "bad step index");
    e->t = (uint64_t)t;
    return RAFT_OK;
}
int64_t raft_engine_device_bytes(raft_engine* e) {
    return e ? (int64_t)(e->bytes + e->bst_bytes + e->bio_bytes + e->aux_bytes + e->hpart_bytes) : -1;
}
int raft_engine_trim_staging(raft_engine* e) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->bst) HIP_TRY(hipFree(e->bst));
    if (e->bio) HIP_TRY(hipFree(e->bio));
    if (e->aux) HIP_TRY(hipFree(e->aux));
    if (e->hst) HIP_TRY(hipHostFree(e->hst));
    e->bst = e->bio = e->aux = e->hst = nullptr;
    e->bst_bytes = e->bio_bytes = e->aux_bytes = e->hst_bytes = 0;
    return RAFT_OK;
}

// Grow-only engine staging (the batch path, the state / log / digest accessors) (no allocation, and so no
// device-wide hipFree synchronisation, once a batch size has been seen).
static int grow_dev(raft_engine* e, char** buf, size_t* have, size_t need) {
    if (need <= *have) return RAFT_OK;
    if (*buf) HIP_TRY(hipFree(*buf));
    *buf = nullptr;
    *have = 0;
    need = std::max(need, (size_t)1 << 20) * 5 / 4;
    HIP_TRY(hipMalloc((void**)buf, need));
    *have = need;
    return RAFT_OK;
}
static int grow_host(raft_engine* e, char** buf, size_t* have, size_t need) {
    if (need <= *have) return RAFT_OK;
    if (*buf) HIP_TRY(hipHostFree(*buf));
    *buf = nullptr;
    *have = 0;
    need = std::max(need, (size_t)1 << 20) * 5 / 4;
    HIP_TRY(hipHostMalloc((void**)buf, need, hipHostMallocDefault));
    *have = need;
    return RAFT_OK;
}
int raft_internal_grow_dev(raft_engine* e, char** buf, size_t* have, size_t need) {
    return grow_dev(e, buf, have, need);
}
int raft_internal_grow_host(raft_engine* e, char** buf, size_t* have, size_t need) {
    return grow_host(e, buf, have, need);
}

static int check_range(raft_engine* e, int64_t g0, int64_t n) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    if (g0 < 0 || n < 0 || g0 + n > e->p.G) return fail(RAFT_ERANGE, "group range outside the engine");
    return RAFT_OK;
}

int raft_engine_read_state(raft_engine* e, int64_t g0, int64_t n, int32_t* out) {
    if (int rc = check_range(e, g0, n)) return rc;
    if (n == 0) return RAFT_OK;
    if (!out) return fail(RAFT_EINVAL, "null buffer");
    HIP_TRY(hipSetDevice(e->device));
    e->fork_needed = true;
    const size_t bytes = (size_t)n * raft_group_words(e->p.R) * 4;
    if (int rc = grow_dev(e, &e->aux, &e->aux_bytes, bytes)) return rc;
    int32_t* buf = (int32_t*)e->aux;
    dispatch_R<PackL>(e->p.R, e, g0, n, buf);
    hipError_t err = hipMemcpyAsync(out, buf, bytes, hipMemcpyDeviceToHost, e->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) return fail(RAFT_EDEVICE, hipGetErrorString(err));
    return RAFT_OK;
}

int raft_engine_write_state(raft_engine* e, int64_t g0, int64_t n, const int32_t* in) {
    if (int rc = check_range(e, g0, n)) return rc;
    if (n == 0) return RAFT_OK;
    if (!in) return fail(RAFT_EINVAL, "null buffer");
    const int W = raft_group_words(e->p.R);
    for (int64_t j = 0; j < n; ++j)              // invariant 0 <= lastIndex <= physLen <= log_cap
        for (int r = 0; r < e->p.R; ++r) {
            const int32_t* f = in + j * W + r * RAFT_NUM_FIELDS;
            if (f[RAFT_F_LAST] < 0 || f[RAFT_F_LAST] > f[RAFT_F_PHYS] || f[RAFT_F_PHYS] > e->p.log_cap)
                return fail(RAFT_EINVAL, "state violates 0 <= lastIndex <= physLen <= log_cap");
        }
    for (int64_t j = 0; j < n; ++j)              // an isolation word: only kernels with NET_ISO from now on
        if (in[j * W + W - 2] != 0) e->iso_written = true;
    HIP_TRY(hipSetDevice(e->device));
    e->fork_needed = true;
    const size_t bytes = (size_t)n * W * 4;
    if (int rc = grow_dev(e, &e->aux, &e->aux_bytes, bytes)) return rc;
    int32_t* buf = (int32_t*)e->aux;
    hipError_t err = hipMemcpyAsync(buf, in, bytes, hipMemcpyHostToDevice, e->stream);
    e->cache_valid = false;
    if (err == hipSuccess) {
        dispatch_R<UnpackL>(e->p.R, e, g0, n, buf);
        err = hipStreamSynchronize(e->stream);
    }
    if (err != hipSuccess) return fail(RAFT_EDEVICE, hipGetErrorString(err));
    return RAFT_OK;
}

// the [n][R][log_cap] host image of groups [g0, g0+n) through a device buffer
static int log_image(raft_engine* e, int64_t g0, int64_t n, std::vector<uint2>& tmp, bool to_ring) {
    e->fork_needed = true;
    const size_t cnt = (size_t)n * e->p.R * e->p.log_cap;
    if (int rc = grow_dev(e, &e->aux, &e->aux_bytes, cnt * 8)) return rc;
    uint2* buf = (uint2*)e->aux;
    hipError_t err = hipSuccess;
    if (to_ring) err = hipMemcpyAsync(buf, tmp.data(), cnt * 8, hipMemcpyHostToDevice, e->stream);
    if (err == hipSuccess) {
        const unsigned grid = (unsigned)std::min<size_t>((cnt + BLOCK - 1) / BLOCK, 65536);
        log_image_kernel<<<grid, BLOCK, 0, e->stream>>>(e->dp, g0, n, buf, to_ring ? 1 : 0);
        err = hipGetLastError();
    }
    if (err == hipSuccess && !to_ring) err = hipMemcpyAsync(tmp.data(), buf, cnt * 8, hipMemcpyDeviceToHost, e->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) return fail(RAFT_EDEVICE, hipGetErrorString(err));
    return RAFT_OK;
}

int raft_engine_read_log(raft_engine* e, int64_t g0, int64_t n, int32_t* terms, uint32_t* cmds) {
    if (int rc = check_range(e, g0, n)) return rc;
    if (n == 0) return RAFT_OK;
    if (!terms || !cmds) return fail(RAFT_EINVAL, "null buffer");
    HIP_TRY(hipSetDevice(e->device));
    const size_t cnt = (size_t)n * e->p.R * e->p.log_cap;
    std::vector<uint2> tmp(cnt);
    if (int rc = log_image(e, g0, n, tmp, false)) return rc;
    for (size_t k = 0; k < cnt; ++k) { terms[k] = (int32_t)tmp[k].x; cmds[k] = tmp[k].y; }
    return RAFT_OK;
}

int raft_engine_write_log(raft_engine* e, int64_t g0, int64_t n, const int32_t* terms, const uint32_t* cmds) {
    if (int rc = check_range(e, g0, n)) return rc;
    if (n == 0) return RAFT_OK;
    if (!terms || !cmds) return fail(RAFT_EINVAL, "null buffer");
    HIP_TRY(hipSetDevice(e->device));
    const size_t cnt = (size_t)n * e->p.R * e->p.log_cap;
    std::vector<uint2> tmp(cnt);
    for (size_t k = 0; k < cnt; ++k) tmp[k] = make_uint2((uint32_t)terms[k], cmds[k]);
    e->cache_valid = false;
    return log_image(e, g0, n, tmp, true);
}

int raft_engine_digest(raft_engine* e, uint64_t* out) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    return raft_engine_digest_range(e, 0, e->p.G, out);
}

int raft_engine_digest_range(raft_engine* e, int64_t g0, int64_t n, uint64_t* out) {
    if (int rc = check_range(e, g0, n)) return rc;
    if (!out) return fail(RAFT_EINVAL, "null argument");
    *out = 0;
    if (n == 0) return RAFT_OK;
    HIP_TRY(hipSetDevice(e->device));
    e->fork_needed = true;
    if (int rc = grow_dev(e, &e->aux, &e->aux_bytes, 8)) return rc;
    unsigned long long* d = (unsigned long long*)e->aux;
    hipError_t err = hipMemsetAsync(d, 0, 8, e->stream);
    if (err == hipSuccess) {
        dispatch_R<DigestL>(e->p.R, e, g0, n, d);
        err = hipMemcpyAsync(out, d, 8, hipMemcpyDeviceToHost, e->stream);
    }
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) return fail(RAFT_EDEVICE, hipGetErrorString(err));
    return RAFT_OK;
}

int raft_engine_traffic_probe(raft_engine* e, int32_t kind, int64_t* bytes_read, int64_t* bytes_written) {
    if (!e || !bytes_read || !bytes_written) return fail(RAFT_EINVAL, "null argument");
    if (kind < 0 || kind > 3)
        return fail(RAFT_EINVAL, "kind must be 0 (state), 1 (log stores), 2 (scattered loads) or 3 (scattered stores)");
    if (kind == 1 && e->p.log_window) return fail(RAFT_EINVAL, "the log-store probe needs a flat log (log_window 0)");
    HIP_TRY(hipSetDevice(e->device));
    e->fork_needed = true;
    if (kind >= 2) {
        // engine-owned scratch (the accessors' staging, grow-only): the state is untouched
        const size_t sz = (size_t)32 << SCATTER_LOG2;
        if (int rc = grow_dev(e, &e->aux, &e->aux_bytes, sz)) return rc;
        scatter_probe_kernel<<<SCATTER_N / BLOCK, BLOCK, 0, e->stream>>>((uint32_t*)e->aux, (int)kind);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(e->stream));
        *bytes_read = kind == 2 ? (int64_t)SCATTER_N * 32 : 0;
        *bytes_written = kind == 3 ? (int64_t)SCATTER_N * 32 : 0;
        return RAFT_OK;
    }
    if (int rc = grow_dev(e, &e->aux, &e->aux_bytes, 8)) return rc;
    unsigned long long* d = (unsigned long long*)e->aux;
    unsigned long long h = 0;
    hipError_t err = hipMemsetAsync(d, 0, 8, e->stream);
    if (err == hipSuccess) {
        dispatch_R<ProbeL>(e->p.R, e, (int)kind, d);
        err = hipGetLastError();
    }
    if (err == hipSuccess) err = hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, e->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) return fail(RAFT_EDEVICE, hipGetErrorString(err));
    const int64_t state = e->p.G * ((int64_t)e->p.R * 16 * ST_QUADS + 4 * GX_WORDS);
    *bytes_read = kind == 0 ? state : 4 * e->p.G * e->p.R;               // kind 1 reads physLen
    *bytes_written = kind == 0 ? state : 8 * (int64_t)h;
    return RAFT_OK;
}

int raft_engine_check_log_matching(raft_engine* e, int64_t g0, int64_t n, uint8_t* flags, int64_t* mismatched) {
    if (int rc = check_range(e, g0, n)) return rc;
    if (!mismatched) return fail(RAFT_EINVAL, "null argument");
    HIP_TRY(hipSetDevice(e->device));
    e->fork_needed = true;
    *mismatched = 0;
    if (n == 0) return RAFT_OK;
    if (int rc = grow_dev(e, &e->aux, &e->aux_bytes, 8 + (flags ? (size_t)n : 0))) return rc;
    void* d = e->aux;
    unsigned long long* cnt = (unsigned long long*)d;
    uint8_t* fl = flags ? (uint8_t*)d + 8 : nullptr;
    unsigned long long h = 0;
    hipError_t err = hipMemsetAsync(d, 0, 8, e->stream);
    if (err == hipSuccess) {
        dispatch_R<LogMatchL>(e->p.R, e, g0, n, fl, cnt);
        err = hipGetLastError();
    }
    if (err == hipSuccess) err = hipMemcpyAsync(&h, cnt, 8, hipMemcpyDeviceToHost, e->stream);
    if (err == hipSuccess && flags) err = hipMemcpyAsync(flags, fl, (size_t)n, hipMemcpyDeviceToHost, e->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) return fail(RAFT_EDEVICE, hipGetErrorString(err));
    *mismatched = (int64_t)h;
    return RAFT_OK;
}


}  // extern "C"
