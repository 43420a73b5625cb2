// raft_batch.hip — the handler batches (include/raft_engine.h raft_*_batch,
// raft_*_batch_dev): RaftServer.vote() / append() / appendCommand()
// (RaftServer.kt:228-287, :100-107) for n messages, each to one (group,
// replica), messages to one replica applied in batch order.
// Two orderings: the bucketed path (a stable partition of each tile into
// buckets of 2^S consecutive replicas, then one workgroup per bucket) and the
// sorted path (a rocprim radix sort of every message).  The handlers are the
// step kernel's own (raft_step.h), applied one message at a time.  Kept apart
// from raft_engine.hip so that the step kernel's source id (build.py
// kernel_source_id, the key of its rocprofv3 rows) does not move with it.
#include <hip/hip_runtime.h>
#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/block/block_scan.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "raft_engine_impl.h"

namespace {

int fail(int code, const std::string& msg) { return raft_internal_fail(code, msg); }

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return fail(RAFT_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

int grow_dev(raft_engine* e, char** buf, size_t* have, size_t need) { return raft_internal_grow_dev(e, buf, have, need); }
int grow_host(raft_engine* e, char** buf, size_t* have, size_t need) { return raft_internal_grow_host(e, buf, have, need); }

// ---------------------------------------------------------------------------
// single-handler batches: one lane per distinct (group, replica), its
// messages applied in batch order
// ---------------------------------------------------------------------------
struct RepState {
    int32_t term, voted, role, commit, last, phys, elec, phase, retry;
    uint32_t fl;
    int32_t t1, t2;
    uint32_t c1;
    __device__ Rep ref() { return Rep{term, voted, role, commit, last, phys, elec, phase, retry, fl, t1, t2, c1}; }
};

// The replica's state quads a handler needs (raft_step.h FIELD_SLOT), one
// 16-B access and one 32-B sector each: quad 0 (term, votedFor, state, flags)
// and quad 1 (lastIndex, physLen, t1, electionMs) for vote() and the timer
// re-arm (RaftServer.kt:228-251); quad 2 (commitIndex, t2, c1, phaseMs) too
// for append() and appendCommand (:253-287, :100-107).  Quad 3 (retryMs and
// the primary session) no handler touches.  The log-tail cache (t1, t2, c1)
// is the HBM copy: the batch path keeps it valid (run_batch_dev rebuilds it
// first when a host write left it stale, and every run stores it back), so
// vote() reads no log slot at all.
struct RepQuads {
    int4 q0, q1, q2;
};
template <bool VOTE_ONLY = false>
__device__ __forceinline__ void load_rep(RepState& x, RepQuads& o, const DevParams& p, int64_t idx) {
    o.q0 = *quad(p, 0, idx);
    o.q1 = *quad(p, 1, idx);
    o.q2 = VOTE_ONLY ? make_int4(0, 0, 0, 0) : *quad(p, 2, idx);
    x.term = o.q0.x; x.voted = o.q0.y; x.role = o.q0.z; x.fl = (uint32_t)o.q0.w;
    x.last = o.q1.x; x.phys = o.q1.y; x.t1 = o.q1.z; x.elec = o.q1.w;
    x.commit = o.q2.x; x.t2 = o.q2.y; x.c1 = (uint32_t)o.q2.z; x.phase = o.q2.w;
    x.retry = 0;                                                        // (quad 3: no handler touches it)
}

// Only the quads that changed are written back, whole (the run's thread owns
// the replica): a random replica's quad is a 32-B sector of its own.
template <bool VOTE_ONLY = false>
__device__ __forceinline__ void store_rep(const RepState& x, const RepQuads& o, const DevParams& p, int64_t idx) {
    const int4 q0 = make_int4(x.term, x.voted, x.role, (int32_t)(x.fl & FL_EXPORT_MASK));
    const int4 q1 = make_int4(x.last, x.phys, x.t1, x.elec);
    const int4 q2 = make_int4(x.commit, x.t2, (int32_t)x.c1, x.phase);
    auto differ = [](int4 a, int4 b) { return a.x != b.x || a.y != b.y || a.z != b.z || a.w != b.w; };
    if (differ(q0, o.q0)) *quad(p, 0, idx) = q0;
    if (differ(q1, o.q1)) *quad(p, 1, idx) = q1;
    if (!VOTE_ONLY && differ(q2, o.q2)) *quad(p, 2, idx) = q2;
}

__device__ __forceinline__ bool resolve_rep_draw(RepState& x, const DevParams& p, uint32_t t, uint32_t gid, int r) {
    if (x.fl & FL_DRAW) {
        const u32x4 w = draw(p, t, gid, RAFT_RNG_TIMER, (uint32_t)(r >> 2));
        x.elec = scale_range(word_of(w, r & 3), p.emin, p.emax);
        x.fl &= ~FL_DRAW;
        return true;
    }
    return false;
}

enum { BATCH_VOTE = 0, BATCH_APPEND = 1, BATCH_COMMAND = 2 };

// The batch handlers report one thing: reference accesses below the window
// (the run is then invalid, RAFT_EWINDOW).  Called in divergent control flow:
// a mask's bit for this lane is read with ib().
struct BatchCounters {
    uint32_t miss = 0;
    __device__ __forceinline__ void add(uint64_t m, int c) {
        if (c == RAFT_C_LOG_WINDOW_MISS) miss += ib(m) ? 1u : 0u;
    }
};

// The batch path on the device (raft_*_batch, raft_*_batch_dev).  Messages
// to one (group, replica) must be applied in batch order, and messages to
// different replicas are independent.  batch_keys_kernel turns each message
// into its key g * R + d (a message outside the engine sets flags[0]); a
// stable radix sort of (key, message index) then puts each replica's messages
// next to each other in batch order, and batch_kernel runs one thread per
// sorted position: the first position of each key's run loads that replica,
// applies the run's messages in order and stores it back.
// Key: uint32_t while G * R fits (half the sort's key traffic), else uint64_t.
template <class Key>
__global__ __launch_bounds__(BLOCK) void batch_keys_kernel(const int64_t* __restrict__ group,
                                                           const int32_t* __restrict__ dst, int n, int64_t G, int R,
                                                           Key* __restrict__ keys, uint32_t* __restrict__ ord,
                                                           unsigned int* flags) {
    const int m = blockIdx.x * BLOCK + threadIdx.x;
    if (m >= n) return;
    const int64_t g = group[m];
    const int32_t d = dst[m];
    const bool ok = g >= 0 && g < G && d >= 0 && d < R;
    keys[m] = ok ? (Key)((uint64_t)g * (uint64_t)R + (uint64_t)d) : (Key)0;
    ord[m] = (uint32_t)m;
    if (!ok) atomicOr(&flags[0], 1u);
}

// One replica's run of messages, in batch order: load the replica (idx =
// g * R + r), apply message ord(m) for m = m0, m0 + 1, ... while more(m), store
// it back.  Shared by both batch paths (batch_kernel, bucket_batch_kernel).
// flags[1]: accesses below the retained log window (RAFT_EWINDOW)
template <bool TB, int kind, class More, class Ord>
__device__ __forceinline__ void apply_run(const DevParams& p, uint32_t t, int64_t idx, int m0, More more, Ord ord,
                                          const void* req, void* resp, unsigned int* flags,
                                          unsigned int* hmiss = nullptr) {
    using Req = std::conditional_t<kind == BATCH_VOTE, raft_vote_req,
                                   std::conditional_t<kind == BATCH_APPEND, raft_append_req, uint32_t>>;
    const int R = p.R;
    const int64_t i = idx / R;
    const int r = (int)(idx - i * R);
    const uint32_t gid = (uint32_t)(p.g0 + i);
    constexpr bool VO = kind == BATCH_VOTE;
    // the run's first request is fetched with the replica's fields (one round
    // trip for both); each later one while the previous message is applied
    uint32_t om = ord(m0);
    Req q = ((const Req*)req)[om];
    RepState x;
    RepQuads o;
    load_rep<VO>(x, o, p, idx);
    const LogView lv = log_of(p, idx);
    BatchCounters cnt;
    for (int m = m0;;) {
        const Req qm = q;
        const uint32_t oc = om;
        if (more(m + 1)) {
            om = ord(m + 1);
            q = ((const Req*)req)[om];
        }
        if constexpr (kind == BATCH_VOTE) {
            int32_t rt;
            uint64_t gr;
            vote_handler<TB, true>(x.ref(), __ballot(1), r + 1, qm.term, qm.candidate_id, qm.last_log_index,
                                   qm.last_log_term, __ballot(x.phys - x.last >= p.W), __ballot(x.last >= 1),
                                   follower_sent(x.fl), cnt, rt, gr);
            ((raft_vote_resp*)resp)[oc] = raft_vote_resp{rt, ib(gr) ? 1 : 0};
        } else if constexpr (kind == BATCH_APPEND) {
            int32_t rt = 0;
            uint64_t su = 0, st = 0;
            const int32_t pv = qm.prev_log_index;
            // log[prev] (and TB: log[prev + 1]) from the tail cache when it
            // holds them, else from the log
            const int32_t dprev = pv == x.last - 1 ? x.t1 : pv == x.last - 2 ? x.t2
                                  : (pv >= 0 && pv < x.last) ? (int32_t)lv.at(pv)->x : 0;
            const int32_t dnext = !TB ? 0 : pv + 1 == x.last - 1 ? x.t1 : pv + 1 == x.last - 2 ? x.t2
                                  : (pv + 1 >= 0 && pv + 1 < x.last) ? (int32_t)lv.at(pv + 1)->x : 0;
            const uint64_t thrown = append_handler<TB, true>(x.ref(), __ballot(1), r + 1, lv, qm.term, qm.leader_id,
                                                       pv, qm.prev_log_term, __ballot(qm.has_entry != 0),
                                                       Entry{qm.entry_term, qm.entry_cmd}, qm.leader_commit, dprev,
                                                       dnext, __ballot(pv + 1 == x.last), __ballot(pv >= 0),
                                                       __ballot(qm.leader_id != r + 1), follower_sent(x.fl),
                                                       cnt, rt, su, st);
            ((raft_append_resp*)resp)[oc] = raft_append_resp{rt, ib(su) ? 1 : 0, ib(thrown) ? 1 : 0};
        } else {
            append_command<TB, true>(x.ref(), __ballot(1), lv, qm, cnt);
        }
        resolve_rep_draw(x, p, t, gid, r);
        if (!more(++m)) break;
    }
    store_rep<VO>(x, o, p, idx);
    if (cnt.miss) {
        atomicAdd(&flags[1], cnt.miss);
        if (hmiss) *(volatile unsigned int*)hmiss = 1u;                 // (bucket path: the host copies the count)
    }
}

// The sorted path: one thread per sorted position; the first position of each
// key's run applies the run.  flags[0]: a message was outside the engine
// (nothing is applied)
template <bool TB, class Key, int kind>
__global__ __launch_bounds__(BLOCK) void batch_kernel(DevParams p, uint32_t t, int n,
                                                      const Key* __restrict__ keys,
                                                      const uint32_t* __restrict__ order, const void* req, void* resp,
                                                      unsigned int* flags) {
    const int m0 = blockIdx.x * BLOCK + threadIdx.x;
    if (m0 >= n || *(volatile unsigned int*)&flags[0]) return;
    const Key key = keys[m0];
    if (m0 > 0 && keys[m0 - 1] == key) return;                          // not the first of its run
    apply_run<TB, kind>(p, t, (int64_t)key, m0, [&](int m) { return m < n && keys[m] == key; },
                        [&](int m) { return order[m]; }, req, resp, flags);
}

// ---- the bucketed path (uint32 keys): a stable partition of each tile instead
// of a full radix sort.  Bucket b holds the keys [b << S, (b + 1) << S) -- 2^S
// consecutive replicas, ~BUCKET_MEAN messages of a random batch.  Two kernels:
//   bucket_tile_kernel:  per tile of TILE messages, its messages stably
//                        partitioned by bucket inside the tile's own region,
//                        and the tile's (offset, count) of every bucket, written
//                        tile-major (coalesced): seg[tile][b]
//   bucket_batch_kernel: per bucket, the tiles' segments in tile order (a
//                        block scan of their counts) -- the bucket's messages
//                        in batch order -- gathered into LDS a chunk of BLOCK
//                        at a time, sorted stably by key, one thread per run
// A bucket is applied by one workgroup, chunk after chunk, so a replica's
// messages keep batch order across chunks too.  Nothing global is scanned or
// scattered: the only cross-tile step is each bucket's scan of its ntile
// counts.
// a tile's workgroup (build-time: 512 threads x 8 messages; 256 x 16 ran the
// tile kernel at one wave per SIMD, 16 serial ballot rounds per wave)
#ifndef RAFT_TILE_THREADS
#define RAFT_TILE_THREADS 512
#endif
#ifndef RAFT_TILE_IPT
#define RAFT_TILE_IPT 8
#endif
constexpr int TILE_THREADS = RAFT_TILE_THREADS, TILE_WAVES = TILE_THREADS / 64;
constexpr int TILE_IPT = RAFT_TILE_IPT, TILE = TILE_THREADS * TILE_IPT;
constexpr int BUCKETS_MAX = 3072;                                       // bucket_tile_kernel's LDS: TILE * 8 + (TILE_WAVES + 1) * NB * 2
constexpr int BUCKET_MEAN = 320;                                        // target messages per bucket
constexpr uint64_t SEG_MAX = 1ull << 27;                                // segment-table entries (1 GB)
constexpr size_t BST_HEAD = 256;                                        // the staging's head: the bucketed path's status words
// bucket_batch_kernel's workgroup: a bucket's chunk, one message per thread
// (per 10^6-message batch, 512 threads at 320 per bucket beat 256 at 160 and
// 1,024 at 640 by 5-10 %, profiles/r5_h)
constexpr int BUCKET_THREADS = 512;
constexpr int GATHER_TILES = 2 * BUCKET_THREADS;                        // bucket_batch_kernel's direct gather

// Wave w of the tile's workgroup takes messages [w * 64 * TILE_IPT, (w + 1) *
// 64 * TILE_IPT) of it, 64 consecutive ones per round.  A message's place in
// its bucket's segment: the lanes of its round with its bucket below it (a
// match by ballots over the bucket bits), plus the wave's earlier rounds (the
// wave's LDS count, read by every lane of the match and then advanced by its
// lowest lane), plus the earlier waves (their counts, summed after the tile).
__global__ __launch_bounds__(TILE_THREADS) void bucket_tile_kernel(const int64_t* __restrict__ group,
                                                            const int32_t* __restrict__ dst, int n, int64_t G, int R,
                                                            int S, int NB, int bbits, uint2* __restrict__ tiles,
                                                            uint2* __restrict__ seg, unsigned int* dflags,
                                                            unsigned int* hflags) {
    // LDS: the tile's output staged (written out coalesced: one 8-B store per
    // message to its place would cost a 32-B sector each), then the waves'
    // counts and the tile's bucket offsets, [TILE_WAVES + 1][NB] (<= TILE)
    extern __shared__ uint2 stage[];                                    // [TILE]
    uint16_t* const cnt = (uint16_t*)(stage + TILE);
    for (int b = threadIdx.x; b < TILE_WAVES * NB; b += TILE_THREADS) cnt[b] = 0;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint16_t* const cw = cnt + w * NB;
    uint16_t* const off = cnt + TILE_WAVES * NB;                    // the tile's bucket offsets
    const uint64_t below = (1ull << lane) - 1ull;
    const int t0 = blockIdx.x * TILE;
    const int base = t0 + w * 64 * TILE_IPT + lane;
    // every round's message loaded up front (the rounds' ballots and LDS
    // updates would otherwise serialise the loads)
    // (unconditional loads at a clamped index: a load under a branch is
    // waited for inside it, which serialised the 2 * TILE_IPT round trips)
    uint32_t key[TILE_IPT], rk[TILE_IPT];
    int64_t gg[TILE_IPT];
    int32_t dd[TILE_IPT];
#pragma unroll
    for (int j = 0; j < TILE_IPT; ++j) {
        const int m = min(base + j * 64, n - 1);
        gg[j] = group[m];
        dd[j] = dst[m];
    }
    bool bad = false;
#pragma unroll
    for (int j = 0; j < TILE_IPT; ++j) {
        const bool in = base + j * 64 < n;
        const bool ok = gg[j] >= 0 && gg[j] < G && dd[j] >= 0 && dd[j] < R;
        key[j] = in && ok ? (uint32_t)((uint64_t)gg[j] * (uint64_t)R + (uint64_t)dd[j]) : 0u;
        bad |= in && !ok;
    }
    if (bad) {                                                          // (idempotent plain stores)
        *(volatile unsigned int*)&dflags[0] = 1u;
        *(volatile unsigned int*)&hflags[0] = 1u;
    }
    __syncthreads();                                                    // the counts are zero
#pragma unroll
    for (int j = 0; j < TILE_IPT; ++j) {
        const bool in = base + j * 64 < n;
        const uint32_t b = key[j] >> S;
        uint64_t peers = __ballot(in);
        for (int i = 0; i < bbits; ++i) {
            const uint64_t x = __ballot((b >> i) & 1u);
            peers &= ((b >> i) & 1u) ? x : ~x;
        }
        uint32_t old = 0;
        if (in) {
            old = cw[b];                                                // every lane of the match reads it,
            if (lane == __builtin_ctzll(peers)) cw[b] = (uint16_t)(old + (uint32_t)__popcll(peers));   // then its first lane
        }
        rk[j] = old + (uint32_t)__popcll(peers & below);
    }
    __syncthreads();
    // the waves' counts -> their prefixes; the tile's count per bucket, and
    // its exclusive scan over the buckets (each thread a contiguous range of
    // buckets, then a block scan of the ranges' sums)
    const int per = (NB + TILE_THREADS - 1) / TILE_THREADS, b0 = threadIdx.x * per, b1 = min(NB, b0 + per);
    uint32_t sum = 0;
    for (int b = b0; b < b1; ++b) {
        uint32_t c = 0;
        for (int q = 0; q < TILE_WAVES; ++q) {
            const uint32_t x = cnt[q * NB + b];
            cnt[q * NB + b] = (uint16_t)c;
            c += x;
        }
        off[b] = (uint16_t)c;                                           // (the count, for now)
        sum += c;
    }
    uint32_t pre;
    rocprim::block_scan<uint32_t, TILE_THREADS>().exclusive_scan(sum, pre, 0u);
    for (int b = b0; b < b1; ++b) {
        const uint32_t c = off[b];
        off[b] = (uint16_t)pre;
        seg[(int64_t)blockIdx.x * NB + b] = make_uint2(pre, c);
        pre += c;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TILE_IPT; ++j) {
        const int m = base + j * 64;
        if (m < n) {
            const uint32_t b = key[j] >> S;
            stage[off[b] + cw[b] + rk[j]] = make_uint2(key[j], (uint32_t)m);   // (key, message index)
        }
    }
    __syncthreads();
    const int len = min(TILE, n - t0);
    for (int q = threadIdx.x; 2 * q < len; q += TILE_THREADS) {                 // two messages per 16-B store
        if (2 * q + 1 < len) *(uint4*)&tiles[t0 + 2 * q] = *(const uint4*)&stage[2 * q];
        else tiles[t0 + 2 * q] = stage[2 * q];
    }
}

// Latency-bound (a workgroup's dependent round trips), so residency counts:
// the vote kernel is built for 8 waves per SIMD (61 VGPRs: 4 workgroups per
// CU instead of 3, +3.6 %, profiles/r6_occ); the append kernel keeps its 90
// (at 6 waves: 80 with spills, no faster; at 8: 25 spills, -18 %)
template <bool TB, int kind, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(kind == BATCH_VOTE ? 8 : 1)))
void bucket_batch_kernel(DevParams p, uint32_t t, int n, int S, int NB, int ntile,
                                                          const uint2* __restrict__ tiles,
                                                          const uint2* __restrict__ seg, const void* req,
                                                          void* resp, unsigned int* dflags, unsigned int* hflags) {
    static_assert(2 * NT >= GATHER_TILES, "the direct gather holds at most two tiles per thread");
    using Sort = rocprim::block_radix_sort<uint32_t, NT, 1, uint32_t>;
    using Scan = rocprim::block_scan<uint32_t, NT>;
    __shared__ union {
        typename Sort::storage_type sort;
        typename Scan::storage_type scan;
    } sm;
    __shared__ uint2 buf[NT];
    __shared__ uint32_t lk[NT], lo[NT];
    __shared__ uint32_t spos[GATHER_TILES], soff[GATHER_TILES];
    // a message outside the engine (bucket_tile_kernel): nothing is applied
    const bool bad = *(volatile unsigned int*)&dflags[0] != 0u;         // the same for the whole grid
    // XCD-aware: workgroups b and b + 8 share an XCD (dealt round-robin), so
    // XCD b % 8 takes the contiguous buckets [(b % 8) * C, (b % 8 + 1) * C) in
    // order; neighbouring buckets share the 64-B lines of each tile's segment
    // row and of its partitioned messages, which then come from one L2
    const int xcb = (NB + 7) >> 3;
    const int bk = (int)(blockIdx.x & 7u) * xcb + (int)(blockIdx.x >> 3);
    if (bk >= NB) return;                                               // (the grid rounds NB up to 8 * C)
    const uint32_t kb = (uint32_t)bk << S;
    // this thread's tiles [tt0, tt1): their segments of this bucket, and
    // where they start in the bucket's batch order
    const int per = (ntile + NT - 1) / NT, tt0 = threadIdx.x * per, tt1 = min(ntile, tt0 + per);
    // up to GATHER_TILES tiles, their segments' starts and offsets go to LDS
    // and every message of a chunk is fetched by its own thread (a binary
    // search for its tile): one round trip.  (A thread walking its tiles'
    // segments waits for each message in turn.)
    const bool direct = ntile <= GATHER_TILES;
    uint32_t mine = 0;
    uint2 sg0 = make_uint2(0u, 0u), sg1 = make_uint2(0u, 0u);
    if (direct) {                                                       // per <= 2
        if (tt0 < tt1) sg0 = seg[(int64_t)tt0 * NB + bk];
        if (tt0 + 1 < tt1) sg1 = seg[(int64_t)(tt0 + 1) * NB + bk];
        mine = sg0.y + sg1.y;
    } else {
        for (int q = tt0; q < tt1; ++q) mine += seg[(int64_t)q * NB + bk].y;
    }
    uint32_t pos, len_all;
    Scan().exclusive_scan(mine, pos, 0u, len_all, sm.scan, rocprim::plus<uint32_t>());
    if (direct) {
        if (tt0 < tt1) { spos[tt0] = pos; soff[tt0] = sg0.x; }
        if (tt0 + 1 < tt1) { spos[tt0 + 1] = pos + sg0.y; soff[tt0 + 1] = sg1.x; }
    }
    for (uint32_t c0 = 0; c0 < (bad ? 0u : len_all); c0 += NT) {    // workgroup-uniform
        const int len = (int)min(len_all - c0, (uint32_t)NT);
        if (!direct) {
            // the chunk's messages [c0, c0 + len) of the bucket into buf, in batch order
            uint32_t at = pos;
            for (int q = tt0; q < tt1 && at < c0 + len; ++q) {
                const uint2 sg = seg[(int64_t)q * NB + bk];
                const uint32_t lo_i = max(at, c0), hi_i = min(at + sg.y, c0 + (uint32_t)len);
                for (uint32_t i = lo_i; i < hi_i; ++i) buf[i - c0] = tiles[(int64_t)q * TILE + sg.x + (i - at)];
                at += sg.y;
            }
        }
        __syncthreads();                                                // buf / spos complete (sm.scan / sm.sort free)
        const int q = threadIdx.x;
        uint2 x = make_uint2(kb + (1u << S), 0u);                      // padding sorts last
        if (q < len) {
            if (direct) {
                // the last tile whose segment starts at or before position i
                const uint32_t i = c0 + (uint32_t)q;
                int lo_t = 0, hi_t = ntile;
                while (hi_t - lo_t > 1) {
                    const int mid = (lo_t + hi_t) >> 1;
                    if (spos[mid] <= i) lo_t = mid; else hi_t = mid;
                }
                x = tiles[(int64_t)lo_t * TILE + soff[lo_t] + (i - spos[lo_t])];
            } else {
                x = buf[q];
            }
        }
        uint32_t k[1] = {x.x - kb}, v[1] = {x.y};
        Sort().sort(k, v, sm.sort, 0, S + 1);
        lk[q] = k[0];
        lo[q] = v[0];
        __syncthreads();
        if (q < len && (q == 0 || lk[q - 1] != lk[q])) {
            const uint32_t key = lk[q];
            apply_run<TB, kind>(p, t, (int64_t)(kb + key), q, [&](int m) { return m < len && lk[m] == key; },
                                [&](int m) { return lo[m]; }, req, resp, dflags + 1,    // misses -> dflags[2]
                                hflags + 1);
        }
        // another chunk of this bucket: the barrier (a workgroup-scope fence:
        // one CU, one L1) makes this chunk's replica stores visible to it, and
        // frees buf / lk / lo
        if (c0 + NT < len_all) __syncthreads();
    }
}

}  // namespace

// rocprim's radix sort takes its merge-sort path up to 2^20 items (one
// block sort and ~10 merge passes over the whole array, 21 dispatches at 10^6
// messages); a merge limit of 0 keeps it on the onesweep path (a histogram
// pass and one pass per 8 key bits).
using BatchSortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                   rocprim::default_config, 0>;
template <class Key>
static int run_batch_keys(raft_engine* e, int kind, const int64_t* group, const int32_t* dst, const void* req,
                          void* resp, int n, int bits) {
    const int R = e->p.R;
    size_t sort_tmp = 0;
    HIP_TRY(rocprim::radix_sort_pairs<BatchSortConfig>(nullptr, sort_tmp, (const Key*)nullptr, (Key*)nullptr,
                                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, n, 0u,
                                                       (unsigned)bits, e->stream));
    const size_t b_keys = al256((size_t)n * sizeof(Key)), b_ord = al256((size_t)n * 4);
    const size_t sz0 = e->bst_bytes;
    if (int rc = grow_dev(e, &e->bst, &e->bst_bytes, BST_HEAD + 2 * b_keys + 2 * b_ord + al256(sort_tmp) + 256))
        return rc;
    if (e->bst_bytes != sz0) HIP_TRY(hipMemsetAsync(e->bst, 0, BST_HEAD, e->stream));   // (the bucketed path's words)
    char* b = e->bst + BST_HEAD;
    Key* k_in = (Key*)b; b += b_keys;
    Key* k_out = (Key*)b; b += b_keys;
    uint32_t* o_in = (uint32_t*)b; b += b_ord;
    uint32_t* o_out = (uint32_t*)b; b += b_ord;
    unsigned int* flags = (unsigned int*)b; b += 256;
    void* tmp = b;
    HIP_TRY(hipMemsetAsync(flags, 0, 8, e->stream));
    const unsigned grid = (unsigned)((n + BLOCK - 1) / BLOCK);
    batch_keys_kernel<Key><<<grid, BLOCK, 0, e->stream>>>(group, dst, n, e->p.G, R, k_in, o_in, flags);
    HIP_TRY(rocprim::radix_sort_pairs<BatchSortConfig>(tmp, sort_tmp, k_in, k_out, o_in, o_out, n, 0u, (unsigned)bits,
                                                       e->stream));
    using BK = void (*)(DevParams, uint32_t, int, const Key*, const uint32_t*, const void*, void*, unsigned int*);
    const bool tb = e->p.mode == RAFT_MODE_TEXTBOOK;
    BK kern = kind == BATCH_VOTE     ? (tb ? batch_kernel<true, Key, BATCH_VOTE> : batch_kernel<false, Key, BATCH_VOTE>)
              : kind == BATCH_APPEND ? (tb ? batch_kernel<true, Key, BATCH_APPEND> : batch_kernel<false, Key, BATCH_APPEND>)
                                     : (tb ? batch_kernel<true, Key, BATCH_COMMAND> : batch_kernel<false, Key, BATCH_COMMAND>);
    kern<<<grid, BLOCK, 0, e->stream>>>(e->dp, (uint32_t)e->t, n, k_out, o_out, req, resp, flags);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(e->bflags_host, flags, 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return RAFT_OK;
}

using BK = void (*)(DevParams, uint32_t, int, int, int, int, const uint2*, const uint2*, const void*, void*,
                    unsigned int*, unsigned int*);
static BK bucket_kernel_of(int kind, bool tb) {
    constexpr int NT = BUCKET_THREADS;
    return kind == BATCH_VOTE     ? (tb ? bucket_batch_kernel<true, BATCH_VOTE, NT> : bucket_batch_kernel<false, BATCH_VOTE, NT>)
           : kind == BATCH_APPEND ? (tb ? bucket_batch_kernel<true, BATCH_APPEND, NT> : bucket_batch_kernel<false, BATCH_APPEND, NT>)
                                  : (tb ? bucket_batch_kernel<true, BATCH_COMMAND, NT> : bucket_batch_kernel<false, BATCH_COMMAND, NT>);
}

// The bucketed path (bucket_tile_kernel, bucket_batch_kernel): buckets of 2^S
// keys, S the smallest shift that gives ~BUCKET_MEAN messages per bucket of a
// uniform batch and at most BUCKETS_MAX buckets.
static int run_batch_buckets(raft_engine* e, int kind, const int64_t* group, const int32_t* dst, const void* req,
                             void* resp, int n, uint64_t nkeys) {
    int S = 0;
    while (S < 31 && ((uint64_t)n << S) < (uint64_t)BUCKET_MEAN * nkeys) ++S;
    // at most BUCKETS_MAX buckets, and a segment table (NB x ntile entries of
    // 8 B) of at most SEG_MAX entries: very large batches take larger buckets
    const uint64_t ntile64 = ((uint64_t)n + TILE - 1) / TILE;
    auto nb_of = [&](int s) { return (nkeys + (1ull << s) - 1) >> s; };
    while (S < 31 && (nb_of(S) > (uint64_t)BUCKETS_MAX || nb_of(S) * ntile64 > SEG_MAX)) ++S;
    const int NB = (int)nb_of(S);
    int bbits = 1;
    while ((uint64_t)(NB - 1) >> bbits) ++bbits;
    const int ntile = (int)ntile64;
    const size_t b_t = al256((size_t)ntile * TILE * 8), b_s = al256((size_t)NB * ntile * 8);
    const size_t sz0 = e->bst_bytes;                                    // grow_dev reallocates only to grow
    if (int rc = grow_dev(e, &e->bst, &e->bst_bytes, BST_HEAD + b_t + b_s)) return rc;
    char* b = e->bst + BST_HEAD;
    uint2* tiles = (uint2*)b; b += b_t;
    uint2* seg = (uint2*)b; b += b_s;
    // status words: dflags (device: [0] a message outside the engine, [2]
    // the window misses), zero between batches; hflags = the engine's
    // page-locked words [0], [1] (RAFT_ERANGE; "some miss was counted"),
    // written by the kernels with plain stores and read after the
    // synchronisation.  A batch without either needs no memset and no copy;
    // one with them copies the count and resets the device words (rare).
    unsigned int* dflags = (unsigned int*)e->bst;                       // at a fixed place: the staging's head
    // new staging, or an earlier batch that returned an error after its
    // kernels were enqueued (its words may still be set): zero them first
    if (e->bst_bytes != sz0 || e->bst_dirty) HIP_TRY(hipMemsetAsync(dflags, 0, BST_HEAD, e->stream));
    e->bst_dirty = true;                                                // until this batch ends cleanly
    unsigned int* hflags = (unsigned int*)e->dp.status - 8;             // device view of bflags_host
    e->bflags_host[0] = e->bflags_host[1] = 0u;
    const size_t tile_lds = (size_t)TILE * 8 + (size_t)(TILE_WAVES + 1) * NB * 2;
    // (more than 64 KB of dynamic LDS: allowed once per device)
    static std::atomic<bool> lds_set[64];
    if (e->device < 0 || e->device >= 64 || !lds_set[e->device].load(std::memory_order_acquire)) {
        HIP_TRY(hipFuncSetAttribute((const void*)bucket_tile_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)((size_t)TILE * 8 + (size_t)(TILE_WAVES + 1) * BUCKETS_MAX * 2)));
        if (e->device >= 0 && e->device < 64) lds_set[e->device].store(true, std::memory_order_release);
    }
    bucket_tile_kernel<<<ntile, TILE_THREADS, tile_lds, e->stream>>>(
        group, dst, n, e->p.G, e->p.R, S, NB, bbits, tiles, seg, dflags, hflags);
    const BK kern = bucket_kernel_of(kind, e->p.mode == RAFT_MODE_TEXTBOOK);
    kern<<<8 * ((NB + 7) >> 3), BUCKET_THREADS, 0, e->stream>>>(e->dp, (uint32_t)e->t, n, S, NB, ntile, tiles, seg, req, resp, dflags,
                                               hflags);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (e->bflags_host[0] | e->bflags_host[1]) {
        unsigned int w[4] = {0u, 0u, 0u, 0u};
        HIP_TRY(hipMemcpy(w, dflags, 16, hipMemcpyDeviceToHost));
        e->bflags_host[1] = w[2];                                       // the count, for RAFT_EWINDOW
        HIP_TRY(hipMemsetAsync(dflags, 0, 16, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
    }
    e->bst_dirty = false;
    return RAFT_OK;
}

// The batch on device buffers: keys, the bucketed partition or a stable radix
// sort over the key bits, the handlers; one synchronisation at the end for the
// status flags.
static int run_batch_dev(raft_engine* e, int kind, const int64_t* group, const int32_t* dst, const void* req,
                         void* resp, int64_t n64) {
    e->fork_needed = true;
    // the handlers read and write the HBM tail cache: rebuilt first if a host
    // write left it stale (then it stays valid: the batches keep it)
    raft_internal_ensure_cache(e);
    const int n = (int)n64;
    const uint64_t nkeys = (uint64_t)e->p.G * (uint64_t)e->p.R;
    int bits = 1;
    while (bits < 64 && (nkeys - 1) >> bits) ++bits;
    if (e->batch_path == RAFT_BATCH_PATH_BUCKETED && bits > 32)
        return fail(RAFT_EINVAL, "the bucketed batch path needs G * R <= 2^32");
    const int rc = e->batch_path != RAFT_BATCH_PATH_SORTED && bits <= 32
                       ? run_batch_buckets(e, kind, group, dst, req, resp, n, nkeys)
                   : bits <= 32 ? run_batch_keys<uint32_t>(e, kind, group, dst, req, resp, n, bits)
                                : run_batch_keys<uint64_t>(e, kind, group, dst, req, resp, n, bits);
    if (rc) return rc;
    if (e->bflags_host[0]) return fail(RAFT_ERANGE, "a message's group or replica index is outside the engine; "
                                                    "nothing was applied");
    if (e->bflags_host[1])
        return fail(RAFT_EWINDOW, std::to_string(e->bflags_host[1]) + " log accesses below the retained log_window: "
                                  "the batch's results are not the reference's");
    return RAFT_OK;
}

static int check_batch_args(raft_engine* e, int64_t n, const void* group, const void* dst, const void* req,
                            size_t resp_sz, const void* resp) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    if (n < 0) return fail(RAFT_EINVAL, "negative batch");
    if (n > 0x7FFFFFFF) return fail(RAFT_EINVAL, "batch larger than 2^31 - 1 messages");
    if (n > 0 && (!group || !dst || !req || (resp_sz && !resp))) return fail(RAFT_EINVAL, "null buffer");
    return RAFT_OK;
}

// The caller's buffer is page-locked host memory (hipHostMalloc / registered):
// the DMA engines can read and write it directly.
static bool host_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();                   // pageable memory: not an error of the batch
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// memcpy of a large batch array into or out of the pinned staging, split
// over a few threads (one core copies ≈10 GB/s; a 10^6-message batch moves
// 28-40 MB each way)
static void batch_memcpy(void* d, const void* s, size_t n) {
    constexpr size_t PAR_MIN = 4u << 20;
    const unsigned hw = std::thread::hardware_concurrency();
    const unsigned T = (unsigned)std::min<size_t>({8u, hw ? hw : 1u, n / PAR_MIN + 1});
    if (T <= 1) {
        std::memcpy(d, s, n);
        return;
    }
    const size_t chunk = (n + T - 1) / T;
    std::vector<std::thread> th;
    for (unsigned t = 1; t < T; ++t) {
        const size_t o = t * chunk;
        if (o < n) th.emplace_back([=] { std::memcpy((char*)d + o, (const char*)s + o, std::min(chunk, n - o)); });
    }
    std::memcpy(d, s, std::min(chunk, n));
    for (auto& x : th) x.join();
}

// Host buffers: moved to device staging with one DMA per array and run on the
// device, the responses copied back the same way.  Page-locked caller buffers
// are read and written by the DMA directly; pageable ones go through the
// engine-owned pinned staging (a multi-threaded memcpy per array).
static int run_batch(raft_engine* e, int kind, const int64_t* group, const int32_t* dst, const void* req,
                     size_t req_sz, void* resp, size_t resp_sz, int64_t n) {
    if (int rc = check_batch_args(e, n, group, dst, req, resp_sz, resp)) return rc;
    if (n == 0) return RAFT_OK;
    HIP_TRY(hipSetDevice(e->device));
    const size_t b_g = al256((size_t)n * 8), b_d = al256((size_t)n * 4), b_q = al256((size_t)n * req_sz);
    const size_t b_s = al256((size_t)n * resp_sz), in_b = b_g + b_d + b_q;
    if (int rc = grow_dev(e, &e->bio, &e->bio_bytes, in_b + b_s)) return rc;
    const bool pinned = host_pinned(group) && host_pinned(dst) && host_pinned(req) && (!resp_sz || host_pinned(resp));
    if (pinned) {
        HIP_TRY(hipMemcpyAsync(e->bio, group, (size_t)n * 8, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipMemcpyAsync(e->bio + b_g, dst, (size_t)n * 4, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipMemcpyAsync(e->bio + b_g + b_d, req, (size_t)n * req_sz, hipMemcpyHostToDevice, e->stream));
    } else {
        if (int rc = grow_host(e, &e->hst, &e->hst_bytes, in_b + b_s)) return rc;
        batch_memcpy(e->hst, group, (size_t)n * 8);
        batch_memcpy(e->hst + b_g, dst, (size_t)n * 4);
        batch_memcpy(e->hst + b_g + b_d, req, (size_t)n * req_sz);
        HIP_TRY(hipMemcpyAsync(e->bio, e->hst, in_b, hipMemcpyHostToDevice, e->stream));
    }
    const int rc = run_batch_dev(e, kind, (const int64_t*)e->bio, (const int32_t*)(e->bio + b_g), e->bio + b_g + b_d,
                                 resp_sz ? e->bio + in_b : nullptr, n);
    if (rc != RAFT_OK && rc != RAFT_EWINDOW) return rc;
    if (resp_sz) {
        HIP_TRY(hipMemcpyAsync(pinned ? resp : (void*)(e->hst + in_b), e->bio + in_b, (size_t)n * resp_sz,
                               hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        if (!pinned) batch_memcpy(resp, e->hst + in_b, (size_t)n * resp_sz);
    }
    return rc;
}

static int run_batch_on_device(raft_engine* e, int kind, const int64_t* group, const int32_t* dst, const void* req,
                               size_t resp_sz, void* resp, int64_t n) {
    if (int rc = check_batch_args(e, n, group, dst, req, resp_sz, resp)) return rc;
    if (n == 0) return RAFT_OK;
    HIP_TRY(hipSetDevice(e->device));
    return run_batch_dev(e, kind, group, dst, req, resp, n);
}

extern "C" {

// the handler batches' provenance: build.py's batch_source_id plus the
// compile-time knobs of their kernels, so a variant build's rocprofv3 rows
// never carry the production build's key
#ifndef RAFT_BUILD_BATCH_ID
#define RAFT_BUILD_BATCH_ID "unknown"
#endif
#define RAFT_STR2(x) #x
#define RAFT_STR(x) RAFT_STR2(x)
const char* raft_build_batch_source_id(void) {
    return RAFT_BUILD_BATCH_ID "-t" RAFT_STR(RAFT_TILE_THREADS) "x" RAFT_STR(RAFT_TILE_IPT);
}

int raft_vote_batch(raft_engine* e, const int64_t* group, const int32_t* dst, const raft_vote_req* req,
                    raft_vote_resp* resp, int64_t n) {
    return run_batch(e, BATCH_VOTE, group, dst, req, sizeof(raft_vote_req), resp, sizeof(raft_vote_resp), n);
}

int raft_append_batch(raft_engine* e, const int64_t* group, const int32_t* dst, const raft_append_req* req,
                      raft_append_resp* resp, int64_t n) {
    return run_batch(e, BATCH_APPEND, group, dst, req, sizeof(raft_append_req), resp, sizeof(raft_append_resp), n);
}

int raft_append_command_batch(raft_engine* e, const int64_t* group, const int32_t* replica, const uint32_t* cmd,
                              int64_t n) {
    return run_batch(e, BATCH_COMMAND, group, replica, cmd, sizeof(uint32_t), nullptr, 0, n);
}

int raft_vote_batch_dev(raft_engine* e, const int64_t* group, const int32_t* dst, const raft_vote_req* req,
                        raft_vote_resp* resp, int64_t n) {
    return run_batch_on_device(e, BATCH_VOTE, group, dst, req, sizeof(raft_vote_resp), resp, n);
}

int raft_append_batch_dev(raft_engine* e, const int64_t* group, const int32_t* dst, const raft_append_req* req,
                          raft_append_resp* resp, int64_t n) {
    return run_batch_on_device(e, BATCH_APPEND, group, dst, req, sizeof(raft_append_resp), resp, n);
}

int raft_append_command_batch_dev(raft_engine* e, const int64_t* group, const int32_t* replica, const uint32_t* cmd,
                                  int64_t n) {
    return run_batch_on_device(e, BATCH_COMMAND, group, replica, cmd, 0, nullptr, n);
}


int raft_engine_set_batch_path(raft_engine* e, int32_t path) {
    if (!e) return fail(RAFT_EINVAL, "null engine");
    if (path < RAFT_BATCH_PATH_AUTO || path > RAFT_BATCH_PATH_BUCKETED) return fail(RAFT_EINVAL, "unknown batch path");
    e->batch_path = path;
    return RAFT_OK;
}

}  // extern "C"
