// raft_engine_impl.h — internal to the engine library: what raft_engine.hip
// (the step kernel, the accessors, the C-ABI) and raft_batch.hip (the handler
// batches, include/raft_engine.h raft_*_batch*) share -- the engine object, the
// HBM indexing helpers and the error / staging entry points.  Not installed.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "raft_step.h"

using namespace raft;

// raft_engine.hip: set raft_last_error() and return `code`; grow-only engine
// staging (device / page-locked host), kept for the engine's lifetime
int raft_internal_fail(int code, const std::string& msg);
extern "C" int raft_internal_grow_dev(raft_engine* e, char** buf, size_t* have, size_t need);
extern "C" int raft_internal_grow_host(raft_engine* e, char** buf, size_t* have, size_t need);
// raft_engine.hip: enqueue the log-tail cache's rebuild on the engine stream
// if a host write left it stale (cache_valid false)
void raft_internal_ensure_cache(raft_engine* e);

namespace {

constexpr int BLOCK = 256;
constexpr int WAVES_PER_BLOCK = BLOCK / 64;

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// field f of replica idx = g * R + r in the state quads (DevParams::st,
// raft_step.h FIELD_SLOT): word f & 3 of quad f >> 2 of the replica's slots
__device__ __forceinline__ int64_t fidx(const DevParams& p, int f, int64_t idx) {
    const int s = FIELD_SLOT[f];
    return ((int64_t)(s >> 2) * p.GR + idx) * 4 + (s & 3);
}
// quad q of replica idx (16-B aligned: the state array starts on 256 B)
__device__ __forceinline__ int4* quad(const DevParams& p, int q, int64_t idx) {
    return (int4*)p.st + (int64_t)q * p.GR + idx;
}

// the log of replica idx = g * R + r outside the step kernel: lane
// (g % GPW) * R + r of the block of step-kernel wave g / GPW
__device__ __forceinline__ LogView log_of(const DevParams& p, int64_t idx) {
    const int64_t g = idx / p.R;
    const int gpw = 64 / p.R;
    const int64_t w = g / gpw;
    const int lane = (int)(g - w * gpw) * p.R + (int)(idx - g * p.R);
    return LogView{p.log + (w * 64 + lane) * (int64_t)p.nslots, (uint32_t)p.nslots, p.wmask, p.cap, p.W};
}
}  // namespace

struct raft_engine {
    raft_params p;
    DevParams dp;
    int device;
    hipStream_t stream;
    void* base;
    size_t bytes;
    uint64_t t;
    int K;                      // steps per launch
    int nwaves;                 // chunks: ceil(G / (64 / R)), one wave's groups (and log block) each
    int nblocks;                // step-kernel workgroups of the one-chunk-per-wave schedule: ceil(nwaves / STEP_WAVES)
    int ncu;                    // compute units of the device
    // the launch schedule (raft_params.schedule, schedule_workgroups; step_kernel)
    int schedule, sched_wg;
    bool part_only;             // the workload's kernel is partitions-only (auto_subranges)
    raft_kernel_info last;      // the last step launch (raft_engine_kernel_info)
    static constexpr int OCC_SLOTS = 4;
    const void* occ_kern[OCC_SLOTS];   // workgroups per CU of occ_kern at occ_lds bytes of LDS (cached)
    size_t occ_lds[OCC_SLOTS];
    int occ_wg[OCC_SLOTS];
    uint32_t occ_next;
    uint32_t* partials;         // [K][NCW][nblocks] packed per-workgroup counter partials (buffer 0)
    uint32_t* partials2;        // buffer 1: launches alternate between the two when nsub > 1
    uint32_t* hpart;            // [K][NCW][workgroups] partials of a launch run as epochs (grow-only,
    size_t hpart_bytes;         // raft_engine_step_async)
    // launch sub-ranges (raft_engine_step_async): the step workgroups split
    // into nsub contiguous ranges, each launched on its own stream, so one
    // range's last waves overlap another's next launch instead of leaving
    // the chip part-empty at every launch boundary
    int nsub;
    int sub_b0[RAFT_MAX_SUBRANGES + 1];       // workgroup boundaries
    hipStream_t sub_stream[RAFT_MAX_SUBRANGES];
    hipEvent_t ev_fork, ev_sub_done[RAFT_MAX_SUBRANGES], ev_red_done[2];
    hipEvent_t ev_wait;         // raft_engine_wait_stream
    uint64_t launches_issued;   // step launches (all sub-ranges) so far: the partials buffer parity
    bool fork_needed;           // the engine stream holds work the sub-range streams have not waited for
    // batch path staging, grow-only: device scratch (keys, sort), device
    // copies of host batches, pinned host staging, pinned status flags
    char* bst;
    size_t bst_bytes;
    bool bst_dirty;             // the bucketed path's device status words may be nonzero (a batch failed mid-way)
    char* bio;
    size_t bio_bytes;
    char* hst;
    size_t hst_bytes;
    unsigned int* bflags_host;
    int batch_path;             // RAFT_BATCH_PATH_* (raft_engine_set_batch_path)
    char* aux;                  // device staging of the state / log / digest accessors, grow-only
    size_t aux_bytes;
    int64_t* counters_dev;      // [K][STRIDE] scratch
    unsigned long long* accum;  // [K * NC] counter accumulators: sum + chunks done << 48 (zero between launches)
    // step-kernel event timing
    bool cache_valid;           // log-tail cache (F_T1, F_T2, F_C1) matches state + logs: the step kernel and the
                                // handler batches keep it; write_state / write_log make it stale
    bool iso_written;           // write_state stored a nonzero isolation word (step_fn: NET_ISO kernels)
    bool timing;
    std::vector<hipEvent_t> ev;  // pool, pairs (one per sub-range launch)
    size_t ev_used;
    int64_t timed_launches;     // K-step launches of the whole grid timed since the last kernel_time()
};
