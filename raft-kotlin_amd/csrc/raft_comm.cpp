// raft_comm.cpp — the engine's one collective: the RCCL all-reduce of the
// per-step counter rows over the GPUs of a sharded run (SURVEY.md §8(e);
// include/raft_engine.h raft_comm_*).  Groups never exchange anything, so the
// counters are the only cross-GPU data, and they never feed back into state.
//
// RCCL is loaded at the first raft_comm call (dlopen), not linked: one-GPU
// users never load it, and in a process that already holds an RCCL (torch's
// backend "nccl") dlopen returns that library, so there is one RCCL per
// process.  The all-reduce is enqueued on the engine's stream, after the
// step launches and counter reductions already there: nothing runs beside
// the RCCL kernel (a balanced step launch holds exactly the workgroups the
// GPU keeps resident), and the host cost is one library call.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "../../include/raft_engine.h"

int raft_internal_fail(int code, const std::string& msg);   // raft_engine.hip
extern "C" int raft_internal_device(const raft_engine* e);   // raft_engine.hip: the engine's GPU

static_assert(RAFT_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "raft_comm ids are ncclUniqueId");

namespace {

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    std::string err;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"librccl.so.1", "librccl.so"}) {
            r.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (r.h) break;
        }
        if (!r.h) {
            r.err = std::string("RCCL not found (dlopen librccl.so.1): ") + dlerror();
            return;
        }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.h, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
        r.all_reduce = (decltype(r.all_reduce))dlsym(r.h, "ncclAllReduce");
        r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
        if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.error_string) {
            r.err = "RCCL is missing an entry point (ncclGetUniqueId / ncclCommInitRank / ncclAllReduce)";
            r.h = nullptr;
        }
    });
    return r;
}

int rccl_fail(const Rccl& r, ncclResult_t rc, const char* what) {
    return raft_internal_fail(RAFT_EDEVICE, std::string(what) + ": " + r.error_string(rc));
}

}  // namespace

struct raft_comm {
    ncclComm_t comm;
    int nranks, rank, device;
};

extern "C" {

int raft_comm_get_unique_id(uint8_t id[RAFT_COMM_ID_BYTES]) {
    if (!id) return raft_internal_fail(RAFT_EINVAL, "null id");
    const Rccl& r = rccl();
    if (!r.h) return raft_internal_fail(RAFT_ENODEV, r.err);
    ncclUniqueId u;
    if (ncclResult_t rc = r.get_unique_id(&u)) return rccl_fail(r, rc, "ncclGetUniqueId");
    std::memcpy(id, u.internal, RAFT_COMM_ID_BYTES);
    return RAFT_OK;
}

int raft_comm_create(const uint8_t id[RAFT_COMM_ID_BYTES], int32_t nranks, int32_t rank, int device,
                     raft_comm** out) {
    if (!id || !out) return raft_internal_fail(RAFT_EINVAL, "null argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return raft_internal_fail(RAFT_EINVAL, "rank outside 0..nranks-1");
    const Rccl& r = rccl();
    if (!r.h) return raft_internal_fail(RAFT_ENODEV, r.err);
    // ncclCommInitRank binds the communicator to the current device: switch
    // to `device` for it and give the caller back its own current device
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) return raft_internal_fail(RAFT_EDEVICE, "hipGetDevice failed");
    if (hipSetDevice(device) != hipSuccess) return raft_internal_fail(RAFT_EINVAL, "bad device index");
    ncclUniqueId u;
    std::memcpy(u.internal, id, RAFT_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    const ncclResult_t rc = r.comm_init_rank(&c, nranks, u, rank);
    (void)hipSetDevice(prev);
    if (rc) return rccl_fail(r, rc, "ncclCommInitRank");
    *out = new raft_comm{c, nranks, rank, device};
    return RAFT_OK;
}

int raft_comm_destroy(raft_comm* c) {
    if (!c) return RAFT_OK;
    const Rccl& r = rccl();
    if (r.h) (void)r.comm_destroy(c->comm);
    delete c;
    return RAFT_OK;
}

int raft_engine_allreduce_counters(raft_engine* e, raft_comm* c, const int64_t* counters_dev, int64_t* out_dev,
                                   int32_t n_steps) {
    if (!e || !c || !counters_dev || !out_dev || n_steps < 0) return raft_internal_fail(RAFT_EINVAL, "bad argument");
    if (n_steps == 0) return RAFT_OK;
    const Rccl& r = rccl();
    if (!r.h) return raft_internal_fail(RAFT_ENODEV, r.err);    // (a communicator implies RCCL; defensive)
    // the all-reduce runs on the engine's stream: the communicator must be on the engine's GPU
    if (raft_internal_device(e) != c->device)
        return raft_internal_fail(RAFT_EINVAL, "the communicator and the engine are on different GPUs");
    if (hipSetDevice(c->device) != hipSuccess) return raft_internal_fail(RAFT_EDEVICE, "hipSetDevice failed");
    const size_t count = (size_t)n_steps * RAFT_COUNTER_STRIDE;
    if (ncclResult_t rc = r.all_reduce(counters_dev, out_dev, count, ncclInt64, ncclSum, c->comm,
                                       (hipStream_t)raft_engine_stream(e)))
        return rccl_fail(r, rc, "ncclAllReduce");
    return RAFT_OK;
}

}  // extern "C"
