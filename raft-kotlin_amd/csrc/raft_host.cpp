// raft_host.cpp — host-only utilities of the C-ABI (include/raft_engine.h):
// page-locked memory for the handler batches' arrays.  raft_vote_batch /
// raft_append_batch move arrays that live in it by direct DMA instead of
// copying them through the engine's pinned staging (raft_engine.hip
// run_batch).  Kept out of raft_engine.hip: no kernel or launch code here.
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>

#include "raft_engine.h"

int raft_internal_fail(int code, const std::string& msg);   // raft_engine.hip: sets raft_last_error()

extern "C" {

void* raft_host_alloc(int64_t bytes) {
    if (bytes <= 0) {
        raft_internal_fail(RAFT_EINVAL, "raft_host_alloc: bytes must be positive");
        return nullptr;
    }
    void* p = nullptr;
    const hipError_t err = hipHostMalloc(&p, (size_t)bytes, hipHostMallocDefault);
    if (err != hipSuccess) {
        raft_internal_fail(RAFT_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(err));
        return nullptr;
    }
    return p;
}

int raft_host_free(void* p) {
    if (!p) return RAFT_OK;
    const hipError_t err = hipHostFree(p);
    if (err != hipSuccess) return raft_internal_fail(RAFT_EDEVICE, std::string("hipHostFree: ") + hipGetErrorString(err));
    return RAFT_OK;
}

}  // extern "C"
