// Microbenchmark (experiments only): does the gfx950 L2 merge successive
// 8-byte stores to one line, as the step kernel's log appends are (one 8-B
// entry per replica every few steps, consecutive slots of the replica's row)?
// Each lane appends N entries of 8 B to consecutive slots of its own row, with
// `spin` dependent VALU operations between appends (the other waves' traffic
// interleaves).  Run under `rocprofv3 --pmc WRITE_SIZE` (and FETCH_SIZE in a
// separate pass): if the L2 merged the stores, a kernel would write about
// N * 8 B per lane; one sector per store is N * 32 B.  The variants set the
// store's cache-policy bits (gfx950 `sc0`, `sc1`, `nt`) with inline asm.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int BITS>
__device__ __forceinline__ void store8(uint2* p, uint2 v) {
    if constexpr (BITS == 0) {
        *p = v;
    } else if constexpr (BITS == 1) {
        asm volatile("global_store_dwordx2 %0, %1, off nt" :: "v"(p), "v"(v) : "memory");
    } else if constexpr (BITS == 2) {
        asm volatile("global_store_dwordx2 %0, %1, off sc0" :: "v"(p), "v"(v) : "memory");
    } else if constexpr (BITS == 3) {
        asm volatile("global_store_dwordx2 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
    } else {
        asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" :: "v"(p), "v"(v) : "memory");
    }
}

// rows: [waves][64][row] uint2 (the step kernel's log layout: lane-major rows)
template <int BITS>
__global__ __launch_bounds__(256) void append_rows(uint2* rows, int row, int n, int spin) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    uint2* r = rows + (wave * 64 + lane) * row;
    uint32_t x = threadIdx.x;
    for (int i = 0; i < n; ++i) {
        for (int k = 0; k < spin; ++k) asm volatile("v_add_u32 %0, %0, 1" : "+v"(x));
        store8<BITS>(r + i, make_uint2(x, (uint32_t)i));
    }
}

int main() {
    const int blocks = 20834, row = 256, n = 64;          // 83,336 waves x 64 lanes, like the step kernel
    const size_t bytes = (size_t)blocks * 4 * 64 * row * 8;
    uint2* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) { printf("hipMalloc failed\n"); return 1; }
    hipMemset(d, 0, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[5] = {"default", "nt", "sc0", "sc1", "sc0_sc1"};
    for (int spin : {0, 256}) {
        for (int v = 0; v < 5; ++v) {
            hipEventRecord(a, 0);
            switch (v) {
                case 0: append_rows<0><<<blocks, 256>>>(d, row, n, spin); break;
                case 1: append_rows<1><<<blocks, 256>>>(d, row, n, spin); break;
                case 2: append_rows<2><<<blocks, 256>>>(d, row, n, spin); break;
                case 3: append_rows<3><<<blocks, 256>>>(d, row, n, spin); break;
                default: append_rows<4><<<blocks, 256>>>(d, row, n, spin); break;
            }
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0.f;
            hipEventElapsedTime(&ms, a, b);
            printf("%-8s spin=%3d  %.3f ms  stored %.1f MB\n", names[v], spin, ms,
                   (double)blocks * 256 * n * 8 / 1e6);
        }
    }
    hipFree(d);
    return 0;
}
