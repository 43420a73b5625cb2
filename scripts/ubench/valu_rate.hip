// Microbenchmark: issue cost of a few VALU opcodes on gfx950 (8 independent
// chains per lane, full occupancy).  Experiments only; prints cycles per
// wave-instruction per SIMD assuming 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__global__ void kern(unsigned long long* out, int iters) {
    unsigned long long a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;
    unsigned long long a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
    unsigned b0 = threadIdx.x, b1 = b0 * 3, b2 = b0 * 5, b3 = b0 * 7, b4 = b0 * 11, b5 = b0 * 13, b6 = b0 * 17,
             b7 = b0 * 19;
    for (int i = 0; i < iters; ++i) {
        if constexpr (K == 0) {
            asm volatile(
                "v_lshrrev_b64 %0, 1, %0\n v_lshrrev_b64 %1, 1, %1\n v_lshrrev_b64 %2, 1, %2\n v_lshrrev_b64 %3, 1, %3\n"
                "v_lshrrev_b64 %4, 1, %4\n v_lshrrev_b64 %5, 1, %5\n v_lshrrev_b64 %6, 1, %6\n v_lshrrev_b64 %7, 1, %7\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        } else if constexpr (K == 1) {
            asm volatile(
                "v_lshrrev_b32 %0, 1, %0\n v_lshrrev_b32 %1, 1, %1\n v_lshrrev_b32 %2, 1, %2\n v_lshrrev_b32 %3, 1, %3\n"
                "v_lshrrev_b32 %4, 1, %4\n v_lshrrev_b32 %5, 1, %5\n v_lshrrev_b32 %6, 1, %6\n v_lshrrev_b32 %7, 1, %7\n"
                : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7));
        } else if constexpr (K == 2) {
            asm volatile(
                "v_mad_u64_u32 %0, s[0:1], %8, %8, %0\n v_mad_u64_u32 %1, s[0:1], %9, %9, %1\n"
                "v_mad_u64_u32 %2, s[0:1], %10, %10, %2\n v_mad_u64_u32 %3, s[0:1], %11, %11, %3\n"
                "v_mad_u64_u32 %4, s[0:1], %12, %12, %4\n v_mad_u64_u32 %5, s[0:1], %13, %13, %5\n"
                "v_mad_u64_u32 %6, s[0:1], %14, %14, %6\n v_mad_u64_u32 %7, s[0:1], %15, %15, %7\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(b0), "v"(b1), "v"(b2), "v"(b3), "v"(b4), "v"(b5), "v"(b6), "v"(b7)
                : "s0", "s1");
        } else if constexpr (K == 3) {
            asm volatile(
                "v_bcnt_u32_b32 %0, %0, 1\n v_bcnt_u32_b32 %1, %1, 1\n v_bcnt_u32_b32 %2, %2, 1\n v_bcnt_u32_b32 %3, %3, 1\n"
                "v_bcnt_u32_b32 %4, %4, 1\n v_bcnt_u32_b32 %5, %5, 1\n v_bcnt_u32_b32 %6, %6, 1\n v_bcnt_u32_b32 %7, %7, 1\n"
                : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7));
        } else if constexpr (K == 4) {
            asm volatile(
                "v_alignbit_b32 %0, %1, %0, 3\n v_alignbit_b32 %1, %2, %1, 3\n v_alignbit_b32 %2, %3, %2, 3\n"
                "v_alignbit_b32 %3, %4, %3, 3\n v_alignbit_b32 %4, %5, %4, 3\n v_alignbit_b32 %5, %6, %5, 3\n"
                "v_alignbit_b32 %6, %7, %6, 3\n v_alignbit_b32 %7, %0, %7, 3\n"
                : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7));
        } else if constexpr (K == 5) {
            asm volatile(
                "v_mul_lo_u32 %0, %0, %0\n v_mul_lo_u32 %1, %1, %1\n v_mul_lo_u32 %2, %2, %2\n v_mul_lo_u32 %3, %3, %3\n"
                "v_mul_lo_u32 %4, %4, %4\n v_mul_lo_u32 %5, %5, %5\n v_mul_lo_u32 %6, %6, %6\n v_mul_lo_u32 %7, %7, %7\n"
                : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7));
        } else if constexpr (K == 6) {
            asm volatile(
                "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n v_bitop3_b32 %1, %1, %2, %3 bitop3:0x96\n"
                "v_bitop3_b32 %2, %2, %3, %4 bitop3:0x96\n v_bitop3_b32 %3, %3, %4, %5 bitop3:0x96\n"
                "v_bitop3_b32 %4, %4, %5, %6 bitop3:0x96\n v_bitop3_b32 %5, %5, %6, %7 bitop3:0x96\n"
                "v_bitop3_b32 %6, %6, %7, %0 bitop3:0x96\n v_bitop3_b32 %7, %7, %0, %1 bitop3:0x96\n"
                : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0 + b1 + b2 + b3 + b4 +
                                                 b5 + b6 + b7;
}

template <int K>
static float run(unsigned long long* out, int blocks, int threads, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    kern<K><<<blocks, threads>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    unsigned long long* out;
    const int blocks = 256 * 24, threads = 256, iters = 2048;
    if (hipMalloc(&out, (size_t)blocks * threads * 8) != hipSuccess) return 1;
    const char* names[] = {"v_lshrrev_b64", "v_lshrrev_b32", "v_mad_u64_u32", "v_bcnt_u32_b32",
                           "v_alignbit_b32", "v_mul_lo_u32", "v_bitop3_b32"};
    for (int rep = 0; rep < 2; ++rep)
        for (int k = 0; k < 7; ++k) {
            float ms = 0.f;
            switch (k) {
                case 0: ms = run<0>(out, blocks, threads, iters); break;
                case 1: ms = run<1>(out, blocks, threads, iters); break;
                case 2: ms = run<2>(out, blocks, threads, iters); break;
                case 3: ms = run<3>(out, blocks, threads, iters); break;
                case 4: ms = run<4>(out, blocks, threads, iters); break;
                case 5: ms = run<5>(out, blocks, threads, iters); break;
                case 6: ms = run<6>(out, blocks, threads, iters); break;
            }
            const double waves = (double)blocks * threads / 64, instr = waves * iters * 8;
            printf("%-16s %8.3f ms  %6.2f cycles/instr/SIMD\n", names[k], ms, ms * 1e-3 * 2.4e9 * 1024 / instr);
        }
    return 0;
}
