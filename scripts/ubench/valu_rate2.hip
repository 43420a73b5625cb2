// Microbenchmark, part 2: more VALU opcodes (see valu_rate.hip). Experiments only.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int K> __global__ void kern(unsigned* out, int iters) {
    unsigned b0 = threadIdx.x, b1 = b0 * 3, b2 = b0 * 5, b3 = b0 * 7, b4 = b0 * 11, b5 = b0 * 13, b6 = b0 * 17, b7 = b0 * 19;
    unsigned long long a0 = b0, a1 = b1, a2 = b2, a3 = b3;
    for (int i = 0; i < iters; ++i) {
        if constexpr (K == 0) asm volatile("v_xor_b32 %0, %0, %1\nv_xor_b32 %1, %1, %2\nv_xor_b32 %2, %2, %3\nv_xor_b32 %3, %3, %4\nv_xor_b32 %4, %4, %5\nv_xor_b32 %5, %5, %6\nv_xor_b32 %6, %6, %7\nv_xor_b32 %7, %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 1) asm volatile("v_and_b32 %0, %0, %1\nv_and_b32 %1, %1, %2\nv_and_b32 %2, %2, %3\nv_and_b32 %3, %3, %4\nv_and_b32 %4, %4, %5\nv_and_b32 %5, %5, %6\nv_and_b32 %6, %6, %7\nv_and_b32 %7, %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 2) asm volatile("v_or_b32 %0, %0, %1\nv_or_b32 %1, %1, %2\nv_or_b32 %2, %2, %3\nv_or_b32 %3, %3, %4\nv_or_b32 %4, %4, %5\nv_or_b32 %5, %5, %6\nv_or_b32 %6, %6, %7\nv_or_b32 %7, %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 3) asm volatile("v_add_u32 %0, %0, %1\nv_add_u32 %1, %1, %2\nv_add_u32 %2, %2, %3\nv_add_u32 %3, %3, %4\nv_add_u32 %4, %4, %5\nv_add_u32 %5, %5, %6\nv_add_u32 %6, %6, %7\nv_add_u32 %7, %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 4) asm volatile("v_sub_u32 %0, %0, %1\nv_sub_u32 %1, %1, %2\nv_sub_u32 %2, %2, %3\nv_sub_u32 %3, %3, %4\nv_sub_u32 %4, %4, %5\nv_sub_u32 %5, %5, %6\nv_sub_u32 %6, %6, %7\nv_sub_u32 %7, %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 5) asm volatile("v_lshlrev_b32 %0, 1, %0\nv_lshlrev_b32 %1, 1, %1\nv_lshlrev_b32 %2, 1, %2\nv_lshlrev_b32 %3, 1, %3\nv_lshlrev_b32 %4, 1, %4\nv_lshlrev_b32 %5, 1, %5\nv_lshlrev_b32 %6, 1, %6\nv_lshlrev_b32 %7, 1, %7" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 6) asm volatile("v_lshrrev_b32 %0, %1, %0\nv_lshrrev_b32 %1, %2, %1\nv_lshrrev_b32 %2, %3, %2\nv_lshrrev_b32 %3, %4, %3\nv_lshrrev_b32 %4, %5, %4\nv_lshrrev_b32 %5, %6, %5\nv_lshrrev_b32 %6, %7, %6\nv_lshrrev_b32 %7, %0, %7" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 7) asm volatile("v_mov_b32 %0, %1\nv_mov_b32 %1, %2\nv_mov_b32 %2, %3\nv_mov_b32 %3, %4\nv_mov_b32 %4, %5\nv_mov_b32 %5, %6\nv_mov_b32 %6, %7\nv_mov_b32 %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 8) asm volatile("s_mov_b32 s2, 0x55555555\ns_mov_b32 s3, 0x55555555\nv_cndmask_b32 %0, %0, %1, s[2:3]\nv_cndmask_b32 %1, %1, %2, s[2:3]\nv_cndmask_b32 %2, %2, %3, s[2:3]\nv_cndmask_b32 %3, %3, %4, s[2:3]\nv_cndmask_b32 %4, %4, %5, s[2:3]\nv_cndmask_b32 %5, %5, %6, s[2:3]\nv_cndmask_b32 %6, %6, %7, s[2:3]\nv_cndmask_b32 %7, %7, %0, s[2:3]" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 9) asm volatile("v_cmp_gt_i32 s[4:5], %0, %1\nv_cmp_gt_i32 s[4:5], %1, %2\nv_cmp_gt_i32 s[4:5], %2, %3\nv_cmp_gt_i32 s[4:5], %3, %4\nv_cmp_gt_i32 s[4:5], %4, %5\nv_cmp_gt_i32 s[4:5], %5, %6\nv_cmp_gt_i32 s[4:5], %6, %7\nv_cmp_gt_i32 s[4:5], %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 10) asm volatile("v_bfe_u32 %0, %0, 3, 5\nv_bfe_u32 %1, %1, 3, 5\nv_bfe_u32 %2, %2, 3, 5\nv_bfe_u32 %3, %3, 3, 5\nv_bfe_u32 %4, %4, 3, 5\nv_bfe_u32 %5, %5, 3, 5\nv_bfe_u32 %6, %6, 3, 5\nv_bfe_u32 %7, %7, 3, 5" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 11) asm volatile("v_min_i32 %0, %0, %1\nv_min_i32 %1, %1, %2\nv_min_i32 %2, %2, %3\nv_min_i32 %3, %3, %4\nv_min_i32 %4, %4, %5\nv_min_i32 %5, %5, %6\nv_min_i32 %6, %6, %7\nv_min_i32 %7, %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 12) asm volatile("v_add3_u32 %0, %0, %1, 7\nv_add3_u32 %1, %1, %2, 7\nv_add3_u32 %2, %2, %3, 7\nv_add3_u32 %3, %3, %4, 7\nv_add3_u32 %4, %4, %5, 7\nv_add3_u32 %5, %5, %6, 7\nv_add3_u32 %6, %6, %7, 7\nv_add3_u32 %7, %7, %0, 7" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 13) asm volatile("v_lshl_add_u32 %0, %0, 2, %1\nv_lshl_add_u32 %1, %1, 2, %2\nv_lshl_add_u32 %2, %2, 2, %3\nv_lshl_add_u32 %3, %3, 2, %4\nv_lshl_add_u32 %4, %4, 2, %5\nv_lshl_add_u32 %5, %5, 2, %6\nv_lshl_add_u32 %6, %6, 2, %7\nv_lshl_add_u32 %7, %7, 2, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 14) asm volatile("v_mul_u32_u24 %0, %0, %1\nv_mul_u32_u24 %1, %1, %2\nv_mul_u32_u24 %2, %2, %3\nv_mul_u32_u24 %3, %3, %4\nv_mul_u32_u24 %4, %4, %5\nv_mul_u32_u24 %5, %5, %6\nv_mul_u32_u24 %6, %6, %7\nv_mul_u32_u24 %7, %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 15) asm volatile("s_mov_b32 s2, 0x55555555\ns_mov_b32 s3, 0x55555555\nv_addc_co_u32 %0, s[4:5], %0, 0, s[2:3]\nv_addc_co_u32 %1, s[4:5], %1, 0, s[2:3]\nv_addc_co_u32 %2, s[4:5], %2, 0, s[2:3]\nv_addc_co_u32 %3, s[4:5], %3, 0, s[2:3]\nv_addc_co_u32 %4, s[4:5], %4, 0, s[2:3]\nv_addc_co_u32 %5, s[4:5], %5, 0, s[2:3]\nv_addc_co_u32 %6, s[4:5], %6, 0, s[2:3]\nv_addc_co_u32 %7, s[4:5], %7, 0, s[2:3]" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 16) asm volatile("v_readlane_b32 s6, %0, 5\nv_readlane_b32 s6, %1, 5\nv_readlane_b32 s6, %2, 5\nv_readlane_b32 s6, %3, 5\nv_readlane_b32 s6, %4, 5\nv_readlane_b32 s6, %5, 5\nv_readlane_b32 s6, %6, 5\nv_readlane_b32 s6, %7, 5" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 17) asm volatile("v_writelane_b32 %0, s7, 5\nv_writelane_b32 %1, s7, 5\nv_writelane_b32 %2, s7, 5\nv_writelane_b32 %3, s7, 5\nv_writelane_b32 %4, s7, 5\nv_writelane_b32 %5, s7, 5\nv_writelane_b32 %6, s7, 5\nv_writelane_b32 %7, s7, 5" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 18) asm volatile("v_lshl_add_u64 %0, %0, 3, %0\nv_lshl_add_u64 %1, %1, 3, %1\nv_lshl_add_u64 %2, %2, 3, %2\nv_lshl_add_u64 %3, %3, 3, %3\nv_lshl_add_u64 %0, %0, 3, %0\nv_lshl_add_u64 %1, %1, 3, %1\nv_lshl_add_u64 %2, %2, 3, %2\nv_lshl_add_u64 %3, %3, 3, %3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) :: "s2", "s3", "s4", "s5", "s6", "s7");
        if constexpr (K == 19) asm volatile("v_pk_add_u16 %0, %0, %1\nv_pk_add_u16 %1, %1, %2\nv_pk_add_u16 %2, %2, %3\nv_pk_add_u16 %3, %3, %4\nv_pk_add_u16 %4, %4, %5\nv_pk_add_u16 %5, %5, %6\nv_pk_add_u16 %6, %6, %7\nv_pk_add_u16 %7, %7, %0" : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7) :: "s2", "s3", "s4", "s5", "s6", "s7");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7 + (unsigned)(a0 + a1 + a2 + a3);
}
template <int K> static float run(unsigned* out, int blocks, int threads, int iters) {
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); (void)hipEventRecord(e0);
    kern<K><<<blocks, threads>>>(out, iters); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms = 0.f; (void)hipEventElapsedTime(&ms, e0, e1); return ms; }
int main() {
    unsigned* out; const int blocks = 256 * 24, threads = 256, iters = 2048;
    if (hipMalloc(&out, (size_t)blocks * threads * 4) != hipSuccess) return 1;
    const double instr = (double)blocks * threads / 64 * iters * 8;
    for (int rep = 0; rep < 2; ++rep) {
        { float ms = run<0>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_xor_b32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<1>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_and_b32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<2>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_or_b32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<3>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_add_u32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<4>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_sub_u32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<5>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_lshlrev_b32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<6>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_lshrrev_b32v", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<7>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_mov_b32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<8>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_cndmask_b32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<9>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_cmp_gt_i32_e64", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<10>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_bfe_u32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<11>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_min_i32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<12>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_add3_u32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<13>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_lshl_add_u32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<14>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_mul_u32_u24", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<15>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_addc_co_u32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<16>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_readlane_b32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<17>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_writelane_b32", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<18>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_lshl_add_u64", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
        { float ms = run<19>(out, blocks, threads, iters); printf("%-18s %8.3f ms %6.2f cycles/instr/SIMD\n", "v_pk_add_u16", ms, ms * 1e-3 * 2.4e9 * 1024 / instr); }
    }
    return 0;
}
