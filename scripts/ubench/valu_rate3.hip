// Microbenchmark, part 3: the issue cost of the step kernel's Philox
// instructions (v_mad_u64_u32, v_bitop3_b32) and of the 32-bit multiplies
// that could replace them, on 24 resident waves per CU (6 per SIMD).
// Experiments only; cycles at the measured clock come from the kernel's own
// s_memtime / s_memrealtime stamps.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CH8(OP) OP(0, 1) OP(1, 2) OP(2, 3) OP(3, 4) OP(4, 5) OP(5, 6) OP(6, 7) OP(7, 0)
template <int K>
__global__ __launch_bounds__(256) void kern(unsigned* out, unsigned long long* clk, int iters) {
    unsigned b[8];
    unsigned long long a[8];
    for (int i = 0; i < 8; ++i) { b[i] = threadIdx.x * (2 * i + 3); a[i] = b[i]; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#define MAD(i, j) asm volatile("v_mad_u64_u32 %0, s[4:5], %1, %2, 0" : "=v"(a[i]) : "v"(b[i]), "v"(b[j]) : "s4", "s5"); b[i] = (unsigned)(a[i] >> 32);
#define MULHI(i, j) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define MULLO(i, j) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define BOP3(i, j) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(b[i]) : "v"(b[j]));
#define XOR3(i, j) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define CMP(i, j) asm volatile("v_cmp_lt_i32_e64 s[6:7], %0, %1" : : "v"(b[i]), "v"(b[j]) : "s6", "s7");
#define CND(i, j) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[8:9]" : "+v"(b[i]) : "v"(b[j]) : "s8", "s9");
#define ADD(i, j) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define MU24(i, j) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define MHU24(i, j) asm volatile("v_mul_hi_u32_u24_e32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define BPERM(i, j) asm volatile("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)" : "+v"(b[i]) : "v"(b[j]));
        if constexpr (K == 0) { CH8(MAD) }
        if constexpr (K == 1) { CH8(MULHI) }
        if constexpr (K == 2) { CH8(MULLO) }
        if constexpr (K == 3) { CH8(BOP3) }
        if constexpr (K == 4) { CH8(XOR3) }
        if constexpr (K == 5) { CH8(CMP) }
        if constexpr (K == 6) { CH8(CND) }
        if constexpr (K == 7) { CH8(ADD) }
        if constexpr (K == 8) { CH8(MU24) }
        if constexpr (K == 9) { CH8(MHU24) }
        if constexpr (K == 10) { CH8(MAD) CH8(BOP3) }          // a Philox-like mix: 1 mad : 1 bitop3
        if constexpr (K == 11) { CH8(CMP) CH8(CND) }           // compare + select
        if constexpr (K == 12) { CH8(ADD) CH8(CND) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s += b[i] + (unsigned)a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

static const char* NAMES[] = {"v_mad_u64_u32", "v_mul_hi_u32", "v_mul_lo_u32", "v_bitop3_b32", "v_xor_b32_e32",
                              "v_cmp_lt_i32_e64", "v_cndmask_b32_e64", "v_add_u32_e32", "v_mul_u32_u24",
                              "v_mul_hi_u32_u24", "mad+bitop3 (pair)", "cmp+cndmask (pair)", "add+cndmask (pair)"};
static const int PER_IT[] = {8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 16, 16, 16};

template <int K>
static void run(unsigned* out, unsigned long long* clk, int blocks, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    kern<K><<<blocks, 256>>>(out, clk, 16);
    (void)hipEventRecord(e0);
    kern<K><<<blocks, 256>>>(out, clk, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;   // s_memtime ticks / s_memrealtime (100 MHz)
    const double instr = (double)blocks * 4 * iters * PER_IT[K];     // wave-instructions
    printf("%-22s %8.3f ms  clock %.2f GHz  %6.2f cycles/instr/SIMD\n", NAMES[K], ms, ghz,
           ms * 1e-3 * ghz * 1e9 * 1024 / instr);
}

int main() {
    unsigned* out;
    unsigned long long* clk;
    const int blocks = 256 * 6, iters = 4096;     // 6 workgroups of 4 waves per CU: 6 waves per SIMD
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    if (hipMalloc(&clk, (size_t)blocks * 16) != hipSuccess) return 1;
    for (int rep = 0; rep < 2; ++rep) {
        run<0>(out, clk, blocks, iters); run<1>(out, clk, blocks, iters); run<2>(out, clk, blocks, iters);
        run<3>(out, clk, blocks, iters); run<4>(out, clk, blocks, iters); run<5>(out, clk, blocks, iters);
        run<6>(out, clk, blocks, iters); run<7>(out, clk, blocks, iters); run<8>(out, clk, blocks, iters);
        run<9>(out, clk, blocks, iters); run<10>(out, clk, blocks, iters); run<11>(out, clk, blocks, iters);
        run<12>(out, clk, blocks, iters);
    }
    return 0;
}
