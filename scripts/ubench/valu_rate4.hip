// Microbenchmark, part 4 (round 6): the issue cost per instruction CLASS of
// the step kernel's VALU mix, on 24 resident waves per CU (6 per SIMD, the
// step kernel runs 7), so DESIGN.md §4.6 can weight its per-phase budget by
// cycles instead of instruction counts.  Part 3 (valu_rate3.hip) wrote every
// compare into ONE SGPR pair and read every select mask from one; here the
// e64 forms also rotate over 8 SGPR pairs (no write-after-write chain), and
// the VCC forms (e32: v_cmp_*_e32 writes VCC, v_cndmask_b32_e32 reads it) are
// measured beside them, with the min / max / med3 / bfi / bitop forms that
// could replace compare + select sequences, and SALU beside VALU.
// Cycles come from each workgroup's own s_memtime stamps (the launch's
// overhead is not in them); experiments only.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CH8(OP) OP(0, 1) OP(1, 2) OP(2, 3) OP(3, 4) OP(4, 5) OP(5, 6) OP(6, 7) OP(7, 0)
// one SGPR pair per chain position: s[8+2i : 9+2i]
template <int K>
__global__ __launch_bounds__(256) void kern(unsigned* out, unsigned long long* clk, int iters) {
    unsigned b[8];
    for (int i = 0; i < 8; ++i) b[i] = threadIdx.x * (2 * i + 3);
    unsigned long long m0 = __ballot(threadIdx.x & 1), m1 = __ballot(threadIdx.x & 2);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#define CMP64_1(i, j) asm volatile("v_cmp_lt_i32_e64 s[6:7], %0, %1" : : "v"(b[i]), "v"(b[j]) : "s6", "s7");
#define SPAIR0 "s[8:9]"
#define SPAIR1 "s[10:11]"
#define SPAIR2 "s[12:13]"
#define SPAIR3 "s[14:15]"
#define SPAIR4 "s[16:17]"
#define SPAIR5 "s[18:19]"
#define SPAIR6 "s[20:21]"
#define SPAIR7 "s[22:23]"
#define CMP64_8(i, j) asm volatile("v_cmp_lt_i32_e64 " SPAIR##i ", %0, %1" : : "v"(b[i]), "v"(b[j]) : "s8", "s9", "s10", "s11", "s12", "s13", "s14", "s15", "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23");
#define CMP32(i, j) asm volatile("v_cmp_lt_i32_e32 vcc, %0, %1" : : "v"(b[i]), "v"(b[j]) : "vcc");
#define CND64(i, j) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(b[i]) : "v"(b[j]), "s"(i & 1 ? m0 : m1));
#define CND32(i, j) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(b[i]) : "v"(b[j]));   /* vcc: whatever it holds (timing only) */
#define ADD(i, j) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define ADD64(i, j) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define MIN(i, j) asm volatile("v_min_i32_e32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define MED3(i, j) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
#define BFI(i, j) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
#define AND(i, j) asm volatile("v_and_b32_e32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define OR3(i, j) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(b[j]), "v"(b[(j + 1) & 7]));
#define ADDC(i, j) asm volatile("v_addc_co_u32_e64 %0, s[4:5], 0, %0, %1" : "+v"(b[i]) : "s"(i & 1 ? m0 : m1) : "s4", "s5");
#define SUBBREV(i, j) asm volatile("v_subbrev_co_u32_e64 %0, s[4:5], 0, %0, %1" : "+v"(b[i]) : "s"(i & 1 ? m0 : m1) : "s4", "s5");
#define CMPX(i, j) asm volatile("v_cmp_lt_u32_e64 " SPAIR##i ", %0, %1" : : "v"(b[i]), "v"(b[j]) : "s8", "s9", "s10", "s11", "s12", "s13", "s14", "s15", "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23");
#define LSH(i, j) asm volatile("v_lshlrev_b32_e32 %0, 1, %0" : "+v"(b[i]));
#define BFE(i, j) asm volatile("v_bfe_u32 %0, %0, %1, 1" : "+v"(b[i]) : "v"(b[j]));
#define BCNT(i, j) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define BPERM(i, j) asm volatile("ds_bpermute_b32 %0, %1, %0" : "+v"(b[i]) : "v"(b[j]));
#define SAND(i, j) asm volatile("s_and_b64 s[4:5], s[4:5], %0" : : "s"(i & 1 ? m0 : m1) : "s4", "s5", "scc");
#define SBCNT(i, j) asm volatile("s_bcnt1_i32_b64 s6, %0\n s_add_u32 s7, s7, s6" : : "s"(i & 1 ? m0 : m1) : "s6", "s7", "scc");
#define WAITL asm volatile("s_waitcnt lgkmcnt(0)");
        if constexpr (K == 0) { CH8(ADD) }
        if constexpr (K == 1) { CH8(ADD64) }
        if constexpr (K == 2) { CH8(CMP64_1) }
        if constexpr (K == 3) { CH8(CMP64_8) }
        if constexpr (K == 4) { CH8(CMP32) }
        if constexpr (K == 5) { CH8(CND64) }
        if constexpr (K == 6) { CH8(CND32) }
        if constexpr (K == 7) { CH8(MIN) }
        if constexpr (K == 8) { CH8(MED3) }
        if constexpr (K == 9) { CH8(BFI) }
        if constexpr (K == 10) { CH8(AND) }
        if constexpr (K == 11) { CH8(OR3) }
        if constexpr (K == 12) { CH8(ADDC) }
        if constexpr (K == 13) { CH8(SUBBREV) }
        if constexpr (K == 14) { CH8(LSH) }
        if constexpr (K == 15) { CH8(BFE) }
        if constexpr (K == 16) { CH8(BCNT) }
        if constexpr (K == 17) { CH8(CMP64_8) CH8(CND64) }      // the kernel's compare + select pair, e64
        if constexpr (K == 18) { CH8(CMP32) CH8(CND32) }        // the same through VCC
        if constexpr (K == 19) { CH8(ADD) CH8(SAND) }           // VALU beside SALU: is the SALU free?
        if constexpr (K == 20) { CH8(ADD) CH8(SBCNT) }          // VALU beside the counter adds (2 SALU each)
        if constexpr (K == 21) { CH8(SAND) }                    // SALU alone
        if constexpr (K == 22) { CH8(CMPX) CH8(SAND) CH8(CND64) }   // mask, SALU combine, select
        if constexpr (K == 23) { CH8(BPERM) WAITL }             // lane broadcasts (LDS crossbar)
        if constexpr (K == 24) { CH8(ADD) CH8(BPERM) WAITL }    // broadcasts beside VALU
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s += b[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

static const char* NAMES[] = {
    "v_add_u32_e32", "v_add_u32_e64", "v_cmp_e64 (1 sgpr pair)", "v_cmp_e64 (8 sgpr pairs)", "v_cmp_e32 (vcc)",
    "v_cndmask_b32_e64", "v_cndmask_b32_e32 (vcc)", "v_min_i32_e32", "v_med3_i32", "v_bfi_b32", "v_and_b32_e32",
    "v_or3_b32", "v_addc_co_u32_e64 (inc_if)", "v_subbrev_co_u32_e64 (dec_if)", "v_lshlrev_b32_e32", "v_bfe_u32",
    "v_bcnt_u32_b32", "cmp_e64+cndmask_e64 (pair)", "cmp_e32+cndmask_e32 (pair)", "add + s_and_b64 (VALU/SALU)",
    "add + s_bcnt1+s_add", "s_and_b64 alone", "cmp_e64 + s_and + cndmask", "ds_bpermute_b32 (+wait)",
    "add + ds_bpermute"};
// instructions per iteration, and how many of them are VALU
static const int PER_IT[] = {8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 16, 16, 16, 24, 8, 24, 8, 16};
static const int VALU_IT[] = {8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 16, 16, 8, 8, 0, 16, 0, 8};

template <int K>
static void run(unsigned* out, unsigned long long* clk, int blocks, int iters) {
    kern<K><<<blocks, 256>>>(out, clk, 16);
    kern<K><<<blocks, 256>>>(out, clk, iters);
    (void)hipDeviceSynchronize();
    static unsigned long long c[256 * 8];
    (void)hipMemcpy(c, clk, (size_t)blocks * 8, hipMemcpyDeviceToHost);
    double cyc = 0;
    for (int b = 0; b < blocks; ++b) cyc += (double)c[b];
    cyc /= blocks;                                  // cycles of one workgroup's loop (all run concurrently)
    const double per_simd = 6.0 * iters;            // 6 waves per SIMD x iterations
    printf("%-32s %7.2f cycles/instr/SIMD  %7.2f cycles/VALU/SIMD\n", NAMES[K], cyc / (per_simd * PER_IT[K]),
           VALU_IT[K] ? cyc / (per_simd * VALU_IT[K]) : 0.0);
}

template <int... Ks>
static void run_all(unsigned* out, unsigned long long* clk, int blocks, int iters, std::integer_sequence<int, Ks...>) {
    (run<Ks>(out, clk, blocks, iters), ...);
}

int main() {
    unsigned* out;
    unsigned long long* clk;
    const int blocks = 256 * 6, iters = 4096;     // 6 workgroups of 4 waves per CU: 6 waves per SIMD
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    if (hipMalloc(&clk, (size_t)blocks * 8) != hipSuccess) return 1;
    for (int rep = 0; rep < 2; ++rep) {
        printf("-- rep %d\n", rep);
        run_all(out, clk, blocks, iters, std::make_integer_sequence<int, 25>{});
    }
    return 0;
}
