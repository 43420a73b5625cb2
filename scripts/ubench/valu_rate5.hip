// Microbenchmark, part 5 (round 6): is the scalar ALU's issue free beside the
// vector ALU's?  Part 4 (valu_rate4.hip) mixed VALU with ONE dependent SALU
// chain per wave, which measures the SALU's dependent-issue latency, not its
// throughput.  Here every SALU stream is 8 independent chains (8 SGPR pairs)
// and the VALU streams 8 independent VGPR chains, at 6 waves per SIMD (and 1
// for the single-wave issue rates); VALU -> SALU mask hand-off (a compare's
// SGPR result consumed by s_and) and not-taken scalar branches, as the step
// kernel's predicated code has them.  Cycles from each workgroup's own
// s_memtime stamps; experiments only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>

#define CH8(OP) OP(0, 1) OP(1, 2) OP(2, 3) OP(3, 4) OP(4, 5) OP(5, 6) OP(6, 7) OP(7, 0)
#define SP0 "s[8:9]"
#define SP1 "s[10:11]"
#define SP2 "s[12:13]"
#define SP3 "s[14:15]"
#define SP4 "s[16:17]"
#define SP5 "s[18:19]"
#define SP6 "s[20:21]"
#define SP7 "s[22:23]"
#define SCLOB "s8", "s9", "s10", "s11", "s12", "s13", "s14", "s15", "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23", "scc"
template <int K>
__global__ __launch_bounds__(256) void kern(unsigned* out, unsigned long long* clk, int iters) {
    unsigned b[8];
    for (int i = 0; i < 8; ++i) b[i] = threadIdx.x * (2 * i + 3);
    const unsigned long long m0 = __ballot(threadIdx.x & 1);
    asm volatile("s_mov_b64 " SP0 ", -1\n s_mov_b64 " SP1 ", -1\n s_mov_b64 " SP2 ", -1\n s_mov_b64 " SP3 ", -1\n"
                 " s_mov_b64 " SP4 ", -1\n s_mov_b64 " SP5 ", -1\n s_mov_b64 " SP6 ", -1\n s_mov_b64 " SP7 ", -1" ::: SCLOB);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#define ADD(i, j) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
#define SAND(i, j) asm volatile("s_and_b64 " SP##i ", " SP##i ", %0" : : "s"(m0) : SCLOB);
#define SAND_DEP(i, j) asm volatile("s_and_b64 s[4:5], s[4:5], %0" : : "s"(m0) : "s4", "s5", "scc");
#define CMP(i, j) asm volatile("v_cmp_lt_u32_e64 " SP##i ", %0, %1" : : "v"(b[i]), "v"(b[j]) : SCLOB);
#define CMPAND(i, j) asm volatile("v_cmp_lt_u32_e64 " SP##i ", %0, %1\n s_and_b64 " SP##i ", " SP##i ", %2" : : "v"(b[i]), "v"(b[j]), "s"(m0) : SCLOB);
#define BR(i, j) asm volatile("s_cmp_eq_u64 " SP##i ", 0\n s_cbranch_scc1 1f\n1:" : : : SCLOB);
#define BCNT(i, j) asm volatile("s_bcnt1_i32_b64 s" #i ", %0" : : "s"(m0) : "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "scc");
        if constexpr (K == 0) { CH8(ADD) }
        if constexpr (K == 1) { CH8(SAND) }
        if constexpr (K == 2) { CH8(ADD) CH8(SAND) }
        if constexpr (K == 3) { CH8(ADD) SAND(0, 0) SAND(1, 0) SAND(2, 0) SAND(3, 0) }
        if constexpr (K == 4) { CH8(ADD) CH8(SAND) CH8(SAND) }
        if constexpr (K == 5) { CH8(SAND_DEP) }
        if constexpr (K == 6) { CH8(CMP) }
        if constexpr (K == 7) { CH8(CMPAND) }
        if constexpr (K == 8) { CH8(ADD) CH8(CMPAND) }
        if constexpr (K == 9) { CH8(BR) }
        if constexpr (K == 10) { CH8(ADD) CH8(BR) }
        if constexpr (K == 11) { CH8(BCNT) }
        if constexpr (K == 12) { CH8(ADD) CH8(BCNT) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s += b[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

static const char* NAMES[] = {"8 v_add", "8 s_and (independent)", "8 v_add + 8 s_and", "8 v_add + 4 s_and",
                              "8 v_add + 16 s_and", "8 s_and (one chain)", "8 v_cmp_e64", "8 (v_cmp -> s_and)",
                              "8 v_add + 8 (v_cmp -> s_and)", "8 (s_cmp + s_cbranch not taken)",
                              "8 v_add + 8 (s_cmp + s_cbranch)", "8 s_bcnt1", "8 v_add + 8 s_bcnt1"};
static const int VALU_IT[] = {8, 0, 8, 8, 8, 0, 8, 8, 16, 0, 8, 0, 8};
static const int SALU_IT[] = {0, 8, 8, 4, 16, 8, 0, 8, 8, 16, 16, 8, 8};

template <int K>
static void run(unsigned* out, unsigned long long* clk, int wps, int iters) {
    const int blocks = 256 * wps;                   // wps workgroups of 4 waves per CU: wps waves per SIMD
    kern<K><<<blocks, 256>>>(out, clk, 16);
    kern<K><<<blocks, 256>>>(out, clk, iters);
    (void)hipDeviceSynchronize();
    static unsigned long long c[256 * 8];
    (void)hipMemcpy(c, clk, (size_t)blocks * 8, hipMemcpyDeviceToHost);
    double cyc = 0;
    for (int b = 0; b < blocks; ++b) cyc += (double)c[b];
    cyc /= blocks;                                  // cycles of one workgroup's loop (all run concurrently)
    const double it = (double)wps * iters;          // wave-iterations per SIMD
    printf("%d wave/SIMD  %-36s %8.2f SIMD-cycles per wave-iteration (%d VALU, %d SALU)\n", wps, NAMES[K], cyc / it,
           VALU_IT[K], SALU_IT[K]);
}

template <int... Ks>
static void run_all(unsigned* out, unsigned long long* clk, int wps, int iters, std::integer_sequence<int, Ks...>) {
    (run<Ks>(out, clk, wps, iters), ...);
}

int main() {
    unsigned* out;
    unsigned long long* clk;
    if (hipMalloc(&out, (size_t)256 * 6 * 256 * 4) != hipSuccess) return 1;
    if (hipMalloc(&clk, (size_t)256 * 6 * 8) != hipSuccess) return 1;
    for (int rep = 0; rep < 2; ++rep)
        for (int wps : {6, 1}) run_all(out, clk, wps, 4096, std::make_integer_sequence<int, 13>{});
    return 0;
}
