// Microbenchmark, part 6 (round 6): lane-mask hand-offs.  Part 4 measured a
// v_cndmask_b32_e32 reading VCC at 12.6 SIMD-cycles (6 waves per SIMD) but
// the same after a v_cmp_*_e32 that writes VCC at ~2.4: what a select costs
// depends on where its mask came from.  The step kernel makes its masks with
// v_cmp (VALU -> SGPR), combines them with s_and / s_or (SALU -> SGPR) and
// consumes them in v_cndmask / v_addc (SGPR -> VALU), so each hand-off is
// timed here in isolation, 8 independent chains per wave, 6 waves per SIMD.
// Cycles from each workgroup's own s_memtime stamps; experiments only.
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
#define SCLOB "s8", "s9", "s10", "s11", "s12", "s13", "s14", "s15", "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23", \
              "s24", "s25", "scc", "vcc"
template <int K>
__global__ __launch_bounds__(256) void kern(unsigned* out, unsigned long long* clk, int iters) {
    unsigned b[8];
    for (int i = 0; i < 8; ++i) b[i] = threadIdx.x * (2 * i + 3);
    asm volatile("s_mov_b64 " SP0 ", 0x5555\n s_mov_b64 " SP1 ", 0x3333\n s_mov_b64 " SP2 ", -1\n s_mov_b64 " SP3 ", -1\n"
                 " s_mov_b64 " SP4 ", -1\n s_mov_b64 " SP5 ", -1\n s_mov_b64 " SP6 ", -1\n s_mov_b64 " SP7 ", -1\n"
                 " s_mov_b64 s[24:25], 0x0f0f\n s_mov_b64 vcc, 0x00ff" ::: SCLOB);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        // selects by mask source
#define CND32(i, j) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define CND64V(i, j) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define CND64S(i, j) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[24:25]" : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define VCMP32_CND32(i, j) asm volatile("v_cmp_lt_u32_e32 vcc, %0, %1\n v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define SAND_VCC_CND32(i, j) asm volatile("s_and_b64 vcc, " SP0 ", " SP1 "\n v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define SAND_S_CND64(i, j) asm volatile("s_and_b64 " SP##i ", " SP0 ", s[24:25]\n v_cndmask_b32_e64 %0, %0, %1, " SP##i : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define VCMP64_CND64(i, j) asm volatile("v_cmp_lt_u32_e64 " SP##i ", %0, %1\n v_cndmask_b32_e64 %0, %0, %1, " SP##i : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define VCMP64_SAND_CND64(i, j) asm volatile("v_cmp_lt_u32_e64 " SP##i ", %0, %1\n s_and_b64 " SP##i ", " SP##i ", s[24:25]\n v_cndmask_b32_e64 %0, %0, %1, " SP##i : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define SAND_ADDC(i, j) asm volatile("s_and_b64 " SP##i ", " SP0 ", s[24:25]\n v_addc_co_u32_e64 %0, s[26:27], 0, %0, " SP##i : "+v"(b[i]) : "v"(b[j]) : SCLOB, "s26", "s27");
#define ADDC32(i, j) asm volatile("v_addc_co_u32_e32 %0, vcc, 0, %0, vcc" : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define SMOV_VCC_CND32(i, j) asm volatile("s_mov_b64 vcc, s[24:25]\n v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(b[i]) : "v"(b[j]) : SCLOB);
#define ADD(i, j) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(b[i]) : "v"(b[j]));
        if constexpr (K == 0) { CH8(CND32) }
        if constexpr (K == 1) { CH8(CND64V) }
        if constexpr (K == 2) { CH8(CND64S) }
        if constexpr (K == 3) { CH8(VCMP32_CND32) }
        if constexpr (K == 4) { CH8(SAND_VCC_CND32) }
        if constexpr (K == 5) { CH8(SAND_S_CND64) }
        if constexpr (K == 6) { CH8(VCMP64_CND64) }
        if constexpr (K == 7) { CH8(VCMP64_SAND_CND64) }
        if constexpr (K == 8) { CH8(SAND_ADDC) }
        if constexpr (K == 9) { CH8(ADDC32) }
        if constexpr (K == 10) { CH8(SMOV_VCC_CND32) }
        if constexpr (K == 11) { CND32(0, 1) ADD(1, 2) ADD(2, 3) ADD(3, 4) ADD(4, 5) ADD(5, 6) ADD(6, 7) ADD(7, 0) }
        if constexpr (K == 12) { CH8(ADD) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned s = 0;
    for (int i = 0; i < 8; ++i) s += b[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

static const char* NAMES[] = {
    "8 v_cndmask_e32 (vcc, set before the loop)", "8 v_cndmask_e64 mask=vcc", "8 v_cndmask_e64 mask=s[24:25]",
    "8 (v_cmp_e32 -> vcc -> v_cndmask_e32)", "8 (s_and -> vcc -> v_cndmask_e32)", "8 (s_and -> sgpr -> v_cndmask_e64)",
    "8 (v_cmp_e64 -> sgpr -> v_cndmask_e64)", "8 (v_cmp_e64 -> s_and -> v_cndmask_e64)",
    "8 (s_and -> sgpr -> v_addc_e64)", "8 v_addc_co_u32_e32 (vcc carry)", "8 (s_mov vcc -> v_cndmask_e32)",
    "1 v_cndmask_e32 (vcc) + 7 v_add", "8 v_add"};

template <int K>
static void run(unsigned* out, unsigned long long* clk, int wps, int iters) {
    const int blocks = 256 * wps;
    kern<K><<<blocks, 256>>>(out, clk, 16);
    kern<K><<<blocks, 256>>>(out, clk, iters);
    (void)hipDeviceSynchronize();
    static unsigned long long c[256 * 8];
    (void)hipMemcpy(c, clk, (size_t)blocks * 8, hipMemcpyDeviceToHost);
    double cyc = 0;
    for (int b = 0; b < blocks; ++b) cyc += (double)c[b];
    cyc /= blocks;
    printf("%d wave/SIMD  %-44s %8.2f SIMD-cycles per wave-iteration\n", wps, NAMES[K], cyc / ((double)wps * iters));
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
