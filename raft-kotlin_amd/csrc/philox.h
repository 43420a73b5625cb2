// philox.h — Philox4x32-10 counter-based RNG for the engine (host + device).
//
// Replaces the reference's unseeded java.util.Random (Commons.kt:33-34) with a
// reproducible stream keyed by (step, global group id, purpose, sub); the
// counter layout is the schedule rule S-9 of DESIGN.md.  Pinned by the
// Random123 known-answer vectors (tests/golden/philox_kat.json).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define RAFT_HD __host__ __device__ __forceinline__
#else
#define RAFT_HD inline
#endif

namespace raft {

struct u32x4 { uint32_t x, y, z, w; };

RAFT_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

RAFT_HD u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                           uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__)
    // Keep the round keys local to this call: without the barrier the
    // optimiser hoists all 20 (uniform) round keys out of the step loop and
    // they pin 20 SGPRs for the whole kernel (spilled to VGPR lanes).
    asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        // one full 32x32->64 product per multiplier (a single v_mad_u64_u32 on gfx950)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#if defined(__HIP_DEVICE_COMPILE__)
        // three-input XOR as one v_bitop3_b32 (gfx950; truth table 0x96):
        // the compiler emits two v_xor_b32 for it
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
#else
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
#endif
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return u32x4{c0, c1, c2, c3};
}

// Word i (0..3) as two bit-selects: a chain of i == k compares would be
// lowered to a branchy switch on the GPU.
RAFT_HD uint32_t sel4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, int i) {
    const uint32_t lo = (i & 1) ? b : a, hi = (i & 1) ? d : c;
    return (i & 2) ? hi : lo;
}
RAFT_HD uint32_t word_of(const u32x4& v, int i) { return sel4(v.x, v.y, v.z, v.w, i); }

// (lo..hi).random() (Commons.kt:33-34), scaled by multiply-shift (S-9)
RAFT_HD int32_t scale_range(uint32_t w, int32_t lo, int32_t hi) {
    return lo + (int32_t)mulhi32(w, (uint32_t)(hi - lo) + 1u);
}

// Bernoulli tests: w / 2^bits < ppm / 1e6, exactly
RAFT_HD bool hit32(uint32_t w, uint32_t ppm) {
    return (uint64_t)w * 1000000ull < ((uint64_t)ppm << 32);
}
RAFT_HD bool hit16(uint32_t u16, uint32_t ppm) {
    return (uint64_t)u16 * 1000000ull < ((uint64_t)ppm << 16);
}

}  // namespace raft
