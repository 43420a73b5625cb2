/*
 * philox_ref.h — TEST INFRASTRUCTURE (oracle side).  Philox4x32-10
 * (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3", SC'11;
 * Random123 constants).  Written independently of the engine's
 * raft-kotlin_amd/csrc/philox.h; both are pinned by the Random123 known-answer
 * vectors in tests/golden/philox_kat.json.
 *
 * It replaces the reference's unseeded java.util.Random draws
 * (Commons.kt:33-34, used at Commons.kt:23 and RaftServer.kt:221), whose
 * values cannot be reproduced.
 */
#ifndef PHILOX_REF_H
#define PHILOX_REF_H
#include <stdint.h>

static inline void philox_ref(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int round = 0; round < 10; ++round) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

#endif
