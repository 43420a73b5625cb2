// Host code under AddressSanitizer + UndefinedBehaviorSanitizer (test
// infrastructure; tests/test_host_sanitize.py builds and runs it).  GPU code
// is never built with a sanitizer here: only the host C / C++ of the
// repository -- the CPU oracle (oracle/raft_oracle.c), the SoA CPU backend
// (oracle/raft_soa.cpp) and the protobuf wire codec (raft_wire.cpp) -- on
// the configurations the tests use, plus malformed and random wire input.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

extern "C" {
#include "raft_oracle.h"
#include "raft_soa.h"
}
#include "raft_wire.h"

// raft_wire.cpp reports errors through this (raft_engine.hip in the product)
std::string g_last;
int raft_internal_fail(int code, const std::string& msg) {
    g_last = msg;
    return code;
}

static int failures = 0;
#define CHECK(cond)                                                         \
    do {                                                                    \
        if (!(cond)) {                                                      \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                     \
        }                                                                   \
    } while (0)

static raft_params base_params() {
    raft_params p;
    std::memset(&p, 0, sizeof p);
    p.R = 5; p.log_cap = 400; p.G = 300; p.g0 = 0; p.seed = 3;
    p.heartbeat_ms = 2000; p.election_min_ms = 20000; p.election_max_ms = 23000;
    p.backoff_min_ms = 2000; p.backoff_max_ms = 3000; p.round_timeout_ms = 25000; p.retry_ms = 5000;
    p.drop_ppm = 50000; p.churn_ppm = 20000; p.churn_steps = 15; p.cmd_ppm = 250000;
    return p;
}

// the oracle and the SoA backend step the same groups: equal digests
static void oracle_vs_soa(raft_params p, int steps) {
    oracle_t* o = nullptr;
    soa_t* s = nullptr;
    CHECK(oracle_create(&p, &o) == 0);
    CHECK(soa_create(&p, &s) == 0);
    std::vector<int64_t> co((size_t)steps * RAFT_COUNTER_STRIDE), cs((size_t)steps * RAFT_COUNTER_STRIDE);
    CHECK(oracle_step(o, steps, co.data(), 3) == 0);
    CHECK(soa_step(s, steps, cs.data(), 3) == 0);
    CHECK(oracle_digest(o) == soa_digest(s));
    for (int k = 0; k < steps; ++k)
        for (int c = 0; c < RAFT_NUM_COUNTERS; ++c)
            CHECK(co[(size_t)k * RAFT_COUNTER_STRIDE + c] == cs[(size_t)k * RAFT_COUNTER_STRIDE + c]);
    oracle_destroy(o);
    soa_destroy(s);
}

// the oracle alone: textbook mode, multi-entry requests, a ring, state/log
// round trips and the single handlers on random requests
static void oracle_paths() {
    raft_params p = base_params();
    p.mode = RAFT_MODE_TEXTBOOK;
    p.ae_max_entries = 8;
    p.partition_period = 40;
    p.partition_len = 10;
    oracle_t* o = nullptr;
    CHECK(oracle_create(&p, &o) == 0);
    CHECK(oracle_step(o, 250, nullptr, 2) == 0);
    oracle_destroy(o);

    p = base_params();
    p.log_window = 64;
    CHECK(oracle_create(&p, &o) == 0);
    CHECK(oracle_step(o, 250, nullptr, 2) == 0);
    oracle_destroy(o);

    p = base_params();
    p.G = 40;
    p.log_cap = 16;
    CHECK(oracle_create(&p, &o) == 0);
    CHECK(oracle_step(o, 60, nullptr, 1) == 0);
    const int W = p.R * RAFT_NUM_FIELDS + 2 * p.R * p.R + RAFT_GROUP_EXTRA;
    std::vector<int32_t> st((size_t)p.G * W), terms((size_t)p.G * p.R * p.log_cap);
    std::vector<uint32_t> cmds(terms.size());
    CHECK(oracle_read_state(o, 0, p.G, st.data()) == 0);
    CHECK(oracle_read_log(o, 0, p.G, terms.data(), cmds.data()) == 0);
    CHECK(oracle_write_state(o, 0, p.G, st.data()) == 0);
    CHECK(oracle_write_log(o, 0, p.G, terms.data(), cmds.data()) == 0);
    std::mt19937 rng(7);
    for (int m = 0; m < 20000; ++m) {
        const int64_t g = rng() % p.G;
        const int32_t d = (int32_t)(rng() % p.R);
        if (m % 3 == 0) {
            raft_vote_req q{(int32_t)(rng() % 6), (int32_t)(1 + rng() % p.R), (int32_t)(rng() % (p.log_cap + 1)),
                            (int32_t)(rng() % 4)};
            raft_vote_resp r;
            CHECK(oracle_vote(o, g, d, &q, &r) == 0);
        } else if (m % 3 == 1) {
            raft_append_req q{(int32_t)(rng() % 6), (int32_t)(1 + rng() % p.R), (int32_t)((int)(rng() % (p.log_cap + 2)) - 2),
                              (int32_t)((int)(rng() % 5) - 1), (int32_t)(rng() % 2), (int32_t)(rng() % 6),
                              (uint32_t)rng(), (int32_t)(rng() % 8)};
            raft_append_resp r;
            CHECK(oracle_append(o, g, d, &q, &r) == 0);
        } else {
            oracle_append_command(o, g, d, (uint32_t)rng());
        }
    }
    (void)oracle_digest(o);
    oracle_destroy(o);
}

// the wire codec: round trips, then random and truncated buffers (any
// verdict, but no out-of-bounds access)
static void wire() {
    std::mt19937 rng(11);
    const int n = 500;
    std::vector<raft_vote_req> vq(n), vq2(n);
    for (auto& q : vq) q = raft_vote_req{(int32_t)rng(), (int32_t)rng(), (int32_t)rng(), (int32_t)rng()};
    std::vector<uint8_t> buf(64 * n);
    std::vector<int64_t> off(n + 1);
    const int64_t len = raft_wire_encode_vote_req(vq.data(), n, buf.data(), (int64_t)buf.size(), off.data());
    CHECK(len > 0);
    CHECK(raft_wire_decode_vote_req(buf.data(), off.data(), n, vq2.data()) == 0);
    CHECK(std::memcmp(vq.data(), vq2.data(), sizeof(raft_vote_req) * n) == 0);
    CHECK(raft_wire_encode_vote_req(vq.data(), n, buf.data(), 10, off.data()) < 0);      // too small: refused

    std::vector<raft_append_req> aq(n), aq2(n);
    std::string cmds;
    std::vector<int64_t> coff(n + 1);
    for (int m = 0; m < n; ++m) {
        aq[m] = raft_append_req{(int32_t)rng(), (int32_t)rng(), (int32_t)rng(), (int32_t)rng(), (int32_t)(rng() % 2),
                                (int32_t)rng(), 0u, (int32_t)rng()};
        coff[m] = (int64_t)cmds.size();
        cmds += std::string(rng() % 40, (char)('a' + m % 26));
    }
    coff[n] = (int64_t)cmds.size();
    std::vector<uint8_t> abuf(128 * n + cmds.size() * 2);
    std::vector<int64_t> aoff(n + 1), dcoff(n);
    std::vector<int32_t> dclen(n), nent(n);
    const int64_t alen = raft_wire_encode_append_req(aq.data(), (const uint8_t*)cmds.data(), coff.data(), n,
                                                     abuf.data(), (int64_t)abuf.size(), aoff.data());
    CHECK(alen > 0);
    CHECK(raft_wire_decode_append_req(abuf.data(), aoff.data(), n, aq2.data(), dcoff.data(), dclen.data(),
                                      nent.data()) == 0);
    for (int m = 0; m < n; ++m) {
        CHECK(aq2[m].term == aq[m].term && aq2[m].leader_commit == aq[m].leader_commit);
        CHECK(aq2[m].has_entry == aq[m].has_entry);
        if (aq[m].has_entry)
            CHECK(dclen[m] == (int32_t)(coff[m + 1] - coff[m]) &&
                  std::memcmp(abuf.data() + dcoff[m], cmds.data() + coff[m], (size_t)dclen[m]) == 0);
    }
    // random bytes and every truncation of a real message: decoders must stay in bounds
    std::vector<uint8_t> junk(4096);
    for (int trial = 0; trial < 2000; ++trial) {
        const int64_t L = rng() % 64;
        for (int64_t k = 0; k < L; ++k) junk[k] = (uint8_t)rng();
        int64_t o2[2] = {0, L};
        raft_vote_req v;
        raft_vote_resp vr;
        raft_append_req a;
        raft_append_resp ar;
        int64_t co;
        int32_t cl, ne;
        (void)raft_wire_decode_vote_req(junk.data(), o2, 1, &v);
        (void)raft_wire_decode_vote_resp(junk.data(), o2, 1, &vr);
        (void)raft_wire_decode_append_req(junk.data(), o2, 1, &a, &co, &cl, &ne);
        (void)raft_wire_decode_append_resp(junk.data(), o2, 1, &ar);
    }
    for (int m = 0; m < 50; ++m) {
        const int64_t a0 = aoff[m], a1 = aoff[m + 1];
        std::vector<uint8_t> one(abuf.begin() + a0, abuf.begin() + a1);
        for (int64_t L = 0; L <= (int64_t)one.size(); ++L) {
            std::vector<uint8_t> cut(one.begin(), one.begin() + L);      // exact-size copy: reads past it are caught
            int64_t o2[2] = {0, L};
            raft_append_req a;
            int64_t co;
            int32_t cl, ne;
            (void)raft_wire_decode_append_req(cut.data(), o2, 1, &a, &co, &cl, &ne);
        }
    }
}

int main() {
    raft_params p = base_params();
    oracle_vs_soa(p, 300);                                   // config 3 semantics
    p = base_params();
    p.R = 7; p.G = 60; p.drop_ppm = 0; p.churn_ppm = 0; p.cmd_ppm = 1000000; p.cmd_mode = RAFT_CMD_ALL_LEADERS;
    p.partition_period = 50; p.partition_len = 25; p.log_cap = 700;
    oracle_vs_soa(p, 300);                                   // config 5 semantics
    for (int R = 1; R <= 8; ++R) {
        p = base_params();
        p.R = R; p.G = 50; p.partition_period = 40; p.partition_len = 10;
        oracle_vs_soa(p, 150);
    }
    oracle_paths();
    wire();
    std::printf("host_check: %d failures\n", failures);
    return failures ? 1 : 0;
}
