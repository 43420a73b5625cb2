/* raft_c_host.c -- a plain C99 host of the engine's C-ABI (include/raft_engine.h),
 * driving it the way the Kotlin JNI shim of INTEGRATION.md would: no Python,
 * no torch, host arrays only.
 *
 *   raft_c_host G R steps seed drop_ppm churn_ppm churn_steps cmd_ppm log_cap nmsg
 *
 * 1. raft_engine_create with raft_params_default() plus the arguments;
 * 2. raft_engine_step(steps) with host counter rows (the timers, RequestVote
 *    rounds, AppendEntries ticks and commits of every group:
 *    RaftServer.kt:109-226, Commons.kt:10-45), then raft_engine_digest;
 * 3. raft_vote_batch and raft_append_batch (RaftServer.kt:228-287) on nmsg
 *    messages each, drawn from a 64-bit LCG (tests/test_gpu_c_host.py draws
 *    the same ones), then raft_engine_digest again.
 * Prints one JSON object: the counter rows, both digests and every response.
 * Any failing call prints raft_last_error() and exits 1 (no GPU: create fails).
 * tests/test_gpu_c_host.py checks every output against the oracle. */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>

#include "raft_engine.h"

static void check(int rc, const char* what) {
    if (rc != RAFT_OK) {
        fprintf(stderr, "%s failed (%d): %s\n", what, rc, raft_last_error());
        exit(1);
    }
}

static uint64_t lcg_state;
static uint32_t draw(uint32_t n) {                       /* uniform-ish in [0, n) */
    lcg_state = lcg_state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)((lcg_state >> 33) % n);
}

static void* xalloc(size_t bytes) {
    void* p = calloc(1, bytes ? bytes : 1);
    if (!p) {
        fprintf(stderr, "out of host memory\n");
        exit(1);
    }
    return p;
}

int main(int argc, char** argv) {
    if (argc != 11) {
        fprintf(stderr, "usage: %s G R steps seed drop_ppm churn_ppm churn_steps cmd_ppm log_cap nmsg\n", argv[0]);
        return 2;
    }
    raft_params p;
    raft_params_default(&p);
    p.G = strtoll(argv[1], NULL, 10);
    p.R = (int32_t)strtol(argv[2], NULL, 10);
    const int32_t steps = (int32_t)strtol(argv[3], NULL, 10);
    p.seed = strtoull(argv[4], NULL, 10);
    p.drop_ppm = (uint32_t)strtoul(argv[5], NULL, 10);
    p.churn_ppm = (uint32_t)strtoul(argv[6], NULL, 10);
    p.churn_steps = (int32_t)strtol(argv[7], NULL, 10);
    p.cmd_ppm = (uint32_t)strtoul(argv[8], NULL, 10);
    p.log_cap = (int32_t)strtol(argv[9], NULL, 10);
    const int64_t n = strtoll(argv[10], NULL, 10);
    if (p.G < 1 || p.R < 1 || steps < 1 || n < 1) {
        fprintf(stderr, "G, R, steps and nmsg must be positive\n");
        return 2;
    }

    raft_engine* e = NULL;
    check(raft_engine_create(&p, 0, &e), "raft_engine_create");
    int64_t* rows = (int64_t*)xalloc((size_t)steps * RAFT_COUNTER_STRIDE * sizeof(int64_t));
    check(raft_engine_step(e, steps, rows), "raft_engine_step");
    uint64_t d_steps = 0, d_end = 0;
    check(raft_engine_digest(e, &d_steps), "raft_engine_digest");

    int64_t* group = (int64_t*)xalloc((size_t)n * sizeof(int64_t));
    int32_t* dst = (int32_t*)xalloc((size_t)n * sizeof(int32_t));
    raft_vote_req* vq = (raft_vote_req*)xalloc((size_t)n * sizeof(raft_vote_req));
    raft_vote_resp* vs = (raft_vote_resp*)xalloc((size_t)n * sizeof(raft_vote_resp));
    raft_append_req* aq = (raft_append_req*)xalloc((size_t)n * sizeof(raft_append_req));
    raft_append_resp* as = (raft_append_resp*)xalloc((size_t)n * sizeof(raft_append_resp));
    lcg_state = p.seed;
    for (int64_t i = 0; i < n; ++i) {
        group[i] = (int64_t)draw((uint32_t)(p.G < 0x7FFFFFFF ? p.G : 0x7FFFFFFF));
        dst[i] = (int32_t)draw((uint32_t)p.R);
        vq[i].term = (int32_t)draw(16);
        vq[i].candidate_id = 1 + (int32_t)draw((uint32_t)p.R);
        vq[i].last_log_index = (int32_t)draw(64);
        vq[i].last_log_term = (int32_t)draw(16);
        aq[i].term = (int32_t)draw(16);
        aq[i].leader_id = 1 + (int32_t)draw((uint32_t)p.R);
        aq[i].prev_log_index = (int32_t)draw(48) - 1;
        aq[i].prev_log_term = (int32_t)draw(16);
        aq[i].has_entry = (int32_t)draw(2);
        aq[i].entry_term = (int32_t)draw(16);
        aq[i].entry_cmd = draw(1u << 31);
        aq[i].leader_commit = (int32_t)draw(48);
    }
    check(raft_vote_batch(e, group, dst, vq, vs, n), "raft_vote_batch");
    check(raft_append_batch(e, group, dst, aq, as, n), "raft_append_batch");
    check(raft_engine_digest(e, &d_end), "raft_engine_digest");

    printf("{\"abi\": %d, \"digest_steps\": %" PRIu64 ", \"digest_end\": %" PRIu64 ", \"counters\": [", raft_abi_version(),
           d_steps, d_end);
    for (int32_t k = 0; k < steps; ++k) {
        printf("%s[", k ? ", " : "");
        for (int c = 0; c < RAFT_NUM_COUNTERS; ++c) printf("%s%" PRId64, c ? ", " : "", rows[(int64_t)k * RAFT_COUNTER_STRIDE + c]);
        printf("]");
    }
    printf("], \"vote\": [");
    for (int64_t i = 0; i < n; ++i) printf("%s[%d, %d]", i ? ", " : "", vs[i].term, vs[i].vote_granted);
    printf("], \"append\": [");
    for (int64_t i = 0; i < n; ++i) printf("%s[%d, %d, %d]", i ? ", " : "", as[i].term, as[i].success, as[i].status);
    printf("]}\n");

    check(raft_engine_destroy(e), "raft_engine_destroy");
    free(rows); free(group); free(dst); free(vq); free(vs); free(aq); free(as);
    return 0;
}
