/*
 * raft_oracle.h — TEST INFRASTRUCTURE ONLY.  Nothing in the product
 * (raft-kotlin_amd/) links or calls this; only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg do, as the checker.
 *
 * Scalar CPU restatement of the reference node (arodionov/raft-kotlin,
 * RaftServer.kt + Commons.kt) under the lockstep schedule of DESIGN.md §3.
 * Parity status: the reference ships no tests or fixtures and cannot be
 * built here (Kotlin/JVM/gradle absent), so this oracle is pinned by the
 * hand-derived known-answer traces K1-K7 of SURVEY.md §4 and the Random123
 * Philox vectors (tests/golden/), not by reference-produced outputs.
 */
#ifndef RAFT_ORACLE_H
#define RAFT_ORACLE_H
#include "../include/raft_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle oracle_t;

int  oracle_create(const raft_params* p, oracle_t** out);
void oracle_destroy(oracle_t* o);
/* counters: nullable [n_steps][RAFT_COUNTER_STRIDE]; nthreads <= 0 -> 1 */
int  oracle_step(oracle_t* o, int32_t n_steps, int64_t* counters, int32_t nthreads);
int64_t oracle_step_index(const oracle_t* o);
int  oracle_set_step_index(oracle_t* o, int64_t t);
int  oracle_read_state(const oracle_t* o, int64_t g0, int64_t n, int32_t* out);
int  oracle_write_state(oracle_t* o, int64_t g0, int64_t n, const int32_t* in);
int  oracle_read_log(const oracle_t* o, int64_t g0, int64_t n, int32_t* terms, uint32_t* cmds);
int  oracle_write_log(oracle_t* o, int64_t g0, int64_t n, const int32_t* terms, const uint32_t* cmds);
uint64_t oracle_digest(const oracle_t* o);
uint64_t oracle_digest_range(const oracle_t* o, int64_t g0, int64_t n);
int oracle_set_log_window(oracle_t* o, int32_t w);

/* single handlers, same semantics as raft_vote_batch & co (applied in order) */
int oracle_vote(oracle_t* o, int64_t group, int32_t dst, const raft_vote_req* req, raft_vote_resp* resp);
int oracle_append(oracle_t* o, int64_t group, int32_t dst, const raft_append_req* req, raft_append_resp* resp);
int oracle_append_command(oracle_t* o, int64_t group, int32_t replica, uint32_t cmd);

/* standalone Log<T> (Commons.kt:47-74) for the K1 trace */
typedef struct oracle_log oracle_log_t;
oracle_log_t* oracle_log_new(int32_t cap);
void    oracle_log_free(oracle_log_t* l);
int32_t oracle_log_add(oracle_log_t* l, int32_t i, int32_t term, uint32_t cmd); /* 1 true, 0 false, -1 overflow, -2 threw */
int32_t oracle_log_get(const oracle_log_t* l, int32_t i, int32_t* term, uint32_t* cmd); /* 1 ok, 0 threw */
int32_t oracle_log_last_index(const oracle_log_t* l);
int32_t oracle_log_size(const oracle_log_t* l);
/* physical slot j < size */
int32_t oracle_log_phys(const oracle_log_t* l, int32_t j, int32_t* term, uint32_t* cmd);

void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
