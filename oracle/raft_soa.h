/*
 * raft_soa.h — CPU BASELINE ONLY (timed by bench.py's cpu_baseline leg and
 * checked against the oracle by tests/test_soa_cpu.py).  Never linked into
 * the product.
 *
 * The same lockstep step as oracle/raft_oracle.c (RaftServer.kt + Commons.kt
 * under DESIGN.md §3's schedule), laid out as structure-of-arrays -- one array
 * per field over all G*R replicas, the logs as two flat [G*R][log_cap] arrays
 * (terms, commands) -- and stepped group by group with std::thread over
 * contiguous group ranges: the CPU analogue of the engine's layout, against
 * which the scalar object-per-replica oracle is the straightforward port.
 * Reference mode only (RAFT_MODE_REFERENCE) and every physical slot kept
 * (log_window 0); bit-exact with the oracle (counters, canonical state, logs,
 * digest).
 */
#ifndef RAFT_SOA_H
#define RAFT_SOA_H
#include "../include/raft_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct soa soa_t;

int  soa_create(const raft_params* p, soa_t** out);       /* RAFT_EINVAL for textbook mode or a log_window */
void soa_destroy(soa_t* s);
/* counters: nullable [n_steps][RAFT_COUNTER_STRIDE]; nthreads <= 0 -> 1 */
int  soa_step(soa_t* s, int32_t n_steps, int64_t* counters, int32_t nthreads);
int  soa_read_state(const soa_t* s, int64_t g0, int64_t n, int32_t* out);
int  soa_read_log(const soa_t* s, int64_t g0, int64_t n, int32_t* terms, uint32_t* cmds);
uint64_t soa_digest(const soa_t* s);
/* Restore a run exported at any step (the canonical [n][raft_group_words(R)]
 * state, the [n][R][log_cap] logs, the next step's index): the steady-state
 * CPU baseline resumes from the engine's state dump.  Every session row,
 * primary or not, is held in full, so no primary owner is implied. */
int  soa_write_state(soa_t* s, int64_t g0, int64_t n, const int32_t* in);
int  soa_write_log(soa_t* s, int64_t g0, int64_t n, const int32_t* terms, const uint32_t* cmds);
int  soa_set_step_index(soa_t* s, int64_t t);

#ifdef __cplusplus
}
#endif
#endif
