/*
 * raft_engine.h — C-ABI of the MI355X batched Raft engine.
 *
 * Drop-in boundary for the consensus core of arodionov/raft-kotlin
 * (reference: src/main/kotlin/ua/org/kug/raft/RaftServer.kt, Commons.kt,
 * src/main/proto/greeter.proto).  The reference exposes one Raft node per JVM
 * process behind the gRPC service
 *
 *     service Raft { rpc Vote(RequestVoteRPC) returns (ResponseVoteRPC);
 *                    rpc Append(RequestAppendEntriesRPC) returns (ResponseAppendEntriesRPC); }
 *                                                             (greeter.proto:46-49)
 *
 * implemented by RaftServer.vote()  (RaftServer.kt:228-251) and
 *                RaftServer.append() (RaftServer.kt:253-287),
 * and drives itself from timers: the election timer (Commons.kt:10-31,
 * RaftServer.kt:180-185), the candidate loop leaderElection()
 * (RaftServer.kt:187-226) and the leader heartbeat/commit loop
 * appendRequestAndLeaderHeartbeat() (RaftServer.kt:109-178).
 *
 * This engine runs that node state machine for G independent groups of R
 * replicas each, in deterministic lockstep (one step = one heartbeat period),
 * with the whole state resident in GPU HBM.  The schedule that turns the
 * racy reference into a deterministic one is specified in DESIGN.md §3.
 *
 * Conventions
 *   - plain C types only; every function returns RAFT_OK (0) or a negative
 *     RAFT_E* code; raft_last_error() gives the text (thread-local).
 *   - the caller owns every host buffer; the engine owns device memory.
 *   - one engine handle is not reentrant: callers serialise per handle.
 *   - the reference's per-message exceptions (Log.get IndexOutOfBounds,
 *     gRPC failures) are per-message status values, never errors.
 */
#ifndef RAFT_ENGINE_H
#define RAFT_ENGINE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: raft_params.schedule / schedule_workgroups / kernel, automatic
 * subranges by workload (1 or 3), raft_engine_kernel_info, raft_engine_set_kernel,
 * raft_engine_reset, raft_engine_wait_stream */
#define RAFT_ABI_VERSION 2

/* ---- status codes ---------------------------------------------------- */
#define RAFT_OK            0
#define RAFT_EINVAL       -1   /* bad argument                               */
#define RAFT_ENOMEM       -2   /* device/host allocation failed              */
#define RAFT_EDEVICE      -3   /* HIP runtime error                          */
#define RAFT_ERANGE       -4   /* group range outside the engine             */
#define RAFT_ENODEV       -5   /* no HIP device / kernel image unavailable   */
#define RAFT_EWINDOW      -6   /* a handler batch touched a log slot below the
                                * retained window (results invalid, like overflow) */

/* ---- node roles: enum class State (RaftServer.kt:24-26) --------------- */
#define RAFT_FOLLOWER  0
#define RAFT_CANDIDATE 1
#define RAFT_LEADER    2

#define RAFT_MAX_R 8
#define RAFT_MAX_STEPS_PER_LAUNCH 16384 /* steps fused into one kernel launch (beyond 512: epochs) */
#define RAFT_MAX_AE_ENTRIES 8           /* textbook mode: entries one AppendEntries request carries */
#define RAFT_MAX_SUBRANGES 4            /* launch sub-ranges (streams) of the step kernel's grid */

/* ---- command-injection modes (harness) ---------------- */
#define RAFT_CMD_LOWEST_LEADER 0   /* appendCommand on the lowest-id LEADER  */
#define RAFT_CMD_ALL_LEADERS   1   /* appendCommand on every LEADER          */

/* ---- protocol modes -------------------------------- */
#define RAFT_MODE_REFERENCE 0   /* the reference's handlers, quirks Q1-Q14 included (parity) */
#define RAFT_MODE_TEXTBOOK  1   /* opt-in, not the reference: append() rejects a stale term,
                                 * truncates only on conflict and advances the follower commit
                                 * after the consistency check; a new leader starts at
                                 * nextIndex = lastIndex + 1; an acked entry sets
                                 * matchIndex = its index; the leader commit is the median of
                                 * matchIndex[] with a current-term guard */

/*
 * Engine parameters.  The *_ms defaults are the reference's hard-coded
 * constants; raft_params_default() fills them in.
 */
typedef struct raft_params {
    int32_t  R;                 /* replicas per group, 1..8 (servers.size, RaftServer.kt:307)      */
    int32_t  log_cap;           /* physical log slots per replica (ghost tail included, §3.2)      */
    int64_t  G;                 /* groups held by this engine                                      */
    int64_t  g0;                /* global id of this engine's first group (sharding offset)         */
    uint64_t seed;              /* Philox key = (seed lo32, seed hi32)                              */

    int32_t  heartbeat_ms;      /* 2000   fixedRateTimer(period = 2000)   RaftServer.kt:115         */
    int32_t  election_min_ms;   /* 20000  (20_000..23_000).random()       Commons.kt:23             */
    int32_t  election_max_ms;   /* 23000                                                            */
    int32_t  backoff_min_ms;    /* 2000   delay((2_000..3_000).random())  RaftServer.kt:221         */
    int32_t  backoff_max_ms;    /* 3000                                                             */
    int32_t  round_timeout_ms;  /* 25000  countDownLatch.await(25, SECONDS) RaftServer.kt:189,:214  */
    int32_t  retry_ms;          /* 5000   retry(delay = 5000)             Commons.kt:37             */

    uint32_t drop_ppm;          /* Bernoulli drop per request and per response (self never dropped) */
    uint32_t churn_ppm;         /* per group-step probability to isolate the lowest-id LEADER      */
    int32_t  churn_steps;       /* isolation length in steps                                        */
    int32_t  partition_period;  /* 0 = off; else a 2-way partition drawn every period steps ...    */
    int32_t  partition_len;     /* ... holding for partition_len steps                              */
    uint32_t cmd_ppm;           /* per group-step probability of one client command               */
    int32_t  cmd_mode;          /* RAFT_CMD_*                                                       */
    int32_t  cmd_limit;         /* 0 = unlimited, else commands per group                           */
    int32_t  steps_per_launch;  /* engine only: steps fused in one kernel launch, 0..RAFT_MAX_STEPS_PER_LAUNCH (0 = 1);
                                   results never depend on it; <= 429 lets the 7-wave kernels (R <= 5, and
                                   R = 7 without drops) run 7 workgroups per CU (LDS), up to 512 run 6; a
                                   longer balanced launch on one sub-range in the reference mode (not a
                                   partitions-only kernel) runs as 400-step epochs (7 per CU), any other
                                   is cut into launches of 512 */
    int32_t  mode;              /* RAFT_MODE_* (0 = the reference)                                  */
    int32_t  log_window;        /* 0 = every physical slot is kept (log_cap slots per replica);
                                 * else a power of two W <= log_cap: only the newest W physical
                                 * slots [physLen - W, physLen) of each replica are kept, in a ring
                                 * (DESIGN.md §4.2).  Every Log.get / Log.add of the reference below
                                 * physLen - W is counted in RAFT_C_LOG_WINDOW_MISS; a run with a
                                 * miss is invalid (its results are not the reference's), as with
                                 * RAFT_C_LOG_OVERFLOW.  log_cap stays the physLen limit.          */
    int32_t  ae_max_entries;    /* RAFT_MODE_TEXTBOOK only: the entries one AppendEntries request
                                 * carries, nextIndex .. up to ae_max_entries of them
                                 * (greeter.proto:37 `repeated LogEntry entries`).  0 or 1 = one
                                 * entry, the reference's shape (RaftServer.kt:130-132); at most
                                 * RAFT_MAX_AE_ENTRIES.  Must be 0 or 1 in reference mode.       */
    int32_t  subranges;         /* engine only: the step kernel's chunks (waves of groups) split into
                                 * this many contiguous ranges, each launched on its own stream, so
                                 * that one range's last waves can overlap another's next launch.
                                 * 0 = automatic (ABI 2): 1 with the balanced schedule, 3 for a
                                 * partitions-only workload (configs 5, 2, 1), whose automatic
                                 * schedule is one chunk per wave; 1..RAFT_MAX_SUBRANGES.  Results
                                 * never depend on it.                                             */
    int32_t  schedule;          /* engine only: RAFT_SCHED_* (0 = automatic: balanced when the
                                 * chunks outnumber the resident wave slots, except for a
                                 * partitions-only workload).  Results never depend on it.        */
    int32_t  schedule_workgroups; /* engine only: workgroups of a balanced launch (0 = as many as
                                 * the GPU holds at once at the launch's LDS; tests set fewer)     */
    int32_t  kernel;            /* engine only: RAFT_KERNEL_AUTO (0): the step kernel built for the
                                 * configured network faults and command harness (the other checks
                                 * compiled out); RAFT_KERNEL_GENERAL: the kernel that decides every
                                 * fault at run time.  Results never depend on it.                 */
} raft_params;
#define RAFT_KERNEL_AUTO    0
#define RAFT_KERNEL_GENERAL 1

/* ---- step-kernel schedules (raft_params.schedule) --------
 * A chunk is one wave's 64 / R groups.  ONE_PER_WAVE launches a wave per
 * chunk for all steps of the launch: when the chunks outnumber the GPU's
 * resident wave slots, the last round of waves runs on a part-empty chip.
 * BALANCED launches only the workgroups the GPU holds at once (nb of them);
 * workgroup b takes the interleaved chunks b, b + nb, b + 2 nb, ... (so the
 * chunks running at one time are neighbours) and its waves split those
 * chunks' chunk-steps into equal parts (a chunk may pass from one wave to
 * the next between steps), so every wave ends together.  AUTO takes BALANCED when the chunks
 * outnumber the resident wave slots, else ONE_PER_WAVE. */
#define RAFT_SCHED_AUTO         0
#define RAFT_SCHED_ONE_PER_WAVE 1
#define RAFT_SCHED_BALANCED     2   /* whenever every workgroup gets >= 4 chunks */

/* What the last step launch ran (raft_engine_kernel_info). */
typedef struct raft_kernel_info {
    int32_t net;                 /* network faults the kernel was built for: bit 0 drops, 1 partitions,
                                  * 2 isolation churn, 3 config 3's command harness compiled in
                                  * (raft_step.h NET_*)                                              */
    int32_t textbook;            /* 1: RAFT_MODE_TEXTBOOK kernel                                   */
    int32_t ring;                /* 1: the log_window ring kernel                                  */
    int32_t steps;               /* steps of the launch                                            */
    int32_t workgroups;          /* workgroups of the launch, all sub-ranges                       */
    int32_t resident_workgroups; /* workgroups of this kernel the GPU holds at once at that LDS    */
    int32_t balanced;            /* sub-ranges that ran the balanced schedule                      */
    int32_t subranges;           /* sub-ranges (streams) of the launch                             */
    int32_t reserved[4];
} raft_kernel_info;

/* ---- per-step counters (sum over the engine's groups) ------------------ */
enum raft_counter {
    RAFT_C_LEADERS = 0,         /* replicas with role LEADER at step end                        */
    RAFT_C_GROUPS_WITH_LEADER,  /* groups with >= 1 LEADER at step end                          */
    RAFT_C_TIMEOUTS,            /* election timers fired (Commons.kt:25-27)                     */
    RAFT_C_ROUNDS,              /* election rounds started (RaftServer.kt:191-193)              */
    RAFT_C_VOTES_GRANTED,       /* vote() handler grants (RaftServer.kt:237-242)                */
    RAFT_C_LEADERS_ELECTED,     /* heartbeat sessions started (RaftServer.kt:66,:109)           */
    RAFT_C_SESSIONS_TICKED,     /* H: leader ticks that built requests (RaftServer.kt:115-122)  */
    RAFT_C_APPEND_SENT,         /* AppendEntries requests built (incl. self)                    */
    RAFT_C_APPEND_SKIPPED,      /* Q11: Log.get threw while building (RaftServer.kt:128)        */
    RAFT_C_ENTRIES_ACKED,       /* successful entry-carrying responses (RaftServer.kt:157-162)  */
    RAFT_C_COMMITS,             /* commitIndex += 1 by the leader rule (RaftServer.kt:161-162)  */
    RAFT_C_MSG_DROPPED,         /* requests + responses lost (drop mask, isolation, partition)  */
    RAFT_C_COMMANDS,            /* client commands appended (RaftServer.kt:100-107)             */
    RAFT_C_COMMIT_REGRESSIONS,  /* Q4: follower commitIndex decreased (RaftServer.kt:270-272)   */
    RAFT_C_DUAL_LEADER_GROUPS,  /* groups with 2+ LEADERs in one term at step end (safety flag) */
    RAFT_C_LOG_OVERFLOW,        /* Log.add refused for lack of physical capacity (run invalid)  */
    RAFT_C_PREV_READS_LEADER,   /* P_L: log[prev].term reads at the leader                      */
    RAFT_C_ENTRY_READS_LEADER,  /* E_L: log[i-1] reads at the leader                            */
    RAFT_C_PREV_READS_FOLLOWER, /* P_F: log[prev].term reads in append()                        */
    RAFT_C_ENTRY_WRITES,        /* E_W: Log.add stores from append()                            */
    RAFT_C_VOTE_LOG_READS,      /* V: last-log-term reads in the vote path                      */
    RAFT_C_LOG_WINDOW_MISS,     /* Log.get/Log.add below physLen - log_window (run invalid)      */
    RAFT_NUM_COUNTERS
};
#define RAFT_COUNTER_STRIDE 32  /* int64 slots per step in counter buffers */

/* ---- canonical state export ------------------------------------------- */
/*
 * Per-replica scalar fields (int32).  Exported per group as
 *   [R][RAFT_NUM_FIELDS] scalars, then next[R][R], match[R][R] (leader
 *   session of replica s towards replica d at [s][d]), then RAFT_GROUP_EXTRA
 *   harness words; i.e. raft_group_words(R) int32 per group.
 */
enum raft_field {
    RAFT_F_TERM = 0,     /* currentTerm        RaftServer.kt:35-36   */
    RAFT_F_VOTED,        /* votedFor (-1/id)   RaftServer.kt:38-39   */
    RAFT_F_ROLE,         /* state              RaftServer.kt:41-42   */
    RAFT_F_COMMIT,       /* commitIndex        RaftServer.kt:46      */
    RAFT_F_LAST,         /* log.lastIndex      Commons.kt:49         */
    RAFT_F_PHYS,         /* physical ArrayList size (ghost tail)     */
    RAFT_F_ELECTION_MS,  /* election timer remaining (0 if disarmed) */
    RAFT_F_FLAGS,        /* RAFT_FL_* bits below                      */
    RAFT_F_PHASE_MS,     /* round elapsed ms, or backoff remaining    */
    RAFT_F_RETRY_MS,     /* vote retry countdown                      */
    RAFT_NUM_FIELDS
};
#define RAFT_FL_ARMED        (1u << 0)   /* election timer scheduled           */
#define RAFT_FL_ELECTING     (1u << 1)   /* consumer busy in leaderElection()  */
#define RAFT_FL_PENDING_RST  (1u << 2)   /* FOLLOWER send queued while busy    */
#define RAFT_FL_HB_ACTIVE    (1u << 3)   /* heartbeat session running          */
#define RAFT_FL_BACKOFF      (1u << 4)   /* election loop in backoff delay     */
#define RAFT_FL_PENDING_SHIFT 8          /* 8 bits: vote dsts awaiting retry   */
#define RAFT_FL_VOTES_SHIFT   16         /* 4 bits: votesGranted               */
#define RAFT_FL_LATCH_SHIFT   20         /* 4 bits: responses counted on latch */

#define RAFT_GROUP_EXTRA 2   /* [0] isolation word (rem<<8 | replica), [1] commands issued */

static inline int32_t raft_group_words(int32_t R) {
    return R * RAFT_NUM_FIELDS + 2 * R * R + RAFT_GROUP_EXTRA;
}

/* ---- single-handler messages (greeter.proto:16-44, fixed width) -------- */
typedef struct raft_vote_req {       /* RequestVoteRPC  greeter.proto:16-21 */
    int32_t term, candidate_id, last_log_index, last_log_term;
} raft_vote_req;
typedef struct raft_vote_resp {      /* ResponseVoteRPC greeter.proto:23-26 */
    int32_t term, vote_granted;
} raft_vote_resp;
typedef struct raft_append_req {     /* RequestAppendEntriesRPC greeter.proto:28-39 */
    int32_t  term, leader_id, prev_log_index, prev_log_term;
    int32_t  has_entry;              /* entriesCount > 0 (only entries[0] is used, RaftServer.kt:278) */
    int32_t  entry_term;             /* LogEntry.term                          */
    uint32_t entry_cmd;              /* LogEntry.command, interned to a u32 id */
    int32_t  leader_commit;
} raft_append_req;
typedef struct raft_append_resp {    /* ResponseAppendEntriesRPC greeter.proto:41-44 */
    int32_t term, success;
    int32_t status;                  /* 0 ok; 1 = handler threw (Log index < -1), no response */
} raft_append_resp;

typedef struct raft_engine raft_engine;

/* ---- lifecycle -------------------------------------------------------- */
void        raft_params_default(raft_params* p);
const char* raft_last_error(void);
int         raft_abi_version(void);
/* The build's provenance: a short hash of every source, header and compiler
 * flag the library was built from (raft-kotlin_amd/build.py
 * library_source_id; abi.load_library refuses a library whose id differs
 * from the sources beside it), and of the step kernel's three sources
 * (kernel_source_id, the key of bench.py's rocprofv3 rows).  "unknown" for a
 * build made without build.py.  raft_build_batch_source_id: the handler
 * batches' sources and the compile-time knobs that shape their kernels
 * (build.py batch_source_id, the key of their rocprofv3 rows). */
const char* raft_build_source_id(void);
const char* raft_build_kernel_source_id(void);
const char* raft_build_batch_source_id(void);
int raft_engine_create(const raft_params* p, int device, raft_engine** out);
int raft_engine_destroy(raft_engine* e);

/* ---- the hot path ------------------------------------------------------ */
/* Advance every group by n_steps lockstep steps.
 * counters_host: nullable, [n_steps][RAFT_COUNTER_STRIDE] int64, filled in
 * step order.  Synchronous: returns after the device finished. */
int raft_engine_step(raft_engine* e, int32_t n_steps, int64_t* counters_host);
/* Same, asynchronous on the engine stream; counters_dev is a nullable
 * DEVICE pointer to [n_steps][RAFT_COUNTER_STRIDE] int64 (overwritten). */
int raft_engine_step_async(raft_engine* e, int32_t n_steps, int64_t* counters_dev);
int raft_engine_sync(raft_engine* e);
/* hipStream_t of the engine, as void* (for event timing by the caller).  Work
 * enqueued on it after a step_async sees that call's steps finished (state,
 * logs and counter rows).  With launch sub-ranges the step kernels run on the
 * engine's own side streams, which wait for this stream only where an engine
 * call other than a step enqueued work on it: caller work on this stream is
 * ordered before the counter reductions of later steps, not before their
 * step kernels (which touch only engine memory). */
void*   raft_engine_stream(raft_engine* e);
/* Kernel timing: while enabled, every step-kernel launch (of every
 * sub-range) carries its own start / stop timestamps.  raft_engine_kernel_time()
 * synchronises and returns, since the last call, the time during which at
 * least one step kernel ran (the union of the launches' intervals: sub-range
 * launches overlap) and the number of K-step launches of the whole grid, then
 * resets both.  With one sub-range the union is the sum of the launches. */
int raft_engine_set_kernel_timing(raft_engine* e, int enable);
int raft_engine_kernel_time(raft_engine* e, double* total_ms, int64_t* launches);
/* The time from the start of the first step launch timed since timing was
 * switched on (the launch's own start timestamp, carried by the dispatch: no
 * marker ahead of it) to `end_event` (a hipEvent_t the caller recorded after
 * its last launch); call before raft_engine_kernel_time, which resets the
 * timed launches. */
int raft_engine_timed_span(raft_engine* e, void* end_event, double* ms);
int64_t raft_engine_step_index(raft_engine* e);   /* steps executed so far */
/* Steps fused into one kernel launch from now on (0 = 1), at most
 * RAFT_MAX_STEPS_PER_LAUNCH.  Results do not depend on it. */
int     raft_engine_set_steps_per_launch(raft_engine* e, int32_t k);
/* Launch sub-ranges from now on (raft_params.subranges; 0 = automatic). */
int     raft_engine_set_subranges(raft_engine* e, int32_t n);
int32_t raft_engine_subranges(raft_engine* e);    /* the sub-ranges in use (-1: null engine) */
/* The step kernel and schedule of the last step launch (zeros before the first). */
int     raft_engine_kernel_info(raft_engine* e, raft_kernel_info* out);
/* The step kernel variant from now on (raft_params.kernel).  Results do not
 * depend on it. */
int     raft_engine_set_kernel(raft_engine* e, int32_t kernel);
/* Every group back to the reference's initial state at step 0, exactly as
 * raft_engine_create leaves it (RaftServer.kt:35-48, the election timers armed
 * as init does, :58). */
int     raft_engine_reset(raft_engine* e);
/* Set the index of the next step (its Philox counter c0); with write_state
 * this resumes a run exported at any step. */
int     raft_engine_set_step_index(raft_engine* e, int64_t t);
/* HBM owned by the engine: the state, logs and counter buffers, plus the
 * grow-only staging of the handler batches and accessors (kept for the
 * engine's lifetime at 1.25x the largest request; raft_engine_trim_staging
 * frees it, page-locked host staging included). */
/* ---- multi-GPU: the counter all-reduce ----------------
 * A sharded run is one engine per GPU, each owning a contiguous range of
 * global group ids (raft_params.g0); groups never exchange anything, and the
 * only cross-GPU data is the per-step counter rows, summed over the ranks by
 * RCCL (over xGMI between MI355X GPUs).  Rank 0 makes an id, the caller
 * passes it to every rank (any channel), and each rank creates its
 * communicator (a collective call: it returns once every rank has joined).
 * raft_engine_allreduce_counters enqueues the sum of n_steps counter rows
 * [n_steps][RAFT_COUNTER_STRIDE] int64 (device pointers; in place when
 * out_dev == counters_dev) on the engine's stream, after every step launch
 * already enqueued there.  RCCL is loaded at the first raft_comm call (never
 * for one-GPU use); without it these return RAFT_ENODEV. */
#define RAFT_COMM_ID_BYTES 128
typedef struct raft_comm raft_comm;
int raft_comm_get_unique_id(uint8_t id[RAFT_COMM_ID_BYTES]);
int raft_comm_create(const uint8_t id[RAFT_COMM_ID_BYTES], int32_t nranks, int32_t rank, int device, raft_comm** out);
int raft_comm_destroy(raft_comm* c);
int raft_engine_allreduce_counters(raft_engine* e, raft_comm* c, const int64_t* counters_dev, int64_t* out_dev,
                                   int32_t n_steps);

/* Traffic probe (rocprofv3 calibration; never part of a step): kind 0 moves
 * every chunk's state into registers and back exactly as a step launch's
 * piece entry and exit does (values unchanged); kind 1 makes one 8-byte store
 * per replica into its own log row past its last entry (a flat log only), the
 * Log.add pattern (Commons.kt:56-68).  Kinds 2 and 3 calibrate the handler
 * batches' scattered accesses: 2^21 threads each load (2) or store (3) one
 * 4-byte word in its own 32-byte sector of a 512 MB engine-owned scratch
 * (sectors spread by an odd multiplicative permutation; the state is not
 * touched), counted as 32 bytes per sector.  Returns the bytes the probe's one
 * dispatch reads and writes, so FETCH_SIZE / WRITE_SIZE of that dispatch
 * give the counters' byte factors for the probed access pattern. */
int raft_engine_traffic_probe(raft_engine* e, int32_t kind, int64_t* bytes_read, int64_t* bytes_written);
int64_t raft_engine_device_bytes(raft_engine* e);
int     raft_engine_trim_staging(raft_engine* e);

/* ---- state access (fixtures, parity) ----------------------------------- */
/* out: [n][raft_group_words(R)] int32, canonical layout above. */
int raft_engine_read_state(raft_engine* e, int64_t g0, int64_t n, int32_t* out);
int raft_engine_write_state(raft_engine* e, int64_t g0, int64_t n, const int32_t* in);
/* terms/cmds: [n][R][log_cap], physical slot j at [j].  read_log returns the
 * retained slots [max(0, physLen - W), physLen) and 0 elsewhere.  write_log to
 * a flat log (log_window 0) stores every slot below log_cap; with a
 * log_window W it stores only the slots [max(0, physLen - W), physLen) of the
 * physLen the engine holds at the call, so call write_state first. */
int raft_engine_read_log(raft_engine* e, int64_t g0, int64_t n, int32_t* terms, uint32_t* cmds);
int raft_engine_write_log(raft_engine* e, int64_t g0, int64_t n, const int32_t* terms, const uint32_t* cmds);
/* Order-independent 64-bit digest of the full canonical state and the
 * retained log slots [max(0, physLen - W), physLen) of every replica (W =
 * log_window, or every slot): sum over groups of a per-group hash (DESIGN.md
 * §3 S-13).  digest_range hashes groups [g0, g0 + n) only. */
int raft_engine_digest(raft_engine* e, uint64_t* out);
int raft_engine_digest_range(raft_engine* e, int64_t g0, int64_t n, uint64_t* out);

/* Log Matching over committed prefixes (safety flag): a
 * group of [g0, g0+n) is flagged when two of its replicas hold different
 * (term, cmd) at an index inside both replicas' committed prefixes, i.e.
 * i < min(commitIndex, lastIndex) of each (and, with a log_window, inside
 * both replicas' retained windows).  The reference's quirks (Q4 commit
 * clamp, Q9 no current-term guard) do not preserve this property, so the
 * count is an observation about the reference's protocol, not an engine
 * error.  *mismatched = flagged groups; flags (nullable, host, n bytes)
 * receives 1 per flagged group. */
int raft_engine_check_log_matching(raft_engine* e, int64_t g0, int64_t n, uint8_t* flags, int64_t* mismatched);

/* ---- single-handler batches: the service boundary ----------------------
 * group: engine-local group index; dst: replica index 0..R-1.  Messages
 * to the same (group, dst) are applied in batch order.  Effects on the
 * consumer (timer reset) use the engine's current step index.  With a
 * log_window, a batch in which some handler touched a slot below its
 * replica's window returns RAFT_EWINDOW after applying it. */
int raft_vote_batch(raft_engine* e, const int64_t* group, const int32_t* dst,
                    const raft_vote_req* req, raft_vote_resp* resp, int64_t n);
int raft_append_batch(raft_engine* e, const int64_t* group, const int32_t* dst,
                      const raft_append_req* req, raft_append_resp* resp, int64_t n);
/* appendCommand (RaftServer.kt:100-107): log.add(lastIndex, (currentTerm, cmd)). */
int raft_append_command_batch(raft_engine* e, const int64_t* group, const int32_t* replica,
                              const uint32_t* cmd, int64_t n);
/* Page-locked host memory for batch arrays: the host entry points above move
 * arrays that live in it by direct DMA (no staging copy; ≈3-5x the rate of
 * pageable arrays at 10^6 messages).  A JNI adapter wraps it in a direct
 * ByteBuffer.  raft_host_alloc returns NULL on failure
 * (raft_last_error() says why). */
void* raft_host_alloc(int64_t bytes);
int   raft_host_free(void* p);
/* The same three on DEVICE buffers of this engine's GPU (group, dst/replica,
 * req, resp: n entries each, in HBM), enqueued on the engine stream; they
 * return once the batch finished.  The engine stream is non-blocking: it does
 * NOT wait for work on other streams, so the device buffers must be complete
 * (and resp no longer in use) before the call -- produced on the engine
 * stream, synchronised, or ordered with raft_engine_wait_stream().  The host
 * entry points above stage their buffers through engine-owned pinned memory
 * and call these.  A message whose group or replica is outside the engine
 * makes the whole batch fail with RAFT_ERANGE before any message is applied.
 * n < 2^31. */
/* Order the engine stream after all work enqueued so far on `stream` (a
 * hipStream_t as void*, NULL = the null stream): later engine calls see that
 * work's results.  Host-side and non-blocking (an event record and wait). */
int raft_engine_wait_stream(raft_engine* e, void* stream);
int raft_vote_batch_dev(raft_engine* e, const int64_t* group, const int32_t* dst,
                        const raft_vote_req* req, raft_vote_resp* resp, int64_t n);
int raft_append_batch_dev(raft_engine* e, const int64_t* group, const int32_t* dst,
                          const raft_append_req* req, raft_append_resp* resp, int64_t n);
int raft_append_command_batch_dev(raft_engine* e, const int64_t* group, const int32_t* replica,
                                  const uint32_t* cmd, int64_t n);
/* How the batches above order messages (results never depend on it):
 * RAFT_BATCH_PATH_SORTED, a stable radix sort of every message by
 * (group, replica); RAFT_BATCH_PATH_BUCKETED, one stable partition into
 * buckets of 2^S consecutive replicas, each bucket sorted in LDS by the
 * workgroup that applies it (G * R <= 2^32 only, else RAFT_EINVAL at the
 * batch); RAFT_BATCH_PATH_AUTO (the default): bucketed where it applies. */
#define RAFT_BATCH_PATH_AUTO     0
#define RAFT_BATCH_PATH_SORTED   1
#define RAFT_BATCH_PATH_BUCKETED 2
int raft_engine_set_batch_path(raft_engine* e, int32_t path);

/* ---- Philox4x32-10 (shared bit-for-bit with the CPU harness) -----------
 * Counter = (c0 = step, c1 = global group id, c2 = purpose, c3 = sub),
 * key = (seed lo32, seed hi32).  Purposes: */
#define RAFT_RNG_TIMER        1u  /* sub = replica >> 2, word replica & 3: the replica's
                                     per-step draw, scaled to the election timeout or to
                                     the backoff (never both in one step)               */
#define RAFT_RNG_BACKOFF      2u  /* reserved (the backoff shares the timer word)      */
#define RAFT_RNG_VOTE_DROP    3u  /* sub = src | chunk << 8: 16-bit drop uniforms */
#define RAFT_RNG_APPEND_DROP  4u  /* sub = src | chunk << 8                        */
#define RAFT_RNG_HARNESS      5u  /* sub = 0: w0 churn, w1 command, w2 command id  */
#define RAFT_RNG_PARTITION    6u  /* c0 = partition window start, sub = 0: w0 mask */
#define RAFT_RNG_INIT_STEP    0xFFFFFFFFu  /* c0 of the initial timer draws        */
void raft_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif /* RAFT_ENGINE_H */
