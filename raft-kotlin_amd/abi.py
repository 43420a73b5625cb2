"""ctypes mirror of include/raft_engine.h (the engine's C-ABI).

Pure data definitions: structs, constants, and the loader of the HIP engine
library.  The loader never falls back to anything: if the in-tree
``lib/libraft_engine.so`` is missing it raises, so a GPU run cannot silently
take another path.
"""
from __future__ import annotations

import ctypes as C
import os
import warnings

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# RAFT_ENGINE_LIB selects an alternative in-tree build (tuning experiments only)
LIB_PATH = os.environ.get("RAFT_ENGINE_LIB") or os.path.join(PKG_DIR, "lib", "libraft_engine.so")

RAFT_OK = 0
RAFT_EINVAL = -1
RAFT_ENOMEM = -2
RAFT_EDEVICE = -3
RAFT_ERANGE = -4
RAFT_ENODEV = -5
RAFT_EWINDOW = -6
COMM_ID_BYTES = 128          # include/raft_engine.h RAFT_COMM_ID_BYTES

# enum class State (RaftServer.kt:24-26)
FOLLOWER, CANDIDATE, LEADER = 0, 1, 2
MAX_R = 8

CMD_LOWEST_LEADER = 0
CMD_ALL_LEADERS = 1
MODE_REFERENCE = 0
MODE_TEXTBOOK = 1

COUNTER_NAMES = [
    "leaders", "groups_with_leader", "timeouts", "rounds", "votes_granted",
    "leaders_elected", "sessions_ticked", "append_sent", "append_skipped",
    "entries_acked", "commits", "msg_dropped", "commands", "commit_regressions",
    "dual_leader_groups", "log_overflow", "prev_reads_leader",
    "entry_reads_leader", "prev_reads_follower", "entry_writes", "vote_log_reads", "log_window_miss",
]
NUM_COUNTERS = len(COUNTER_NAMES)
COUNTER_STRIDE = 32
MAX_STEPS_PER_LAUNCH = 16384          # include/raft_engine.h RAFT_MAX_STEPS_PER_LAUNCH
# the longest launch whose counter rows stay in LDS for the whole launch
# (raft_engine.hip LDS_MAX_STEPS); a longer one runs as 400-step epochs when
# its schedule is balanced on one sub-range in the reference mode (not a
# partitions-only kernel), else the engine cuts it to this
LDS_MAX_STEPS_PER_LAUNCH = 512
# bench.py's launch length for the step kernels built for 7 waves per SIMD
# (R <= 5, or R = 7 without drops; RAFT_STEP_WAVES_PER_EU in raft_engine.hip):
# the longest that keeps 7 step workgroups per CU within the LDS (STEP_K_7WG,
# 429 steps).  The other kernels run 6 workgroups per CU at any length and
# take the longest LDS launch.
BENCH_STEPS_PER_LAUNCH = 400
# bench.py's launch length where the engine runs epochs: the whole default run
# in one launch (a launch boundary costs ~36 us / sqrt(K) of the waves'
# uneven work; an epoch boundary only waits for a workgroup's own waves)
LONG_STEPS_PER_LAUNCH = 10_000


# The network faults (and command harness) a step kernel is built for
# (raft_step.h NET_*): at R = 3, 5, 7 the engine runs a kernel for drops +
# isolation churn without partitions with config 3's command harness (lowest
# LEADER, no limit), or for partitions alone (configs 5, 2, 1), the other
# checks compiled out; else the NET_ALL kernel
NET_DROP, NET_PART, NET_ISO, NET_CMDLOW = 1, 2, 4, 8
NET_ALL = NET_DROP | NET_PART | NET_ISO


def step_net(R: int, drop_ppm: int = 0, partition_period: int = 0, partition_len: int = 0,
             churn_ppm: int = 0, iso_written: bool = False, cmd_mode: int = 0, cmd_limit: int = 0) -> int:
    """The NET of the step kernel the engine launches (raft_engine.hip step_fn);
    iso_written: an isolation word was written into the state."""
    drops, parts = drop_ppm > 0, partition_period > 0 and partition_len > 0
    iso = churn_ppm > 0 or iso_written
    cmdlow = cmd_mode == CMD_LOWEST_LEADER and cmd_limit == 0
    if R in (3, 5, 7):
        if drops and not parts and cmdlow:
            return NET_DROP | NET_ISO | NET_CMDLOW
        if not drops and not iso:
            return NET_PART
    return NET_ALL


def step_net_of(kw: dict) -> int:
    """step_net of a raft_params keyword dict (abi.CONFIGS entries)."""
    return step_net(kw["R"], kw.get("drop_ppm", 0), kw.get("partition_period", 0), kw.get("partition_len", 0),
                    kw.get("churn_ppm", 0), cmd_mode=kw.get("cmd_mode", CMD_LOWEST_LEADER),
                    cmd_limit=kw.get("cmd_limit", 0))


def bench_steps_per_launch(R: int, mode: int = 0, log_window: int = 0, net: int = NET_ALL, groups: int = 0,
                           simds: int = 1024) -> int:
    """Default fused launch length of bench.py for a kernel variant:
    LONG_STEPS_PER_LAUNCH where the engine runs a long launch as epochs (the
    reference mode, one launch sub-range -- not a partitions-only kernel --
    and a balanced schedule: more chunks of 64 // R groups than the resident
    wave slots of `simds` SIMDs); else 400 for the 7-waves-per-SIMD kernels (R
    <= 5, or R = 7 built for partitions only; either protocol mode, flat log or
    ring), the longest LDS launch for the others."""
    seven = R <= 5 or (R == 7 and net == NET_PART)
    balanced = -(-groups // (64 // R)) > simds * (7 if seven else 6)
    if mode == MODE_REFERENCE and net != NET_PART and balanced:
        return LONG_STEPS_PER_LAUNCH
    return BENCH_STEPS_PER_LAUNCH if seven else LDS_MAX_STEPS_PER_LAUNCH
MAX_AE_ENTRIES = 8           # include/raft_engine.h RAFT_MAX_AE_ENTRIES
C_INDEX = {n: i for i, n in enumerate(COUNTER_NAMES)}

FIELD_NAMES = ["term", "voted", "role", "commit", "last", "phys",
               "election_ms", "flags", "phase_ms", "retry_ms"]
NUM_FIELDS = len(FIELD_NAMES)
# the engine's HBM state per replica: 4 quads of int32 (the 10 fields, the
# log-tail cache and the primary session column; raft_step.h FIELD_SLOT), and
# per group: 3 harness words
REPLICA_STATE_BYTES, GROUP_STATE_BYTES = 64, 12
F_INDEX = {n: i for i, n in enumerate(FIELD_NAMES)}
FL_ARMED, FL_ELECTING, FL_PENDING_RST, FL_HB_ACTIVE, FL_BACKOFF = 1, 2, 4, 8, 16
GROUP_EXTRA = 2


def group_words(R: int) -> int:
    return R * NUM_FIELDS + 2 * R * R + GROUP_EXTRA


class raft_params(C.Structure):
    _fields_ = [
        ("R", C.c_int32), ("log_cap", C.c_int32), ("G", C.c_int64), ("g0", C.c_int64),
        ("seed", C.c_uint64),
        ("heartbeat_ms", C.c_int32), ("election_min_ms", C.c_int32), ("election_max_ms", C.c_int32),
        ("backoff_min_ms", C.c_int32), ("backoff_max_ms", C.c_int32),
        ("round_timeout_ms", C.c_int32), ("retry_ms", C.c_int32),
        ("drop_ppm", C.c_uint32), ("churn_ppm", C.c_uint32), ("churn_steps", C.c_int32),
        ("partition_period", C.c_int32), ("partition_len", C.c_int32),
        ("cmd_ppm", C.c_uint32), ("cmd_mode", C.c_int32), ("cmd_limit", C.c_int32),
        ("steps_per_launch", C.c_int32), ("mode", C.c_int32), ("log_window", C.c_int32),
        ("ae_max_entries", C.c_int32), ("subranges", C.c_int32), ("schedule", C.c_int32),
        ("schedule_workgroups", C.c_int32), ("kernel", C.c_int32),
    ]


# step-kernel schedules (raft_params.schedule)
SCHED_AUTO, SCHED_ONE_PER_WAVE, SCHED_BALANCED = 0, 1, 2
# step-kernel variant (raft_params.kernel): built for the workload, or the general one
KERNEL_AUTO, KERNEL_GENERAL = 0, 1
# raft_engine_set_batch_path
BATCH_PATH_AUTO, BATCH_PATH_SORTED, BATCH_PATH_BUCKETED = 0, 1, 2


class raft_kernel_info(C.Structure):
    _fields_ = [("net", C.c_int32), ("textbook", C.c_int32), ("ring", C.c_int32), ("steps", C.c_int32),
                ("workgroups", C.c_int32), ("resident_workgroups", C.c_int32), ("balanced", C.c_int32),
                ("subranges", C.c_int32), ("reserved", C.c_int32 * 4)]


class raft_vote_req(C.Structure):
    _fields_ = [("term", C.c_int32), ("candidate_id", C.c_int32),
                ("last_log_index", C.c_int32), ("last_log_term", C.c_int32)]


class raft_vote_resp(C.Structure):
    _fields_ = [("term", C.c_int32), ("vote_granted", C.c_int32)]


class raft_append_req(C.Structure):
    _fields_ = [("term", C.c_int32), ("leader_id", C.c_int32), ("prev_log_index", C.c_int32),
                ("prev_log_term", C.c_int32), ("has_entry", C.c_int32), ("entry_term", C.c_int32),
                ("entry_cmd", C.c_uint32), ("leader_commit", C.c_int32)]


class raft_append_resp(C.Structure):
    _fields_ = [("term", C.c_int32), ("success", C.c_int32), ("status", C.c_int32)]


# the reference's hard-coded constants
DEFAULTS = dict(
    heartbeat_ms=2000,        # RaftServer.kt:115
    election_min_ms=20000,    # Commons.kt:23
    election_max_ms=23000,
    backoff_min_ms=2000,      # RaftServer.kt:221
    backoff_max_ms=3000,
    round_timeout_ms=25000,   # RaftServer.kt:189, :214
    retry_ms=5000,            # Commons.kt:37
)

# BASELINE.json configs; G/steps are the full sizes
CONFIGS = {
    1: dict(R=5, G=1, seed=1, cmd_ppm=1_000_000, cmd_mode=CMD_LOWEST_LEADER, cmd_limit=1000),
    2: dict(R=3, G=10_000, seed=2, cmd_ppm=250_000, cmd_mode=CMD_LOWEST_LEADER),
    3: dict(R=5, G=1_000_000, seed=3, drop_ppm=50_000, churn_ppm=1_000, churn_steps=15,
            cmd_ppm=250_000, cmd_mode=CMD_LOWEST_LEADER),
    5: dict(R=7, G=100_000, seed=5, partition_period=50, partition_len=25,
            cmd_ppm=1_000_000, cmd_mode=CMD_ALL_LEADERS),
}
CONFIG_STEPS = {1: None, 2: 1_000, 3: 10_000, 5: 10_000}


def make_params(**kw) -> raft_params:
    """raft_params with the reference defaults; keyword overrides."""
    p = raft_params()
    p.R = 5
    p.log_cap = 1024
    p.G = 1
    p.g0 = 0
    p.seed = 1
    for k, v in DEFAULTS.items():
        setattr(p, k, v)
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError(f"unknown raft_params field {k!r}")
        setattr(p, k, v)
    return p


def config_params(cfg: int, **kw) -> raft_params:
    d = dict(CONFIGS[cfg])
    d.update(kw)
    return make_params(**d)


def counters_array(n_steps: int) -> np.ndarray:
    return np.zeros((n_steps, COUNTER_STRIDE), dtype=np.int64)


def ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


_lib = None


def _missing_entry(name: str):
    def stub(*_a, **_k):
        raise RuntimeError(f"{name} is not in this engine build (RAFT_ENGINE_LIB={os.environ.get('RAFT_ENGINE_LIB')})")
    return stub


def check_build(lib, p: str) -> None:
    """Refuse an engine library that was not built from the sources beside it
    (build.py compiles library_source_id() into it): a stale binary would make
    every measurement and parity result describe other code.  Skipped when
    the sources are absent (an installed library)."""
    from . import build as B
    if not B.sources_present():
        return
    lib.raft_build_source_id.restype = C.c_char_p
    have = lib.raft_build_source_id().decode()
    want = B.library_source_id()
    if have != want:
        raise RuntimeError(f"{p} was built from sources {have}, the working tree is {want}: rebuild it "
                           "(`python raft-kotlin_amd/build.py`)")


def build_ids() -> dict:
    """The loaded library's provenance (include/raft_engine.h raft_build_*)."""
    lib = load_library()
    return {"library_source_id": lib.raft_build_source_id().decode(),
            "kernel_source_id": lib.raft_build_kernel_source_id().decode(),
            "batch_source_id": lib.raft_build_batch_source_id().decode(), "path": LIB_PATH}


def load_library(path: str | None = None):
    """Load the HIP engine.  Raises if it is absent: there is no fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            f"HIP engine library not built: {p} (run `python __graft_entry__.py build` "
            "or `python raft-kotlin_amd/build.py`)")
    lib = C.CDLL(p)
    if path is None and not os.environ.get("RAFT_ENGINE_LIB"):
        check_build(lib, p)
    P, I32, I64, U64 = C.POINTER, C.c_int32, C.c_int64, C.c_uint64
    eng = C.c_void_p
    sig = {
        "raft_params_default": (None, [P(raft_params)]),
        "raft_last_error": (C.c_char_p, []),
        "raft_abi_version": (C.c_int, []),
        "raft_build_source_id": (C.c_char_p, []),
        "raft_build_kernel_source_id": (C.c_char_p, []),
        "raft_build_batch_source_id": (C.c_char_p, []),
        "raft_engine_create": (C.c_int, [P(raft_params), C.c_int, P(eng)]),
        "raft_engine_destroy": (C.c_int, [eng]),
        "raft_engine_step": (C.c_int, [eng, I32, P(I64)]),
        "raft_engine_step_async": (C.c_int, [eng, I32, C.c_void_p]),
        "raft_engine_sync": (C.c_int, [eng]),
        "raft_engine_stream": (C.c_void_p, [eng]),
        "raft_engine_set_kernel_timing": (C.c_int, [eng, C.c_int]),
        "raft_engine_kernel_time": (C.c_int, [eng, P(C.c_double), P(I64)]),
        "raft_engine_timed_span": (C.c_int, [eng, C.c_void_p, P(C.c_double)]),
        "raft_engine_step_index": (I64, [eng]),
        "raft_engine_set_step_index": (C.c_int, [eng, I64]),
        "raft_engine_set_steps_per_launch": (C.c_int, [eng, I32]),
        "raft_engine_set_subranges": (C.c_int, [eng, I32]),
        "raft_engine_subranges": (I32, [eng]),
        "raft_engine_kernel_info": (C.c_int, [eng, P(raft_kernel_info)]),
        "raft_engine_wait_stream": (C.c_int, [eng, C.c_void_p]),
        "raft_engine_set_kernel": (C.c_int, [eng, I32]),
        "raft_engine_set_batch_path": (C.c_int, [eng, I32]),
        "raft_engine_reset": (C.c_int, [eng]),
        "raft_engine_trim_staging": (C.c_int, [eng]),
        "raft_engine_device_bytes": (I64, [eng]),
        "raft_engine_read_state": (C.c_int, [eng, I64, I64, P(I32)]),
        "raft_engine_write_state": (C.c_int, [eng, I64, I64, P(I32)]),
        "raft_engine_read_log": (C.c_int, [eng, I64, I64, P(I32), P(C.c_uint32)]),
        "raft_engine_write_log": (C.c_int, [eng, I64, I64, P(I32), P(C.c_uint32)]),
        "raft_engine_digest": (C.c_int, [eng, P(U64)]),
        "raft_engine_digest_range": (C.c_int, [eng, I64, I64, P(U64)]),
        "raft_engine_check_log_matching": (C.c_int, [eng, I64, I64, P(C.c_uint8), P(I64)]),
        "raft_engine_traffic_probe": (C.c_int, [eng, I32, P(I64), P(I64)]),
        "raft_comm_get_unique_id": (C.c_int, [P(C.c_uint8)]),
        "raft_comm_create": (C.c_int, [P(C.c_uint8), I32, I32, C.c_int, P(C.c_void_p)]),
        "raft_comm_destroy": (C.c_int, [C.c_void_p]),
        "raft_engine_allreduce_counters": (C.c_int, [eng, C.c_void_p, C.c_void_p, C.c_void_p, I32]),
        "raft_vote_batch": (C.c_int, [eng, P(I64), P(I32), P(raft_vote_req), P(raft_vote_resp), I64]),
        "raft_append_batch": (C.c_int, [eng, P(I64), P(I32), P(raft_append_req), P(raft_append_resp), I64]),
        "raft_append_command_batch": (C.c_int, [eng, P(I64), P(I32), P(C.c_uint32), I64]),
        "raft_vote_batch_dev": (C.c_int, [eng, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, I64]),
        "raft_append_batch_dev": (C.c_int, [eng, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, I64]),
        "raft_append_command_batch_dev": (C.c_int, [eng, C.c_void_p, C.c_void_p, C.c_void_p, I64]),
        "raft_philox4x32_10": (None, [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]),
        "raft_host_alloc": (C.c_void_p, [I64]),
        "raft_host_free": (C.c_int, [C.c_void_p]),
        # include/raft_wire.h
        "raft_wire_decode_vote_req": (C.c_int, [P(C.c_uint8), P(I64), I64, P(raft_vote_req)]),
        "raft_wire_encode_vote_req": (I64, [P(raft_vote_req), I64, P(C.c_uint8), I64, P(I64)]),
        "raft_wire_decode_vote_resp": (C.c_int, [P(C.c_uint8), P(I64), I64, P(raft_vote_resp)]),
        "raft_wire_encode_vote_resp": (I64, [P(raft_vote_resp), I64, P(C.c_uint8), I64, P(I64)]),
        "raft_wire_decode_append_req": (C.c_int, [P(C.c_uint8), P(I64), I64, P(raft_append_req), P(I64), P(I32),
                                                  P(I32)]),
        "raft_wire_encode_append_req": (I64, [P(raft_append_req), P(C.c_uint8), P(I64), I64, P(C.c_uint8), I64,
                                              P(I64)]),
        "raft_wire_decode_append_resp": (C.c_int, [P(C.c_uint8), P(I64), I64, P(raft_append_resp)]),
        "raft_wire_encode_append_resp": (I64, [P(raft_append_resp), I64, P(C.c_uint8), I64, P(I64)]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("RAFT_ENGINE_LIB") and not hasattr(lib, name):
            # an older experimental build (RAFT_ENGINE_LIB) may lack newer
            # entry points: bind a stub that says so when it is called
            warnings.warn(f"{path or os.environ['RAFT_ENGINE_LIB']}: no {name}; calls to it will raise", stacklevel=2)
            setattr(lib, name, _missing_entry(name))
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib if path is None else _lib
    return lib


# symbols declared in include/*.h (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = [
    "raft_params_default", "raft_last_error", "raft_abi_version", "raft_build_source_id",
    "raft_build_kernel_source_id", "raft_build_batch_source_id", "raft_engine_create",
    "raft_engine_destroy", "raft_engine_step", "raft_engine_step_async", "raft_engine_sync",
    "raft_engine_stream", "raft_engine_set_kernel_timing", "raft_engine_kernel_time", "raft_engine_timed_span",
    "raft_engine_step_index", "raft_engine_set_step_index", "raft_engine_set_steps_per_launch",
    "raft_engine_set_subranges", "raft_engine_subranges", "raft_engine_kernel_info", "raft_engine_wait_stream",
    "raft_engine_set_kernel", "raft_engine_set_batch_path", "raft_engine_reset", "raft_engine_trim_staging",
    "raft_engine_device_bytes",
    "raft_engine_read_state", "raft_engine_write_state", "raft_engine_read_log",
    "raft_engine_write_log", "raft_engine_digest", "raft_engine_digest_range", "raft_engine_check_log_matching", "raft_engine_traffic_probe",
    "raft_comm_get_unique_id", "raft_comm_create", "raft_comm_destroy", "raft_engine_allreduce_counters", "raft_vote_batch", "raft_append_batch",
    "raft_append_command_batch", "raft_vote_batch_dev", "raft_append_batch_dev", "raft_append_command_batch_dev",
    "raft_philox4x32_10", "raft_host_alloc", "raft_host_free",
    # include/raft_wire.h
    "raft_wire_decode_vote_req", "raft_wire_encode_vote_req", "raft_wire_decode_vote_resp",
    "raft_wire_encode_vote_resp", "raft_wire_decode_append_req", "raft_wire_encode_append_req",
    "raft_wire_decode_append_resp", "raft_wire_encode_append_resp",
]
