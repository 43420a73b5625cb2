"""RaftEngine — host-side handle of the HIP batched Raft engine (C-ABI in include/raft_engine.h).

One engine owns G groups x R replicas of Raft node state in the HBM of one
GPU.  ``step(n)`` advances every group by n lockstep heartbeat periods, which
is what each reference node does on its own timers
(RaftServer.kt:109-226, Commons.kt:10-31); the handler batches are the
reference's gRPC service (RaftServer.vote / RaftServer.append,
RaftServer.kt:228-287) applied to chosen replicas.

There is no CPU fallback anywhere in this module: every call goes to the HIP
library and a missing library or device raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


class RaftError(RuntimeError):
    pass


class RaftComm:
    """An RCCL communicator for the counter all-reduce of a sharded run
    (include/raft_engine.h raft_comm_*): rank 0 makes `unique_id()`, every
    rank gets it (any channel) and constructs RaftComm(uid, nranks, rank,
    device); construction returns once every rank has joined."""

    @staticmethod
    def unique_id() -> bytes:
        lib = abi.load_library()
        buf = (C.c_uint8 * abi.COMM_ID_BYTES)()
        if lib.raft_comm_get_unique_id(buf) != abi.RAFT_OK:
            raise RaftError("raft_comm_get_unique_id: " + lib.raft_last_error().decode(errors="replace"))
        return bytes(buf)

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int = 0):
        self._lib = abi.load_library()
        if len(uid) != abi.COMM_ID_BYTES:
            raise ValueError(f"a communicator id is {abi.COMM_ID_BYTES} bytes")
        buf = (C.c_uint8 * abi.COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        if self._lib.raft_comm_create(buf, nranks, rank, device, C.byref(h)) != abi.RAFT_OK:
            raise RaftError("raft_comm_create: " + self._lib.raft_last_error().decode(errors="replace"))
        self._h = h
        self.nranks, self.rank, self.device = nranks, rank, device

    def close(self):
        if getattr(self, "_h", None):
            self._lib.raft_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RaftEngine:
    def __init__(self, params: abi.raft_params, device: int = 0):
        self._lib = abi.load_library()
        self.p = params
        self.R = int(params.R)
        self.G = int(params.G)
        self.g0 = int(params.g0)
        self.cap = int(params.log_cap)
        self.W = abi.group_words(self.R)
        self.device = device
        h = C.c_void_p()
        self._check(self._lib.raft_engine_create(C.byref(params), device, C.byref(h)), "raft_engine_create")
        self._h = h

    # -- plumbing ---------------------------------------------------------
    def _check(self, rc: int, what: str):
        if rc != abi.RAFT_OK:
            msg = self._lib.raft_last_error().decode(errors="replace")
            raise RaftError(f"{what} failed ({rc}): {msg}")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.raft_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def stream(self) -> int:
        """hipStream_t of the engine (for torch.cuda.ExternalStream / events)."""
        return int(self._lib.raft_engine_stream(self._h) or 0)

    @property
    def step_index(self) -> int:
        return int(self._lib.raft_engine_step_index(self._h))

    @step_index.setter
    def step_index(self, t: int):
        self._check(self._lib.raft_engine_set_step_index(self._h, int(t)), "set_step_index")

    def set_steps_per_launch(self, k: int):
        """Steps fused into one kernel launch from now on (results do not depend on it)."""
        self._check(self._lib.raft_engine_set_steps_per_launch(self._h, int(k)), "set_steps_per_launch")

    @property
    def subranges(self) -> int:
        """Launch sub-ranges in use (raft_params.subranges; streams per launch).
        An older experimental build (RAFT_ENGINE_LIB) without them: 1."""
        if getattr(self._lib.raft_engine_subranges, "__name__", "") == "stub":
            return 1
        return int(self._lib.raft_engine_subranges(self._h))

    def set_subranges(self, n: int):
        """Split the step launches over n sub-range streams (0 = automatic)."""
        if getattr(self._lib.raft_engine_set_subranges, "__name__", "") == "stub":
            return                                   # an older experimental build: one range
        self._check(self._lib.raft_engine_set_subranges(self._h, int(n)), "set_subranges")

    def set_kernel(self, kernel: int):
        """The step kernel variant from now on (abi.KERNEL_AUTO / KERNEL_GENERAL;
        results do not depend on it)."""
        self._check(self._lib.raft_engine_set_kernel(self._h, int(kernel)), "set_kernel")

    def set_batch_path(self, path: int):
        """How the handler batches order their messages (abi.BATCH_PATH_AUTO /
        _SORTED / _BUCKETED; results do not depend on it)."""
        self._check(self._lib.raft_engine_set_batch_path(self._h, int(path)), "set_batch_path")
        self._batch_path = int(path)

    @property
    def batch_path(self) -> int:
        """The batch path set with set_batch_path (abi.BATCH_PATH_AUTO unless set)."""
        return getattr(self, "_batch_path", abi.BATCH_PATH_AUTO)

    def reset(self):
        """Every group back to its initial state at step 0 (as created)."""
        self._check(self._lib.raft_engine_reset(self._h), "reset")

    def kernel_info(self) -> dict:
        """The step kernel and schedule of the last step launch
        (raft_engine_kernel_info): net (raft_step.h NET_* bits), textbook, ring,
        steps, workgroups, resident_workgroups, balanced (sub-ranges on the
        balanced schedule), subranges."""
        k = abi.raft_kernel_info()
        self._check(self._lib.raft_engine_kernel_info(self._h, C.byref(k)), "kernel_info")
        return {n: int(getattr(k, n)) for n, _ in abi.raft_kernel_info._fields_ if n != "reserved"}

    @property
    def device_bytes(self) -> int:
        """HBM owned by the engine, the batch / accessor staging included."""
        return int(self._lib.raft_engine_device_bytes(self._h))

    def trim_staging(self):
        """Free the grow-only staging of the handler batches and accessors."""
        self._check(self._lib.raft_engine_trim_staging(self._h), "trim_staging")

    # -- the hot path -----------------------------------------------------
    def step(self, n: int = 1, counters: bool = True) -> np.ndarray | None:
        """Advance n lockstep steps; returns [n, NUM_COUNTERS] int64 counters."""
        c = abi.counters_array(n) if counters else None
        self._check(self._lib.raft_engine_step(self._h, n, abi.ptr(c, C.c_int64) if c is not None else None),
                    "raft_engine_step")
        return c[:, : abi.NUM_COUNTERS] if c is not None else None

    def step_async(self, n: int, counters_dev_ptr: int | None = None):
        """Enqueue n steps on the engine stream; counters to a device buffer
        of [n][COUNTER_STRIDE] int64 (e.g. a torch tensor's data_ptr())."""
        self._check(self._lib.raft_engine_step_async(self._h, n, C.c_void_p(counters_dev_ptr or 0)),
                    "raft_engine_step_async")

    def set_kernel_timing(self, enable: bool = True):
        """Bracket every step-kernel launch with HIP events on the engine stream."""
        self._check(self._lib.raft_engine_set_kernel_timing(self._h, int(enable)), "set_kernel_timing")

    def kernel_time(self):
        """(summed step-kernel ms, launches) since the last call; synchronises."""
        ms, n = C.c_double(), C.c_int64()
        self._check(self._lib.raft_engine_kernel_time(self._h, C.byref(ms), C.byref(n)), "kernel_time")
        return float(ms.value), int(n.value)

    def sync(self):
        self._check(self._lib.raft_engine_sync(self._h), "raft_engine_sync")

    # -- state ------------------------------------------------------------
    def read_state(self, g0: int = 0, n: int | None = None) -> np.ndarray:
        n = self.G - g0 if n is None else n
        out = np.zeros((n, self.W), dtype=np.int32)
        self._check(self._lib.raft_engine_read_state(self._h, g0, n, abi.ptr(out, C.c_int32)), "read_state")
        return out

    def write_state(self, state: np.ndarray, g0: int = 0):
        s = np.ascontiguousarray(state, dtype=np.int32).reshape(-1, self.W)
        self._check(self._lib.raft_engine_write_state(self._h, g0, s.shape[0], abi.ptr(s, C.c_int32)),
                    "write_state")

    def read_log(self, g0: int = 0, n: int | None = None):
        n = self.G - g0 if n is None else n
        t = np.zeros((n, self.R, self.cap), dtype=np.int32)
        c = np.zeros((n, self.R, self.cap), dtype=np.uint32)
        self._check(self._lib.raft_engine_read_log(self._h, g0, n, abi.ptr(t, C.c_int32), abi.ptr(c, C.c_uint32)),
                    "read_log")
        return t, c

    def write_log(self, terms: np.ndarray, cmds: np.ndarray, g0: int = 0):
        t = np.ascontiguousarray(terms, dtype=np.int32)
        c = np.ascontiguousarray(cmds, dtype=np.uint32)
        # the C side reads n * R * log_cap words from both arrays
        if t.ndim != 3 or t.shape[1:] != (self.R, self.cap) or c.shape != t.shape:
            raise ValueError(f"write_log: terms {t.shape} and cmds {c.shape} must both be (n, {self.R}, {self.cap})")
        self._check(self._lib.raft_engine_write_log(self._h, g0, t.shape[0], abi.ptr(t, C.c_int32),
                                                    abi.ptr(c, C.c_uint32)), "write_log")

    def digest(self) -> int:
        out = C.c_uint64()
        self._check(self._lib.raft_engine_digest(self._h, C.byref(out)), "digest")
        return int(out.value)

    def digest_range(self, g0: int, n: int) -> int:
        """The digest of groups [g0, g0 + n) only."""
        out = C.c_uint64()
        self._check(self._lib.raft_engine_digest_range(self._h, g0, n, C.byref(out)), "digest_range")
        return int(out.value)

    def check_log_matching(self, g0: int = 0, n: int | None = None, flags: bool = False):
        """Groups whose replicas disagree inside their common committed prefix
        (safety flag, include/raft_engine.h); returns the count, or (count,
        per-group uint8 flags) with flags=True."""
        n = self.G - g0 if n is None else n
        f = np.zeros(n, dtype=np.uint8) if flags else None
        out = C.c_int64()
        self._check(self._lib.raft_engine_check_log_matching(self._h, g0, n, abi.ptr(f, C.c_uint8) if flags else None,
                                                             C.byref(out)), "check_log_matching")
        return (int(out.value), f) if flags else int(out.value)

    def allreduce_counters(self, comm: RaftComm, counters_ptr: int, out_ptr: int, n_steps: int):
        """raft_engine_allreduce_counters: the sum over the ranks of n_steps
        counter rows (DEVICE pointers, [n_steps][COUNTER_STRIDE] int64; in
        place when out_ptr == counters_ptr), enqueued on the engine stream
        after its step launches."""
        self._check(self._lib.raft_engine_allreduce_counters(self._h, comm._h, C.c_void_p(counters_ptr),
                                                             C.c_void_p(out_ptr), int(n_steps)),
                    "raft_engine_allreduce_counters")

    def timed_span(self, end_event_ptr: int) -> float:
        """raft_engine_timed_span: ms from the first timed step launch's start to
        the caller's event (e.g. torch.cuda.Event.cuda_event); call before
        kernel_time()."""
        ms = C.c_double()
        self._check(self._lib.raft_engine_timed_span(self._h, C.c_void_p(end_event_ptr), C.byref(ms)), "timed_span")
        return float(ms.value)

    def traffic_probe(self, kind: int) -> tuple[int, int]:
        """raft_engine_traffic_probe: one dispatch of the step kernel's own HBM
        access pattern (kind 0: the state into registers and back; kind 1: one
        8-byte log store per replica, flat logs only); returns (bytes read,
        bytes written) for calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE."""
        r, w = C.c_int64(), C.c_int64()
        self._check(self._lib.raft_engine_traffic_probe(self._h, int(kind), C.byref(r), C.byref(w)), "traffic_probe")
        return int(r.value), int(w.value)

    # -- the service boundary (RaftServer.kt:228-287, :100-107) -------------
    @staticmethod
    def _batch_index(group, dst, n: int, what: str):
        """group / dst as contiguous int64 / int32 vectors of exactly n entries
        (the C side reads n of each)."""
        g = np.ascontiguousarray(group, dtype=np.int64)
        d = np.ascontiguousarray(dst, dtype=np.int32)
        if g.ndim != 1 or d.ndim != 1 or g.shape[0] != n or d.shape[0] != n:
            raise ValueError(f"{what}: group {g.shape} and replica {d.shape} must be 1-D with {n} entries")
        return g, d

    @staticmethod
    def _batch_out(out, n: int, w: int, what: str) -> np.ndarray:
        """The response array: a new [n, w] int32 array, or the caller's (e.g. a
        view of page-locked memory, which the engine's DMA writes directly)."""
        if out is None:
            return np.zeros((n, w), dtype=np.int32)
        if out.dtype != np.int32 or out.shape != (n, w) or not out.flags.c_contiguous:
            raise ValueError(f"{what}: out must be a C-contiguous int32 array of shape {(n, w)}")
        return out

    def vote_batch(self, group, dst, req: np.ndarray, out: np.ndarray | None = None) -> np.ndarray:
        """req: [n, 4] int32 (term, candidateId, lastLogIndex, lastLogTerm) ->
        [n, 2] int32 (term, voteGranted), into `out` when given.  Page-locked
        arrays (all four) are moved by DMA with no staging copy."""
        q = np.ascontiguousarray(req, dtype=np.int32).reshape(-1, 4)
        g, d = self._batch_index(group, dst, q.shape[0], "vote_batch")
        out = self._batch_out(out, q.shape[0], 2, "vote_batch")
        self._check(self._lib.raft_vote_batch(self._h, abi.ptr(g, C.c_int64), abi.ptr(d, C.c_int32),
                                              abi.ptr(q, abi.raft_vote_req), abi.ptr(out, abi.raft_vote_resp),
                                              q.shape[0]), "raft_vote_batch")
        return out

    def append_batch(self, group, dst, req: np.ndarray, out: np.ndarray | None = None) -> np.ndarray:
        """req: [n, 8] int32 (term, leaderId, prevLogIndex, prevLogTerm, hasEntry,
        entryTerm, entryCmd(u32 bits), leaderCommit) -> [n, 3] (term, success, status),
        into `out` when given."""
        req = np.asarray(req)
        if req.dtype == np.int32 or req.dtype == np.uint32:       # already the struct's 32-bit words
            q = np.ascontiguousarray(req).view(np.int32).reshape(-1, 8)
        else:
            q = np.ascontiguousarray(req).astype(np.int64).astype(np.uint32).view(np.int32).reshape(-1, 8)
        g, d = self._batch_index(group, dst, q.shape[0], "append_batch")
        out = self._batch_out(out, q.shape[0], 3, "append_batch")
        self._check(self._lib.raft_append_batch(self._h, abi.ptr(g, C.c_int64), abi.ptr(d, C.c_int32),
                                                abi.ptr(q, abi.raft_append_req), abi.ptr(out, abi.raft_append_resp),
                                                q.shape[0]), "raft_append_batch")
        return out

    def append_command_batch(self, group, replica, cmd):
        c = np.ascontiguousarray(cmd, dtype=np.uint32)
        if c.ndim != 1:
            raise ValueError(f"append_command_batch: cmd {c.shape} must be 1-D")
        g, r = self._batch_index(group, replica, c.shape[0], "append_command_batch")
        self._check(self._lib.raft_append_command_batch(self._h, abi.ptr(g, C.c_int64), abi.ptr(r, C.c_int32),
                                                        abi.ptr(c, C.c_uint32), c.shape[0]),
                    "raft_append_command_batch")


    # -- the same batches on device buffers (HBM-resident inputs) ------------
    # The engine stream does not wait for other streams: the buffers must be
    # complete before the call.  `after_stream` (a hipStream_t handle, e.g.
    # torch.cuda.current_stream().cuda_stream) orders the batch after all work
    # enqueued on that stream so far (raft_engine_wait_stream).
    def wait_stream(self, stream: int | None):
        """Order the engine stream after all work enqueued so far on `stream`
        (None / 0: the null stream)."""
        self._check(self._lib.raft_engine_wait_stream(self._h, C.c_void_p(stream or 0)), "wait_stream")

    def vote_batch_dev(self, group_ptr: int, dst_ptr: int, req_ptr: int, resp_ptr: int, n: int,
                       after_stream: int | None = None):
        """raft_vote_batch_dev: DEVICE pointers to n int64 groups, int32
        replicas, raft_vote_req and raft_vote_resp (e.g. torch tensors'
        data_ptr() on this engine's GPU)."""
        if after_stream is not None:
            self.wait_stream(after_stream)
        self._check(self._lib.raft_vote_batch_dev(self._h, group_ptr, dst_ptr, req_ptr, resp_ptr, int(n)),
                    "raft_vote_batch_dev")

    def append_batch_dev(self, group_ptr: int, dst_ptr: int, req_ptr: int, resp_ptr: int, n: int,
                         after_stream: int | None = None):
        if after_stream is not None:
            self.wait_stream(after_stream)
        self._check(self._lib.raft_append_batch_dev(self._h, group_ptr, dst_ptr, req_ptr, resp_ptr, int(n)),
                    "raft_append_batch_dev")

    def append_command_batch_dev(self, group_ptr: int, replica_ptr: int, cmd_ptr: int, n: int,
                                 after_stream: int | None = None):
        if after_stream is not None:
            self.wait_stream(after_stream)
        self._check(self._lib.raft_append_command_batch_dev(self._h, group_ptr, replica_ptr, cmd_ptr, int(n)),
                    "raft_append_command_batch_dev")


def philox4x32_10(ctr, key):
    """The engine's Philox (host side of the shared header), for KAT checks."""
    lib = abi.load_library()
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    out = (C.c_uint32 * 4)()
    lib.raft_philox4x32_10(c, k, out)
    return list(out)
