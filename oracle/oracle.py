"""TEST INFRASTRUCTURE ONLY: ctypes driver for the CPU oracle (oracle/lib/liboracle.so).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker; never by the product package.  Mirrors the engine's Python surface
(step / read_state / read_log / digest / handler batches) so parity tests can
run both side by side.
"""
from __future__ import annotations

import ctypes as C
import importlib
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "lib", "liboracle.so")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
abi = importlib.import_module("raft-kotlin_amd.abi")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P, I32, I64, U32 = C.POINTER, C.c_int32, C.c_int64, C.c_uint32
        o = C.c_void_p
        sig = {
            "oracle_create": (C.c_int, [P(abi.raft_params), P(o)]),
            "oracle_destroy": (None, [o]),
            "oracle_step": (C.c_int, [o, I32, P(I64), I32]),
            "oracle_step_index": (I64, [o]),
            "oracle_set_step_index": (C.c_int, [o, I64]),
            "oracle_read_state": (C.c_int, [o, I64, I64, P(I32)]),
            "oracle_write_state": (C.c_int, [o, I64, I64, P(I32)]),
            "oracle_read_log": (C.c_int, [o, I64, I64, P(I32), P(U32)]),
            "oracle_write_log": (C.c_int, [o, I64, I64, P(I32), P(U32)]),
            "oracle_digest": (C.c_uint64, [o]),
            "oracle_digest_range": (C.c_uint64, [o, I64, I64]),
            "oracle_set_log_window": (C.c_int, [o, I32]),
            "oracle_vote": (C.c_int, [o, I64, I32, P(abi.raft_vote_req), P(abi.raft_vote_resp)]),
            "oracle_append": (C.c_int, [o, I64, I32, P(abi.raft_append_req), P(abi.raft_append_resp)]),
            "oracle_append_command": (C.c_int, [o, I64, I32, U32]),
            "oracle_log_new": (C.c_void_p, [I32]),
            "oracle_log_free": (None, [C.c_void_p]),
            "oracle_log_add": (I32, [C.c_void_p, I32, I32, U32]),
            "oracle_log_get": (I32, [C.c_void_p, I32, P(I32), P(U32)]),
            "oracle_log_last_index": (I32, [C.c_void_p]),
            "oracle_log_size": (I32, [C.c_void_p]),
            "oracle_log_phys": (I32, [C.c_void_p, I32, P(I32), P(U32)]),
            "oracle_philox": (None, [P(U32), P(U32), P(U32)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    out = (C.c_uint32 * 4)()
    lib().oracle_philox(c, k, out)
    return list(out)


class OracleLog:
    """Standalone Log<T> (Commons.kt:47-74) for the K1 trace."""

    def __init__(self, cap: int = 1 << 20):
        self.h = lib().oracle_log_new(cap)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_log_free(self.h)
            self.h = None

    def add(self, i, term, cmd):
        return lib().oracle_log_add(self.h, i, term, cmd)

    def get(self, i):
        t, c = C.c_int32(), C.c_uint32()
        ok = lib().oracle_log_get(self.h, i, C.byref(t), C.byref(c))
        if not ok:
            raise IndexError(i)
        return t.value, c.value

    @property
    def last_index(self):
        return lib().oracle_log_last_index(self.h)

    @property
    def size(self):
        return lib().oracle_log_size(self.h)

    def phys(self):
        out = []
        for j in range(self.size):
            t, c = C.c_int32(), C.c_uint32()
            lib().oracle_log_phys(self.h, j, C.byref(t), C.byref(c))
            out.append((t.value, c.value))
        return out

    def entries(self):
        return self.phys()[: self.last_index]


class Oracle:
    def __init__(self, params: "abi.raft_params"):
        self.p = params
        self.R = params.R
        self.G = params.G
        self.cap = params.log_cap
        self.W = abi.group_words(self.R)
        h = C.c_void_p()
        rc = lib().oracle_create(C.byref(params), C.byref(h))
        if rc != 0:
            raise ValueError(f"oracle_create failed: {rc}")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().oracle_destroy(self.h)
            self.h = None

    __del__ = close

    def step(self, n: int, nthreads: int = 1, counters: bool = True):
        c = abi.counters_array(n) if counters else None
        rc = lib().oracle_step(self.h, n, abi.ptr(c, C.c_int64) if c is not None else None, nthreads)
        if rc != 0:
            raise RuntimeError(rc)
        return c

    @property
    def step_index(self):
        return lib().oracle_step_index(self.h)

    @step_index.setter
    def step_index(self, t):
        if lib().oracle_set_step_index(self.h, int(t)) != 0:
            raise ValueError(t)

    def read_state(self, g0=0, n=None):
        n = self.G - g0 if n is None else n
        out = np.zeros((n, self.W), dtype=np.int32)
        rc = lib().oracle_read_state(self.h, g0, n, abi.ptr(out, C.c_int32))
        if rc != 0:
            raise RuntimeError(rc)
        return out

    def write_state(self, state, g0=0):
        s = np.ascontiguousarray(state, dtype=np.int32)
        rc = lib().oracle_write_state(self.h, g0, s.shape[0], abi.ptr(s, C.c_int32))
        if rc != 0:
            raise RuntimeError(rc)

    def read_log(self, g0=0, n=None):
        n = self.G - g0 if n is None else n
        t = np.zeros((n, self.R, self.cap), dtype=np.int32)
        c = np.zeros((n, self.R, self.cap), dtype=np.uint32)
        rc = lib().oracle_read_log(self.h, g0, n, abi.ptr(t, C.c_int32), abi.ptr(c, C.c_uint32))
        if rc != 0:
            raise RuntimeError(rc)
        return t, c

    def write_log(self, terms, cmds, g0=0):
        t = np.ascontiguousarray(terms, dtype=np.int32)
        c = np.ascontiguousarray(cmds, dtype=np.uint32)
        rc = lib().oracle_write_log(self.h, g0, t.shape[0], abi.ptr(t, C.c_int32), abi.ptr(c, C.c_uint32))
        if rc != 0:
            raise RuntimeError(rc)

    def digest(self) -> int:
        return int(lib().oracle_digest(self.h))

    def digest_range(self, g0: int, n: int) -> int:
        return int(lib().oracle_digest_range(self.h, g0, n))

    def set_log_window(self, w: int):
        """View every log through a log_window of w slots (0: all); the lists keep every slot."""
        if lib().oracle_set_log_window(self.h, int(w)) != 0:
            raise ValueError(w)

    def vote(self, group, dst, term, candidate_id, last_log_index, last_log_term):
        rq = abi.raft_vote_req(term, candidate_id, last_log_index, last_log_term)
        rs = abi.raft_vote_resp()
        rc = lib().oracle_vote(self.h, group, dst, C.byref(rq), C.byref(rs))
        if rc != 0:
            raise RuntimeError(rc)
        return rs.term, bool(rs.vote_granted)

    def append(self, group, dst, term, leader_id, prev_log_index, prev_log_term,
               entry=None, leader_commit=0):
        has = entry is not None
        et, ec = entry if has else (0, 0)
        rq = abi.raft_append_req(term, leader_id, prev_log_index, prev_log_term, int(has), et, ec,
                                 leader_commit)
        rs = abi.raft_append_resp()
        rc = lib().oracle_append(self.h, group, dst, C.byref(rq), C.byref(rs))
        if rc != 0:
            raise RuntimeError(rc)
        return rs.term, bool(rs.success), rs.status

    def append_command(self, group, replica, cmd):
        rc = lib().oracle_append_command(self.h, group, replica, cmd)
        if rc != 0:
            raise RuntimeError(rc)


# ---- the SoA CPU backend (oracle/raft_soa.cpp): CPU BASELINE only ---------
SOA_LIB = os.path.join(HERE, "lib", "libsoa.so")
_soa = None


def soa_lib():
    global _soa
    if _soa is None:
        if not os.path.exists(SOA_LIB):
            build()
        L = C.CDLL(SOA_LIB)
        P, I32, I64, U32 = C.POINTER, C.c_int32, C.c_int64, C.c_uint32
        o = C.c_void_p
        for name, res, args in [
            ("soa_create", C.c_int, [P(abi.raft_params), P(o)]),
            ("soa_destroy", None, [o]),
            ("soa_step", C.c_int, [o, I32, P(I64), I32]),
            ("soa_read_state", C.c_int, [o, I64, I64, P(I32)]),
            ("soa_read_log", C.c_int, [o, I64, I64, P(I32), P(U32)]),
            ("soa_digest", C.c_uint64, [o]),
            ("soa_write_state", C.c_int, [o, I64, I64, P(I32)]),
            ("soa_write_log", C.c_int, [o, I64, I64, P(I32), P(U32)]),
            ("soa_set_step_index", C.c_int, [o, I64]),
        ]:
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _soa = L
    return _soa


class Soa:
    """The SoA multithreaded CPU backend: same step as Oracle, other layout."""

    def __init__(self, params: "abi.raft_params"):
        self.p, self.R, self.G, self.cap = params, params.R, params.G, params.log_cap
        self.W = abi.group_words(self.R)
        h = C.c_void_p()
        rc = soa_lib().soa_create(C.byref(params), C.byref(h))
        if rc != 0:
            raise ValueError(f"soa_create failed: {rc}")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            soa_lib().soa_destroy(self.h)
            self.h = None

    __del__ = close

    def step(self, n: int, nthreads: int = 1, counters: bool = True):
        c = abi.counters_array(n) if counters else None
        rc = soa_lib().soa_step(self.h, n, abi.ptr(c, C.c_int64) if c is not None else None, nthreads)
        if rc != 0:
            raise RuntimeError(rc)
        return c

    def read_state(self, g0=0, n=None):
        n = self.G - g0 if n is None else n
        out = np.zeros((n, self.W), dtype=np.int32)
        if soa_lib().soa_read_state(self.h, g0, n, abi.ptr(out, C.c_int32)) != 0:
            raise RuntimeError("soa_read_state")
        return out

    def read_log(self, g0=0, n=None):
        n = self.G - g0 if n is None else n
        t = np.zeros((n, self.R, self.cap), dtype=np.int32)
        c = np.zeros((n, self.R, self.cap), dtype=np.uint32)
        if soa_lib().soa_read_log(self.h, g0, n, abi.ptr(t, C.c_int32), abi.ptr(c, C.c_uint32)) != 0:
            raise RuntimeError("soa_read_log")
        return t, c

    def digest(self) -> int:
        return int(soa_lib().soa_digest(self.h))

    def write_state(self, state, g0=0):
        a = np.ascontiguousarray(state, dtype=np.int32)
        if soa_lib().soa_write_state(self.h, g0, a.shape[0], abi.ptr(a, C.c_int32)) != 0:
            raise RuntimeError("soa_write_state")

    def write_log(self, terms, cmds, g0=0):
        t = np.ascontiguousarray(terms, dtype=np.int32)
        c = np.ascontiguousarray(cmds, dtype=np.uint32)
        if soa_lib().soa_write_log(self.h, g0, t.shape[0], abi.ptr(t, C.c_int32), abi.ptr(c, C.c_uint32)) != 0:
            raise RuntimeError("soa_write_log")

    def set_step_index(self, t):
        """The index of the next step (its Philox counter c0), as the engine's."""
        if soa_lib().soa_set_step_index(self.h, int(t)) != 0:
            raise RuntimeError("soa_set_step_index")
