"""Batched proto3 codec of the reference's messages (greeter.proto:16-44) over
the C-ABI of include/raft_wire.h: lists of serialized messages <-> the fixed
width arrays of RaftEngine.vote_batch / append_batch.  Host code; no GPU."""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import abi


def _lib():
    return abi.load_library()


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise RuntimeError(f"{what}: {_lib().raft_last_error().decode()} (rc={rc})")
    return rc


# Upper bound of one encoded message without its command bytes: every int32
# field is a 1-byte tag plus at most 10 varint bytes (negative values), i.e.
# 11 B; RequestAppendEntriesRPC has 5 of them (55 B) plus entries[0]: a tag,
# a <= 5-byte length, the entry's term (11 B), the command's tag and <= 5-byte
# length (78 B before the command).  The other messages are smaller.
MAX_FIXED_BYTES = 96


def _pack(msgs: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    off = np.zeros(len(msgs) + 1, dtype=np.int64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    buf = np.frombuffer(b"".join(msgs), dtype=np.uint8) if off[-1] else np.zeros(1, dtype=np.uint8)
    return np.ascontiguousarray(buf), off


def _split(buf: np.ndarray, off: np.ndarray) -> List[bytes]:
    raw = buf.tobytes()
    return [raw[off[m]:off[m + 1]] for m in range(len(off) - 1)]


def _decode(fn: str, msgs: Sequence[bytes], width: int, ctype) -> np.ndarray:
    buf, off = _pack(msgs)
    out = np.zeros((len(msgs), width), dtype=np.int32)
    _check(getattr(_lib(), fn)(abi.ptr(buf, C.c_uint8), abi.ptr(off, C.c_int64), len(msgs), abi.ptr(out, ctype)), fn)
    return out


def _encode(fn: str, arr: np.ndarray, width: int, ctype, extra=()) -> List[bytes]:
    a = np.ascontiguousarray(arr, dtype=np.int32).reshape(-1, width)
    n = a.shape[0]
    off = np.zeros(n + 1, dtype=np.int64)
    cap = MAX_FIXED_BYTES * n + 16 + sum(int(x.nbytes) for x in extra if isinstance(x, np.ndarray))
    buf = np.zeros(cap, dtype=np.uint8)
    used = _check(getattr(_lib(), fn)(abi.ptr(a, ctype), *extra_args(extra), n, abi.ptr(buf, C.c_uint8), cap,
                                      abi.ptr(off, C.c_int64)), fn)
    return _split(buf[:max(used, 1)], off)


def extra_args(extra):
    return [abi.ptr(x, C.c_uint8 if x.dtype == np.uint8 else C.c_int64) for x in extra]


# ---- RequestVoteRPC / ResponseVoteRPC ---------------------------------------
def decode_vote_requests(msgs: Sequence[bytes]) -> np.ndarray:
    """-> [n, 4] int32 (term, candidateId, lastLogIndex, lastLogTerm)"""
    return _decode("raft_wire_decode_vote_req", msgs, 4, abi.raft_vote_req)


def encode_vote_requests(req: np.ndarray) -> List[bytes]:
    return _encode("raft_wire_encode_vote_req", req, 4, abi.raft_vote_req)


def decode_vote_responses(msgs: Sequence[bytes]) -> np.ndarray:
    """-> [n, 2] int32 (term, voteGranted)"""
    return _decode("raft_wire_decode_vote_resp", msgs, 2, abi.raft_vote_resp)


def encode_vote_responses(resp: np.ndarray) -> List[bytes]:
    return _encode("raft_wire_encode_vote_resp", resp, 2, abi.raft_vote_resp)


# ---- RequestAppendEntriesRPC / ResponseAppendEntriesRPC ---------------------
def decode_append_requests(msgs: Sequence[bytes]) -> Tuple[np.ndarray, List[Optional[bytes]], np.ndarray]:
    """-> ([n, 8] int32 rows of RaftEngine.append_batch with entryCmd = 0,
    entries[0].command bytes per message (None without an entry),
    [n] entry counts)."""
    buf, off = _pack(msgs)
    n = len(msgs)
    out = np.zeros((n, 8), dtype=np.int32)
    co = np.zeros(n, dtype=np.int64)
    cl = np.zeros(n, dtype=np.int32)
    ne = np.zeros(n, dtype=np.int32)
    _check(_lib().raft_wire_decode_append_req(abi.ptr(buf, C.c_uint8), abi.ptr(off, C.c_int64), n,
                                              abi.ptr(out, abi.raft_append_req), abi.ptr(co, C.c_int64),
                                              abi.ptr(cl, C.c_int32), abi.ptr(ne, C.c_int32)),
           "raft_wire_decode_append_req")
    raw = buf.tobytes()
    cmds = [raw[co[m]:co[m] + cl[m]] if out[m, 4] else None for m in range(n)]
    return out, cmds, ne


def encode_append_requests(req: np.ndarray, commands: Sequence[Optional[bytes]]) -> List[bytes]:
    """req: [n, 8] rows (entryCmd ignored); commands[m]: entries[0].command bytes."""
    cs = [c or b"" for c in commands]
    cbuf, coff = _pack(cs)
    return _encode("raft_wire_encode_append_req", req, 8, abi.raft_append_req, extra=(cbuf, coff))


def decode_append_responses(msgs: Sequence[bytes]) -> np.ndarray:
    """-> [n, 3] int32 (term, success, status = 0)"""
    return _decode("raft_wire_decode_append_resp", msgs, 3, abi.raft_append_resp)


def encode_append_responses(resp: np.ndarray) -> List[bytes]:
    return _encode("raft_wire_encode_append_resp", resp, 3, abi.raft_append_resp)
