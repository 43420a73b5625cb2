"""RaftService — the reference's per-node API over the batched engine.

The reference node is ``class RaftServer(val id: Int, val servers: List<RaftClient>)``
(RaftServer.kt:28) serving ``service Raft { Vote; Append }`` (greeter.proto:46-49)
plus ``appendCommand`` / ``entries`` (RaftServer.kt:96-107).  Here a node is one
(group, replica) slot of a RaftEngine; ``RaftNode`` has the same method names,
argument meaning and error behaviour:

* ``vote(RequestVoteRPC) -> ResponseVoteRPC``           (RaftServer.kt:228-251)
* ``append(RequestAppendEntriesRPC) -> ResponseAppendEntriesRPC``
  (RaftServer.kt:253-287); raises ``IndexError`` where the reference's
  ``Log.get`` throws (prevLogIndex < -1), after the handler's earlier effects
* ``appendCommand(command: str) -> str``                 (RaftServer.kt:100-107)
* ``entries() -> list[str]`` in the reference's ``"term: command"`` format
  (RaftServer.kt:96-97)

Commands are strings in the reference (LogEntry.command, greeter.proto:31); the
engine stores a u32 id per entry, interned here.  Every call is one HIP batch;
``RaftService.vote_many`` / ``append_many`` batch many nodes per launch.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import abi, wire
from .engine import RaftEngine


@dataclass
class LogEntry:                        # RequestAppendEntriesRPC.LogEntry, greeter.proto:29-32
    term: int
    command: str


@dataclass
class RequestVoteRPC:                  # greeter.proto:16-21
    term: int
    candidateId: int
    lastLogIndex: int
    lastLogTerm: int


@dataclass
class ResponseVoteRPC:                 # greeter.proto:23-26
    term: int
    voteGranted: bool


@dataclass
class RequestAppendEntriesRPC:         # greeter.proto:28-39
    term: int
    leaderId: int
    prevLogIndex: int
    prevLogTerm: int
    entries: List[LogEntry] = field(default_factory=list)
    leaderCommit: int = 0


@dataclass
class ResponseAppendEntriesRPC:        # greeter.proto:41-44
    term: int
    success: bool


class CommandTable:
    """Interns LogEntry.command strings to the engine's u32 command ids."""

    BASE = 0x80000000

    def __init__(self):
        self._ids: dict[str, int] = {}
        self._names: dict[int, str] = {}

    def intern(self, s: str) -> int:
        i = self._ids.get(s)
        if i is None:
            i = self.BASE + len(self._ids)
            if i > 0xFFFFFFFF:
                raise OverflowError("command table full")
            self._ids[s] = i
            self._names[i] = s
        return i

    def name(self, i: int) -> str:
        # commands injected by the lockstep harness carry Philox ids
        return self._names.get(int(i), f"cmd#{int(i):08x}")


class RaftNode:
    """One reference RaftServer: replica ``replica`` (id = replica + 1) of ``group``."""

    def __init__(self, service: "RaftService", group: int, replica: int):
        self.s = service
        self.group = group
        self.replica = replica
        self.id = replica + 1

    # -- RaftGrpcKt.RaftImplBase overrides ---------------------------------
    def vote(self, request: RequestVoteRPC) -> ResponseVoteRPC:
        return self.s.vote_many([self.group], [self.replica], [request])[0]

    def append(self, request: RequestAppendEntriesRPC) -> ResponseAppendEntriesRPC:
        return self.s.append_many([self.group], [self.replica], [request])[0]

    def appendCommand(self, command: str) -> str:      # RaftServer.kt:100-107
        self.s.engine.append_command_batch([self.group], [self.replica], [self.s.commands.intern(command)])
        return command

    def entries(self) -> List[str]:                      # RaftServer.kt:96-97
        return [f"{t}: {c}" for t, c in self.log()]

    # -- inspection ----------------------------------------------------------
    def log(self) -> List[tuple]:
        """Visible entries log[0 .. lastIndex) as (term, command) (Commons.kt:71-72)."""
        st = self._fields()
        terms, cmds = self.s.engine.read_log(self.group, 1)
        n = int(st[abi.F_INDEX["last"]])
        return [(int(terms[0, self.replica, j]), self.s.commands.name(cmds[0, self.replica, j])) for j in range(n)]

    def _fields(self) -> np.ndarray:
        w = self.s.engine.read_state(self.group, 1)[0]
        return w[self.replica * abi.NUM_FIELDS:(self.replica + 1) * abi.NUM_FIELDS]

    @property
    def currentTerm(self) -> int:
        return int(self._fields()[abi.F_INDEX["term"]])

    @property
    def votedFor(self) -> int:
        return int(self._fields()[abi.F_INDEX["voted"]])

    @property
    def state(self) -> str:
        return ("FOLLOWER", "CANDIDATE", "LEADER")[int(self._fields()[abi.F_INDEX["role"]])]

    @property
    def commitIndex(self) -> int:
        return int(self._fields()[abi.F_INDEX["commit"]])


class RaftService:
    """The `service Raft` surface of every node of a RaftEngine."""

    def __init__(self, engine: RaftEngine):
        self.engine = engine
        self.commands = CommandTable()

    def node(self, group: int, replica: int) -> RaftNode:
        if not (0 <= group < self.engine.G and 0 <= replica < self.engine.R):
            raise IndexError((group, replica))
        return RaftNode(self, group, replica)

    def vote_many(self, groups, replicas, requests: List[RequestVoteRPC]) -> List[ResponseVoteRPC]:
        q = np.array([[r.term, r.candidateId, r.lastLogIndex, r.lastLogTerm] for r in requests],
                     dtype=np.int32).reshape(-1, 4)
        out = self.engine.vote_batch(groups, replicas, q)
        return [ResponseVoteRPC(int(t), bool(g)) for t, g in out]

    def append_many(self, groups, replicas, requests: List[RequestAppendEntriesRPC]) -> List[ResponseAppendEntriesRPC]:
        rows = []
        for r in requests:
            # the reference appends only entries[0] (RaftServer.kt:278)
            e = r.entries[0] if r.entries else None
            rows.append([r.term, r.leaderId, r.prevLogIndex, r.prevLogTerm, int(e is not None),
                         e.term if e else 0, self.commands.intern(e.command) if e else 0, r.leaderCommit])
        out = self.engine.append_batch(groups, replicas, np.array(rows, dtype=np.int64).reshape(-1, 8))
        res = []
        for t, s, status in out:
            if status != 0:
                raise IndexError("Log.get: prevLogIndex out of bounds (RaftServer.kt:276, Commons.kt:53-54)")
            res.append(ResponseAppendEntriesRPC(int(t), bool(s)))
        return res

    # -- the gRPC-facing wire form (include/raft_wire.h) --------------------
    # RaftImplBase.vote()/append() (RaftServer.kt:228, :253) receive and return
    # serialized protobufs; these batch them through the engine unchanged.
    def vote_wire(self, groups, replicas, requests: List[bytes]) -> List[bytes]:
        """Serialized RequestVoteRPCs -> serialized ResponseVoteRPCs."""
        q = wire.decode_vote_requests(requests)
        return wire.encode_vote_responses(self.engine.vote_batch(groups, replicas, q))

    def append_wire(self, groups, replicas, requests: List[bytes]) -> List[Optional[bytes]]:
        """Serialized RequestAppendEntriesRPCs -> serialized responses; None where
        the handler threw (Log.get, RaftServer.kt:276): that call has no response,
        which the reference's caller swallows (RaftServer.kt:170-172)."""
        rows, cmds, _ = wire.decode_append_requests(requests)
        rows = rows.astype(np.int64)
        for m, c in enumerate(cmds):
            if c is not None:
                rows[m, 6] = self.commands.intern(c.decode("utf-8"))
        out = self.engine.append_batch(groups, replicas, rows)
        enc = wire.encode_append_responses(out)
        return [None if out[m, 2] else enc[m] for m in range(len(enc))]
