"""raft-kotlin_amd — MI355X-native batched Raft engine.

Drop-in for the consensus core of arodionov/raft-kotlin (RaftServer.vote /
RaftServer.append / the leader commit loop / the election timer) run for up
to millions of independent groups in lockstep on gfx950.  The compute path
is the HIP library ``lib/libraft_engine.so`` behind the C-ABI in
``include/raft_engine.h``; this package is its host-side mirror.
"""
from . import abi  # noqa: F401

__all__ = ["abi", "RaftEngine", "RaftService"]


def __getattr__(name):
    if name == "RaftEngine":
        from .engine import RaftEngine
        return RaftEngine
    if name == "RaftService":
        from .service import RaftService
        return RaftService
    raise AttributeError(name)
