"""Build the in-tree HIP engine library for gfx950 (hipcc cross-compiles; no GPU needed).

    python raft-kotlin_amd/build.py          -> raft-kotlin_amd/lib/libraft_engine.so
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "raft_engine.hip")
SRCS = [SRC, os.path.join(PKG, "csrc", "raft_wire.cpp"),           # the wire codec is host code
        os.path.join(PKG, "csrc", "raft_host.cpp")]                  # page-locked batch memory
HDRS = [os.path.join(PKG, "csrc", h) for h in ("raft_step.h", "philox.h")] + [
    os.path.join(ROOT, "include", h) for h in ("raft_engine.h", "raft_wire.h")]
OUT = os.path.join(PKG, "lib", "libraft_engine.so")
ARCH = os.environ.get("RAFT_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(f) > t for f in [*SRCS, *HDRS, __file__])


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics",
           "-I", os.path.join(ROOT, "include"), "-o", OUT + ".tmp", *SRCS]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="-f" in sys.argv, verbose=True))
