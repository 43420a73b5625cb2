"""Build the in-tree HIP engine library for gfx950 (hipcc cross-compiles; no GPU needed).

    python raft-kotlin_amd/build.py          -> raft-kotlin_amd/lib/libraft_engine.so

The build is keyed on the sources, not on mtimes: `library_source_id()` hashes
every source and header the library is compiled from plus the compiler flags,
the id is compiled into the library (`raft_build_source_id()`) and written
beside it (`libraft_engine.so.srcid`), and a build whose id differs from the
working tree's is rebuilt here and refused by `abi.load_library`.  The step
kernel's own id (`kernel_source_id()`, the step kernel's sources -- not the
handler batches' raft_batch.hip; bench.py keys its rocprofv3 rows on it) is
compiled in too (`raft_build_kernel_source_id()`).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
SRC = os.path.join(CSRC, "raft_engine.hip")
SRCS = [SRC, os.path.join(CSRC, "raft_batch.hip"),                   # the handler batches
        os.path.join(CSRC, "raft_wire.cpp"),                         # the wire codec is host code
        os.path.join(CSRC, "raft_host.cpp"),                         # page-locked batch memory
        os.path.join(CSRC, "raft_comm.cpp")]                         # the RCCL counter all-reduce (dlopen)
HDRS = [os.path.join(CSRC, h) for h in ("raft_step.h", "philox.h", "raft_engine_impl.h")] + [
    os.path.join(ROOT, "include", h) for h in ("raft_engine.h", "raft_wire.h")]
# the step kernel's sources (bench.py's kernel_source_id, the key of its
# rocprofv3 rows): not raft_batch.hip, which holds no step-kernel code
KERNEL_SOURCES = ("raft_step.h", "raft_engine.hip", "philox.h", "raft_engine_impl.h")
# the handler batches' sources (bench.py keys their rocprofv3 rows on them)
BATCH_SOURCES = [os.path.join(CSRC, f) for f in ("raft_batch.hip", "raft_engine_impl.h", "raft_step.h", "philox.h")] + [
    os.path.join(ROOT, "include", "raft_engine.h")]
OUT = os.path.join(PKG, "lib", "libraft_engine.so")
ARCH = os.environ.get("RAFT_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics", "-ldl"]


def kernel_source_id() -> str:
    """Short hash of the step kernel's sources (bench.py's PMC-row key)."""
    h = hashlib.sha1()
    for f in KERNEL_SOURCES:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


def batch_source_id() -> str:
    """Short hash of the handler batches' sources.  The library reports it
    with its kernels' compile-time knobs appended (raft_build_batch_source_id,
    e.g. "<hash>-t512x8"): bench.py keys their PMC rows on the loaded
    library's id, so a variant build never matches a production row."""
    h = hashlib.sha1()
    for f in BATCH_SOURCES:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


def library_source_id() -> str:
    """Short hash of everything the library is built from: sources, headers,
    target and flags."""
    h = hashlib.sha1()
    for f in [*SRCS, *HDRS]:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join([ARCH, *FLAGS]).encode())
    return h.hexdigest()[:12]


def sources_present() -> bool:
    return all(os.path.exists(f) for f in [*SRCS, *HDRS])


def built_source_id(path: str = OUT) -> str | None:
    """The id the build at `path` was made from (its .srcid file), or None."""
    try:
        with open(path + ".srcid") as fh:
            return fh.read().strip() or None
    except OSError:
        return None


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    return not os.path.exists(OUT) or built_source_id() != library_source_id()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        if verbose:
            print(f"{OUT} is current (sources {library_source_id()})", flush=True)
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    sid, kid, bid = library_source_id(), kernel_source_id(), batch_source_id()
    cmd = [hipcc(), f"--offload-arch={ARCH}", *FLAGS, f'-DRAFT_BUILD_SOURCE_ID="{sid}"',
           f'-DRAFT_BUILD_KERNEL_ID="{kid}"', f'-DRAFT_BUILD_BATCH_ID="{bid}"', "-I", os.path.join(ROOT, "include"),
           "-o", OUT + ".tmp", *SRCS]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    with open(OUT + ".srcid.tmp", "w") as fh:
        fh.write(sid + "\n")
    os.replace(OUT + ".srcid.tmp", OUT + ".srcid")
    return OUT


if __name__ == "__main__":
    print(build(force="-f" in sys.argv, verbose=True))
