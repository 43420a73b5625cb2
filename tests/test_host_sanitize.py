"""The repository's host C / C++ under sanitizers (CPU): the oracle
(oracle/raft_oracle.c), the SoA backend (oracle/raft_soa.cpp) and the wire
codec (raft-kotlin_amd/csrc/raft_wire.cpp), driven by
tests/sanitize/host_check.cpp -- oracle vs SoA on config 3 / config 5 / every
R, textbook mode, a ring, the single handlers on random requests, wire round
trips, random and truncated wire input.  Once with AddressSanitizer +
UndefinedBehaviorSanitizer, once with ThreadSanitizer (the oracle and the SoA
backend step groups on worker threads).  GPU code is never built with a
sanitizer."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = {"asan_ubsan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
       "tsan": ["-fsanitize=thread"]}


@pytest.mark.parametrize("kind", sorted(SAN))
def test_host_code_under_sanitizers(kind, tmp_path):
    if not (shutil.which("gcc") and shutil.which("g++")):
        pytest.skip("gcc / g++ not available")
    flags = SAN[kind] + ["-g", "-O1"]
    inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle")]
    objs = []
    for src, cc, std in (("oracle/raft_oracle.c", "gcc", "-std=c11"), ("oracle/raft_soa.cpp", "g++", "-std=c++17"),
                         ("raft-kotlin_amd/csrc/raft_wire.cpp", "g++", "-std=c++17")):
        obj = str(tmp_path / (os.path.basename(src) + ".o"))
        subprocess.run([cc, *flags, std, "-pthread", *inc, "-c", os.path.join(ROOT, src), "-o", obj], check=True)
        objs.append(obj)
    exe = str(tmp_path / "host_check")
    subprocess.run(["g++", *flags, "-std=c++17", "-pthread", *inc, os.path.join(ROOT, "tests", "sanitize", "host_check.cpp"),
                    *objs, "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "0 failures" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
