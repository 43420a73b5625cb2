#!/bin/bash
# Build the engine with a rewrite of raft_engine.hip's device ISA between
# codegen and assembly (experiments: scripts/sessions/r6.sh A/B runs):
#   scripts/build_asm_variant.sh NAME REWRITE      -> raft-kotlin_amd/lib/libraft_engine_NAME.so
# REWRITE is a python script filtering stdin -> stdout (the gfx950 .s).  The
# device code is compiled once with --save-temps, rewritten, assembled
# (clang -cc1as), linked (lld), bundled (clang-offload-bundler) and embedded
# into the host object (-fcuda-include-gpubinary); the other translation
# units are compiled as build.py compiles them.
set -e
NAME=${1:?name}; RW=${2:?rewrite script}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LLVM=/opt/rocm/lib/llvm/bin
D=$(mktemp -d)
FL="-O3 -std=c++17 -fPIC -Wno-unused-function -munsafe-fp-atomics -I $ROOT/include ${EXTRA:-}"
(cd "$D" && /opt/rocm/bin/hipcc --offload-arch=gfx950 $FL --save-temps -c -o eng.o "$ROOT/raft-kotlin_amd/csrc/raft_engine.hip" 2>&1 | grep -v warning || true)
python3 "$RW" < "$D/raft_engine-hip-amdgcn-amd-amdhsa-gfx950.s" > "$D/dev.s"
$LLVM/clang -cc1as -triple amdgcn-amd-amdhsa -target-cpu gfx950 -filetype obj -mrelocation-model pic -o "$D/dev.o" "$D/dev.s"
$LLVM/lld -flavor gnu -m elf64_amdgpu --no-undefined -shared -o "$D/dev.out" "$D/dev.o"
$LLVM/clang-offload-bundler -type=o -bundle-align=4096 -targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--gfx950 \
    -input=/dev/null -input="$D/dev.out" -output="$D/dev.hipfb"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $FL --cuda-host-only -Xclang -fcuda-include-gpubinary -Xclang "$D/dev.hipfb" \
    -c -o "$D/host.o" "$ROOT/raft-kotlin_amd/csrc/raft_engine.hip" 2>&1 | grep -v warning || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 $FL -shared -ldl -o "$ROOT/raft-kotlin_amd/lib/libraft_engine_$NAME.so" "$D/host.o" \
    "$ROOT/raft-kotlin_amd/csrc/raft_batch.hip" "$ROOT/raft-kotlin_amd/csrc/raft_wire.cpp" \
    "$ROOT/raft-kotlin_amd/csrc/raft_host.cpp" "$ROOT/raft-kotlin_amd/csrc/raft_comm.cpp"
rm -rf "$D"
ls -la "$ROOT/raft-kotlin_amd/lib/libraft_engine_$NAME.so"
