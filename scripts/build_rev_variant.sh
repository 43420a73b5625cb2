#!/bin/bash
# Build the engine of a git revision (default HEAD) as an A/B variant next to
# the working tree's: raft-kotlin_amd/lib/libraft_engine_<name>.so, selected
# with RAFT_ENGINE_LIB (scripts/ab.sh, scripts/ab_session.sh VARIANTS).
#   scripts/build_rev_variant.sh head [REV]
set -e
cd "$(dirname "$0")/.."
name=${1:-head}; rev=${2:-HEAD}
d=$(mktemp -d)
git archive "$rev" raft-kotlin_amd/csrc include | tar -x -C "$d"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I "$d/include" \
    -o raft-kotlin_amd/lib/libraft_engine_$name.so "$d/raft-kotlin_amd/csrc/raft_engine.hip" \
    "$d/raft-kotlin_amd/csrc/raft_wire.cpp"
rm -rf "$d"
echo "built raft-kotlin_amd/lib/libraft_engine_$name.so from $rev"
