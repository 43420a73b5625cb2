#!/bin/bash
# Build tuning variants of the engine next to the real one, for
# scripts/variant_sweep.sh (RAFT_ENGINE_LIB selects one; experiments only):
#   scripts/build_variants.sh "w6:-DRAFT_STEP_WAVES_PER_EU(R,TB,RING)=6"
cd "$(dirname "$0")/.."
for spec in "$@"; do rm -f raft-kotlin_amd/lib/libraft_engine_${spec%%:*}.so; done
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include $flags \
      -o raft-kotlin_amd/lib/libraft_engine_$name.so raft-kotlin_amd/csrc/raft_engine.hip raft-kotlin_amd/csrc/raft_wire.cpp &
done
wait
ls raft-kotlin_amd/lib/
