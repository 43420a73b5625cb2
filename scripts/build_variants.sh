#!/bin/bash
# Build experiment variants of the engine next to the real one
# (raft-kotlin_amd/lib/libraft_engine_<name>.so, selected with RAFT_ENGINE_LIB
# by scripts/ab.sh / scripts/ab_session.sh).  The product sources carry no
# experiment switches: a variant is the working tree's csrc plus
#   name:-DFLAGS ...        compiler flags (e.g. "w6:-DRAFT_STEP_WAVES_PER_EU(R,TB,RING,NET)=6")
#   name:patch=P[+P2...]    patches from scripts/variants/P.patch (e.g. "replay:patch=commit_replay")
#   name:rev=REV            the csrc of a git revision instead of the working tree
# Specs may combine parts with ';' ("nc7:patch=no_counters;-DRAFT_STEP_BLOCK=256").
#   scripts/build_variants.sh "nocnt:patch=no_counters" "head:rev=HEAD"
set -e
cd "$(dirname "$0")/.."
ROOT=$PWD
build_one() {
  local name=$1 spec=$2 d flags="" part
  d=$(mktemp -d)
  mkdir -p "$d/raft-kotlin_amd"
  cp -r include "$d/"; cp -r raft-kotlin_amd/csrc "$d/raft-kotlin_amd/"
  IFS=';' read -ra parts <<< "$spec"
  for part in "${parts[@]}"; do
    case "$part" in
      rev=*) rm -rf "$d/include" "$d/raft-kotlin_amd/csrc"
             git archive "${part#rev=}" raft-kotlin_amd/csrc include | tar -x -C "$d" ;;
      patch=*) IFS='+' read -ra ps <<< "${part#patch=}"
               for p in "${ps[@]}"; do (cd "$d" && patch -s -p1 < "$ROOT/scripts/variants/$p.patch"); done ;;
      *) flags="$flags $part" ;;
    esac
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -I "$d/include" $flags \
      -o "raft-kotlin_amd/lib/libraft_engine_$name.so" "$d/raft-kotlin_amd/csrc/raft_engine.hip" \
      $( [ -f "$d/raft-kotlin_amd/csrc/raft_batch.hip" ] && echo "$d/raft-kotlin_amd/csrc/raft_batch.hip" ) \
      "$d/raft-kotlin_amd/csrc/raft_wire.cpp" $( [ -f "$d/raft-kotlin_amd/csrc/raft_host.cpp" ] && echo "$d/raft-kotlin_amd/csrc/raft_host.cpp" ) \
      $( [ -f "$d/raft-kotlin_amd/csrc/raft_comm.cpp" ] && echo "$d/raft-kotlin_amd/csrc/raft_comm.cpp -ldl" )
  rm -rf "$d"
}
for spec in "$@"; do build_one "${spec%%:*}" "${spec#*:}" & done
wait
ls raft-kotlin_amd/lib/
