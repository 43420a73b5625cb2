#!/bin/bash
# Ballots (lm()) of a comparison made in another basic block: the backend
# re-materialises each through a VGPR (v_cndmask 0/1 + v_cmp, two VALU), so the
# step kernel should have none on its hot paths.  Lists them for step_kernel<R>.
R=${R:-5}; TB=${TB:-0}; RING=${RING:-0}; D=$PWD/gpurun_out/ir; mkdir -p $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -emit-llvm -I include ${EXTRA:-} \
    -o $D/k.ll raft-kotlin_amd/csrc/raft_engine.hip 2>&1 | grep -v warning | head -3
python3 - "$D/k.ll" "step_kernelILi${R}ELb${TB}ELb${RING}E" <<'PY'
import re, sys
s = open(sys.argv[1]).read().split('\n')
start = next(i for i, l in enumerate(s) if l.startswith('define') and sys.argv[2] in l)
fn = []
for l in s[start:]:
    fn.append(l)
    if l == '}': break
defs, blk, uses = {}, 'entry', []
for i, l in enumerate(fn):
    m = re.match(r'^(\S+):', l)
    if m: blk = m.group(1); continue
    m = re.match(r'\s+(%\S+) = (.*)', l)
    if m: defs[m.group(1)] = (blk, m.group(2)[:90])
    m = re.search(r'@llvm.amdgcn.ballot.i64\(i1 (%[\w.]+)\)', l)
    if m: uses.append((m.group(1), blk, i))
cross = [(v, b, i) for v, b, i in uses if v in defs and defs[v][0] != b]
print(f"{sys.argv[2]}: {len(uses)} ballots, {len(cross)} of a comparison from another block")
for v, b, i in cross: print(f"  line {i}: {v} = {defs[v][1]}  (block {defs[v][0]} -> {b})")
PY
