#!/bin/bash
# Static instruction counts per step phase of step_kernel<R> (asm markers in a scratch copy).
R=${R:-5}; D=$PWD/gpurun_out/mk; rm -rf $D; mkdir -p $D
cp raft-kotlin_amd/csrc/raft_engine.hip raft-kotlin_amd/csrc/philox.h raft-kotlin_amd/csrc/raft_step.h $D/
sed -i 's#../../include/raft_engine.h#/root/repo/include/raft_engine.h#' $D/raft_step.h
python3 - "$D" <<'PY'
import sys
p=sys.argv[1]+'/raft_step.h'; s=open(p).read()
for k,v in {'T: timers':'T',"the step's Philox":'JOBS','H: harness':'H','V: RequestVote':'V','D: latch':'D',
            'A: leader ticks':'A','C: client':'C','K: end-of-step':'K'}.items():
    s=s.replace('        // ---------------- '+k,'        asm volatile(";MARK_%s" ::: "memory");\n        // ---------------- %s'%(v,k))
s=s.replace('        // the deferred ResettableCountdownTimer draws','        asm volatile(";MARK_TDRAW" ::: "memory");\n        // the deferred ResettableCountdownTimer draws')
open(p,'w').write(s)
PY
cd $D && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I /root/repo/include --save-temps -o x.so raft_engine.hip 2>&1 | grep -v warn | head -3
python3 - $R "$D" <<'PY'
import re, sys, collections
R=sys.argv[1]
s=open(sys.argv[2]+'/raft_engine-hip-amdgcn-amd-amdhsa-gfx950.s').read().split('\n')
cur=False; region='PRE'; c=collections.defaultdict(collections.Counter)
for l in s:
    if re.match(r'^_Z\S*step_kernelILi%sELb0ELb0E\S*:'%R,l): cur=True; continue
    if cur and '; -- End function' in l: break
    if not cur: continue
    m=re.search(r';MARK_(\w+)',l)
    if m: region=m.group(1); continue
    t=l.strip().split()
    if not t or t[0].startswith(('.',';')) or t[0].endswith(':'): continue
    k='v' if t[0].startswith('v_') else 's' if t[0].startswith('s_') else 'ds' if t[0].startswith('ds_') else 'mem'
    c[region][k]+=1
    if t[0] in ('v_readlane_b32','v_writelane_b32'): c[region]['lane']+=1
    if t[0].startswith('v_mov'): c[region]['vmov']+=1
for r,v in c.items(): print(f"{r:6s}", dict(v))
PY
