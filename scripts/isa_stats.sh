#!/bin/bash
# Per-R step_kernel ISA statistics (VGPRs, SGPR spills via v_readlane/v_writelane, code size).
set -e
D=${1:-$PWD/gpurun_out/isa}; mkdir -p $D; cd $D; rm -f raft_engine-*
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared ${EXTRA:-} -I /root/repo/include --save-temps \
    -o $D/x.so /root/repo/raft-kotlin_amd/csrc/raft_engine.hip 2>&1 | grep -v warning | head -5 || true
python3 - "$D" "${KERNEL:-step_kernel}" <<'PY'
import re, sys, collections
d, kn = sys.argv[1], sys.argv[2]
s = open(f'{d}/raft_engine-hip-amdgcn-amd-amdhsa-gfx950.s').read().split('\n')
cur = None; st = {}
for i, l in enumerate(s):
    m = re.match(r'^(_Z\S*' + kn + r'ILi(\d)ELb(\d)ELb(\d)E(?:Li(\d+)E)?\S*):', l)
    if m:
        cur = m.group(2) + ("t" if m.group(3) == "1" else "") + ("r" if m.group(4) == "1" else "") + \
              (("/net" + m.group(5)) if m.group(5) else "")
        st[cur] = collections.Counter(); continue
    if cur and '; -- End function' in l:
        blk = '\n'.join(s[i:i + 30])
        for k in ['codeLenInByte', 'NumVgprs', 'NumSgprs', 'ScratchSize', 'Occupancy']:
            m2 = re.search(k + r'(?: = |: )(\d+)', blk)
            if m2: st[cur][k] = int(m2.group(1))
        cur = None; continue
    if cur:
        t = l.strip().split()
        if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'): continue
        st[cur]['v' if t[0].startswith('v_') else 's' if t[0].startswith('s_') else 'other'] += 1
        if t[0] in ('v_readlane_b32', 'v_writelane_b32'): st[cur]['lane'] += 1
        if t[0].startswith(('global_', 'buffer_')): st[cur]['mem'] += 1
        if t[0].startswith('ds_'): st[cur]['ds'] += 1
        if t[0] == 'v_mul_hi_u32': st[cur]['mulhi'] += 1
for k, v in st.items():
    print(f"R={k}: vgpr={v['NumVgprs']} sgpr={v['NumSgprs']} occ={v['Occupancy']} scratch={v['ScratchSize']} "
          f"code={v['codeLenInByte']} valu={v['v']} salu={v['s']} lanemov={v['lane']} mem={v['mem']} ds={v['ds']} mulhi={v['mulhi']}")
PY
