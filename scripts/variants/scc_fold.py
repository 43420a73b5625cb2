"""ISA rewrite (scripts/build_asm_variant.sh): drop the scalar compare that
tests a lane mask the instruction just before it computed.

The compiler tests a wave-uniform mask as

    s_and_b64     s[24:25], s[22:23], s[70:71]     ; SCC = (result != 0)
    s_cmp_eq_u64  s[24:25], 0                      ; SCC = (result == 0)
    s_cbranch_scc0 .LBB..

but the logic op already set SCC from the same result: the compare is one
SALU instruction of pure overhead (gfx950 prices a SALU instruction at ~2
SIMD-cycles beside the VALU stream).  `s_cmp_lg_* X, 0` has
the logic op's own polarity and is dropped as is; `s_cmp_eq_* X, 0` is dropped
and its branch inverted (scc0 <-> scc1), only where no later instruction reads
SCC before writing it (both ways out of the branch).

A compare is dropped only where it is provably redundant and removing it
shortens no hazard window:
  * the last SCC writer before it is a logic op (and/or/xor/andn2/orn2/nand/
    nor/xnor/not) whose destination is exactly the compared register, with
    only VALU, memory and SCC-neutral scalar instructions between and
    nothing in between writing that register;
  * its only SCC reader before the next SCC write is the s_cbranch_scc* that
    follows it;
  * no label, EXEC / M0 writer or transcendental among the 5 instructions
    before it, and no SGPR / VCC that a VALU among them wrote is read within
    6 instructions of that VALU on any path after the compare: every gfx9
    wait-state window the compare may count in is at most 5 instructions, so
    nothing it padded loses a wait state.
"""
import re
import sys

LOGIC = re.compile(r"s_(and|or|xor|andn2|orn2|nand|nor|xnor|not)_b(32|64)$")
CMP = re.compile(r"s_cmp_(eq|lg)_u(32|64)$")
SCC_READERS = re.compile(r"s_(cselect|cmov|cmovk|addc|subb|cbranch_scc[01])")
# scalar instructions that neither read nor write SCC
SCC_NEUTRAL = re.compile(r"s_(mov_b32|mov_b64|movk_i32|nop|waitcnt|setprio|sleep|load_\w+|buffer_load_\w+|"
                         r"mul_i32|mul_hi_u32|brev_b32|ff1_i32_b32|ff1_i32_b64|flbit_\w+|sext_\w+|getpc_b64|"
                         r"barrier|dcache_inv)$")
VALU_SDST = re.compile(r"v_(cmp|cmpx|readlane|readfirstlane|add_co|sub_co|subrev_co|addc_co|subb_co|subbrev_co|"
                       r"mad_u64_u32|mad_i64_i32|div_scale|cndmask_b32_e64_unused)")
TRANS = re.compile(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_")
LABEL = re.compile(r"^(\.?[\w.$]+):")


def parse(lines):
    """Per line: ('i', mnemonic, operands) for instructions, ('l', name) for
    labels, ('f',) for function ends, None otherwise."""
    out = []
    for ln in lines:
        st = ln.strip()
        if not st or st.startswith(";"):
            out.append(None)
            continue
        if "; -- End function" in ln:
            out.append(("f",))
            continue
        m = LABEL.match(st)
        if m and not ln.startswith(("\t", " ")):
            out.append(("l", m.group(1)))
            continue
        if st.startswith("."):
            out.append(None)
            continue
        code = st.split(";")[0].strip()
        parts = code.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        out.append(("i", parts[0], ops))
    return out


def writes_exec_or_m0(mn, ops):
    if "saveexec" in mn or "wrexec" in mn or mn.startswith("v_cmpx"):
        return True
    return bool(ops) and ops[0] in ("exec", "exec_lo", "exec_hi", "m0")


IMPLICIT_VCC_READERS = re.compile(r"(v_cndmask_b32_e32|v_addc_co_u32_e32|v_subb_co_u32_e32|v_subbrev_co_u32_e32|"
                                  r"s_cbranch_vccz|s_cbranch_vccnz)$")


def sgpr_dsts(mn, ops):
    """The SGPRs (or VCC) a VALU instruction writes."""
    if not ops:
        return set()
    out = set()
    if mn.startswith("v_cmp") and mn.endswith("_e32"):
        out |= regs("vcc")
    if mn.startswith(("v_add_co", "v_sub_co", "v_subrev_co", "v_addc_co", "v_subb_co", "v_subbrev_co")) and \
            mn.endswith("_e32"):
        out |= regs("vcc")
    for d in ops[:2] if VALU_SDST.match(mn) else ops[:1]:
        if d == "vcc" or d.startswith("s[") or re.fullmatch(r"s\d+", d):
            out |= regs(d)
    return out


def reads(e, rs):
    """Does e read any register of rs where a wait state applies (a VALU
    operand or mask, a memory instruction's address; the scalar ALU
    interlocks on SGPRs a VALU wrote)?"""
    mn, ops = e[1], e[2]
    if not mn.startswith(("v_", "global_", "buffer_", "flat_", "scratch_", "ds_")):
        return False
    if (rs & regs("vcc")) and IMPLICIT_VCC_READERS.match(mn):
        return True
    srcs = ops if mn.startswith(("global_store", "buffer_store", "flat_store", "scratch_store", "ds_")) else ops[1:]
    return any(regs(x) & rs for x in srcs if x)


def window_after(p, k, labels, n, depth=0):
    """The next n instructions on every path from index k (labels skipped)."""
    out = []
    while k < len(p) and n > 0:
        e = p[k]
        k += 1
        if e is None or e[0] == "l":
            continue
        if e[0] == "f":
            break
        out.append(e)
        n -= 1
        if e[1] == "s_endpgm":
            break
        if e[1].startswith(("s_branch", "s_cbranch")) and depth < 3:
            t = labels.get(e[2][0]) if e[2] else None
            if t is None:
                out.append(("i", "?", []))
            else:
                out += window_after(p, t, labels, n, depth + 1)
            if e[1] == "s_branch":
                break
    return out


def hazard_free(p, k, labels):
    """Dropping instruction k shortens no wait-state window: no label among
    the 5 instructions before it, no EXEC / M0 writer or transcendental there,
    and no SGPR / VCC a VALU wrote there read within the window after it."""
    seen, j = 0, k - 1
    while seen < 5 and j >= 0:
        e = p[j]
        j -= 1
        if e is None:
            continue
        if e[0] != "i":
            return False
        mn, ops = e[1], e[2]
        seen += 1
        if TRANS.match(mn) or writes_exec_or_m0(mn, ops):
            return False
        if mn.startswith("v_"):
            rs = sgpr_dsts(mn, ops)
            if rs:
                for f in window_after(p, k + 1, labels, 6 - seen):
                    if f[1] == "?" or reads(f, rs):
                        return False
    return True


def regs(x):
    """The 32-bit registers of an operand (s[4:5] -> {s4, s5})."""
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", x)
    if m:
        return {f"s{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1)}
    if re.fullmatch(r"s\d+", x):
        return {x}
    if x == "vcc":
        return {"vcc_lo", "vcc_hi"}
    return {x}


def writes(e, rs):
    """Does instruction e write any register of rs (its first operand, or a
    VALU's carry / compare SGPR destination)?"""
    mn, ops = e[1], e[2]
    if not ops:
        return False
    dsts = [ops[0]]
    if mn.startswith("v_") and len(ops) > 1 and VALU_SDST.match(mn):
        dsts.append(ops[1])
    if mn.startswith(("s_store", "s_buffer_store", "global_store", "buffer_store", "ds_write", "ds_add",
                      "s_cbranch", "s_branch")):
        return False
    return any(regs(d) & rs for d in dsts)


def scc_dead_after(p, k, labels, depth=0):
    """From index k on (one path, following unconditional branches and both
    ways of non-SCC conditional branches), is SCC written before it is read?"""
    if depth > 4:
        return False
    n = 0
    while k < len(p) and n < 64:
        e = p[k]
        k += 1
        if e is None or e[0] == "l":
            continue
        if e[0] == "f":
            return True
        mn, ops = e[1], e[2]
        n += 1
        if mn == "s_endpgm":
            return True
        if SCC_READERS.match(mn):
            return False
        if mn == "s_branch":
            t = labels.get(ops[0])
            return t is not None and scc_dead_after(p, t, labels, depth + 1)
        if mn.startswith("s_cbranch_"):
            t = labels.get(ops[0])
            if t is None or not scc_dead_after(p, t, labels, depth + 1):
                return False
            continue
        if mn.startswith("s_") and not SCC_NEUTRAL.match(mn):
            return True                                              # a writer (readers matched above)
    return False


def rewrite(text):
    lines = text.split("\n")
    p = parse(lines)
    labels = {e[1]: i + 1 for i, e in enumerate(p) if e and e[0] == "l"}
    drop, flip = set(), set()
    stats = {"eq": 0, "lg": 0, "kept": 0}
    for k, e in enumerate(p):
        if not e or e[0] != "i":
            continue
        m = CMP.match(e[1])
        if not m or len(e[2]) != 2 or e[2][1] != "0":
            continue
        x, width = e[2][0], m.group(2)
        rs = regs(x)
        ok = False
        # backward: the last SCC writer must be a logic op into x
        j = k - 1
        while j >= 0:
            f = p[j]
            j -= 1
            if f is None:
                continue
            if f[0] != "i":
                break
            mn = f[1]
            lm = LOGIC.match(mn)
            if lm:
                ok = lm.group(2) == width and f[2] and f[2][0] == x
                break
            if mn.startswith("s_") and not SCC_NEUTRAL.match(mn):
                break
            if writes(f, rs):
                break
        if ok:
            ok = hazard_free(p, k, labels)
        # forward: the branch that reads it, with nothing touching SCC between
        br = None
        if ok:
            j = k + 1
            while j < len(p):
                f = p[j]
                if f is None:
                    j += 1
                    continue
                if f[0] != "i":
                    break
                mn = f[1]
                if mn in ("s_cbranch_scc0", "s_cbranch_scc1"):
                    br = j
                    break
                if mn.startswith("s_") and not SCC_NEUTRAL.match(mn):
                    break
                j += 1
            ok = br is not None
        if ok and m.group(1) == "eq":
            # the inverted SCC must be dead on both ways out of the branch
            t = labels.get(p[br][2][0])
            ok = t is not None and scc_dead_after(p, br + 1, labels) and scc_dead_after(p, t, labels)
        if not ok:
            stats["kept"] += 1
            continue
        drop.add(k)
        if m.group(1) == "eq":
            flip.add(br)
        stats[m.group(1)] += 1
    out = []
    for i, ln in enumerate(lines):
        if i in drop:
            continue
        if i in flip:
            ln = ln.replace("s_cbranch_scc0", "s_cbranch_sccX").replace("s_cbranch_scc1", "s_cbranch_scc0") \
                   .replace("s_cbranch_sccX", "s_cbranch_scc1")
        out.append(ln)
    return "\n".join(out), stats


if __name__ == "__main__":
    out, st = rewrite(sys.stdin.read())
    sys.stdout.write(out)
    print(f"scc_fold: dropped {st['eq']} eq (branch inverted) + {st['lg']} lg compares, kept {st['kept']}",
          file=sys.stderr)
