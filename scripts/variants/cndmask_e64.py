"""ISA rewrite (scripts/build_asm_variant.sh): every v_cndmask_b32_e32 (the
VOP2 form, whose lane mask is VCC, read implicitly) becomes the same select in
the VOP3 form with VCC as an explicit operand.  scripts/ubench/valu_rate6.hip
measures the VOP2 form at ~13 SIMD-cycles per instruction when its VCC was
written by the scalar ALU (or before a run of them), the VOP3 form at ~3.2
(profiles/r6_c).  src0 must be a VGPR or an inline constant in VOP3 (gfx9: no
literal, and VCC already takes the one constant-bus read)."""
import re
import sys

PAT = re.compile(r"^(\s+)v_cndmask_b32_e32(\s+)(v\d+),\s*([^,]+),\s*(v\d+),\s*vcc\s*$", re.M)


def ok_src0(x: str) -> bool:
    x = x.strip()
    if re.fullmatch(r"v\d+", x):
        return True
    try:
        return -16 <= int(x, 0) <= 64
    except ValueError:
        return False


def rewrite(s: str) -> tuple[str, int, int]:
    n = [0, 0]

    def rep(m):
        if ok_src0(m.group(4)):
            n[0] += 1
            return f"{m.group(1)}v_cndmask_b32_e64{m.group(2)}{m.group(3)}, {m.group(4)}, {m.group(5)}, vcc"
        n[1] += 1
        return m.group(0)
    return PAT.sub(rep, s), n[0], n[1]


if __name__ == "__main__":
    out, a, b = rewrite(sys.stdin.read())
    sys.stdout.write(out)
    print(f"cndmask_e64: {a} selects rewritten, {b} kept", file=sys.stderr)
