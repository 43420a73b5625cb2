"""ISA rewrite that changes nothing: the control build of scripts/build_asm_variant.sh (the
assembler pipeline itself must not move the timing)."""
import sys
sys.stdout.write(sys.stdin.read())
