"""VALU / SALU per chunk-step of the last step_kernel dispatch of each
rocprofv3 --pmc run given (`<dir>` with `<dir>.log` holding bench.py's line):
the A/B of kernel variants by dynamic instruction count.

    python scripts/pmc_valu.py gpurun_out/r5_e/pmc_prod_d20 gpurun_out/r5_e/pmc_m1_d20 ...
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from phase_budget import last_dispatch  # noqa: E402


def main(dirs):
    out = {}
    for d in dirs:
        line = json.loads([ln for ln in open(d + ".log") if ln.startswith("{")][-1])
        unit = line["config"]["step_waves_per_rank"] * line["roofline"]["launch_steps"]
        x = last_dispatch(d)
        out[os.path.basename(d)] = {"valu": x["SQ_INSTS_VALU"] / unit, "salu": x["SQ_INSTS_SALU"] / unit,
                                    "kernel_avg_ms": line["roofline"]["kernel_avg_ms"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
