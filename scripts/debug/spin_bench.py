"""bench.py with the HIP runtime told to spin-wait in synchronisations
(hipSetDeviceFlags(hipDeviceScheduleSpin) before any other HIP call): a probe
of how much of a short timed region is the host's wake-up after the device
finishes.   python scripts/debug/spin_bench.py <bench.py args>"""
import ctypes
import os
import sys

hip = ctypes.CDLL("libamdhip64.so")
rc = hip.hipSetDeviceFlags(ctypes.c_uint(int(os.environ.get("RAFT_HIP_FLAGS", "1"))))   # 1 = hipDeviceScheduleSpin
print(f"hipSetDeviceFlags rc={rc}", file=sys.stderr, flush=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

sys.exit(bench.main(sys.argv[1:]))
