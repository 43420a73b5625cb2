import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


# torch ships its own HIP runtime (same soname as /opt/rocm's): import it
# before the engine library is loaded, so every test process uses one HIP
# runtime whatever order its tests run in (bench.py imports torch first too).
# Importing torch does not initialise a GPU.
try:
    import torch  # noqa: F401,E402
except ImportError:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP engine on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
