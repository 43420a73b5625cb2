"""The ring-buffered log (raft_params.log_window) on the CPU
oracle: a window changes what is retained and hashed, never the protocol.
While no access misses the window, the run is the flat run: same per-step
counters, same state, same digest of the full lists; the retained slots read
back identically; and the window-miss count is exactly the accesses of the
reference (Log.get / Log.add) below physLen - W (Commons.kt:53-68)."""
import numpy as np
import pytest

import oracle as O
from helpers import abi, fld

KW = dict(abi.CONFIGS[3], G=400, churn_ppm=20_000)


def test_window_does_not_change_the_protocol():
    flat = O.Oracle(abi.make_params(log_cap=320, **KW))
    ring = O.Oracle(abi.make_params(log_cap=320, log_window=64, **KW))
    cf, cr = flat.step(900), ring.step(900)
    assert cr[:, abi.C_INDEX["log_window_miss"]].sum() == 0
    np.testing.assert_array_equal(cf, cr)
    np.testing.assert_array_equal(flat.read_state(), ring.read_state())
    assert flat.digest() != ring.digest()                  # the ring hashes the retained window only
    ring.set_log_window(0)
    assert flat.digest() == ring.digest()
    ring.set_log_window(64)
    st = ring.read_state()
    (tf, cmf), (tr, cmr) = flat.read_log(), ring.read_log()
    phys = np.stack([fld(st, 5, r, "phys") for r in range(5)], 1)
    j = np.arange(320)[None, None, :]
    keep = (j >= phys[:, :, None] - 64) & (j < phys[:, :, None])
    assert np.array_equal(np.where(keep, tf, 0), tr) and np.array_equal(np.where(keep, cmf, 0), cmr)
    assert phys.max() > 3 * 64                              # the ring wrapped several times


@pytest.mark.parametrize("w", [3, 6, -1, 128])
def test_bad_windows_are_refused(w):
    with pytest.raises(ValueError):
        O.Oracle(abi.make_params(R=3, G=1, log_cap=64, log_window=w))
