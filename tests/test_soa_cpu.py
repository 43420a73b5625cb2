"""The SoA multithreaded CPU backend (oracle/raft_soa.cpp, bench.py's CPU
baseline) is bit-exact with the scalar oracle: per-step counters, canonical
state, logs and digest, on every configuration's semantics and thread count."""
import numpy as np
import pytest

import oracle as O
from helpers import abi

CASES = {
    "c2": dict(abi.CONFIGS[2], G=300),
    "c3": dict(abi.CONFIGS[3], G=300, churn_ppm=20_000),
    "c5": dict(abi.CONFIGS[5], G=60),
    "r_mix": dict(R=4, G=200, seed=9, drop_ppm=100_000, churn_ppm=20_000, churn_steps=15, cmd_ppm=500_000,
                  partition_period=40, partition_len=10),
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("threads", [1, 3])
def test_soa_equals_oracle(name, threads):
    kw = CASES[name]
    cap = 700 if name == "c5" else 300
    o = O.Oracle(abi.make_params(log_cap=cap, **kw))
    s = O.Soa(abi.make_params(log_cap=cap, **kw))
    np.testing.assert_array_equal(o.read_state(), s.read_state())
    for chunk in (1, 37, 200, 262):
        np.testing.assert_array_equal(o.step(chunk, nthreads=2), s.step(chunk, nthreads=threads))
        assert o.digest() == s.digest()
    np.testing.assert_array_equal(o.read_state(), s.read_state())
    for a, b in zip(o.read_log(), s.read_log()):
        np.testing.assert_array_equal(a, b)


def test_soa_refuses_what_it_does_not_model():
    with pytest.raises(ValueError):
        O.Soa(abi.make_params(R=3, G=4, mode=abi.MODE_TEXTBOOK))
    with pytest.raises(ValueError):
        O.Soa(abi.make_params(R=3, G=4, log_cap=64, log_window=16))


def test_soa_restore_resumes_bit_exact():
    """soa_write_state / soa_write_log / soa_set_step_index (the steady-state
    CPU baseline's restore, bench_legs.cpu_baseline): a run exported at step
    t and restored into a fresh backend continues exactly as the original."""
    kw = dict(abi.CONFIGS[3], G=300)
    a = O.Soa(abi.make_params(log_cap=200, **kw))
    a.step(300, nthreads=4)
    b = O.Soa(abi.make_params(log_cap=200, **kw))
    b.write_state(a.read_state())
    b.write_log(*a.read_log())
    b.set_step_index(300)
    assert b.digest() == a.digest()
    assert np.array_equal(a.step(50, nthreads=4), b.step(50, nthreads=2))
    assert a.digest() == b.digest()
    a.close()
    b.close()
