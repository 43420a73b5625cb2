"""Committed golden vectors (tests/golden/make_golden.py) vs the oracle (CPU)
and vs the HIP engine (GPU)."""
import importlib
import json
import os

import numpy as np
import pytest

import oracle as O
from helpers import abi, masked_logs

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "oracle_golden.npz"))   # allow_pickle=False
META = json.load(open(os.path.join(HERE, "golden", "oracle_golden.json")))


def replay(make, name):
    spec = dict(META[name]["spec"])
    spec.pop("steps")
    every = spec.pop("digest_every")
    x = make(abi.make_params(**spec))
    counters, digests = [], []
    for _ in META[name]["digests"]:
        counters.append(x.step(every)[:, : abi.NUM_COUNTERS])
        digests.append(f"{x.digest():016x}")
    st = x.read_state()
    t, c = masked_logs(st, *x.read_log(), x.R)
    np.testing.assert_array_equal(np.concatenate(counters), GOLD[f"{name}_counters"])
    assert digests == META[name]["digests"]
    np.testing.assert_array_equal(st, GOLD[f"{name}_state"])
    np.testing.assert_array_equal(t, GOLD[f"{name}_log_terms"])
    np.testing.assert_array_equal(c, GOLD[f"{name}_log_cmds"])


@pytest.mark.parametrize("name", sorted(META))
def test_oracle_matches_golden(name):
    replay(O.Oracle, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(META))
def test_engine_matches_golden(name):
    RaftEngine = importlib.import_module("raft-kotlin_amd.engine").RaftEngine
    replay(RaftEngine, name)


def test_config1_golden_outcome():
    """Config 1's end state: one leader, all 1000 commands committed everywhere."""
    st = GOLD["c1_state"][0]
    R = 5
    roles = [st[r * abi.NUM_FIELDS + abi.F_INDEX["role"]] for r in range(R)]
    commits = [st[r * abi.NUM_FIELDS + abi.F_INDEX["commit"]] for r in range(R)]
    assert roles.count(abi.LEADER) == 1 and min(commits) == 1000
