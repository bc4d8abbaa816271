"""GPU vote tally vs the CPU restatement of TrackedMsgs + Quorums."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tally_oracle  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nv", [1, 4, 7, 25, 31])
def test_tally_matches_oracle(gpu_engine, nv):
    rng = np.random.default_rng(nv)
    n_keys = 1000
    nvotes = n_keys * nv * 2
    k = rng.integers(0, n_keys, nvotes).astype(np.uint32)
    v = rng.integers(0, nv, nvotes).astype(np.uint8)
    ph = rng.integers(0, 2, nvotes).astype(np.uint8)
    ok = (rng.random(nvotes) < 0.95).astype(np.uint8)
    counts, prep, com = gpu_engine.tally(k, v, ph, ok, n_keys, nv)
    c2, p2, m2 = tally_oracle.tally(k, v, ph, ok, n_keys, nv)
    assert (counts == c2).all() and (prep == p2).all() and (com == m2).all()


def test_tally_duplicates_count_once(gpu_engine):
    k = np.zeros(50, np.uint32)
    v = np.array([3] * 50, np.uint8)
    ph = np.zeros(50, np.uint8)
    counts, prep, com = gpu_engine.tally(k, v, ph, np.ones(50, np.uint8), 1, 4)
    assert counts.tolist() == [[1, 0]] and not prep[0]


def test_tally_c4_shape(gpu_engine):
    """configs[4] tally shape on one GPU: K = 160,000 keys x 25 validators x 2 phases, ~5% invalid."""
    rng = np.random.default_rng(4)
    n_keys, nv = 160_000, 25
    k = np.repeat(np.arange(n_keys, dtype=np.uint32), nv * 2)
    v = np.tile(np.repeat(np.arange(nv, dtype=np.uint8), 2), n_keys)
    ph = np.tile(np.array([0, 1], np.uint8), n_keys * nv)
    ok = (rng.random(k.size) >= 0.05).astype(np.uint8)
    counts, prep, com = gpu_engine.tally(k, v, ph, ok, n_keys, nv)
    c2, p2, m2 = tally_oracle.tally(k, v, ph, ok, n_keys, nv)
    assert (counts == c2).all() and (prep == p2).all() and (com == m2).all()
