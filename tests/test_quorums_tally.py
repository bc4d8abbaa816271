"""Quorum thresholds (plenum/server/quorums.py:15-32 with getMaxFailures,
plenum/common/util.py:217-228) and the distinct-voter tally semantics
(plenum/server/models.py:21-37).  The reference's quorums.py cannot be
imported here (util.py:337 is a SyntaxError on Python >= 3.7), so the values
are pinned by the formula table below, which matches the thresholds the
reference's tests assume (n=4: f=1, prepare 2, commit 3; n=25: f=8)."""
import sys
import os

import numpy as np

from conftest import ROOT
from plenum_amd.quorums import Quorums, getMaxFailures
from plenum_amd.tally import ballots_from_votes

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tally_oracle  # noqa: E402


def test_quorum_table():
    table = {1: (0, 0, 1), 3: (0, 2, 3), 4: (1, 2, 3), 7: (2, 4, 5), 10: (3, 6, 7), 25: (8, 16, 17), 31: (10, 20, 21)}
    for n, (f, prep, com) in table.items():
        q = Quorums(n)
        assert (q.f, q.prepare.value, q.commit.value) == (f, prep, com)
        assert q.propagate.value == f + 1 and q.checkpoint.value == 2 * f
        assert tally_oracle.thresholds(n) == (prep, com)
    for n in range(1, 64):
        assert getMaxFailures(n) == tally_oracle.max_failures(n)
        assert Quorums(n).commit.is_reached(n - getMaxFailures(n))
        assert not Quorums(n).commit.is_reached(n - getMaxFailures(n) - 1)


def test_tally_oracle_set_semantics():
    votes = [(0, 1, 0, 1), (0, 1, 0, 1), (0, 2, 0, 1), (0, 3, 0, 0), (1, 1, 1, 1)]
    counts, qp, qc = tally_oracle.tally_sets(votes, 4)
    assert counts == {(0, 0): 2, (1, 1): 1} and (qp, qc) == (2, 3)
    k, v, p, ok = map(np.array, zip(*votes))
    c, prep, com = tally_oracle.tally(k, v, p, ok, 2, 4)
    assert c.tolist() == [[2, 0], [0, 1]] and prep.tolist() == [True, False] and com.tolist() == [False, False]


def test_ballot_union_equals_set_union():
    rng = np.random.default_rng(0)
    n_keys, nv = 50, 25
    k = rng.integers(0, n_keys, 4000)
    v = rng.integers(0, nv, 4000)
    p = rng.integers(0, 2, 4000)
    ok = rng.random(4000) < 0.95
    half = 2000
    b = np.maximum(ballots_from_votes(k[:half], v[:half], p[:half], ok[:half], n_keys, nv),
                   ballots_from_votes(k[half:], v[half:], p[half:], ok[half:], n_keys, nv))
    counts, _, _ = tally_oracle.tally(k, v, p, ok, n_keys, nv)
    assert (b.sum(axis=2) == counts).all()
