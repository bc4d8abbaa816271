"""Quorum thresholds (plenum/server/quorums.py:15-32 with getMaxFailures,
plenum/common/util.py:217-228) and the distinct-voter tally semantics
(plenum/server/models.py:21-106, primary PREPARE rejected per
replica.py:1289-1291).  Pinned by tests/golden/quorums_kat.json and
tally_kat.json, which gen_ref_quorums.py produced by running the reference's
own quorums.py / models.py (Prepares, Commits) under Python 3.9."""
import json
import os
import sys

import numpy as np

from conftest import GOLDEN, ROOT
from plenum_amd.quorums import Quorums, getMaxFailures
from plenum_amd.tally import ThreePhaseTally

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import tally_oracle  # noqa: E402


def quorums_kat():
    return json.load(open(os.path.join(GOLDEN, "quorums_kat.json")))


def tally_kat():
    return json.load(open(os.path.join(GOLDEN, "tally_kat.json")))


def test_quorum_table_matches_reference():
    rows = quorums_kat()
    assert [r["n"] for r in rows] == list(range(1, 64))
    for r in rows:
        q = Quorums(r["n"])
        assert q.f == r["f"] == getMaxFailures(r["n"]) == tally_oracle.max_failures(r["n"])
        for name, v in r.items():
            if name not in ("n", "f"):
                assert getattr(q, name).value == v, (r["n"], name)
        assert tally_oracle.thresholds(r["n"]) == (r["prepare"], r["commit"])
        assert q.commit.is_reached(r["commit"]) and not q.commit.is_reached(r["commit"] - 1)


def _arrays(case):
    v = np.array(case["votes"], np.int64).reshape(-1, 4)
    return v[:, 0], v[:, 1], v[:, 2], v[:, 3]


def test_tally_oracle_matches_reference_vote_sets():
    for case in tally_kat():
        k, v, ph, ok = _arrays(case)
        counts, prep, com = tally_oracle.tally(k, v, ph, ok, len(case["keys"]), case["n"], primary=case["primary"])
        e = case["expect"]
        assert counts.tolist() == e["counts"], case["name"]
        assert prep.tolist() == e["prepared"] and com.tolist() == e["committed"], case["name"]
        assert (e["prepare_quorum"], e["commit_quorum"]) == tally_oracle.thresholds(case["n"])


def test_primary_prepare_never_counts():
    case = next(c for c in tally_kat() if c["name"] == "primary-prepare-would-reach-quorum")
    k, v, ph, ok = _arrays(case)
    without, prep_wo, _ = tally_oracle.tally(k, v, ph, ok, len(case["keys"]), case["n"])
    assert prep_wo[0] and not case["expect"]["prepared"][0]  # counting the primary would be one vote early


class _OracleTallyEngine:
    def tally(self, key, voter, phase, valid, n_keys, n_validators, primary=None):
        return tally_oracle.tally(key, voter, phase, valid, n_keys, n_validators, primary=primary)


def test_three_phase_tally_host_mapping():
    """ThreePhaseTally's name/key mapping and primary rule (rank (view + inst) % n,
    primary_selector.py:353-354) against the reference's vote sets."""
    for case in tally_kat():
        n = case["n"]
        names = ["Node%d" % (i + 1) for i in range(n)]
        # the fixture's primary of key k is view % n, i.e. instance 0
        assert all(p == view % n for p, (view, _) in zip(case["primary"], case["keys"]))
        t = ThreePhaseTally(_OracleTallyEngine(), names)
        for view, seq in case["keys"]:  # fixture key order
            t._keys.setdefault((view, seq), len(t._keys))
        for kk, voter, phase, valid in case["votes"]:
            view, seq = case["keys"][kk]
            t.add(view, seq, names[voter], phase, bool(valid))
        res = t.run()
        e = case["expect"]
        for i, (view, seq) in enumerate(case["keys"]):
            assert res[(view, seq)] == (e["counts"][i][0], e["counts"][i][1], e["prepared"][i], e["committed"][i])


def test_ballot_union_equals_set_union():
    rng = np.random.default_rng(0)
    n_keys, nv = 50, 25
    k = rng.integers(0, n_keys, 4000)
    v = rng.integers(0, nv, 4000)
    p = rng.integers(0, 2, 4000)
    ok = rng.random(4000) < 0.95
    half = 2000
    b = np.maximum(tally_oracle.ballots_from_votes(k[:half], v[:half], p[:half], ok[:half], n_keys, nv),
                   tally_oracle.ballots_from_votes(k[half:], v[half:], p[half:], ok[half:], n_keys, nv))
    counts, _, _ = tally_oracle.tally(k, v, p, ok, n_keys, nv)
    assert (b.sum(axis=2) == counts).all()


def test_c4_vote_classes_decide_at_the_thresholds():
    """synth.c4_votes (bench configs[4], tests/test_gpu_tally.py): on the CPU
    oracle every class decides as constructed at n = 25, identically on any
    split of the global vote range into ranks."""
    import numpy as np
    import tally_oracle
    from plenum_amd import synth
    n_keys, V = 4000, 25
    g = np.arange(n_keys * 2 * V)
    k, ph, v, pres, cls = synth.c4_votes(g, V)
    prim = synth.c4_primary(n_keys, V)
    c, p, m = tally_oracle.tally(k, v, ph, pres.astype(np.uint8), n_keys, V, primary=prim)
    kc = cls[::2 * V]
    names = synth.C4_CLASSES
    assert not p[kc == names.index("prepare_below")].any() and p[kc == names.index("prepare_at")].all()
    assert not m[kc == names.index("commit_below")].any() and m[kc == names.index("commit_at")].all()
    halves = [synth.c4_votes(part, V) for part in np.array_split(g, 3)]
    assert all((np.concatenate([h[i] for h in halves]) == x).all() for i, x in enumerate((k, ph, v, pres, cls)))
