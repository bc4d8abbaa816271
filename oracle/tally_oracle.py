"""TEST INFRASTRUCTURE ONLY: CPU restatement of the vote tally the GPU
edv_tally_* kernels implement.

  plenum/server/models.py:21-37   TrackedMsgs.addMsg / hasEnoughVotes: a
      distinct-voter SET per key; a duplicate vote counts once; quorum when
      len(voters) >= count.
  plenum/server/quorums.py:15-21  prepare = n - f - 1, commit = n - f,
  plenum/common/util.py:217-228   f = (n - 1) // 3 for n >= 4, else 0.
  plenum/server/replica.py:1289-1291  a PREPARE from the primary of the
      key's view is rejected before Prepares.addVote (never counts).
Pinned by tests/golden/quorums_kat.json / tally_kat.json, produced by running
the reference's own quorums.py and models.py (gen_ref_quorums.py).
Only tests/ and bench.py's checker may import this."""
import numpy as np


def max_failures(n):
    return (n - 1) // 3 if n >= 4 else 0


def thresholds(n):
    f = max_failures(n)
    return n - f - 1, n - f


def tally(key, voter, phase, valid, n_keys, n_validators, primary=None):
    """Returns (counts[n_keys, 2], prepare_quorum[n_keys], commit_quorum[n_keys])."""
    key = np.asarray(key, np.int64)
    voter = np.asarray(voter, np.int64)
    phase = np.asarray(phase, np.int64)
    ok = (np.asarray(valid) != 0) & (key < n_keys) & (voter < n_validators) & (phase < 2)
    if primary is not None:
        prim = np.asarray(primary, np.int64)[np.minimum(key, n_keys - 1)]
        ok &= ~((phase == 0) & (voter == prim))
    trip = np.unique(np.stack([key[ok], phase[ok], voter[ok]], axis=1), axis=0) if ok.any() else np.zeros((0, 3), np.int64)
    counts = np.zeros((n_keys, 2), np.uint32)
    np.add.at(counts, (trip[:, 0], trip[:, 1]), 1)
    qp, qc = thresholds(n_validators)
    return counts, counts[:, 0] >= qp, counts[:, 1] >= qc


def tally_sets(votes, n_validators, primary=None):
    """Pure-Python twin (small cases): votes = [(key, voter, phase, valid)]."""
    sets = {}
    for k, v, ph, ok in votes:
        if ph == 0 and primary is not None and primary[k] == v:
            continue
        if ok:
            sets.setdefault((k, ph), set()).add(v)
    qp, qc = thresholds(n_validators)
    return {k: len(s) for k, s in sets.items()}, qp, qc


def ballots_from_votes(key, voter, phase, valid, n_keys, n_validators):
    """numpy ballot array [key][phase][voter] (the CPU-side sharding tests)."""
    b = np.zeros((n_keys, 2, n_validators), np.uint8)
    ok = np.asarray(valid) != 0
    b[np.asarray(key)[ok], np.asarray(phase)[ok], np.asarray(voter)[ok]] = 1
    return b
