"""TEST INFRASTRUCTURE ONLY: CPU restatement of the vote tally the GPU
edv_tally_* kernels implement.

  plenum/server/models.py:21-37   TrackedMsgs.addMsg / hasEnoughVotes: a
      distinct-voter SET per key; a duplicate vote counts once; quorum when
      len(voters) >= count.
  plenum/server/quorums.py:15-21  prepare = n - f - 1, commit = n - f,
  plenum/common/util.py:217-228   f = (n - 1) // 3 for n >= 4, else 0.
Only tests/ and bench.py's checker may import this."""
import numpy as np


def max_failures(n):
    return (n - 1) // 3 if n >= 4 else 0


def thresholds(n):
    f = max_failures(n)
    return n - f - 1, n - f


def tally(key, voter, phase, valid, n_keys, n_validators):
    """Returns (counts[n_keys, 2], prepare_quorum[n_keys], commit_quorum[n_keys])."""
    key = np.asarray(key, np.int64)
    voter = np.asarray(voter, np.int64)
    phase = np.asarray(phase, np.int64)
    ok = (np.asarray(valid) != 0) & (key < n_keys) & (voter < n_validators) & (phase < 2)
    trip = np.unique(np.stack([key[ok], phase[ok], voter[ok]], axis=1), axis=0) if ok.any() else np.zeros((0, 3), np.int64)
    counts = np.zeros((n_keys, 2), np.uint32)
    np.add.at(counts, (trip[:, 0], trip[:, 1]), 1)
    qp, qc = thresholds(n_validators)
    return counts, counts[:, 0] >= qp, counts[:, 1] >= qc


def tally_sets(votes, n_validators):
    """Pure-Python twin (small cases): votes = [(key, voter, phase, valid)]."""
    sets = {}
    for k, v, ph, ok in votes:
        if ok:
            sets.setdefault((k, ph), set()).add(v)
    qp, qc = thresholds(n_validators)
    return {k: len(s) for k, s in sets.items()}, qp, qc
