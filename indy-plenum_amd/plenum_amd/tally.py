"""PREPARE/COMMIT vote tally on the GPU with the reference's semantics.

Reference: Replica.processPrepare/processCommit add votes to per-(viewNo,
ppSeqNo) distinct-voter sets (plenum/server/models.py:21-106) and order when
the set size reaches Quorums(n).prepare / .commit (replica.py:1379-1401,
1456-1488; quorums.py:15-32).  Here a batch of votes -- (key, voter, phase,
valid) with valid = the vote's signature/precondition verdict -- becomes a
uint8 ballot array [key][phase][voter] (set semantics: duplicates write the
same 1), then per-key counts and quorum flags.  Across GPUs ballots are
combined with an RCCL all-reduce(MAX) (dist.py), which is set union; SUM
would double-count duplicates.
"""
import numpy as np

from .quorums import Quorums

PREPARE, COMMIT = 0, 1


class VoteTally:
    def __init__(self, engine, n_validators):
        self.engine = engine
        self.n_validators = n_validators
        self.quorums = Quorums(n_validators)

    def tally(self, key, voter, phase, valid, n_keys):
        """Host-array form -> (counts[n_keys, 2], prepared[n_keys], committed[n_keys])."""
        return self.engine.tally(key, voter, phase, valid, n_keys, self.n_validators)

    def thresholds(self):
        return self.quorums.prepare.value, self.quorums.commit.value


def ballots_from_votes(key, voter, phase, valid, n_keys, n_validators):
    """numpy ballot array (used by the CPU-side sharding tests)."""
    b = np.zeros((n_keys, 2, n_validators), np.uint8)
    ok = np.asarray(valid) != 0
    b[np.asarray(key)[ok], np.asarray(phase)[ok], np.asarray(voter)[ok]] = 1
    return b
