"""PREPARE/COMMIT vote tally on the GPU with the replica's semantics.

Reference: Replica.processPrepare / processCommit add votes to per-(viewNo,
ppSeqNo) distinct-voter sets (plenum/server/models.py:21-106) and the batch
orders when the set sizes reach Quorums(n).prepare / .commit
(replica.py:1379-1401, 1456-1488; quorums.py:15-32).  Before a PREPARE is
added, Replica.validatePrepare rejects one sent by the primary of its view
(replica.py:1289-1291); the primary of view v on protocol instance i is the
node of rank (v + i) % n (primary_selector.py:353-354).

ThreePhaseTally collects a batch of votes (as the replica would receive them,
each with the verdict of its signature / preconditions) and resolves them in
one edv_tally launch: key and voter names become indices, the primary of each
key's view is passed along, and the device builds the uint8 ballot
[key][phase][voter] (set semantics), counts it and compares with the
thresholds.  Across GPUs ballots combine with all-reduce(MAX) (dist.py).
"""
import numpy as np

from .quorums import Quorums

PREPARE, COMMIT = 0, 1
NO_PRIMARY = 0xFF


class ThreePhaseTally:
    """validators: node names in rank order (the pool's nodeReg order);
    inst_id: the protocol instance the votes belong to (0 = master)."""

    def __init__(self, engine, validators, inst_id=0):
        if not 0 < len(validators) < NO_PRIMARY:
            raise ValueError("1..254 validators")
        self.engine = engine
        self.validators = list(validators)
        self.rank = {name: i for i, name in enumerate(self.validators)}
        self.inst_id = inst_id
        self.quorums = Quorums(len(self.validators))
        self.clear()

    def clear(self):
        self._keys = {}
        self._key = []
        self._voter = []
        self._phase = []
        self._valid = []

    def primary_rank(self, view_no):
        return (view_no + self.inst_id) % len(self.validators)

    def add(self, view_no, pp_seq_no, voter, phase, valid=True):
        """One PREPARE (phase 0) or COMMIT (phase 1) from node `voter`."""
        key = (view_no, pp_seq_no)
        k = self._keys.setdefault(key, len(self._keys))
        self._key.append(k)
        self._voter.append(self.rank[voter])
        self._phase.append(phase)
        self._valid.append(1 if valid else 0)

    def run(self):
        """-> {(viewNo, ppSeqNo): (prepare voters, commit voters, prepared, committed)}."""
        keys = list(self._keys)
        if not keys:
            return {}
        primary = np.array([self.primary_rank(v) for v, _ in keys], np.uint8)
        counts, prepared, committed = self.engine.tally(
            np.array(self._key, np.uint32), np.array(self._voter, np.uint8), np.array(self._phase, np.uint8),
            np.array(self._valid, np.uint8), len(keys), len(self.validators), primary=primary)
        return {key: (int(counts[i, 0]), int(counts[i, 1]), bool(prepared[i]), bool(committed[i]))
                for i, key in enumerate(keys)}

    def thresholds(self):
        return self.quorums.prepare.value, self.quorums.commit.value
