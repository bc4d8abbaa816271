"""BFT quorum thresholds, restated from plenum/server/quorums.py:4-32 and
getMaxFailures (plenum/common/util.py:217-228)."""
from math import floor


def getMaxFailures(nodeCount: int) -> int:
    if nodeCount >= 4:
        return int(floor((nodeCount - 1) / 3))
    return 0


class Quorum:
    def __init__(self, value: int):
        self.value = value

    def is_reached(self, msg_count: int) -> bool:
        return msg_count >= self.value

    def __repr__(self):
        return "{}({!r})".format(self.__class__.__name__, self.value)


class Quorums:
    def __init__(self, n):
        f = getMaxFailures(n)
        self.f = f
        self.propagate = Quorum(f + 1)
        self.prepare = Quorum(n - f - 1)
        self.commit = Quorum(n - f)
        self.reply = Quorum(f + 1)
        self.view_change = Quorum(n - f)
        self.election = Quorum(n - f)
        self.view_change_done = Quorum(n - f)
        self.propagate_primary = Quorum(f + 1)
        self.same_consistency_proof = Quorum(f + 1)
        self.consistency_proof = Quorum(f + 1)
        self.ledger_status = Quorum(n - f - 1)
        self.checkpoint = Quorum(2 * f)
        self.timestamp = Quorum(f + 1)
        self.bls_signatures = Quorum(n - f)

    def __str__(self):
        return "{}".format(self.__dict__)
