"""BFT quorum thresholds of plenum/server/quorums.py:15-32 with getMaxFailures
(plenum/common/util.py:217-228).

When the reference package is importable (inside a Plenum node) its own
Quorum / Quorums classes are re-exported, so thresholds come from the node's
code.  Otherwise the table below restates them; tests/golden/quorums_kat.json
(produced by running the reference's quorums.py, gen_ref_quorums.py) pins
every value for n = 1..63.  The verify path itself uses prepare (n - f - 1)
and commit (n - f) -- edv_tally_* compute the same two on the device."""

try:  # pragma: no cover - only inside a Plenum installation
    from plenum.server.quorums import Quorum, Quorums  # noqa: F401
    from plenum.common.util import getMaxFailures  # noqa: F401
    REFERENCE = True
except Exception:
    REFERENCE = False

if not REFERENCE:
    def getMaxFailures(nodeCount: int) -> int:
        """f = floor((n - 1) / 3) for n >= 4, else 0."""
        return (nodeCount - 1) // 3 if nodeCount >= 4 else 0

    class Quorum:
        def __init__(self, value: int):
            self.value = value

        def is_reached(self, msg_count: int) -> bool:
            return msg_count >= self.value

        def __repr__(self):
            return "{}({!r})".format(self.__class__.__name__, self.value)

    # name -> threshold as a function of (n, f), in the reference's attribute order
    _F1 = lambda n, f: f + 1  # noqa: E731
    _NF = lambda n, f: n - f  # noqa: E731
    _NF1 = lambda n, f: n - f - 1  # noqa: E731
    THRESHOLDS = (("propagate", _F1), ("prepare", _NF1), ("commit", _NF), ("reply", _F1),
                  ("view_change", _NF), ("election", _NF), ("view_change_done", _NF),
                  ("propagate_primary", _F1), ("same_consistency_proof", _F1), ("consistency_proof", _F1),
                  ("ledger_status", _NF1), ("checkpoint", lambda n, f: 2 * f), ("timestamp", _F1),
                  ("bls_signatures", _NF))

    class Quorums:
        def __init__(self, n):
            self.f = getMaxFailures(n)
            for name, rule in THRESHOLDS:
                setattr(self, name, Quorum(rule(n, self.f)))

        def __str__(self):
            return "{}".format(self.__dict__)
