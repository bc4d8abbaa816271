"""Verify-ahead extraction from a receive-loop drain (plenum_amd/batching.py)."""
import json

from plenum_amd.batching import VerifyAheadMixin, prefetch_drain, requests_in_drain


def test_requests_in_drain():
    req = {"identifier": "a", "reqId": 1, "operation": {"type": "1"}, "signature": "s"}
    drain = [(json.dumps(req), b"c1"), ("not json", b"c2"), (json.dumps({"op": "PROPAGATE", "request": req,
                                                                         "senderClient": "x"}), b"n1"),
             (json.dumps({"op": "PREPARE", "viewNo": 0}), b"n2"), (json.dumps([1, 2]), b"n3"),
             (json.dumps({"identifier": "b"}), b"c3")]
    got = requests_in_drain(drain)
    assert got == [req, req]
    assert requests_in_drain(drain, limit=1) == [req]


class _Stack:
    def __init__(self, msgs):
        self.rxMsgs = list(msgs)
        self.processed = 0

    def deserializeMsg(self, m):
        return json.loads(m)

    def processReceived(self, limit):
        self.processed += min(limit, len(self.rxMsgs))
        return self.processed


class _Auth:
    def __init__(self):
        self.batches = []

    def prefetch(self, reqs):
        self.batches.append(reqs)
        return len(reqs)


def test_verify_ahead_mixin_prefetches_then_processes():
    class S(VerifyAheadMixin, _Stack):
        pass
    req = {"identifier": "a", "signature": "s"}
    st = S([(json.dumps(req), 1)] * 3)
    st.authnr = _Auth()
    assert st.processReceived(2) == 2
    assert st.authnr.batches == [[req, req]]
    assert prefetch_drain(st.authnr, st.rxMsgs) == 3
