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
    assert st.authnr.batches == [[req]]  # the two entries are the same text: one copy prefetched
    assert prefetch_drain(st.authnr, st.rxMsgs) == 3


def _batch(msgs):
    """A node's flushed outbox as the reference frames it: Batched._make_batch
    (plenum/common/batched.py:141-144) wraps the already-serialized messages in
    Batch(msgs, None) (node_messages.py:30-36), serialized by ZStack.serializeMsg."""
    return json.dumps({"op": "BATCH", "messages": [json.dumps(m) for m in msgs], "signature": None})


def test_requests_inside_batch_messages():
    """node.py:1333-1337: each entry of a BATCH re-enters handleOneNodeMsg, so
    PROPAGATEs inside a BATCH are authenticated like bare ones."""
    r1 = {"identifier": "a", "reqId": 1, "operation": {"type": "1"}, "signature": "s1"}
    r2 = {"identifier": "b", "reqId": 2, "operation": {"type": "1"}, "signature": "s2"}
    prop = [{"op": "PROPAGATE", "request": r, "senderClient": "c"} for r in (r1, r2)]
    other = {"op": "PREPARE", "instId": 0, "viewNo": 0, "ppSeqNo": 1}
    drain = [(json.dumps(r1), b"c1"),
             (_batch([prop[0], other, prop[1]]), b"Node2"),
             (json.dumps({"op": "BATCH", "messages": ["not json", json.dumps(prop[1])], "signature": None}), b"N3"),
             (json.dumps({"op": "BATCH", "messages": "oops", "signature": None}), b"N4"),
             (json.dumps({"op": "BATCH", "messages": [_batch([prop[0]])], "signature": None}), b"N5")]
    assert requests_in_drain(drain) == [r1, r1, r2, r2, r1]
    # a BATCH is one rxMsgs entry for processReceived's limit
    assert requests_in_drain(drain, limit=2) == [r1, r1, r2]
    # bytes entries (the wire form) decode like str ones
    assert requests_in_drain([(_batch(prop).encode(), b"n")], deserialize=lambda m: json.loads(m)) == [r1, r2]


def test_verify_ahead_stack_binds_authenticator():
    """verify_ahead_stack(base, authnr): the class a Node subclass returns from
    nodeStackClass / clientStackClass (node.py:536-541); the node constructs it
    as cls(**kwargs) (node.py:182-196)."""
    from plenum_amd.batching import verify_ahead_stack

    class Base(_Stack):
        def __init__(self, msgs=(), **kw):
            _Stack.__init__(self, msgs)
            self.kw = kw

    auth = _Auth()
    cls = verify_ahead_stack(Base, auth)
    assert verify_ahead_stack(Base, auth) is cls and issubclass(cls, Base)
    req = {"identifier": "a", "signature": "s"}
    st = cls(msgs=[(_batch([{"op": "PROPAGATE", "request": req}] * 2), b"n")], stackParams={"name": "x"})
    assert st.kw == {"stackParams": {"name": "x"}}
    st.processReceived(100)
    assert auth.batches == [[req]]  # identical PROPAGATE texts inside the BATCH: one copy
    other = _Auth()
    st2 = verify_ahead_stack(Base, auth)(msgs=[(json.dumps(req), 1)], authnr=other)
    st2.processReceived(1)
    assert other.batches == [[req]] and len(auth.batches) == 1


def test_memo_decode_edge_cases():
    """The verify-ahead's decode memo: the same raw object twice in rxMsgs (the
    second is decoded afresh, never the same dict twice), ping / pong entries
    (left to the reference loop), an undecodable entry, and deserializeMsg on
    the class (a static call, as the reference's own tests make)."""
    from plenum_amd.batching import verify_ahead_stack
    from plenum_amd.nodeloop import PING, NodeCounters, Stack

    class Auth:
        def __init__(self):
            self.seen = []

        def prefetch(self, reqs):
            return len(reqs)

        def authenticate(self, req):
            self.seen.append(req)
            return req["identifier"]
    a = Auth()
    cls = verify_ahead_stack(Stack, a)
    assert cls.deserializeMsg('{"a": 1}') == {"a": 1}  # class-level: the base's static method
    nc = NodeCounters()
    st = cls(a, "node", nc)
    req = {"identifier": "i", "reqId": 1, "operation": {"type": "1"}, "signature": "s"}
    prop = json.dumps({"op": "PROPAGATE", "request": req, "senderClient": "c"})
    batch = json.dumps({"op": "BATCH", "messages": [prop, PING.decode(), prop], "signature": None})
    st.rxMsgs.extend([(prop, "n1"), (prop, "n1"), (PING, "n2"), ("{not json", "n3"), (batch, "n4")])
    assert st.processReceived(10) == 5
    assert len(a.seen) == 4 and all(r == req for r in a.seen)
    assert len({id(r) for r in a.seen}) == 4  # every authenticate() got its own dict
    assert st._va_memo is None
