"""Verify-ahead for the node's receive loop.

Reference: ZStack.processReceived (stp_zmq/zstack.py:528-549) pops
(json_text, ident) pairs from rxMsgs -- up to LISTENER_MESSAGE_QUOTA = 100 per
listener per cycle (plenum/config.py:179) -- and hands each to the node, which
authenticates client REQUESTs (node.py:1439-1440) and the request inside each
PROPAGATE (node.py:1313-1316, 2304-2306) one at a time.

Under load the node-to-node traffic does not arrive as bare messages: a
sender's outbox of more than one message is flushed as ONE signed BATCH
(Batched.flushOutBoxes -> _make_batch, plenum/common/batched.py:99-125,
141-144; Batch = {"op": "BATCH", "messages": [serialized message, ...],
"signature": ...}, node_messages.py:30-36), kept whole by doProcessReceived
(batched.py:149-162, which only drops pings / pongs) and unpacked by
Node.unpackNodeMsg, which deserializes every entry of `messages` with
nodestack.deserializeMsg and re-enters handleOneNodeMsg for it
(node.py:1333-1337).  So the n - 1 PROPAGATE copies of a request mostly sit
INSIDE BATCH entries.  `requests_in_drain` descends into them the same way, so
one GPU batch (`prefetch`) covers client REQUESTs, bare PROPAGATEs and batched
PROPAGATEs alike; the unchanged per-message authenticate() then hits the
verdict cache."""
import json
from itertools import islice

PROPAGATE = "PROPAGATE"
BATCH = "BATCH"
_MAX_BATCH_DEPTH = 2  # the reference never nests batches; bounded anyway


def _decode(raw, deserialize):
    try:
        return deserialize(raw) if isinstance(raw, (str, bytes)) else raw
    except Exception:
        return None


def _collect(m, deserialize, out, depth, seen):
    if not isinstance(m, dict):
        return
    op = m.get("op")
    if op == BATCH:  # node.py:1333-1337: each entry re-enters handleOneNodeMsg
        inner = m.get("messages")
        if depth < _MAX_BATCH_DEPTH and isinstance(inner, list):
            for raw in inner:
                _visit(raw, deserialize, out, depth + 1, seen)
        return
    if op == PROPAGATE:
        m = m.get("request")
        if not isinstance(m, dict):
            return
    if "signature" in m:
        out.append(m)


def _visit(raw, deserialize, out, depth, seen):
    """Decode one entry (every entry: the node loop gets the object back from
    the memo) and collect its requests -- once per distinct raw text: the
    n - 1 PROPAGATEs of a request usually arrive as the same text from every
    node, and one copy is all the prefetch needs (authenticate() recomputes
    every message's own bytes anyway)."""
    m = _decode(raw, deserialize)
    if seen is not None and isinstance(raw, (str, bytes)):
        if raw in seen:
            return
        seen.add(raw)
    _collect(m, deserialize, out, depth, seen)


def requests_in_drain(raw_msgs, deserialize=json.loads, limit=None, distinct=False):
    """Signed request dicts inside a list of raw rxMsgs entries
    ((text, ident) pairs or bare texts): client requests themselves, the
    `request` of PROPAGATE messages, and both of those inside BATCH messages.
    `limit` counts rxMsgs entries (a BATCH is one entry, as in
    processReceived).  Undecodable entries are skipped (the reference logs and
    drops them, zstack.py:541-545).  distinct=True: entries whose raw text
    was already seen in this drain contribute nothing more (they are still
    decoded)."""
    out = []
    seen = set() if distinct else None
    for n, item in enumerate(raw_msgs):
        if limit is not None and n >= limit:
            break
        raw = item[0] if isinstance(item, tuple) else item
        _visit(raw, deserialize, out, 0, seen)
    return out


def prefetch_drain(authnr, raw_msgs, deserialize=json.loads, limit=None):
    """One batched verification for everything the next processReceived(limit)
    will authenticate; returns the number of distinct signatures verified."""
    return authnr.prefetch(requests_in_drain(raw_msgs, deserialize, limit))


class _Memo:
    """Decoded messages of one drain, by the identity of their raw text: the
    verify-ahead decodes each rxMsgs entry (and each entry of a BATCH) once,
    and the stack's deserializeMsg hands that object back when the reference
    loop asks for the same raw object (zstack.py:538, node.py:1335) -- one
    json decode per message instead of two.  An entry is used once; anything
    not found (another object, a second copy) is decoded as before."""

    __slots__ = ("d", "deserialize")

    def __init__(self, deserialize):
        self.d = {}
        self.deserialize = deserialize

    def __call__(self, raw):
        obj = self.deserialize(raw)
        self.d[id(raw)] = (raw, obj)  # raw kept alive, so its id is not reused while held
        return obj

    def take(self, raw):
        e = self.d.pop(id(raw), None)
        if e is not None and e[0] is raw:
            return e[1]
        return _NONE


_NONE = object()


class _MemoDeserialize:
    """VerifyAheadMixin.deserializeMsg: on an instance, the memo's object for a
    raw message it decoded (else the base class's decode); on the class (the
    reference calls ZStack.deserializeMsg(...) as a static method, e.g.
    plenum/test/input_validation/test_message_serialization.py:15), the base
    class's static method itself."""

    def __set_name__(self, owner, name):
        self.owner, self.name = owner, name

    def __get__(self, obj, objtype=None):
        base = getattr(super(self.owner, objtype if objtype is not None else type(obj)), self.name)
        if obj is None:
            return base
        memo = obj._va_memo
        if memo is None:
            return base

        def deserialize(msg):
            o = memo.take(msg)
            return base(msg) if o is _NONE else o
        return deserialize


class VerifyAheadMixin:
    """Mix in front of a ZStack subclass (e.g. plenum.common.stacks.ClientZStack
    / NodeZStack).  The authenticator is the class attribute `authnr`
    (verify_ahead_stack binds it) or a constructor keyword `authnr=`.

    processReceived(limit) first decodes the next `limit` rxMsgs entries
    (descending into BATCH entries) and prefetches their signed requests in one
    GPU batch, then runs the reference loop; deserializeMsg returns the
    objects decoded for the prefetch, so every message is decoded once."""

    authnr = None
    _va_memo = None

    def __init__(self, *args, authnr=None, **kwargs):
        if authnr is not None:
            self.authnr = authnr
        super().__init__(*args, **kwargs)

    def processReceived(self, limit):
        if self.authnr is None or limit <= 0:
            return super().processReceived(limit)
        memo = _Memo(super().deserializeMsg)
        self.authnr.prefetch(requests_in_drain(islice(self.rxMsgs, limit), memo, limit, distinct=True))
        self._va_memo = memo
        try:
            return super().processReceived(limit)
        finally:
            self._va_memo = None

    deserializeMsg = _MemoDeserialize()


_stack_classes = {}


def verify_ahead_stack(base, authnr):
    """A subclass of the stack class `base` whose processReceived prefetches
    for `authnr`: what a Node subclass returns from its nodeStackClass /
    clientStackClass properties (node.py:536-541; the node constructs its
    stacks as cls(**kwargs) at node.py:182-196, after clientAuthNr is set at
    :168), see INTEGRATION.md section 4."""
    key = (base, id(authnr))
    cls = _stack_classes.get(key)
    if cls is None or cls.authnr is not authnr:
        cls = type("VerifyAhead" + base.__name__, (VerifyAheadMixin, base), {"authnr": authnr})
        _stack_classes[key] = cls
    return cls
