"""Verify-ahead for the node's receive loop.

Reference: ZStack.processReceived (stp_zmq/zstack.py:528-549) pops
(json_text, ident) pairs from rxMsgs -- up to LISTENER_MESSAGE_QUOTA = 100 per
listener per cycle (plenum/config.py:179) -- and hands each to the node, which
authenticates client REQUESTs (node.py:1439-1440) and the request inside each
PROPAGATE (node.py:1313-1316, 2304-2306) one at a time.  `requests_in_drain`
pulls those requests out of a drain so one GPU batch (`prefetch`) covers them;
the unchanged per-message authenticate() then hits the verdict cache."""
import json

PROPAGATE = "PROPAGATE"


def requests_in_drain(raw_msgs, deserialize=json.loads, limit=None):
    """Signed request dicts inside a list of raw rxMsgs entries
    ((text, ident) pairs or bare texts): client requests themselves and the
    `request` of PROPAGATE messages.  Undecodable entries are skipped (the
    reference logs and drops them, zstack.py:541-545)."""
    out = []
    for n, item in enumerate(raw_msgs):
        if limit is not None and n >= limit:
            break
        raw = item[0] if isinstance(item, tuple) else item
        try:
            m = deserialize(raw) if isinstance(raw, (str, bytes)) else raw
        except Exception:
            continue
        if not isinstance(m, dict):
            continue
        if m.get("op") == PROPAGATE:
            m = m.get("request")
            if not isinstance(m, dict):
                continue
        if "signature" in m:
            out.append(m)
    return out


def prefetch_drain(authnr, raw_msgs, deserialize=json.loads, limit=None):
    """One batched verification for everything the next processReceived(limit)
    will authenticate; returns the number of distinct signatures verified."""
    return authnr.prefetch(requests_in_drain(raw_msgs, deserialize, limit))


class VerifyAheadMixin:
    """Mix in front of a ZStack subclass (e.g. plenum.common.stacks.ClientZStack
    / NodeZStack) constructed with `authnr=<GpuAuthMixin instance>`."""

    authnr = None

    def processReceived(self, limit):
        if self.authnr is not None and limit > 0:
            prefetch_drain(self.authnr, list(self.rxMsgs), self.deserializeMsg, limit)
        return super().processReceived(limit)
