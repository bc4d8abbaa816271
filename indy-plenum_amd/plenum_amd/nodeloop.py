"""The receive loop a Plenum node runs over its two stacks, restated so the
drop-in can be driven (bench.py's end_to_end.node_drain leg, the drain tests)
exactly the way a node drives it, without the rest of the node.

What a node does per rxMsgs entry (reference files):
  ZStack.processReceived(limit)      stp_zmq/zstack.py:528-549
    popleft (text, ident); ping / pong dropped (handlePingPong :655-666);
    msg = self.deserializeMsg(text) (json, :776-780); doProcessReceived
    (plenum/common/batched.py:149-162: pings / pongs dropped from a BATCH's
    messages); msgHandler((msg, frm))
  client stack -> Node.handleOneClientMsg -> validateClientMsg
    (plenum/server/node.py:1399-1451): a request (operation, identifier,
    reqId present) becomes SafeRequest(**msg); verifySignature(cMsg)
    (node.py:2294-2314) authenticates cMsg.as_dict (request.py:27-39: a NEW
    dict of identifier / reqId / operation / signature / protocolVersion)
  node stack -> Node.handleOneNodeMsg -> validateNodeMsg (node.py:1270-1320):
    verifySignature(message): a PROPAGATE authenticates message.request (the
    decoded dict itself); a BATCH is whitelisted; then unpackNodeMsg
    (node.py:1322-1337) re-enters handleOneNodeMsg for every entry of
    `messages`, each decoded with self.nodestack.deserializeMsg
  an authenticate() error: the client gets a REQNACK (node.py:2568-2571); a
    node's message is SuspiciousNode (node.py:1313-1316) -- counted here.

Message validation (schemas), the 3PC handlers and the outboxes are not part
of the path and are left out; the loop calls authenticate() with the same
objects in the same order as the node.  `Stack` is the bare ZStack loop;
`verify_ahead_stack(Stack, authnr)` (batching.py) gives the node's stack with
the verify-ahead wired in, as INTEGRATION.md section 4 does for the real one.
"""
import json
from collections import deque

PING, PONG = b"pi", b"po"  # zstack.py pingMessage / pongMessage
OPERATION, IDENTIFIER, REQ_ID, SIGNATURE, PROTOCOL_VERSION = (
    "operation", "identifier", "reqId", "signature", "protocolVersion")


class NodeCounters:
    """What the node's handlers did with a drain's messages."""

    def __init__(self):
        self.authenticated = 0   # authenticate() returned the identifier
        self.rejected = 0        # authenticate() raised (REQNACK / SuspiciousNode)
        self.messages = 0        # messages handed to a handler (BATCH entries included)
        self.outcomes = []       # (kind, identifier or exception class name), when record=True
        self.record = False


class Stack:
    """ZStack's receive loop (zstack.py:528-549) with the node's handler for
    this stack (client: node.py:1363-1451; node: node.py:1270-1337)."""

    def __init__(self, authnr, kind="node", counters=None):
        assert kind in ("node", "client")
        self.rxMsgs = deque()
        self.kind = kind
        self.auth = authnr       # Node.clientAuthNr (node.authNr(req), node.py:2320)
        self.nc = counters or NodeCounters()

    @staticmethod
    def deserializeMsg(msg):  # zstack.py:776-780
        if isinstance(msg, bytes):
            msg = msg.decode()
        return json.loads(msg)

    def handlePingPong(self, msg, frm, ident):
        return msg in (PING, PONG)

    def doProcessReceived(self, msg, frm, ident):  # batched.py:149-162
        if msg.get("op") == "BATCH" and isinstance(msg.get("messages"), list):
            relevant = [m for m in msg["messages"] if not self.handlePingPong(m, frm, ident)]
            if not relevant:
                return None
            msg["messages"] = relevant
        return msg

    def processReceived(self, limit):  # zstack.py:528-549
        if limit <= 0:
            return 0
        num_processed = 0
        for num_processed in range(limit):
            if len(self.rxMsgs) == 0:
                return num_processed
            msg, ident = self.rxMsgs.popleft()
            frm = ident
            if self.handlePingPong(msg, frm, ident):
                continue
            try:
                msg = self.deserializeMsg(msg)
            except Exception:
                continue
            msg = self.doProcessReceived(msg, frm, ident)
            if msg:
                self.msgHandler((msg, frm))
        return num_processed + 1

    # -- the node's handlers ----------------------------------------------------
    def msgHandler(self, wrapped):
        if self.kind == "client":
            self.handleOneClientMsg(wrapped)
        else:
            self.handleOneNodeMsg(wrapped)

    def _authenticate(self, req, kind):
        nc = self.nc
        try:
            idr = self.auth.authenticate(req)
        except Exception as ex:  # REQNACK to the client / SuspiciousNode for a node
            nc.rejected += 1
            if nc.record:
                nc.outcomes.append((kind, type(ex).__name__))
            return False
        nc.authenticated += 1
        if nc.record:
            nc.outcomes.append((kind, idr))
        return True

    def handleOneClientMsg(self, wrapped):  # node.py:1399-1451, a request
        msg, frm = wrapped
        self.nc.messages += 1
        if not isinstance(msg, dict) or not all(k in msg for k in (OPERATION, IDENTIFIER, REQ_ID)):
            return
        # SafeRequest(**msg).as_dict (request.py:27-39): a new dict with the request's fields
        req = {IDENTIFIER: msg[IDENTIFIER], REQ_ID: msg[REQ_ID], OPERATION: msg[OPERATION]}
        if msg.get(SIGNATURE) is not None:
            req[SIGNATURE] = msg[SIGNATURE]
        if msg.get(PROTOCOL_VERSION) is not None:
            req[PROTOCOL_VERSION] = msg[PROTOCOL_VERSION]
        self._authenticate(req, "request")

    def handleOneNodeMsg(self, wrapped):  # node.py:1270-1337
        msg, frm = wrapped
        self.nc.messages += 1
        if not isinstance(msg, dict):
            return
        op = msg.get("op")
        if op == "PROPAGATE":
            req = msg.get("request")
            if isinstance(req, dict):
                self._authenticate(req, "propagate")
        elif op == "BATCH":  # whitelisted; unpackNodeMsg re-enters for every entry
            for m in msg.get("messages") or ():
                try:
                    m = self.deserializeMsg(m)
                except Exception:
                    continue
                self.handleOneNodeMsg((m, frm))


def batch_text(texts):
    """A node's flushed outbox (Batched._make_batch, batched.py:141-144):
    Batch(messages=[serialized message, ...], signature=None), serialized."""
    return json.dumps({"op": "BATCH", "messages": list(texts), "signature": None})


def propagate_text(req, sender_client):
    """A PROPAGATE of a client request (node_messages.py Propagate), serialized."""
    return json.dumps({"op": "PROPAGATE", "request": req, "senderClient": sender_client})


def drain_texts(reqs, n_nodes=25, client_names=None):
    """One drain's rxMsgs of a node in an n-node pool: the clients' REQUESTs
    (client stack) and, from each of the other n - 1 nodes, one BATCH with
    its PROPAGATE of every request (node stack).  Returns (client, node)
    lists of (text, ident) pairs."""
    client = [(json.dumps(r), "client%d" % i) for i, r in enumerate(reqs)]
    props = [propagate_text(r, (client_names or {}).get(i, "client%d" % i)) for i, r in enumerate(reqs)]
    node = [(batch_text(props), "Node%d" % k) for k in range(2, n_nodes + 1)]
    return client, node
