"""The node's per-message path (CPU, oracle engine double):

* authn_key: authenticate()'s host steps up to getVerkey in one native call --
  (identifier, b58decode(signature) || serialization) or None exactly where the
  Python path must decide (it raises the reference's exception);
* authenticate()'s native form == the per-message Python form on every
  reference KAT, the verdict-cache hit included;
* distinct_sm: one verify per distinct (identifier, sig || ser) of a drain;
* the verify-ahead stack over the restated node loop (plenum_amd/nodeloop.py):
  one prefetch per drain, one decode per message (the reference loop gets the
  prefetch's objects back), one engine launch for the drain's distinct
  requests, and authenticate() outcomes identical to the bare loop's."""

import pytest
from engine_double import OracleEngine
from test_client_authn import _outcome, _signed

from plenum_amd import _hostpack
from plenum_amd.base58 import b58decode
from plenum_amd.batching import verify_ahead_stack
from plenum_amd.client_authn import GpuAuthNr
from plenum_amd.nodeloop import NodeCounters, Stack, drain_texts
from plenum_amd.serialization import serialize_msg_for_signing


def test_authn_key_matches_python_steps():
    idrs, vks, msgs = _signed(3, 50)
    odd = [dict(msgs[0], operation={"type": "1", "x": 1.5, "n": None, "l": [1, True, "é"]}),
           dict(msgs[1], reqId=2 ** 80), dict(msgs[2], identifier="ünicode")]
    for m in msgs + odd:
        k = _hostpack.authn_key(m, ("signature",))
        assert k is not None
        assert k[0] == m["identifier"]
        assert k[1] == b58decode(m["signature"]) + serialize_msg_for_signing(m, topLevelKeysToIgnore=["signature"])
    # the Python path decides: missing / empty / non-str fields, bad base58, non-dict, unserializable
    base = msgs[0]
    for bad in ({k: v for k, v in base.items() if k != "signature"}, dict(base, signature=""),
                {k: v for k, v in base.items() if k != "identifier"}, dict(base, identifier=""),
                dict(base, signature="0OIl"), dict(base, signature=b"abc"), dict(base, identifier=5),
                dict(base, signature="ü"), dict(base, operation={"t": (1, 2)}), dict(base, operation={1: "x"}),
                [base], None):
        assert _hostpack.authn_key(bad, ("signature",)) is None, bad


class _PyOnly(GpuAuthNr):
    """authenticate() pinned to the per-message Python path."""

    def _native_host_steps(self):
        return False


def test_native_authenticate_equals_python_path_on_kats(oracle):
    """Every reference KAT through authenticate(): the native host steps and the
    per-message Python path give the same identifier or exception (class,
    args, cause), first call and verdict-cache hit alike, and both match the
    reference's recorded outcome."""
    from test_client_authn import check_result, fix_case, kat
    n = 0
    for c in kat()["cases"]:
        outs = []
        for cls in (GpuAuthNr, _PyOnly):
            a = cls(engine=OracleEngine(oracle))
            if c["register"]:
                a.addIdr(c["msg"].get("identifier") if c["identifier"] is None else c["identifier"], c["verkey"])
            for _ in range(2):
                try:
                    r = a.authenticate(fix_case(c), c["identifier"], c["signature"])
                except Exception as ex:
                    r = ex
                check_result(c, r)
                outs.append(_outcome(r))
        assert outs[:2] == outs[2:], c["name"]
        n += 1
    assert n >= 20


def test_native_authenticate_uses_one_native_call(oracle, monkeypatch):
    """The node's call (no identifier / signature arguments) on a prefetched
    request: no _prepare, no engine call, a verdict-cache hit; a changed
    verkey for the identifier is seen at the next call (getVerkey runs every
    time, as in the reference)."""
    idrs, vks, msgs = _signed(2, 6)
    a = GpuAuthNr(engine=OracleEngine(oracle))
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    assert a.prefetch(msgs) == 6
    calls = a.engine.calls
    from plenum_amd import client_authn as CA
    monkeypatch.setattr(CA, "b58decode", lambda *x: pytest.fail("python path"))  # only _prepare uses it
    assert [a.authenticate(dict(m)) for m in msgs] == [m["identifier"] for m in msgs]
    assert a.engine.calls == calls and a.stats["cache_hits"] == 6
    a.addIdr(idrs[0], vks[1])  # the identifier's key changes: its requests no longer verify
    from plenum_amd.exceptions import InvalidSignature
    with pytest.raises(InvalidSignature):
        a.authenticate(dict(msgs[0]))
    assert a.authenticate(dict(msgs[1])) == idrs[1]


def test_distinct_sm_dedupes_copies():
    idrs, vks, msgs = _signed(2, 10)
    batch = [dict(m) for m in msgs] * 3 + [dict(msgs[0], reqId=99)]
    scan = _hostpack.scan_batch_u(batch, ["signature"], 1, None, 64)
    fast, uidx, uniq, sig, msgbuf, off, short = scan
    picks, sms = _hostpack.distinct_sm(memoryview(sig)[:64 * len(batch)], msgbuf, off, short, uidx, fast)
    assert picks == list(range(10)) + [30]
    for i, sm in zip(picks, sms):
        m = batch[i]
        assert sm == b58decode(m["signature"]) + serialize_msg_for_signing(m, topLevelKeysToIgnore=["signature"])


def _node(oracle, n_signers=4, n_reqs=40, n_nodes=7):
    idrs, vks, reqs = _signed(n_signers, n_reqs)
    eng = OracleEngine(oracle)
    a = GpuAuthNr(engine=eng)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    a.keys_settle()
    return a, eng, idrs, vks, reqs


@pytest.mark.parametrize("n_nodes", [4, 7])
def test_verify_ahead_node_loop(oracle, monkeypatch, n_nodes):
    a, eng, idrs, vks, reqs = _node(oracle, n_nodes=n_nodes)
    reqs = [dict(r) for r in reqs]
    reqs[5]["reqId"] += 1                  # forged: InvalidSignature at every copy
    reqs[6]["identifier"] = "Unknown11111"  # UnknownIdentifier
    client, node = drain_texts(reqs, n_nodes=n_nodes)
    decodes = []
    real = Stack.deserializeMsg

    def counting(msg):
        decodes.append(1)
        return real(msg)
    monkeypatch.setattr(Stack, "deserializeMsg", staticmethod(counting))
    nc = NodeCounters()
    nc.record = True
    ns = verify_ahead_stack(Stack, a)(a, "node", nc)
    cs = verify_ahead_stack(Stack, a)(a, "client", nc)
    ns.rxMsgs.extend(node)
    cs.rxMsgs.extend(client)
    calls0, prep = eng.calls, []
    orig = GpuAuthNr._authenticate_sm
    monkeypatch.setattr(GpuAuthNr, "_authenticate_sm", lambda self, *x: prep.append(1) or orig(self, *x))
    assert ns.processReceived(100) == n_nodes - 1
    assert cs.processReceived(100) == len(reqs)
    # every raw message decoded once: the BATCHes, their PROPAGATEs, the REQUESTs
    assert len(decodes) == (n_nodes - 1) * (1 + len(reqs)) + len(reqs)
    assert eng.calls - calls0 == 1         # one launch: the node drain's distinct requests
    assert a.stats["single_verifies"] == 0
    assert nc.messages == (n_nodes - 1) * (1 + len(reqs)) + len(reqs)
    assert len(prep) == n_nodes * len(reqs)  # every authenticate() took the native host steps
    # the same outcomes as the bare reference loop with a fresh authenticator
    b, _, _, _, _ = _node(oracle, n_nodes=n_nodes)
    nb = NodeCounters()
    nb.record = True
    s1, s2 = Stack(b, "node", nb), Stack(b, "client", nb)
    s1.rxMsgs.extend(node)
    s2.rxMsgs.extend(client)
    s1.processReceived(100)
    s2.processReceived(100)
    assert nc.outcomes == nb.outcomes
    want = [r["identifier"] for r in reqs]
    want[5], want[6] = "InvalidSignature", "UnknownIdentifier"
    assert [o[1] for o in nc.outcomes] == want * (n_nodes - 1) + want


def test_distinct_sm_rejects_bad_offsets():
    import numpy as np
    sig = bytes(64 * 2)
    off = np.array([0, 10, 5], np.uint64).tobytes()
    with pytest.raises(ValueError):
        _hostpack.distinct_sm(sig, bytes(20), off, bytes(2), bytes(8), b"\x01\x01")
    off = np.array([0, 10, 30], np.uint64).tobytes()
    with pytest.raises(ValueError):
        _hostpack.distinct_sm(sig, bytes(20), off, bytes(2), bytes(8), b"\x01\x01")
