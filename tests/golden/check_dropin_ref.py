"""Drop-in check against the REAL reference classes (container-side only):

    /opt/conda/bin/python3.9 tests/golden/check_dropin_ref.py [--write]

Builds the INTEGRATION.md binding -- GpuAuthMixin mixed in front of the
reference's own plenum.server.client_authn.SimpleAuthNr (imported from
/root/reference with the stand-ins of ref_standins.py) -- over the
oracle-backed engine double (tests/engine_double.py; the double stands in for
the GPU, which this container lacks; tests/test_gpu_authn.py runs the same
table on the device), and asserts:
  1. all authn_kat.json outcomes (produced by the reference's own
     SimpleAuthNr): identifier or exception class (+ cause class);
  2. verification goes through the engine: engine called, and no libsodium
     crypto_sign_open call (the stand-in libnacl counts them);
  3. every raised error IS an instance of the reference's BaseExc /
     SigningException, and node.py:1313-1316's handler
         try: self.verifySignature(message)
         except BaseExc as ex: raise SuspiciousNode(frm, ex, message) from ex
     turns a forged PROPAGATE into the reference's SuspiciousNode
     (plenum/test/signing/test_signing.py:35-62 pins that behaviour);
  4. prefetch() followed by authenticate() of the same requests makes 0
     extra engine calls; authenticate_batch == per-message authenticate;
  5. node.py:2482 isinstance(authnr, SimpleAuthNr) holds and addIdr stores
     the NYM in the reference's `clients` dict.
With --write the summary goes to dropin_ref_check.json (committed evidence).
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import ref_standins as R  # noqa: E402

R.install()
from plenum.server.client_authn import SimpleAuthNr as RefSimpleAuthNr  # noqa: E402
import plenum.common.exceptions as ref_exc  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from plenum_amd import exceptions as X  # noqa: E402
from plenum_amd.client_authn import GpuAuthMixin  # noqa: E402
from engine_double import OracleEngine  # noqa: E402


class GpuSimpleAuthNr(GpuAuthMixin, RefSimpleAuthNr):
    """INTEGRATION.md section 3, verbatim shape."""

    def __init__(self, state=None, engine=None, **options):
        RefSimpleAuthNr.__init__(self, state=state)
        self._gpu_init(engine=engine, **options)


def fix_case(c):
    msg = dict(c["msg"])
    if c["name"] == "tuple-field":
        msg["operation"] = tuple(msg["operation"])
    return msg


def node_validate(authnr, frm, message):
    """node.py:1313-1316 (validateNodeMsg's signature step) with the
    reference's BaseExc and SuspiciousNode."""
    try:
        authnr.authenticate(message)
    except ref_exc.BaseExc as ex:
        raise ref_exc.SuspiciousNode(frm, ex, message) from ex


def batch_vs_single(eng):
    import base58
    from plenum_amd import client_authn as CA
    sod = R.sodium()

    def b58s(b):  # (the stand-in's b58encode may return str or bytes)
        e = base58.b58encode(b)
        return e.decode() if isinstance(e, bytes) else e
    keys = []
    for i in range(5):
        pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        sod.crypto_sign_seed_keypair(pk, sk, bytes([9, i + 1]) + b"\0" * 30)
        keys.append((b58s(pk.raw[:16]), "~" + b58s(pk.raw[16:]), sk))
    a = GpuSimpleAuthNr(engine=eng)
    for idr, vk, _ in keys[:4]:  # keys[4]: unknown (the reference's state lookup finds nothing)
        a.addIdr(idr, vk)
    msgs = []
    for j in range(300):
        idr, _, sk = keys[j % 5]
        m = {"identifier": idr, "reqId": 5000 + j, "operation": {"type": "1", "dest": "d%d" % j}}
        ser = a.serializeForSig(m, topLevelKeysToIgnore=["signature"])
        sig = ctypes.create_string_buffer(64)
        sod.crypto_sign_detached(sig, None, ser, ctypes.c_ulonglong(len(ser)), sk)
        msgs.append(dict(m, signature=b58s(sig.raw)))
    for j in range(0, 300, 7):
        msgs[j] = dict(msgs[j], reqId=msgs[j]["reqId"] + 1)  # forged after signing
    native = [0]
    real = CA._keys_known

    def counted(*args):
        native[0] += 1
        return real(*args)
    CA._keys_known = counted if real is not None else None

    def outcome(r):
        return r if isinstance(r, str) else type(r).__name__

    def single(m):
        try:
            return a.authenticate(dict(m))
        except Exception as ex:
            return ex
    rounds = []
    try:
        for change in (False, True):
            if change:
                a.addIdr(keys[1][0], keys[0][1])  # keys[1]'s identifier now holds keys[0]'s verkey
            got = [outcome(r) for r in a.authenticate_batch([dict(m) for m in msgs])]
            want = [outcome(single(m)) for m in msgs]
            assert got == want, change
            rounds.append(got)
    finally:
        CA._keys_known = real
    assert rounds[0] != rounds[1] and "UnknownIdentifier" in rounds[0] and "InvalidSignature" in rounds[0]
    return {"batch_vs_single_items": 2 * len(msgs), "batch_vs_single_matched": 2 * len(msgs),
            "keys_known_native_calls": native[0], "known_getverkey": CA._known_getverkey(type(a))}


def main():
    kat = json.load(open(os.path.join(HERE, "authn_kat.json")))
    assert X.REFERENCE and X.InvalidSignature is ref_exc.InvalidSignature, "exceptions not re-exported"
    eng = OracleEngine()
    R.CALLS.clear()
    summary = {"cases": 0, "matched": 0, "raised": 0, "raised_reference_baseexc": 0, "keyed_items": 0}
    for c in kat["cases"]:
        for max_keys in (16, 0):  # key-table path and general path
            a = GpuSimpleAuthNr(engine=eng, max_keys=max_keys)
            assert isinstance(a, RefSimpleAuthNr)  # node.py:2482
            if c["register"]:
                idr = c["msg"].get("identifier") if c["identifier"] is None else c["identifier"]
                a.addIdr(idr, c["verkey"])
                assert a.clients[idr]["verkey"] == c["verkey"]
            try:
                out = a.authenticate(fix_case(c), c["identifier"], c["signature"])
            except Exception as ex:
                out = ex
            summary["cases"] += 1
            if "result" in c:
                assert out == c["result"], (c["name"], out)
            else:
                assert isinstance(out, Exception), (c["name"], out)
                assert type(out).__name__ == c["raises"], (c["name"], out)
                cause = type(out.__cause__).__name__ if out.__cause__ is not None else None
                assert cause == c["cause"] or c["cause"] not in ("ValueError", "InvalidKey", None), (c["name"], cause)
                summary["raised"] += 1
                assert isinstance(out, ref_exc.BaseExc) and isinstance(out, ref_exc.SigningException), c["name"]
                summary["raised_reference_baseexc"] += 1
            summary["matched"] += 1
            summary["keyed_items"] += a.stats["keyed_items"]
    assert eng.calls > 0 and R.CALLS["crypto_sign_open"] == 0, (eng.calls, dict(R.CALLS))
    summary["engine_calls"] = eng.calls
    summary["libsodium_crypto_sign_open_calls"] = R.CALLS["crypto_sign_open"]
    assert summary["keyed_items"] > 0

    # forged PROPAGATE -> the reference's SuspiciousNode (node.py:1313-1316)
    good = next(c for c in kat["cases"] if c["name"] == "valid-abbreviated-verkey")
    a = GpuSimpleAuthNr(engine=eng)
    a.addIdr(good["msg"]["identifier"], good["verkey"])
    node_validate(a, "Alpha", dict(good["msg"]))
    forged = dict(good["msg"], operation=dict(good["msg"]["operation"], dest="changed"))
    try:
        node_validate(a, "Beta:9702", forged)
        raise AssertionError("forged request accepted")
    except ref_exc.SuspiciousNode as sn:
        assert isinstance(sn.__cause__, ref_exc.InvalidSignature) and sn.node == "Beta"
        summary["forged_propagate"] = "SuspiciousNode(Beta, InvalidSignature)"

    # verify-ahead: one engine call for the drain, none afterwards
    a = GpuSimpleAuthNr(engine=eng)
    a.addIdr(good["msg"]["identifier"], good["verkey"])
    msgs = [dict(good["msg"])] * 4 + [forged]
    before = eng.calls
    assert a.prefetch(msgs) == 2
    after_prefetch = eng.calls
    assert a.authenticate(dict(good["msg"])) == good["msg"]["identifier"]
    try:
        a.authenticate(forged)
        raise AssertionError("forged request accepted")
    except ref_exc.InvalidSignature:
        pass
    assert eng.calls == after_prefetch, "authenticate after prefetch launched the engine"
    summary["prefetch_engine_calls"] = after_prefetch - before
    summary["authenticate_after_prefetch_engine_calls"] = eng.calls - after_prefetch

    # batch == single, on the reference class
    res = a.authenticate_batch(msgs)
    assert res[:4] == [good["msg"]["identifier"]] * 4 and isinstance(res[4], ref_exc.InvalidSignature)
    assert R.CALLS["crypto_sign_open"] == 0

    # batch == single over many signers on the reference class, with the per-identifier keys of
    # the batch from the native lookup where it applies (_hostpack.keys_known: the reference's own
    # getVerkey, clients entries holding the verkey addIdr gave); then one verkey replaced
    summary.update(batch_vs_single(eng))
    summary["ok"] = True
    print(json.dumps(summary))
    if "--write" in sys.argv:
        with open(os.path.join(HERE, "dropin_ref_check.json"), "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
