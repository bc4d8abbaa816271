"""Host-side logic of the drop-in authenticator: check order, exception
classes and causes, batching, verify-ahead, multi-signature extension.

Verdicts come from an oracle-backed test double (conftest.OracleEngine); the
same table runs against the real GPU engine in test_gpu_authn.py.  The
expectations are tests/golden/authn_kat.json, produced by running the
reference's own NaclAuthNr/SimpleAuthNr/DidVerifier (gen_ref_kats.py)."""
import json
import os

import pytest

from conftest import GOLDEN
from engine_double import OracleEngine
from plenum_amd import exceptions as X
from plenum_amd.client_authn import GpuAuthNr, ReqAuthenticator, SimpleAuthNr
from plenum_amd.verifier import DidVerifier


def kat():
    return json.load(open(os.path.join(GOLDEN, "authn_kat.json")))


def fix_case(c):
    msg = dict(c["msg"])
    if c["name"] == "tuple-field":
        msg["operation"] = tuple(msg["operation"])  # JSON turned the tuple into a list
    return msg


def make(engine, c):
    a = GpuAuthNr(engine=engine)
    if c["register"]:
        a.addIdr(c["msg"].get("identifier") if c["identifier"] is None else c["identifier"], c["verkey"])
    return a


def check_result(c, outcome):
    if "result" in c:
        assert outcome == c["result"], c["name"]
    else:
        assert isinstance(outcome, Exception), (c["name"], outcome)
        assert type(outcome).__name__ == c["raises"], (c["name"], outcome)
        cause = type(outcome.__cause__).__name__ if outcome.__cause__ is not None else None
        if c["cause"] in ("AttributeError", "ValueError", "Exception", "InvalidKey", None):
            assert cause == c["cause"], (c["name"], cause)


def run_single(a, c):
    try:
        return a.authenticate(fix_case(c), c["identifier"], c["signature"])
    except Exception as ex:
        return ex


def test_authenticate_matches_reference_kats(oracle_engine):
    for c in kat()["cases"]:
        check_result(c, run_single(make(oracle_engine, c), c))


def test_authenticate_batch_equals_single(oracle_engine):
    cases = [c for c in kat()["cases"] if c["register"]]
    # one authenticator holding every identity the cases use (same verkey per idr)
    by_idr = {}
    for c in cases:
        idr = c["msg"].get("identifier") if c["identifier"] is None else c["identifier"]
        by_idr.setdefault((idr, c["verkey"]), []).append(c)
    for (idr, vk), group in by_idr.items():
        a = GpuAuthNr(engine=oracle_engine)
        a.addIdr(idr, vk)
        res = a.authenticate_batch([fix_case(c) for c in group], [c["identifier"] for c in group],
                                   [c["signature"] for c in group])
        for c, r in zip(group, res):
            check_result(c, r)


def test_batch_is_one_engine_call(oracle_engine):
    good = next(c for c in kat()["cases"] if c["name"] == "valid-abbreviated-verkey")
    a = make(oracle_engine, good)
    msgs = [good["msg"]] * 5 + [dict(good["msg"], reqId=7)] * 3
    before = oracle_engine.calls
    res = a.authenticate_batch(msgs)
    assert oracle_engine.calls == before + 1
    assert res[:5] == [good["msg"]["identifier"]] * 5
    assert all(isinstance(r, X.InvalidSignature) for r in res[5:])


def test_prefetch_then_authenticate_hits_cache(oracle_engine):
    good = next(c for c in kat()["cases"] if c["name"] == "valid-abbreviated-verkey")
    a = make(oracle_engine, good)
    bad = dict(good["msg"], reqId=9)
    assert a.prefetch([good["msg"], bad, good["msg"], {"no": "sig"}]) == 2  # deduped, unsigned skipped
    calls = oracle_engine.calls
    assert a.authenticate(good["msg"]) == good["msg"]["identifier"]
    with pytest.raises(X.InvalidSignature):
        a.authenticate(bad)
    assert oracle_engine.calls == calls and a.stats["cache_hits"] == 2
    with pytest.raises(X.MissingSignature):
        a.authenticate({"no": "sig"})


def test_did_verifier_reference_kats():
    for d in kat()["did_expand"]:
        assert DidVerifier(d["verkey"], identifier=d["identifier"]).verkey == d["expanded"]
    with pytest.raises(X.InvalidKey, match="verkey FFFF"):
        DidVerifier('FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF')  # test_verifier.py:18-23


def test_reference_dummy_authenticator(oracle_engine):
    # plenum/test/client/test_client_authn.py:39-52: getVerkey -> None
    class Dummy(GpuAuthNr):
        def getVerkey(self, _):
            return None
    good = next(c for c in kat()["cases"] if c["name"] == "valid-abbreviated-verkey")
    with pytest.raises(X.CouldNotAuthenticate):
        Dummy(engine=oracle_engine).authenticate(good["msg"])


def test_simpleauthnr_state_lookup(oracle_engine):
    good = next(c for c in kat()["cases"] if c["name"] == "valid-abbreviated-verkey")
    idr = good["msg"]["identifier"]
    a = GpuAuthNr(state="S", nym_lookup=lambda st, i: {"verkey": good["verkey"]} if (st, i) == ("S", idr) else {},
                  engine=oracle_engine)
    assert a.authenticate(good["msg"]) == idr
    assert isinstance(a, SimpleAuthNr)


def test_reqid_reason_text():
    ex = X.CouldNotAuthenticate()
    ex.__cause__ = X.InvalidKey("verkey abc")
    assert X.reasonForClientFromException(ex) == \
        "client request invalid: CouldNotAuthenticate() [caused by verkey abc]"


# --- authenticate_multi (extension; parity unpinned: only per-signature
# verdicts are pinned, by libsodium through the oracle) ----------------------
def _multi_fixture(oracle_engine):
    import ctypes
    from plenum_amd.base58 import b58encode
    from plenum_amd.serialization import serialize_msg_for_signing
    from conftest import sodium
    s = sodium()
    if s is None:
        pytest.skip("needs libsodium to sign")
    a = GpuAuthNr(engine=oracle_engine)
    msg = {"identifier": "x", "reqId": 1, "operation": {"type": "1"}}
    ser = serialize_msg_for_signing(msg, topLevelKeysToIgnore=["signature", "signatures"])
    sigs = {}
    for i in range(4):
        pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        s.crypto_sign_seed_keypair(pk, sk, bytes([i + 1]) * 32)
        idr = b58encode(pk.raw[:16])
        a.addIdr(idr, "~" + b58encode(pk.raw[16:]))
        sig = ctypes.create_string_buffer(64)
        s.crypto_sign_detached(sig, None, ser, ctypes.c_ulonglong(len(ser)), sk)
        sigs[idr] = b58encode(sig.raw)
    return a, msg, sigs


def test_authenticate_multi(oracle_engine):
    a, msg, sigs = _multi_fixture(oracle_engine)
    idrs = list(sigs)
    assert a.authenticate_multi(msg, sigs) == idrs
    assert a.authenticate_multi(msg, sigs, threshold=2) == idrs[:2]
    with pytest.raises(X.InsufficientSignatures):
        a.authenticate_multi(msg, sigs, threshold=5)
    bad = dict(sigs)
    bad[idrs[0]] = sigs[idrs[1]]
    assert a.authenticate_multi(msg, bad, threshold=3) == idrs[1:]
    with pytest.raises(X.InsufficientCorrectSignatures):
        a.authenticate_multi(msg, bad)
    fmt = dict(sigs)
    fmt[idrs[0]] = "0OIl"
    with pytest.raises(X.InvalidSignatureFormat):
        a.authenticate_multi(msg, fmt)
    res = a.authenticate_multi_batch([(msg, sigs, None), (msg, bad, None), (msg, bad, 3), (msg, sigs, 9)])
    assert res[0] == idrs and res[2] == idrs[1:]
    assert isinstance(res[1], X.InsufficientCorrectSignatures) and isinstance(res[3], X.InsufficientSignatures)


def test_req_authenticator(oracle_engine):
    good = next(c for c in kat()["cases"] if c["name"] == "valid-abbreviated-verkey")
    ra = ReqAuthenticator()
    ra.register_authenticator(make(oracle_engine, good))
    assert ra.authenticate(good["msg"]) == {good["msg"]["identifier"]}
    assert isinstance(ra.core_authenticator, GpuAuthNr)


def _outcomes(engine, max_keys):
    out, keyed = [], 0
    for c in kat()["cases"]:
        a = GpuAuthNr(engine=engine, max_keys=max_keys)
        if c["register"]:
            a.addIdr(c["msg"].get("identifier") if c["identifier"] is None else c["identifier"], c["verkey"])
        r = run_single(a, c)
        out.append(r if not isinstance(r, Exception) else (type(r).__name__,
                                                            type(r.__cause__).__name__ if r.__cause__ else None))
        keyed += a.stats["keyed_items"]
    return out, keyed


def test_keyed_and_general_paths_agree(oracle):
    """addIdr registers verkeys in the engine's key store (key-table path);
    with no store (max_keys = 0) the same requests take the general path. The
    reference KAT outcomes (incl. 63/65-byte signatures split at byte 64 on
    the host for the keyed path) are identical either way."""
    with_keys, n_keyed = _outcomes(OracleEngine(oracle), 16)
    without, n_general = _outcomes(OracleEngine(oracle), 0)
    assert with_keys == without
    assert n_keyed > 0 and n_general == 0


def _signed(n_signers, n_msgs, seed=1):
    """n_msgs NYM-like requests from n_signers libsodium keys: (idrs, verkeys, msgs)."""
    import ctypes
    from plenum_amd.base58 import b58encode
    from plenum_amd.serialization import serialize_msg_for_signing
    from conftest import sodium
    s = sodium()
    if s is None:
        pytest.skip("needs libsodium to sign")
    keys = []
    for i in range(n_signers):
        pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        s.crypto_sign_seed_keypair(pk, sk, bytes([seed, i + 1]) + b"\0" * 30)
        keys.append((b58encode(pk.raw[:16]), "~" + b58encode(pk.raw[16:]), sk))
    msgs = []
    for j in range(n_msgs):
        idr, _, sk = keys[j % n_signers]
        m = {"identifier": idr, "reqId": 1000 + j, "operation": {"type": "1", "dest": "d%d" % j}}
        ser = serialize_msg_for_signing(m, topLevelKeysToIgnore=["signature"])
        sig = ctypes.create_string_buffer(64)
        s.crypto_sign_detached(sig, None, ser, ctypes.c_ulonglong(len(ser)), sk)
        msgs.append(dict(m, signature=b58encode(sig.raw)))
    return [k[0] for k in keys], [k[1] for k in keys], msgs


def test_hot_keys_get_registered_after_verifying(oracle_engine):
    idrs, vks, msgs = _signed(1, 8)
    a = GpuAuthNr(engine=oracle_engine, nym_lookup=lambda st, idr: {"verkey": vks[0]}, hot_key_uses=2)
    assert a.authenticate_batch(msgs[:4]) == [idrs[0]] * 4      # general path, 4 verified uses
    assert len(a._g.hot) == 1 and a.stats["keyed_items"] == 0   # earned a slot
    assert a.authenticate_batch(msgs[4:]) == [idrs[0]] * 4      # registered, now keyed
    assert a.stats["keys_registered"] == 1 and a.stats["keyed_items"] == 4


def test_bad_signatures_do_not_promote_keys(oracle_engine):
    idrs, vks, msgs = _signed(1, 6)
    a = GpuAuthNr(engine=oracle_engine, nym_lookup=lambda st, idr: {"verkey": vks[0]}, hot_key_uses=2)
    forged = [dict(m, reqId=m["reqId"] + 1) for m in msgs]
    for _ in range(3):
        assert all(isinstance(r, X.InvalidSignature) for r in a.authenticate_batch(forged))
    assert a.stats["keys_registered"] == 0 and len(a._g.hot) == 0


def test_two_authenticators_share_one_engine(oracle_engine):
    """ids of one authenticator must never point at another's keys."""
    idrs, vks, msgs = _signed(2, 4)
    a, b = GpuAuthNr(engine=oracle_engine), GpuAuthNr(engine=oracle_engine)
    a.addIdr(idrs[0], vks[0])
    b.addIdr(idrs[1], vks[1])
    assert a.authenticate_batch([msgs[0], msgs[2]]) == [idrs[0]] * 2
    assert b.authenticate_batch([msgs[1], msgs[3]]) == [idrs[1]] * 2
    assert a.authenticate_batch([msgs[0], msgs[2]]) == [idrs[0]] * 2   # a's id still bound to a's key
    assert a.stats["keyed_items"] == 4 and b.stats["keyed_items"] == 2
    # b's identity cannot authenticate through a (a has no NYM for it)
    r = a.authenticate_batch([msgs[1]])[0]
    assert isinstance(r, X.UnknownIdentifier)
    # a reset of the engine's store by anyone: ids are dropped, verdicts stay right
    oracle_engine.keys_reset()
    assert b.authenticate_batch([msgs[1]]) == [idrs[1]]


def test_key_store_lru_eviction(oracle_engine):
    idrs, vks, msgs = _signed(3, 30)
    table = dict(zip(idrs, vks))
    a = GpuAuthNr(engine=oracle_engine, nym_lookup=lambda st, idr: {"verkey": table[idr]}, max_keys=2,
                  hot_key_uses=1)
    for k in range(0, 30, 3):  # one signer per batch, cycling over 3 signers with room for 2
        s = (k // 3) % 3
        assert a.authenticate_batch([msgs[k + s]] * 2) == [idrs[s]] * 2
    assert len(oracle_engine.keys) == 2 and a.stats["keys_registered"] >= 3
    assert a.stats["keyed_items"] > 0


def test_registration_failure_falls_back_to_general(oracle_engine):
    idrs, vks, msgs = _signed(1, 6)
    oracle_engine.fail_keys_add = True
    a = GpuAuthNr(engine=oracle_engine)
    a.addIdr(idrs[0], vks[0])
    assert a.authenticate_batch(msgs[:3]) == [idrs[0]] * 3
    assert a.authenticate_batch(msgs[3:]) == [idrs[0]] * 3
    assert a.stats["keyed_items"] == 0 and a.stats["keys_registered"] == 0


def _outcome(r):
    if isinstance(r, Exception):
        return (type(r).__name__, r.args, type(r.__cause__).__name__ if r.__cause__ else None)
    return r


def test_scanned_batch_equals_single_on_kats(oracle):
    """authenticate_batch's native-scan path (hostpack.scan_batch) gives, per
    message, exactly what authenticate() gives -- including every reference
    KAT error case, in one mixed batch over one authenticator."""
    from plenum_amd import client_authn as CA
    assert CA._scan_batch is not None
    cases = [c for c in kat()["cases"] if c["identifier"] is None and c["signature"] is None]
    for max_keys in (16, 0):
        eng = OracleEngine(oracle)
        a = GpuAuthNr(engine=eng, max_keys=max_keys)
        b = GpuAuthNr(engine=OracleEngine(oracle), max_keys=max_keys)
        for c in cases:
            if c["register"] and c["name"] not in ("verkey-31-bytes", "verkey-hex-encoded", "verkey-none",
                                                   "verkey-non-base58", "verkey-abbrev-15-bytes"):
                idr = c["msg"].get("identifier")
                a.addIdr(idr, c["verkey"])
                b.addIdr(idr, c["verkey"])
        msgs = [fix_case(c) for c in cases] * 3
        got = [_outcome(r) for r in a.authenticate_batch(msgs)]
        want = []
        for m in msgs:
            try:
                want.append(_outcome(b.authenticate(m)))
            except Exception as ex:
                want.append(_outcome(ex))
        assert got == want


def test_concurrent_batches_serialised_on_the_engine(oracle):
    """A batch from another thread waits for the engine lock (held from key
    routing through the verify), so it neither overwrites the reused scan
    buffers nor rebinds key ids an in-flight batch resolved."""
    import threading
    import time
    from plenum_amd.client_authn import _engine_lock
    idrs, vks, msgs = _signed(2, 30, seed=4)
    eng = OracleEngine(oracle)
    a = GpuAuthNr(engine=eng)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    want = [_outcome(r) for r in a.authenticate_batch(msgs)]
    assert all(isinstance(x, str) for x in want)
    got = []
    with _engine_lock(eng):  # a first batch in flight
        t = threading.Thread(target=lambda: got.append([_outcome(r) for r in a.authenticate_batch(msgs)]))
        t.start()
        time.sleep(0.3)
        assert t.is_alive() and not got
    t.join(30)
    assert got == [want]


def test_concurrent_batches_with_evictions(oracle):
    """Threads on two authenticators sharing one engine whose key store holds
    2 keys of 6 hot signers (every batch evicts): every verdict stays right."""
    import threading
    idrs, vks, msgs = _signed(6, 36, seed=8)
    bad = [dict(m, reqId=m["reqId"] + 1) if i % 5 == 0 else m for i, m in enumerate(msgs)]
    eng = OracleEngine(oracle)
    auths = [GpuAuthNr(engine=eng, max_keys=2, hot_key_uses=1) for _ in range(2)]
    for a in auths:
        for idr, vk in zip(idrs, vks):
            a.addIdr(idr, vk)
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for idr, vk in zip(idrs, vks):
        ref.addIdr(idr, vk)
    want = [_outcome(r) for r in ref.authenticate_batch(bad)]
    assert sum(1 for w in want if w[0] == "InvalidSignature") == 8
    errors = []

    def work(a, k):
        for it in range(6):
            batch = bad[k % 6:] + bad[:k % 6]
            got = [_outcome(r) for r in a.authenticate_batch(batch)]
            if got != want[k % 6:] + want[:k % 6]:
                errors.append((k, it))
            k += 1

    th = [threading.Thread(target=work, args=(auths[i % 2], i)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors and eng.keyed_calls > 0


def test_overridden_serializer_keeps_the_per_message_path(oracle):
    """A host class with its own serializeForSig: authenticate_batch uses it
    (the native scan would restate the mixin's), so batch == per-message."""
    idrs, vks, msgs = _signed(1, 4, seed=2)

    class Custom(GpuAuthNr):
        def serializeForSig(self, msg, topLevelKeysToIgnore=None):
            return b"custom" + super().serializeForSig(msg, topLevelKeysToIgnore)

    a = Custom(engine=OracleEngine(oracle))
    a.addIdr(idrs[0], vks[0])
    assert not a._native_host_steps() and GpuAuthNr(engine=OracleEngine(oracle))._native_host_steps()
    got = [_outcome(r)[0] for r in a.authenticate_batch(msgs)]
    assert got == ["InvalidSignature"] * 4  # signed over the plain bytes
    for m in msgs:
        with pytest.raises(Exception) as ei:
            a.authenticate(m)
        assert type(ei.value).__name__ == "InvalidSignature"


def test_scanned_batch_fuzz(oracle):
    """Random request dicts (valid, tampered, odd field types, missing / empty
    fields, non-base58, short signatures): scanned batch == per-message."""
    import random
    idrs, vks, msgs = _signed(3, 60, seed=9)
    rnd = random.Random(5)
    pool = []
    for m in msgs:
        m = dict(m)
        r = rnd.random()
        if r < 0.1:
            m["reqId"] += 1
        elif r < 0.15:
            m["signature"] = ""
        elif r < 0.2:
            del m["signature"]
        elif r < 0.25:
            m["identifier"] = ""
        elif r < 0.3:
            m["signature"] = m["signature"][:20]
        elif r < 0.35:
            m["signature"] = "0" + m["signature"]
        elif r < 0.4:
            m["operation"] = {"type": "1", "x": (1, 2)}
        elif r < 0.45:
            m["extra"] = [1, 2.5, None, True, {"k": "v"}]
        elif r < 0.5:
            m["identifier"] = "unknownIdr"
        elif r < 0.55:
            m["signature"] = 12345
        pool.append(m)
    for max_keys in (16, 0):
        a = GpuAuthNr(engine=OracleEngine(oracle), max_keys=max_keys)
        b = GpuAuthNr(engine=OracleEngine(oracle), max_keys=max_keys)
        for idr, vk in zip(idrs, vks):
            a.addIdr(idr, vk)
            b.addIdr(idr, vk)
        got = [_outcome(r) for r in a.authenticate_batch(pool)]
        want = []
        for m in pool:
            try:
                want.append(_outcome(b.authenticate(m)))
            except Exception as ex:
                want.append(_outcome(ex))
        assert got == want
        assert sum(isinstance(x, str) for x in got) > 10


def test_scan_slots_into_engine_buffers(oracle):
    """A batch large enough for the engine's (pinned) host buffers: the scan
    writes signature slots (base58 text for signatures that decode to 64
    bytes, raw R || S otherwise) straight into host_alloc memory; verdicts ==
    authenticate() per message, including 63- / 65-byte signatures (split at
    byte 64 on the host) and non-base58 ones."""
    from plenum_amd.base58 import b58decode, b58encode
    idrs, vks, msgs = _signed(4, 64, seed=6)
    pool = []
    for k in range(4200):
        m = dict(msgs[k % 64])
        r = k % 50
        if r == 1:
            m["reqId"] += 7  # tampered
        elif r == 2:
            m["signature"] = b58encode(b58decode(m["signature"])[:63])  # 63 bytes: ser[0] joins the signature
        elif r == 3:
            m["signature"] = b58encode(b58decode(m["signature"]) + b"\x01")  # 65 bytes: spills into M
        elif r == 4:
            m["signature"] = "0OIl" + m["signature"][4:]  # not base58
        elif r == 5:
            m["signature"] = b58encode(b"\0\0" + b58decode(m["signature"])[2:])  # leading '1's, 64 bytes
        pool.append(m)
    eng = OracleEngine(oracle)
    a = GpuAuthNr(engine=eng)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    got = [_outcome(r) for r in a.authenticate_batch(pool)]
    assert getattr(eng, "host_allocs", 0) == 2 and eng.slot_text_items > 3800
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for idr, vk in zip(idrs, vks):
        ref.addIdr(idr, vk)
    want = []
    for m in pool[:400]:
        try:
            want.append(_outcome(ref.authenticate(m)))
        except Exception as ex:
            want.append(_outcome(ex))
    assert got[:400] == want
    assert got == got[:200] * 21
    # a second, larger batch grows the buffers; a smaller one reuses them
    a.authenticate_batch(pool + pool[:3000])
    a.authenticate_batch(pool[:4100])
    assert eng.host_allocs == 4


def test_pipelined_parts_equal_per_message(oracle):
    """A batch scanned in parts (pipeline_part): steady-state parts are
    submitted asynchronously (verify_submit / verify_collect), a part with an
    unknown identifier, a non-base58 signature, a missing field and a
    registered-later key takes the ordinary path; verdicts == authenticate()
    per message, and getVerkey runs once per identifier of the whole batch."""
    idrs, vks, msgs = _signed(5, 80, seed=11)
    pool = []
    for k in range(6000):
        m = dict(msgs[k % 80])
        if k % 37 == 0:
            m["reqId"] += 1
        pool.append(m)
    pool[2500] = dict(pool[2500], identifier="UnknownIdr1111111111")
    pool[2600] = dict(pool[2600], signature="0OIl" + pool[2600]["signature"][4:])
    del pool[2700]["identifier"]
    eng = OracleEngine(oracle)
    a = GpuAuthNr(engine=eng, pipeline_part=1024)
    for idr, vk in zip(idrs[:4], vks[:4]):
        a.addIdr(idr, vk)
    a.clients[idrs[4]] = {"verkey": vks[4], "role": None}  # known, not queued for a key slot
    calls = []
    orig = a.getVerkey
    a.getVerkey = lambda idr: calls.append(idr) or orig(idr)
    got = [_outcome(r) for r in a.authenticate_batch(pool)]
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for idr, vk in zip(idrs, vks):
        ref.addIdr(idr, vk)
    want = []
    for m in pool:
        try:
            want.append(_outcome(ref.authenticate(m)))
        except Exception as ex:
            want.append(_outcome(ex))
    assert got == want
    assert getattr(eng, "submits", 0) >= 2
    assert sorted(calls) == sorted(set(calls))  # once per identifier
    # the next batch: idrs[4] promoted by use earlier, everything steady -> every part asynchronous
    eng.submits = 0
    got2 = [_outcome(r) for r in a.authenticate_batch(pool[:4096])]
    assert got2 == want[:4096] and eng.submits >= 3


def _ref_outcomes(oracle, batches, lookup=None):
    """The same batches through an authenticator with no key store (general path only)."""
    ref = GpuAuthNr(engine=OracleEngine(oracle), nym_lookup=lookup, max_keys=0)
    return [[_outcome(r) for r in ref.authenticate_batch(b)] for b in batches]


def test_async_key_builds_stay_off_the_request_path(oracle):
    """VERDICT r2 'keep hot-key table builds off the request path': an addIdr
    key and a key promoted by use register with keys_add_async / keys_set_async
    (the double raises on the synchronous forms); until a build completes its
    requests take the general path, and the verdicts are the general path's at
    every step, across an eviction too."""
    from engine_double import AsyncOracleEngine
    eng = AsyncOracleEngine(oracle)
    idrs, vks, msgs = _signed(3, 48)
    table = dict(zip(idrs, vks))
    a = GpuAuthNr(engine=eng, nym_lookup=lambda st, idr: {"verkey": table[idr]}, max_keys=2, hot_key_uses=1)
    a.addIdr(idrs[0], vks[0])
    batches = [[msgs[k + s] for k in range(j, j + 12, 3) for s in range(2)] for j in range(0, 48, 12)]
    lookup = lambda st, idr: {"verkey": table[idr]}  # noqa: E731
    want = _ref_outcomes(oracle, batches + [[m for m in msgs if m["identifier"] == idrs[2]][:4]], lookup)
    # batch 1: idrs[0]'s key (addIdr) is queued, not built: everything general; idrs[1] earns a slot
    assert [_outcome(r) for r in a.authenticate_batch(batches[0])] == want[0]
    assert a.stats["keyed_items"] == 0 and eng.issued == 1
    # batch 2: idrs[1]'s build is queued in this batch, idrs[0]'s still running: still general
    assert [_outcome(r) for r in a.authenticate_batch(batches[1])] == want[1]
    assert a.stats["keyed_items"] == 0 and eng.issued == 2
    eng.finish_builds()
    # batch 3: both built -> keyed
    assert [_outcome(r) for r in a.authenticate_batch(batches[2])] == want[2]
    assert a.stats["keyed_items"] == len(batches[2])
    # idrs[2] earns a slot with the store full: an eviction rebuild (keys_set_async), its requests general
    third = [m for m in msgs if m["identifier"] == idrs[2]][:4]
    assert [_outcome(r) for r in a.authenticate_batch(third)] == want[4]
    before = a.stats["keyed_items"]
    assert [_outcome(r) for r in a.authenticate_batch(third)] == want[4]
    assert eng.issued == 3 and a.stats["keyed_items"] == before  # evicted into, still building
    assert eng.sync_calls == 0  # no batch ever waited on a build
    eng.finish_builds()
    assert [_outcome(r) for r in a.authenticate_batch(third)] == want[4]
    assert a.stats["keyed_items"] == before + len(third)


def test_keys_settle_waits_for_queued_builds(oracle):
    from engine_double import AsyncOracleEngine
    eng = AsyncOracleEngine(oracle)
    idrs, vks, msgs = _signed(2, 8)
    a = GpuAuthNr(engine=eng)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    assert a.keys_settle() == 2 and eng.sync_calls == 1 and not eng.building
    assert a.authenticate_batch(msgs) == [m["identifier"] for m in msgs]
    assert a.stats["keyed_items"] == len(msgs)


def test_streamed_batch_equals_whole(oracle, monkeypatch):
    """authenticate_batch's streamed path (scan with the pack deferred, then per
    library chunk pack_range + verify_submit, so a chunk's DMA overlaps the
    next chunk's pack): the same outcome per message as the unstreamed path,
    in the steady state (keys registered) and when the batch leaves it (an
    unknown identifier, a missing signature, a forgery)."""
    from plenum_amd import client_authn as CA
    idrs, vks, msgs = _signed(3, 5000)
    monkeypatch.setattr(CA, "_STREAM_CHUNK", 1024)
    eng = OracleEngine(oracle)
    a = GpuAuthNr(engine=eng)
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
        ref.addIdr(i, v)
    a.keys_settle()
    batch = [dict(m) for m in msgs]
    batch[17]["reqId"] += 1  # forged
    subs = getattr(eng, "submits", 0)
    got = [_outcome(r) for r in a.authenticate_batch(batch)]
    assert got == [_outcome(r) for r in ref.authenticate_batch(batch)]
    assert eng.submits - subs == 5 and a.stats["keyed_items"] == 5000  # 5 chunks streamed, all keyed
    odd = [dict(m) for m in msgs]
    odd[3]["identifier"] = "UnknownIdentifier1111"
    del odd[4000]["signature"]
    got = [_outcome(r) for r in a.authenticate_batch(odd)]
    assert got == [_outcome(r) for r in ref.authenticate_batch(odd)]


def test_staged_batch_equals_whole(oracle, monkeypatch):
    """authenticate_batch's staged path (the scan's workers place each chunk's
    messages at a bump cursor and queue its messages and slots to the device
    with edv_stage_put -- here the CPU stand-in, called from the same worker
    threads -- then edv_verify_staged over the item spans): the same outcome
    per message as the unstaged path in the steady state, when the batch
    leaves it (messages repacked from the spans), and when the pinned message
    buffer is too small (the batch is scanned again the ordinary way)."""
    from engine_double import StagingOracleEngine
    from plenum_amd import client_authn as CA
    idrs, vks, msgs = _signed(3, 5000)
    monkeypatch.setattr(CA, "_STAGE_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PINNED_MIN_BATCH", 1000)
    eng = StagingOracleEngine(oracle)
    a = GpuAuthNr(engine=eng, stage=True)
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
        ref.addIdr(i, v)
    a.keys_settle()
    batch = [dict(m) for m in msgs]
    batch[17]["reqId"] += 1                       # forged
    batch[99]["signature"] = batch[99]["signature"][:-2]   # decodes to < 64 bytes: raw slot, split at 64
    assert [_outcome(r) for r in a.authenticate_batch(batch)] == [_outcome(r) for r in ref.authenticate_batch(batch)]
    assert eng.staged_calls == 1 and a.stats["keyed_items"] == 5000
    odd = [dict(m) for m in msgs]
    odd[3]["identifier"] = "UnknownIdentifier1111"
    del odd[4000]["signature"]
    assert [_outcome(r) for r in a.authenticate_batch(odd)] == [_outcome(r) for r in ref.authenticate_batch(odd)]
    assert eng.staged_calls == 1  # left the steady state: repacked, ordinary path
    small = GpuAuthNr(engine=StagingOracleEngine(oracle), stage=True)
    for i, v in zip(idrs, vks):
        small.addIdr(i, v)
    small.keys_settle()
    small._g.msg_bytes_per_item = 10.0           # pinned message buffer far too small for this batch
    assert [_outcome(r) for r in small.authenticate_batch(batch)] == \
        [_outcome(r) for r in ref.authenticate_batch(batch)]
    assert small.engine.staged_calls == 0


def test_staged_batch_one_scan_thread(oracle, monkeypatch):
    """The staged scan with scan_threads=1 over more than one 4k-item stage
    chunk: the serial scan still publishes every chunk's slots (run_chunks
    walks the chunks in order instead of one call over the whole batch), so
    items past the first chunk are verified against their own slots."""
    from engine_double import StagingOracleEngine
    from plenum_amd import client_authn as CA
    idrs, vks, msgs = _signed(3, 9000)
    monkeypatch.setattr(CA, "_STAGE_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PINNED_MIN_BATCH", 1000)
    eng = StagingOracleEngine(oracle)
    a = GpuAuthNr(engine=eng, stage=True, scan_threads=1)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    a.keys_settle()
    batch = [dict(m) for m in msgs]
    batch[8500]["reqId"] += 1  # forged, in the third stage chunk
    got = a.authenticate_batch(batch)
    assert eng.staged_calls == 1
    assert [_outcome(r) for r in got] == [m["identifier"] if i != 8500 else ("InvalidSignature", (), None)
                                          for i, m in enumerate(msgs)]


def test_streamed_batch_bounded_in_flight(oracle, monkeypatch):
    """More streamed chunks than the in-flight window: the oldest submissions
    are collected before new ones go out (the library refuses a 65th
    uncollected ticket), and the verdicts stay in request order."""
    from plenum_amd import client_authn as CA
    idrs, vks, msgs = _signed(3, 5000)
    monkeypatch.setattr(CA, "_STREAM_CHUNK", 128)
    monkeypatch.setattr(CA, "_STREAM_WINDOW", 4)
    eng = OracleEngine(oracle)
    a = GpuAuthNr(engine=eng)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    a.keys_settle()
    batch = [dict(m) for m in msgs]
    batch[4321]["reqId"] += 1
    got = a.authenticate_batch(batch)
    assert eng.max_in_flight <= 4
    assert [_outcome(r) for r in got] == [m["identifier"] if i != 4321 else ("InvalidSignature", (), None)
                                          for i, m in enumerate(msgs)]


def test_pipelined_parts_bounded_in_flight(oracle, monkeypatch):
    """a pipelined batch of more parts than the library holds
    tickets (kMaxPending = 64): the oldest parts are collected before new ones
    go out, every verdict in request order."""
    from plenum_amd import client_authn as CA
    idrs, vks, msgs = _signed(3, 4480)
    monkeypatch.setattr(CA, "_STREAM_WINDOW", 5)
    eng = OracleEngine(oracle)
    a = GpuAuthNr(engine=eng, pipeline_part=64)  # 70 parts
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    a.keys_settle()
    batch = [dict(m) for m in msgs]
    batch[4400]["reqId"] += 1
    got = a.authenticate_batch(batch)
    assert eng.submits >= 70 and eng.max_in_flight <= 5 and eng.in_flight == 0
    assert [_outcome(r) for r in got] == [m["identifier"] if i != 4400 else ("InvalidSignature", (), None)
                                          for i, m in enumerate(msgs)]


@pytest.mark.parametrize("where", ["streamed", "pipelined"])
def test_batch_raising_between_submit_and_collect_frees_tickets(oracle, monkeypatch, where):
    """an exception after some chunks were submitted and before they
    were collected (here in the pack, or in a later part's scan) leaves no
    ticket outstanding, so the next batch on the same engine still runs."""
    from plenum_amd import client_authn as CA
    idrs, vks, msgs = _signed(3, 5000)
    eng = OracleEngine(oracle)
    if where == "streamed":
        monkeypatch.setattr(CA, "_STREAM_CHUNK", 512)
        a = GpuAuthNr(engine=eng)
        real, name = CA._pack_range, "_pack_range"
    else:
        a = GpuAuthNr(engine=eng, pipeline_part=512)
        real, name = CA._scan_batch, "_scan_batch"
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    a.keys_settle()
    calls = []

    def flaky(*args):
        calls.append(1)
        if len(calls) == 4:
            raise MemoryError("injected")
        return real(*args)
    monkeypatch.setattr(CA, name, flaky)
    with pytest.raises(MemoryError):
        a.authenticate_batch([dict(m) for m in msgs])
    assert eng.submits >= 2 and eng.in_flight == 0
    monkeypatch.setattr(CA, name, real)
    assert a.authenticate_batch(msgs) == [m["identifier"] for m in msgs]
    assert eng.in_flight == 0


def test_authenticate_batches_pipeline(oracle, monkeypatch):
    """authenticate_batches: two batches in flight over the engine's two
    staging sets (the double refuses to reuse a set whose submission was not
    collected), every outcome equal to authenticate_batch's, batch by batch,
    with batches that leave the steady state (a forgery is steady; an unknown
    identifier and a missing signature are not; a batch below the staging
    threshold) finished synchronously in order."""
    from engine_double import StagingOracleEngine
    from plenum_amd import client_authn as CA
    monkeypatch.setattr(CA, "_STAGE_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PINNED_MIN_BATCH", 1000)
    idrs, vks, msgs = _signed(3, 6000)
    eng = StagingOracleEngine(oracle)
    a = GpuAuthNr(engine=eng)
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
        ref.addIdr(i, v)
    a.keys_settle()
    batches = [[dict(m) for m in msgs[k * 1200:(k + 1) * 1200]] for k in range(5)]
    batches[1][7]["reqId"] += 1                           # forged: still the steady state
    batches[2][3]["identifier"] = "UnknownIdentifier1111"  # leaves it: finished synchronously
    del batches[3][5]["signature"]
    batches.insert(4, [dict(m) for m in msgs[:50]])       # below the staging threshold
    got = [[_outcome(r) for r in res] for res in a.authenticate_batches(iter(batches))]
    want = [[_outcome(r) for r in ref.authenticate_batch(b)] for b in batches]
    assert got == want
    # batches 0, 1 and 5 were in flight: 0 submitted, 1 and 5 speculated (their kernels queued
    # under their scans with the ids of the batches before)
    assert eng.submits_staged == 1 and a._g.stats["speculated"] == 2 * 1200 and eng.held == [None, None]
    assert list(a.authenticate_batches([])) == []


def test_authenticate_batches_speculation_hits_and_misses(oracle, monkeypatch):
    """authenticate_batches speculates too: a batch whose identifiers all
    resolved in the batches before runs its kernels under its own scan (and
    is collected when the caller asks for it); a batch bringing an identifier
    the kid map does not hold drops its parts and takes the ordinary submit;
    every outcome equals authenticate_batch's."""
    from engine_double import StagingOracleEngine
    from plenum_amd import client_authn as CA
    monkeypatch.setattr(CA, "_STAGE_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PINNED_MIN_BATCH", 1000)
    idrs, vks, msgs = _signed(4, 7200)
    eng = StagingOracleEngine(oracle)
    a = GpuAuthNr(engine=eng)
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
        ref.addIdr(i, v)
    a.keys_settle()
    three = [dict(m) for m in msgs if m["identifier"] != idrs[3]]
    batches = [three[k * 1200:(k + 1) * 1200] for k in range(3)]  # signers 0-2 only
    batches.insert(2, [dict(m) for m in msgs[:1200]])             # signer 3 appears: a miss
    batches[1][11]["signature"] = batches[1][12]["signature"]      # a forgery in a speculated batch
    got = [[_outcome(r) for r in res] for res in a.authenticate_batches(iter(batches))]
    want = [[_outcome(r) for r in ref.authenticate_batch(b)] for b in batches]
    assert got == want
    # batch 0: no kid map yet; batch 2: the miss -- both submitted; batches 1 and 3 speculated
    assert eng.submits_staged == 2 and a._g.stats["speculated"] == 2 * 1200 and eng.held == [None, None]


def test_authenticate_batches_abandoned_frees_the_set(oracle, monkeypatch):
    """An authenticate_batches iteration closed with a batch in flight collects
    it, so the staging sets are free for the next call."""
    from engine_double import StagingOracleEngine
    from plenum_amd import client_authn as CA
    monkeypatch.setattr(CA, "_STAGE_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PINNED_MIN_BATCH", 1000)
    idrs, vks, msgs = _signed(3, 2400)
    eng = StagingOracleEngine(oracle)
    a = GpuAuthNr(engine=eng)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    a.keys_settle()
    b = [dict(m) for m in msgs[:1200]]
    it = a.authenticate_batches([b, b, b])
    first = next(it)  # batch 0 returned; batch 1 in flight
    it.close()
    assert eng.held[0] is None and eng.held[1] is None
    assert first == [m["identifier"] for m in b]
    assert a.authenticate_batch(b) == first


def test_authenticate_batch_while_an_iteration_holds_set_0(oracle, monkeypatch):
    """an authenticate_batches generator left unfinished (still
    referenced) with its batch in flight in staging set 0; a later
    authenticate_batch does not raise out of the busy set: it takes the
    unpinned path, with the same outcomes, and leaves the batch in flight
    alone until the iteration is finished."""
    from engine_double import StagingOracleEngine
    from plenum_amd import client_authn as CA
    monkeypatch.setattr(CA, "_STAGE_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PINNED_MIN_BATCH", 1000)
    idrs, vks, msgs = _signed(3, 2400)
    eng = StagingOracleEngine(oracle)
    a = GpuAuthNr(engine=eng)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    a.keys_settle()
    b = [dict(m) for m in msgs[:1200]]
    want = [m["identifier"] for m in b]
    it = a.authenticate_batches([b, b, b, b])
    assert next(it) == want and next(it) == want  # batch 2 now in flight in set 0
    assert eng.held[0] is not None
    forged = [dict(m) for m in b]
    forged[9]["reqId"] += 1
    got = a.authenticate_batch(forged)
    assert [_outcome(r) for r in got] == [m["identifier"] if i != 9 else ("InvalidSignature", (), None)
                                          for i, m in enumerate(b)]
    assert eng.held[0] is not None  # untouched
    assert list(it) == [want, want] and eng.held == [None, None]


def _staged_pair(oracle, monkeypatch, n_msgs=5500, **kw):
    from engine_double import StagingOracleEngine
    from plenum_amd import client_authn as CA
    monkeypatch.setattr(CA, "_STAGE_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PINNED_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PART_ITEMS", 4096)
    idrs, vks, msgs = _signed(5, n_msgs)
    eng = StagingOracleEngine(oracle)
    a = GpuAuthNr(engine=eng, **kw)
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for i, v in zip(idrs[:4], vks[:4]):
        a.addIdr(i, v)
    a.clients[idrs[4]] = {"verkey": vks[4], "role": None}  # known, not queued for a key slot
    for i, v in zip(idrs, vks):
        ref.addIdr(i, v)
    a.keys_settle()
    return eng, a, ref, idrs, vks, msgs


def test_speculative_staged_batches(oracle, monkeypatch):
    """A synchronous staged batch whose kernels run under its own scan (key ids
    from kid_map, edv_verify_staged_part per staged part -- the double
    snapshots each part as the library DMAs it): the first batch builds the
    map, the next ones speculate; forgeries still reject; a new signer, an
    identifier whose key moved (eviction: KeyStore.version) and a failing part
    all fall back to the ordinary verify; every outcome equals the general
    path's."""
    eng, a, ref, idrs, vks, msgs = _staged_pair(oracle, monkeypatch, max_keys=4)
    steady = [m for m in msgs if m["identifier"] in idrs[:4]]
    b = [dict(m) for m in steady]
    b[5]["reqId"] += 1
    b[-1]["reqId"] += 1

    def check(batch):
        assert [_outcome(r) for r in a.authenticate_batch(batch)] == \
            [_outcome(r) for r in ref.authenticate_batch(batch)]
        assert eng.held == [None, None]
    check(b)
    assert getattr(eng, "parts_begun", 0) == 0 and a._g.kid_map is not None  # no map yet: ordinary
    check(b)
    assert eng.parts_begun == 1 and a.stats["speculated"] == len(b) and a._g.last_breakdown["speculated"]
    assert eng.parts_verified == len(b)
    # identifiers[4] is known to the state only: its key is not registered -> not the steady state
    check([dict(m) for m in msgs])
    # a new key registered (evicting one of the four): its requests' ids change -> fallback, then speculate
    a.addIdr(idrs[4], vks[4])
    a.keys_settle()
    v0 = a._key_store().version
    mixed = [dict(m) for m in msgs if m["identifier"] != idrs[0]]
    check(mixed)
    spec0 = a.stats["speculated"]
    check(mixed)
    check(mixed)
    assert a._key_store().version >= v0 and a.stats["speculated"] > spec0
    # a part that fails: the ordinary verify
    eng.part_fail_at = 2
    before = a.stats["speculated"]
    check(mixed)
    assert a.stats["speculated"] == before and not a._g.last_breakdown["speculated"]
    eng.part_fail_at = 0
    check(mixed)
    assert a.stats["speculated"] > before


def test_speculative_staged_batch_raising_scan_frees_the_set(oracle, monkeypatch):
    """A scan that raises inside a speculative batch leaves neither staging
    set held."""
    from plenum_amd import client_authn as CA
    eng, a, ref, idrs, vks, msgs = _staged_pair(oracle, monkeypatch)
    steady = [dict(m) for m in msgs if m["identifier"] in idrs[:4]]
    a.authenticate_batch(steady)
    real = CA._scan_batch

    def boom(*args):
        if len(args) > 8 and args[8] is not None:
            raise MemoryError("injected")
        return real(*args)
    monkeypatch.setattr(CA, "_scan_batch", boom)
    with pytest.raises(MemoryError):
        a.authenticate_batch(steady)
    assert eng.held == [None, None]
    monkeypatch.setattr(CA, "_scan_batch", real)
    assert a.authenticate_batch(steady) == [m["identifier"] for m in steady]


def test_speculative_batch_raising_after_the_scan_frees_the_set(oracle, monkeypatch):
    """Something raising between the scan and the parts' collect (here the key store's lookup)
    propagates and leaves neither staging set held; the next batch speculates again."""
    from plenum_amd import keystore as KS
    eng, a, ref, idrs, vks, msgs = _staged_pair(oracle, monkeypatch)
    steady = [dict(m) for m in msgs if m["identifier"] in idrs[:4]]
    a.authenticate_batch(steady)  # the kid map
    real = KS.KeyStore.lookup_array

    def boom(self, keys, *rest):
        raise MemoryError("injected")
    monkeypatch.setattr(KS.KeyStore, "lookup_array", boom)
    with pytest.raises(MemoryError):
        a.authenticate_batch(steady)
    assert eng.held == [None, None]
    monkeypatch.setattr(KS.KeyStore, "lookup_array", real)
    before = a._g.stats.get("speculated", 0)
    assert a.authenticate_batch(steady) == [m["identifier"] for m in steady]
    assert a._g.stats["speculated"] == before + len(steady) and eng.held == [None, None]


def test_pipelined_speculative_batch_raising_scan_frees_the_sets(oracle, monkeypatch):
    """authenticate_batches: a scan that raises while batch k's kernels are in
    flight and batch k + 1 speculates propagates, and neither staging set
    stays held (the open parts are ended and collected, the batch in flight
    is collected by the generator's close)."""
    from plenum_amd import client_authn as CA
    eng, a, ref, idrs, vks, msgs = _staged_pair(oracle, monkeypatch)
    steady = [dict(m) for m in msgs if m["identifier"] in idrs[:4]]
    a.authenticate_batch(steady)  # the kid map
    real = CA._scan_batch
    calls = [0]

    def boom(*args):
        calls[0] += 1
        if calls[0] == 2 and len(args) > 8 and args[8] is not None:
            raise MemoryError("injected")
        return real(*args)
    monkeypatch.setattr(CA, "_scan_batch", boom)
    it = a.authenticate_batches([steady, steady, steady])
    with pytest.raises(MemoryError):
        list(it)
    assert eng.held == [None, None]
    monkeypatch.setattr(CA, "_scan_batch", real)
    want = [m["identifier"] for m in steady]
    assert list(a.authenticate_batches([steady, steady])) == [want, want]


def test_keys_known_matches_getverkey_path(oracle):
    """The batch's per-identifier keys from the native lookup (_hostpack.keys_known, for
    SimpleAuthNr's getVerkey) equal the per-message path's outcomes: a verkey replaced by
    addIdr after the first batch (old signatures now fail), an identifier known only to the
    state lookup, an unknown one, a clients entry without a verkey, an empty clients entry."""
    from plenum_amd import _hostpack
    idrs, vks, msgs = _signed(6, 600)
    state = {idrs[2]: {"verkey": vks[2]}, idrs[5]: {"verkey": vks[5]}}
    a = GpuAuthNr(engine=OracleEngine(oracle), nym_lookup=lambda st, idr: state.get(idr, {}), max_keys=0)
    for i, v in zip(idrs[:2], vks[:2]):
        a.addIdr(i, v)
    a.clients[idrs[3]] = {"verkey": None}
    a.clients[idrs[5]] = {}  # empty: getVerkey asks the state
    batch = [dict(m) for m in msgs if m["identifier"] != idrs[4]] + [dict(msgs[4], identifier="Unknown111111")]
    first = [_outcome(r) for r in a.authenticate_batch(batch)]
    assert first == [_outcome(_single(a, m)) for m in batch]
    a.addIdr(idrs[1], vks[0])  # idrs[1]'s key replaced: its requests no longer verify
    again = [_outcome(r) for r in a.authenticate_batch(batch)]
    assert again == [_outcome(_single(a, m)) for m in batch]
    assert again != first and ("InvalidSignature", (), None) in again
    uniq = list(dict.fromkeys(m["identifier"] for m in batch))
    keys, holes = _hostpack.keys_known(a.clients, a._g.fast_keys, uniq, "verkey")
    assert [uniq[j] for j in holes] == [i for i in uniq if i not in (idrs[0], idrs[1])]
    assert keys[uniq.index(idrs[0])] == a._g.fast_keys[idrs[0]][1]


def _single(a, m):
    try:
        return a.authenticate(dict(m))
    except Exception as ex:
        return ex


def test_verdict_cache_bounded_by_entries_bytes_and_age(oracle, monkeypatch):
    """The verify-ahead verdict cache (bounded by bytes, trimmed by
    age): entries beyond verdict_cache_size, bytes beyond verdict_cache_bytes
    and entries older than verdict_max_age go, oldest first; the byte count
    stays exact; authenticate() answers the same with or without the entry."""
    from plenum_amd import client_authn as CA
    idrs, vks, msgs = _signed(2, 300)
    clock = [1000.0]
    monkeypatch.setattr(CA, "monotonic", lambda: clock[0])
    a = GpuAuthNr(engine=OracleEngine(oracle), verdict_cache_size=250, verdict_cache_bytes=1 << 30,
                  verdict_max_age=10.0)
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    g = a._g

    def size_of():
        return sum(len(k[0]) + len(k[1]) + CA._VERDICT_ENTRY_BYTES for k in g.verdicts)
    a.prefetch(msgs[:200])
    assert len(g.verdicts) == 200 and g.verdict_bytes == size_of()
    clock[0] += 5
    a.prefetch(msgs[200:])
    assert len(g.verdicts) == 250 and g.verdict_bytes == size_of()  # entries bound: the oldest 50 went
    assert (a._vkey(a._prepare(msgs[0])) not in g.verdicts) and (a._vkey(a._prepare(msgs[299])) in g.verdicts)
    clock[0] += 6  # the first second's entries are now 11 s old
    a.prefetch([msgs[0]])
    assert len(g.verdicts) == 101 and g.verdict_bytes == size_of()  # only the 5-second-old ones and the new one
    g.verdict_cache_bytes = 50 * (size_of() // len(g.verdicts))
    a.prefetch([msgs[1]])
    assert g.verdict_bytes <= g.verdict_cache_bytes and g.verdict_bytes == size_of()
    hits = g.stats["cache_hits"]
    assert [a.authenticate(m) for m in msgs] == [m["identifier"] for m in msgs]
    assert g.stats["cache_hits"] > hits
    a.clear_verdicts()
    assert g.verdict_bytes == 0 and not g.verdict_epochs


def test_promotions_decay_cap_and_one_build_call(oracle):
    """Keys earn slots by verified use counted with decay (a count halves per
    2^18 requests: _use_epoch), at most max_promotions per batch, and a batch's
    evictions go to the engine as one keys_set_many_async call."""
    from engine_double import AsyncOracleEngine
    eng = AsyncOracleEngine(oracle)
    idrs, vks, msgs = _signed(6, 60)
    table = dict(zip(idrs, vks))
    a = GpuAuthNr(engine=eng, nym_lookup=lambda st, idr: {"verkey": table[idr]}, max_keys=2, hot_key_uses=2,
                  max_promotions=3)
    g = a._g
    key_of = {i: a._key_for(i) for i in idrs}
    # fill the two slots
    a._count_verified_keys([key_of[idrs[0]], key_of[idrs[1]]], [5, 5])
    a._register_waiting(a._key_store(), [])
    eng.finish_builds()
    assert len(a._key_store()) == 2 and not g.hot
    # four keys earn a slot at once; the two slots go to the first of them (the batch's cap is 3), both
    # evictions in one call
    a._count_verified_keys([key_of[i] for i in idrs[2:6]], [3, 3, 3, 3])
    assert len(g.hot) == 4
    calls = getattr(eng, "many_calls", 0)
    got = a._key_store().register(list(g.hot)[:g.max_promotions], evict=True, asynchronous=True)
    assert len(got) == 2 and eng.many_calls == calls + 1  # two slots to evict: one set-many call
    # decay: one verified use per 2^18 requests never reaches 2
    g.hot.clear()
    k = key_of[idrs[5]]
    g.key_uses.pop(k, None)
    for _ in range(6):
        a._count_verified_keys([k], [1])
        g.stats["batch_items"] += 1 << 18
    assert k not in g.hot
    a._count_verified_keys([k], [1])
    assert k not in g.hot
    a._count_verified_keys([k], [1])  # a second use in the same epoch: it earns a slot
    assert k in g.hot


@pytest.mark.parametrize("subset", [True, False])
def test_staged_mixed_batch_keyed_and_general(oracle, monkeypatch, subset):
    """A staged batch whose signers outnumber the key store (identifiers known,
    only some keys built): one keyed verify of the staged batch plus the
    general path for the other identifiers' items (on the engine's copy of
    the staged batch, edv_verify_staged_subset, or gathered from the pinned
    spans), forgeries and a short signature among both; every outcome equals
    the general path's, and the general items count towards promotion."""
    from engine_double import StagingOracleEngine
    from plenum_amd import client_authn as CA
    monkeypatch.setattr(CA, "_STAGE_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PINNED_MIN_BATCH", 1000)
    idrs, vks, msgs = _signed(5, 5000)
    table = dict(zip(idrs, vks))
    eng = StagingOracleEngine(oracle)
    eng.supports_staged_subset = subset
    a = GpuAuthNr(engine=eng, nym_lookup=lambda st, idr: {"verkey": table[idr]}, max_keys=2, hot_key_uses=10 ** 4)
    for i, v in zip(idrs[:2], vks[:2]):
        a.addIdr(i, v)
    a.keys_settle()
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for i, v in zip(idrs, vks):
        ref.addIdr(i, v)
    batch = [dict(m) for m in msgs]
    batch[10]["reqId"] += 1
    batch[11]["reqId"] += 1
    batch[12]["signature"] = batch[12]["signature"][:-3]
    got = [_outcome(r) for r in a.authenticate_batch(batch)]
    assert got == [_outcome(r) for r in ref.authenticate_batch(batch)]
    bd = a._g.last_breakdown
    assert bd and bd["general_items"] > 0 and eng.staged_calls == 1 and eng.subset_calls == (1 if subset else 0)
    assert 0 < a.stats["keyed_items"] < len(batch)
    assert a._g.key_uses  # general-path keys counted


def _use_counts_dict(uses, keys, counts, now, h, cap):
    """The promotion policy's counts as first written: an LRU OrderedDict of
    key -> (decayed count, epoch), one key at a time (the checker for
    keystore.UseCounts)."""
    hot = []
    for key, c in zip(keys, counts):
        if not c:
            continue
        u, e = uses.pop(key, (0, now))
        u = (u >> min(62, now - e)) + int(c)
        if u >= h:
            hot.append(key)
            u = 0
        if u:
            uses[key] = (u, now)
    while len(uses) > cap:
        uses.popitem(last=False)
    return hot


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_use_counts_match_the_dict_policy(seed):
    """keystore.UseCounts (vectorized, one pass per batch) gives the same hot
    keys, in the same order, and the same (count, epoch) per key as the
    one-key-at-a-time dict, over random batches with decay epochs, zero
    counts and promotions; with a bound, the kept keys are the most recently
    counted ones."""
    from collections import OrderedDict
    from plenum_amd.keystore import UseCounts
    import numpy as np
    rng = np.random.default_rng(seed)
    universe = [bytes([i % 256, i // 256]) * 16 for i in range(3000)]
    uc, ref = UseCounts(10 ** 6), OrderedDict()
    now = 0
    for step in range(60):
        now += int(rng.integers(0, 2))
        idx = rng.choice(len(universe), int(rng.integers(1, 400)), replace=False)
        keys = [universe[i] for i in idx]
        counts = rng.integers(0, 4, len(keys))
        h = int(rng.integers(2, 9))
        assert uc.add(keys, counts, now, h) == _use_counts_dict(ref, keys, counts, now, h, 10 ** 6)
        assert len(uc) == len(ref)
    for k in list(ref)[:200]:
        assert uc.pop(k, None) == ref.pop(k)
        assert k not in uc
    assert uc.pop(universe[0] + b"x", "none") == "none"
    # bounded: keys counted in later calls outlive earlier ones
    uc = UseCounts(100)
    for b in range(10):
        uc.add(universe[b * 50:(b + 1) * 50], [1] * 50, 0, 10)
        assert len(uc) <= 100
    assert all(k in uc for k in universe[450:500])
    assert not any(k in uc for k in universe[:300])


def test_use_counts_sum_a_repeated_key():
    """Two identifiers sharing a verkey bring it twice in one call: the counts
    add up, and the key is reported hot once."""
    from plenum_amd.keystore import UseCounts
    uc = UseCounts(16)
    k1, k2 = b"a" * 32, b"b" * 32
    assert uc.add([k1, k2, k1], [1, 1, 1], 0, 2) == [k1]
    assert k1 not in uc and uc.pop(k2) == (1, 0)
    assert uc.add([k2, k2], [1, 1], 3, 3) == []
    assert uc.pop(k2) == (2, 3)
    with pytest.raises(TypeError):  # an unhashable key: nothing of that call stays
        uc.add([k1, [1]], [1, 1], 3, 3)
    assert len(uc) == 0 and uc.add([k1], [1], 3, 3) == [] and uc.pop(k1) == (1, 3)


def test_use_counts_native_and_array_forms_agree():
    """UseCounts keeps 32-byte keys in the native table (add_flat over one
    buffer) and other keys in the array form: a call mixing both reports its
    hot keys in input order, counts floor-filtered by add_flat, and both forms
    decay and promote alike."""
    from plenum_amd.keystore import UseCounts, _ArrayUseCounts
    import numpy as np
    uc = UseCounts(1000)
    if not uc.native:
        pytest.skip("native module not built")
    a32, b32, c16 = b"a" * 32, b"b" * 32, b"c" * 16
    assert uc.add([c16, a32, b32], [3, 3, 1], 0, 3) == [c16, a32]
    assert len(uc) == 1 and b32 in uc and uc.pop(b32) == (1, 0)
    # floor: counts below it are not counted at all
    flat = a32 + b32
    assert uc.add_flat(flat, np.array([1, 2]), 1, 10, floor=2).tolist() == []
    assert a32 not in uc and uc.pop(b32) == (2, 1)
    # random sequences: the native table against the array form
    rng = np.random.default_rng(5)
    universe = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(500)]
    nat, arr = UseCounts(300), _ArrayUseCounts(300)
    for step in range(40):
        now = step // 3
        idx = rng.choice(len(universe), int(rng.integers(1, 120)))  # (repeats: summed)
        keys = [universe[i] for i in idx]
        counts = rng.integers(0, 5, len(keys))
        h = int(rng.integers(3, 12))
        assert nat.add(keys, counts, now, h) == arr.add(keys, counts, now, h)
        assert len(nat) == len(arr)
    for k in universe:
        assert nat.pop(k, None) == arr.pop(k, None)


def test_keystore_lookup_array_matches_lookup(oracle):
    """KeyStore.lookup_array is lookup() as an array (-1 for None): unregistered keys, keys
    whose asynchronous builds are still queued, repeated keys; both mark the hits used."""
    import numpy as np
    from engine_double import AsyncOracleEngine
    from plenum_amd.keystore import KeyStore
    eng = AsyncOracleEngine(oracle)
    ks = KeyStore(eng, 10, 8)
    keys = [bytes([i]) * 32 for i in range(12)]
    ks.register(keys[:3], asynchronous=True)
    eng.finish_builds()
    ks.register(keys[3:6], asynchronous=True)  # building until finish_builds
    q = keys + keys[:4]
    want = [-1 if i is None else i for i in ks.lookup(q)]
    t = ks._tick
    assert ks.lookup_array(q).tolist() == want and ks._tick == t + 1
    assert want[3:6] == [-1, -1, -1] and want[:3] == [0, 1, 2]
    eng.finish_builds()
    got = ks.lookup_array(q)
    assert got.tolist() == [-1 if i is None else i for i in ks.lookup(q)] and (got[:6] >= 0).all()
    assert (ks._used[got[got >= 0]] == ks._tick - 1).all()
    assert ks.lookup_array([]).dtype == np.int64


def test_no_speculation_over_a_reused_slot(oracle, monkeypatch):
    """an eviction moves a slot to another key whose table build is
    still in flight; the next all-keyed batch must not queue kernels under its
    scan with the ids of the batches before it (kid_map), which would read that
    slot's old or half-written tables.  The key store's version, bumped by the
    eviction, gates the speculation (the double fails any keyed verify of an id
    still building), and the batches after it speculate again once the map is
    rebuilt."""
    from engine_double import AsyncOracleEngine, StagingOracleEngine
    from plenum_amd import client_authn as CA

    class Eng(StagingOracleEngine, AsyncOracleEngine):
        pass
    monkeypatch.setattr(CA, "_STAGE_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PINNED_MIN_BATCH", 1000)
    monkeypatch.setattr(CA, "_PART_ITEMS", 4096)
    idrs, vks, msgs = _signed(5, 6000)
    eng = Eng(oracle)
    a = GpuAuthNr(engine=eng, max_keys=4, hot_key_uses=1)
    ref = GpuAuthNr(engine=OracleEngine(oracle), max_keys=0)
    for i, v in zip(idrs, vks):
        ref.addIdr(i, v)
    for i, v in zip(idrs[:4], vks[:4]):
        a.addIdr(i, v)
    a.keys_settle()
    a.clients[idrs[4]] = {"verkey": vks[4], "role": None}  # known, no slot: earns one by verified use

    def check(batch):
        assert [_outcome(r) for r in a.authenticate_batch(batch)] == \
            [_outcome(r) for r in ref.authenticate_batch(batch)]
        assert eng.held == [None, None]
    old4 = [dict(m) for m in msgs if m["identifier"] in idrs[:4]]
    check(old4)
    check(old4)
    assert eng.parts_begun == 1  # the steady state speculates
    new4 = [dict(m) for m in msgs if m["identifier"] != idrs[0]]
    check(new4)  # idrs[4] verifies on the general path: it earns a slot ...
    check(new4)  # ... taken here, evicting idrs[0] (the least recently used) with an asynchronous build
    assert eng.building, "the rebuilt slot's table is still in flight"
    begun = eng.parts_begun
    check(old4)  # idrs[0]'s id in kid_map now names a slot being rebuilt for idrs[4]
    assert eng.parts_begun == begun  # no kernels under the scan with the stale map
    eng.finish_builds()
    for _ in range(3):
        check(new4)
    assert eng.parts_begun > begun  # speculating again on the rebuilt map


def test_speculation_after_another_authenticator_reset_the_store(oracle, monkeypatch):
    """the engine's key store reset by someone else sharing it
    (keys_reset bumps keys_generation) while this authenticator's kid_map is
    still set: authenticate_batch neither raises ('no registered keys' from
    edv_verify_staged_begin) nor leaves a staging set held, and the outcomes
    are the general path's."""
    eng, a, ref, idrs, vks, msgs = _staged_pair(oracle, monkeypatch)
    steady = [dict(m) for m in msgs if m["identifier"] in idrs[:4]]
    a.authenticate_batch(steady)
    a.authenticate_batch(steady)
    begun = eng.parts_begun
    eng.keys_reset()
    got = a.authenticate_batch(steady)
    assert [_outcome(r) for r in got] == [_outcome(r) for r in ref.authenticate_batch(steady)]
    assert eng.parts_begun == begun and eng.held == [None, None]


def test_staging_reserve_fault_is_raised_not_read_as_busy(oracle, monkeypatch):
    """only EDV_EBUSY (the set holds an uncollected submission)
    sends a batch to the unstaged path; any other stage_reserve failure (an
    allocation or HIP error) is raised."""
    eng, a, ref, idrs, vks, msgs = _staged_pair(oracle, monkeypatch)
    steady = [dict(m) for m in msgs if m["identifier"] in idrs[:4]]

    def fault(nbytes):
        raise RuntimeError("edverify error -3: hipMalloc failed (test)")
    monkeypatch.setattr(eng, "stage_reserve", fault)
    with pytest.raises(RuntimeError, match="hipMalloc"):
        a.authenticate_batch(steady)
    assert eng.held == [None, None]


def test_batch_calls_pause_and_restore_the_collector(oracle, monkeypatch):
    """authenticate_batch pauses the cyclic collector for its own duration only: enabled again
    after the call, after a call that raises, and left disabled if the caller had disabled it."""
    import gc
    from plenum_amd import client_authn as CA
    idrs, vks, msgs = _signed(2, 40)
    a = GpuAuthNr(engine=OracleEngine(oracle))
    for i, v in zip(idrs, vks):
        a.addIdr(i, v)
    seen = []
    real = a._authenticate_batch_scanned

    def spy(m):
        seen.append(gc.isenabled())
        return real(m)
    monkeypatch.setattr(a, "_authenticate_batch_scanned", spy)
    assert gc.isenabled()
    assert a.authenticate_batch(msgs) == [m["identifier"] for m in msgs]
    assert seen == [False] and gc.isenabled()

    def boom(m):
        raise MemoryError("injected")
    monkeypatch.setattr(a, "_authenticate_batch_scanned", boom)
    with pytest.raises(MemoryError):
        a.authenticate_batch(msgs)
    assert gc.isenabled()
    gc.disable()
    try:
        monkeypatch.setattr(a, "_authenticate_batch_scanned", spy)
        a.authenticate_batch(msgs)
        assert not gc.isenabled()
    finally:
        gc.enable()


def test_fast_invalid_signatures_equal_constructed_ones():
    """_invalid_signatures builds a batch's many InvalidSignature instances without the
    constructor when the classes are this package's: each equals a constructed one in class, args,
    attributes, cause and str, and each is a distinct object."""
    from plenum_amd import client_authn as ca
    from plenum_amd.exceptions import InvalidSignature
    got = ca._invalid_signatures(300)
    ref = InvalidSignature()
    assert len({id(e) for e in got}) == 300
    for e in got:
        assert type(e) is InvalidSignature and e.args == ref.args and e.__dict__ == ref.__dict__
        assert e.__cause__ is None and e.__context__ is None and str(e) == str(ref)
        assert e.code == ref.code and e.reason == ref.reason
    assert len(ca._invalid_signatures(3)) == 3
