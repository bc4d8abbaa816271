"""The drop-in authenticator on the real GPU engine: the reference KAT table
(tests/golden/authn_kat.json from the reference's own NaclAuthNr) and batch
== single, with no CPU verification anywhere on the path."""
import numpy as np
import pytest

import test_client_authn as T
from plenum_amd.client_authn import GpuAuthNr

pytestmark = pytest.mark.gpu


def test_reference_kats_on_gpu(gpu_engine):
    for c in T.kat()["cases"]:
        T.check_result(c, T.run_single(T.make(gpu_engine, c), c))


def test_batch_on_gpu(gpu_engine):
    good = next(c for c in T.kat()["cases"] if c["name"] == "valid-abbreviated-verkey")
    a = T.make(gpu_engine, good)
    msgs = [dict(good["msg"]) for _ in range(1000)]
    for i in range(0, 1000, 3):
        msgs[i]["reqId"] += 1
    res = a.authenticate_batch(msgs)
    for i, r in enumerate(res):
        if i % 3 == 0:
            assert type(r).__name__ == "InvalidSignature"
        else:
            assert r == good["msg"]["identifier"]
    assert a.stats["batches"] == 1


def test_reference_propagate_vector_on_gpu(gpu_engine):
    """The signed PROPAGATE the reference holds (test_valid_message_request.py:
    60-64; cryptonym identifier, so the key is the identifier itself,
    verifier.py:26-28) and its tampered variants, one batch of them repeated
    across a 5,000-request authenticate_batch (the native scan, the GPU) and
    each once through authenticate(), on the key-table and general paths:
    every outcome the reference's own authenticate() gave (authn_kat.json)."""
    cases = [c for c in T.kat()["cases"] if c["name"].startswith("ref-propagate-")]
    assert len(cases) == 7
    with _own_key_store(gpu_engine):
        _propagate_cases(gpu_engine, cases)


def _own_key_store(eng):
    """A test whose authenticators size the engine's key store themselves (the
    first authenticator on an engine fixes its capacity and window): a store
    of their own for the test, and the default store again after it."""
    import contextlib

    @contextlib.contextmanager
    def cm():
        eng.__dict__.pop("_edv_key_store", None)
        try:
            yield
        finally:
            eng.__dict__.pop("_edv_key_store", None)
            eng.keys_reset()
    return cm()


def _propagate_cases(gpu_engine, cases):
    for max_keys in (16, 0):
        a = GpuAuthNr(engine=gpu_engine, max_keys=max_keys)
        idr = cases[0]["msg"]["identifier"]
        a.addIdr(idr, "")  # on record with an empty verkey: the cryptonym resolves to the key
        a.keys_settle()
        pool = [c for c in cases if c["register"] and c["verkey"] == ""]
        batch = [dict(pool[i % len(pool)]["msg"]) for i in range(5000)]
        res = a.authenticate_batch(batch)
        for i, r in enumerate(res):
            c = pool[i % len(pool)]
            if "result" in c:
                assert r == c["result"], (max_keys, c["name"], r)
            else:
                assert type(r).__name__ == c["raises"], (max_keys, c["name"], r)
        for c in cases:
            T.check_result(c, T.run_single(T.make(gpu_engine, c), c))
        if max_keys:
            assert a.stats["keyed_items"] > 0


def test_multi_on_gpu(gpu_engine):
    a, msg, sigs = T._multi_fixture(gpu_engine)
    assert a.authenticate_multi(msg, sigs) == list(sigs)


def test_default_engine_is_gpu():
    from plenum_amd.engine import EdVerifyEngine
    a = GpuAuthNr()
    assert isinstance(a._engine(), EdVerifyEngine)


def test_keyed_and_general_paths_agree_on_gpu(gpu_engine):
    with _own_key_store(gpu_engine):
        with_keys, n_keyed = T._outcomes(gpu_engine, 16)
        without, n_general = T._outcomes(gpu_engine, 0)
    assert with_keys == without
    assert n_keyed > 0 and n_general == 0
    for c, r in zip(T.kat()["cases"], with_keys):
        if "result" in c:
            assert r == c["result"], c["name"]
        else:
            assert r[0] == c["raises"], c["name"]


class _Counting:
    """Pass-through engine proxy counting verify launches."""

    def __init__(self, eng):
        self.eng = eng
        self.launches = 0

    def __getattr__(self, name):
        attr = getattr(self.eng, name)
        if name in ("verify_batch", "verify_batch_keyed", "sign_open_batch"):
            def counted(*a, **k):
                self.launches += 1
                return attr(*a, **k)
            return counted
        return attr


def _drain(gpu_engine, n_req=100, n_nodes=25, n_signers=10):
    """A synthetic rxMsgs drain (stp_zmq/zstack.py:528-549): n_req client
    REQUESTs (every 10th forged after signing) plus, for each, the n_nodes - 1
    PROPAGATE copies other nodes send (node.py:1313-1316, 2304-2306)."""
    import json
    from plenum_amd import pack_messages, synth
    from plenum_amd.base58 import b58encode
    from plenum_amd.serialization import serialize_msg_for_signing
    pks, sks = gpu_engine.seed_keypair_batch(synth.signer_seeds(n_signers))
    idrs = [b58encode(bytes(pk[:16])) for pk in pks]
    vks = ["~" + b58encode(bytes(pk[16:])) for pk in pks]
    reqs = [synth.nym_request(idrs[i % n_signers], 1_600_000_000_000_000 + i, "dest%d" % i, "~vk%d" % i)
            for i in range(n_req)]
    sers = [serialize_msg_for_signing(r, topLevelKeysToIgnore=["signature"]) for r in reqs]
    buf, off = pack_messages(sers)
    sig = gpu_engine.sign_batch(sks, (np.arange(n_req) % n_signers).astype(np.uint32), buf, off)
    for i, r in enumerate(reqs):
        r["signature"] = b58encode(sig[i].tobytes())
        if i % 10 == 3:
            r["operation"]["dest"] += "x"  # forged after signing
    rx = []
    for i, r in enumerate(reqs):
        rx.append((json.dumps(r), b"client%d" % i))
        for node in range(1, n_nodes):
            rx.append((json.dumps({"op": "PROPAGATE", "request": r, "senderClient": "client%d" % i}),
                       b"Node%d" % node))
    return reqs, rx, idrs, vks, pks, sers, sig


def test_verify_ahead_drain_on_gpu(gpu_engine, oracle):
    """One rxMsgs drain of 100 REQUESTs + 24 PROPAGATE copies each: exactly one
    engine launch (the n copies dedupe to one verify each), then authenticate()
    on Request.as_dict-shaped dicts (plenum/common/request.py:27-39) hits the
    cache for all of them (0 single-verify launches); verdicts == the oracle."""
    from plenum_amd.batching import prefetch_drain
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine)
    eng = _Counting(gpu_engine)
    a = GpuAuthNr(engine=eng)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()  # genesis NYMs: their tables built before traffic (batches never wait on builds)
    assert prefetch_drain(a, rx) == 100
    assert eng.launches == 1 and a.stats["keyed_items"] == 100
    for i, r in enumerate(reqs):
        as_dict = {"identifier": r["identifier"], "reqId": r["reqId"], "operation": r["operation"],
                   "signature": r["signature"], "protocolVersion": r["protocolVersion"]}
        ser = sers[i] if i % 10 != 3 else None
        want = ser is not None and oracle.oracle_verify_detached(sig[i].tobytes(), ser, len(ser),
                                                                 pks[i % 10].tobytes()) == 0
        if want:
            assert a.authenticate(as_dict) == r["identifier"]
        else:
            with pytest.raises(Exception) as ei:
                a.authenticate(as_dict)
            assert type(ei.value).__name__ == "InvalidSignature"
    assert eng.launches == 1 and a.stats["single_verifies"] == 0 and a.stats["cache_hits"] == 100


def test_verify_ahead_batch_framed_drain_on_gpu(gpu_engine, oracle):
    """The drain as it looks under load: 100 client REQUESTs plus, from each of
    the 24 other nodes, ONE BATCH message wrapping that node's serialized
    PROPAGATEs (Batched.flushOutBoxes -> _make_batch, batched.py:99-125,
    141-144) interleaved with a 3PC message, unpacked by the node with
    nodestack.deserializeMsg per entry (node.py:1333-1337).  One engine
    launch, 0 single verifies, verdicts == the oracle's."""
    import json
    from plenum_amd.batching import prefetch_drain
    reqs, _rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_nodes=1)
    rx = [(json.dumps(r), b"client%d" % i) for i, r in enumerate(reqs)]
    for node in range(1, 25):
        inner = []
        for i, r in enumerate(reqs):
            inner.append(json.dumps({"op": "PROPAGATE", "request": r, "senderClient": "client%d" % i}))
            if i % 25 == 0:
                inner.append(json.dumps({"op": "PREPARE", "instId": 0, "viewNo": 0, "ppSeqNo": i}))
        rx.append((json.dumps({"op": "BATCH", "messages": inner, "signature": None}).encode(), b"Node%d" % node))
    eng = _Counting(gpu_engine)
    a = GpuAuthNr(engine=eng)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()  # genesis NYMs: their tables built before traffic (batches never wait on builds)
    assert prefetch_drain(a, rx) == 100
    assert eng.launches == 1 and a.stats["keyed_items"] == 100
    # the requests as the node authenticates them after unpacking one node's BATCH
    unpacked = [json.loads(m) for m in json.loads(rx[100 + 5][0])["messages"]]
    props = [m["request"] for m in unpacked if m["op"] == "PROPAGATE"]
    assert len(props) == 100
    for i, r in enumerate(reqs):
        ser = sers[i] if i % 10 != 3 else None
        want = ser is not None and oracle.oracle_verify_detached(sig[i].tobytes(), ser, len(ser),
                                                                 pks[i % 10].tobytes()) == 0
        for m in (r, props[i]):
            if want:
                assert a.authenticate(m) == r["identifier"]
            else:
                with pytest.raises(Exception) as ei:
                    a.authenticate(m)
                assert type(ei.value).__name__ == "InvalidSignature"
    assert eng.launches == 1 and a.stats["single_verifies"] == 0 and a.stats["cache_hits"] == 200


def test_node_loop_drains_on_gpu(gpu_engine, oracle):
    """bench.py's end_to_end.node_drain shape, checked: three drains of an
    n = 25 pool through the verify-ahead stacks over the restated node loop
    (plenum_amd/nodeloop.py): per drain 100 client REQUESTs + 24 BATCHes of
    PROPAGATEs, every raw message decoded once, ONE engine launch per drain,
    0 single verifies, and all 2,500 authenticate() outcomes per drain equal
    to the oracle's verdict (forged payloads, a corrupted S, an unknown
    identifier among them)."""
    from plenum_amd.batching import verify_ahead_stack
    from plenum_amd.nodeloop import NodeCounters, Stack, drain_texts
    reqs, _rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=300, n_nodes=1)
    reqs[7]["signature"] = reqs[8]["signature"]            # another request's signature
    reqs[150]["identifier"] = "UnknownIdentifier111111"   # getVerkey raises
    eng = _Counting(gpu_engine)
    a = GpuAuthNr(engine=eng)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()
    want = []
    for i, r in enumerate(reqs):
        if i == 150:
            want.append("UnknownIdentifier")
            continue
        s = sig[8] if i == 7 else sig[i]
        ser = sers[i]
        ok = i % 10 != 3 and oracle.oracle_verify_detached(s.tobytes(), ser, len(ser), pks[i % 10].tobytes()) == 0
        want.append(r["identifier"] if ok else "InvalidSignature")
    assert want.count("InvalidSignature") == 31
    nc = NodeCounters()
    nc.record = True
    ns = verify_ahead_stack(Stack, a)(a, "node", nc)
    cs = verify_ahead_stack(Stack, a)(a, "client", nc)
    for d in range(3):
        part = reqs[d * 100:(d + 1) * 100]
        client, node = drain_texts(part, 25)
        ns.rxMsgs.extend(node)
        cs.rxMsgs.extend(client)
        l0, s0 = eng.launches, a.stats["single_verifies"]
        nc.outcomes.clear()
        assert ns.processReceived(100) == 24 and cs.processReceived(100) == 100
        assert eng.launches - l0 == 1 and a.stats["single_verifies"] == s0
        w = want[d * 100:(d + 1) * 100]
        assert [o[1] for o in nc.outcomes] == w * 24 + w
    assert a.stats["single_verifies"] == 0 and a.stats["cache_hits"] == 3 * 2500 - 25  # the unknown id never reaches it


def test_multi_engine_one_device(gpu_engine):
    """The single-process multi-GPU path with the devices of this box (one
    here): MultiEngine through the authenticator == the plain engine."""
    from plenum_amd.multi import MultiEngine
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_nodes=1)
    me = MultiEngine(engines=[gpu_engine])
    a, b = GpuAuthNr(engine=me, max_keys=0), GpuAuthNr(engine=gpu_engine, max_keys=0)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
        b.addIdr(idr, vk)
    ra = [r if isinstance(r, str) else type(r).__name__ for r in a.authenticate_batch(reqs)]
    rb = [r if isinstance(r, str) else type(r).__name__ for r in b.authenticate_batch(reqs)]
    assert ra == rb and ra.count("InvalidSignature") == 10
    auto = MultiEngine("all")
    try:
        assert len(auto) >= 1
        c = GpuAuthNr(engine=auto)
        for idr, vk in zip(idrs, vks):
            c.addIdr(idr, vk)
        c.keys_settle()
        rc = [r if isinstance(r, str) else type(r).__name__ for r in c.authenticate_batch(reqs)]
        assert rc == rb and c.stats["keyed_items"] == len(reqs)
    finally:
        auto.close()


def test_reused_scan_buffers_on_gpu(gpu_engine):
    """authenticate_batch over a large, a small and a large batch again on one
    authenticator (the scan writes into the same grown output buffers each
    time; csrc/hostpack.cpp scan_impl), with different forgeries per batch
    and one batch that leaves the whole-batch fast path (a request without a
    signature): every verdict is the construction's."""
    import copy
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=3000, n_nodes=1)
    a = GpuAuthNr(engine=gpu_engine)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    base_bad = {i for i in range(3000) if i % 10 == 3}  # forged after signing by _drain
    for size, extra_bad, drop_sig in ((3000, (7, 2999), None), (500, (11,), 42), (3000, (1, 1500), None)):
        batch = [copy.deepcopy(r) for r in reqs[:size]]
        for i in extra_bad:
            batch[i]["reqId"] += 1
        if drop_sig is not None:
            del batch[drop_sig]["signature"]
        res = a.authenticate_batch(batch)
        for i, r in enumerate(res):
            if i == drop_sig:
                assert type(r).__name__ == "MissingSignature"
            elif i in base_bad or i in extra_bad:
                assert type(r).__name__ == "InvalidSignature", (size, i)
            else:
                assert r == batch[i]["identifier"], (size, i)
    assert len(a._g.scan_out[0]) >= 64 * 3000


def test_pinned_slots_end_to_end_on_gpu(gpu_engine):
    """A batch above the pinned-buffer threshold: the scan writes signature
    slots (base58 text, decoded by edv_b58_sig_kernel) and messages straight
    into the engine's pinned host memory, and the GPU call copies them with no
    staging copy of the bulk (last_host_stats).  Every
    verdict is the construction's, including signatures whose R starts with
    zero bytes (leading '1's in the text) and 63 / 65-byte signatures."""
    import copy
    from plenum_amd.base58 import b58decode, b58encode
    n = 20000
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=n, n_nodes=1)
    a = GpuAuthNr(engine=gpu_engine)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    bad = {i for i in range(n) if i % 10 == 3}  # forged after signing by _drain
    batch = [copy.deepcopy(r) for r in reqs]
    for i in range(5, n, 997):
        batch[i]["signature"] = b58encode(b58decode(batch[i]["signature"])[:63])
        bad.add(i)
    for i in range(6, n, 1999):
        batch[i]["signature"] = b58encode(b58decode(batch[i]["signature"]) + b"\x07")
        bad.add(i)
    lead0 = [i for i in range(n) if sig[i][0] == 0 and i not in bad]
    assert lead0 and all(batch[i]["signature"].startswith("1") for i in lead0)
    for rep in range(2):
        res = a.authenticate_batch(batch)
        for i, r in enumerate(res):
            if i in bad:
                assert type(r).__name__ == "InvalidSignature", (rep, i)
            else:
                assert r == batch[i]["identifier"], (rep, i)
        st = gpu_engine.last_host_stats()
        # the bulk (signature slots, messages) straight from pinned memory; key ids and offsets
        # (4 + 8 B per request, made by numpy / the scan's result bytes) are staged: microseconds
        assert st["direct"]["sig"] and st["direct"]["msgs"] and st["stage_ms"] < 1.0, st
    assert a._g.pinned_out is not None and len(a._g.pinned_out[0]) >= 96 * n


def test_pipelined_parts_on_gpu(gpu_engine):
    """authenticate_batch in parts (pipeline_part = 4096 on 20,000 requests:
    5 parts, more submissions than the library's two copy slots, so slots are
    reused across pending submissions): edv_verify_submit / collect give the
    construction's verdicts, the same as one synchronous call."""
    import copy
    n = 20000
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=n, n_nodes=1, n_signers=16)
    bad = {i for i in range(n) if i % 10 == 3}
    whole = GpuAuthNr(engine=gpu_engine, pipeline_part=0)
    parts = GpuAuthNr(engine=gpu_engine, pipeline_part=4096)
    for a in (whole, parts):
        for idr, vk in zip(idrs, vks):
            a.addIdr(idr, vk)
        a.keys_settle()
    batch = [copy.deepcopy(r) for r in reqs]
    batch[9000]["reqId"] += 1
    bad.add(9000)
    r1 = whole.authenticate_batch(batch)
    for rep in range(2):
        r2 = parts.authenticate_batch(batch)
        assert [type(x).__name__ if not isinstance(x, str) else x for x in r2] == \
               [type(x).__name__ if not isinstance(x, str) else x for x in r1]
        for i, r in enumerate(r2):
            assert (type(r).__name__ == "InvalidSignature") if i in bad else (r == batch[i]["identifier"]), i
    assert parts.stats["keyed_items"] >= n


@pytest.mark.gpu
def test_async_key_promotion_on_gpu(gpu_engine):
    """Hot-key promotion with the table builds off the request path
    (edv_keys_add_async / edv_keys_set_async on the engine's build stream):
    10 signers with room for 4 keys and hot_key_uses = 1; each batch carries 5
    of the signers, rotating, so batches keep promoting keys and evicting the
    ones the batch does not use while earlier builds may still run.  A
    building key's requests take the general path (the proxy records, at each
    verify launch, how many ids were still building); every verdict is the
    construction's, in every batch; once the builds drain, the store's keys
    verify on the key-table path."""
    import copy
    from plenum_amd.engine import EdVerifyEngine
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=3000, n_nodes=1, n_signers=10)
    table = dict(zip(idrs, vks))
    bad = {i for i in range(3000) if i % 10 == 3}

    class Probe(_Counting):
        seen = 0

        def __getattr__(self, name):
            attr = super().__getattr__(name)
            if name in ("verify_batch", "verify_batch_keyed"):
                def probed(*a, **k):
                    ks = self.__dict__.get("_edv_key_store")
                    if ks is not None:
                        Probe.seen = max(Probe.seen, ks.building())
                    return attr(*a, **k)
                return probed
            return attr

    real = EdVerifyEngine(0)  # a store of its own (4 slots at W = 16: 64 MiB tables per key)
    try:
        eng = Probe(real)
        a = GpuAuthNr(engine=eng, nym_lookup=lambda st, idr: {"verkey": table[idr]}, max_keys=4, hot_key_uses=1)
        for rep in range(8):
            signers = {(rep + j) % 10 for j in range(5)}
            idx = [i for i in range(3000) if i % 10 in signers][:600]
            batch = [copy.deepcopy(reqs[i]) for i in idx]
            res = a.authenticate_batch(batch)
            for i, r in zip(idx, res):
                if i in bad:
                    assert type(r).__name__ == "InvalidSignature", (rep, i)
                else:
                    assert r == reqs[i]["identifier"], (rep, i)
        assert a.stats["keys_registered"] > 4, a.stats  # evictions rebuilt slots
        assert Probe.seen > 0  # some verify ran while a table was still building
        a.keys_settle()
        ks = a._key_store()
        assert ks.building() == 0 and len(ks) == 4
        before = a.stats["keyed_items"]
        last = {(7 + j) % 10 for j in range(5)}
        idx = [i for i in range(3000) if i % 10 in last][:600]
        res = a.authenticate_batch([reqs[i] for i in idx])
        assert [r if isinstance(r, str) else type(r).__name__ for r in res] == \
               ["InvalidSignature" if i in bad else reqs[i]["identifier"] for i in idx]
        assert a.stats["keyed_items"] > before
    finally:
        real.close()


@pytest.mark.gpu
def test_bench_e2e_devices_leg_on_gpu(gpu_engine):
    """bench.py's node-shaped multi-GPU leg (end_to_end.by_devices: GpuAuthNr
    over MultiEngine with k engines, one node process) at k = 1 on this box:
    every request of a configs[1]-shaped batch accepted, on the key-table
    path after keys_settle."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import bench
    reqs, idrs, vks = bench.e2e_requests(gpu_engine, 8192, 16, 43)
    out = bench.time_e2e_devices(gpu_engine, reqs, idrs, vks, [1])
    assert out["1"]["accepted"] == 8192 and out["1"]["keyed_items_share"] == 1.0, out


@pytest.mark.gpu
def test_staged_batch_on_gpu(gpu_engine):
    """The staged path on the device (edv_stage_put from the scan's workers,
    edv_verify_staged over the item spans): 70,000 requests (above the 2^16
    staging threshold), every 10th forged, 63- and 65-byte signatures, R with
    leading zero bytes -- every verdict is the construction's, over two
    batches on one authenticator (reused pinned and staging buffers)."""
    import copy
    from plenum_amd.base58 import b58decode, b58encode
    n = 70000
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=n, n_nodes=1)
    a = GpuAuthNr(engine=gpu_engine, stage=True)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()
    bad = {i for i in range(n) if i % 10 == 3}
    batch = [copy.deepcopy(r) for r in reqs]
    for i in range(5, n, 4999):
        batch[i]["signature"] = b58encode(b58decode(batch[i]["signature"])[:63])
        bad.add(i)
    for i in range(6, n, 7001):
        batch[i]["signature"] = b58encode(b58decode(batch[i]["signature"]) + b"\x07")
        bad.add(i)
    before = a.stats["keyed_items"]
    for rep in range(2):
        res = a.authenticate_batch(batch)
        for i, r in enumerate(res):
            if i in bad:
                assert type(r).__name__ == "InvalidSignature", (rep, i)
            else:
                assert r == batch[i]["identifier"], (rep, i)
    assert a.stats["keyed_items"] - before == 2 * n


def _oracle_verdicts(sig64, pk32, msgs, threads=16):
    """The C oracle's crypto_sign_verify_detached over many items, on host
    threads (oracle/cpu_baseline.c with use_sodium=0: the plain-C restatement)."""
    import ctypes
    import os
    from conftest import ROOT
    from plenum_amd import pack_messages
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libcpu_baseline.so"))
    buf, off = pack_messages(msgs)
    buf = np.concatenate([buf, np.zeros(16, np.uint8)])
    n = len(msgs)
    ok = np.zeros(n, np.uint8)
    secs = ctypes.c_double()
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    sig64, pk32 = np.ascontiguousarray(sig64), np.ascontiguousarray(pk32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    assert lib.cpu_baseline_run(P(sig64), P(pk32), P(buf), P(off), ctypes.c_uint64(n), threads, 0, P(ok),
                                ctypes.byref(secs)) == 0
    return ok.astype(bool)


_C3_SIGS = 100_000


def test_configs3_multi_signature_shape_vs_oracle(gpu_engine, sodium_verdicts):
    """BASELINE configs[3] at its real shape through authenticate_multi_batch:
    >= 100k signatures, 1-5 per request (distinct signers), signed payloads
    log-uniform over 64 B - 4 KiB, ~6 % of the signatures corrupted (a bit of
    R or S flipped, a signature moved to another signer, a payload changed
    after signing).  Every per-signature verdict of the GPU path equals the C
    oracle's, and every request's outcome (identifiers up to the threshold, or
    InsufficientCorrectSignatures / InsufficientSignatures) is the one those
    verdicts give; the verdicts are also libsodium 1.0.18's, every one.
    Signers: 48 registered (key-table path) + 16 known only through the state
    lookup (general path)."""
    from plenum_amd import _hostpack, pack_messages, synth
    from plenum_amd.base58 import b58encode
    from plenum_amd.exceptions import InsufficientCorrectSignatures, InsufficientSignatures
    from plenum_amd.serialization import serialize_msg_for_signing
    rng = np.random.default_rng(33)
    S = 64
    pks, sks = gpu_engine.seed_keypair_batch(synth.signer_seeds(S + 77)[77:])
    idrs = [b58encode(bytes(pk[:16])) for pk in pks]
    vks = ["~" + b58encode(bytes(pk[16:])) for pk in pks]
    state = {idrs[j]: {"verkey": vks[j]} for j in range(48, S)}
    a = GpuAuthNr(engine=gpu_engine, nym_lookup=lambda st, idr: state.get(idr, {}))
    for j in range(48):
        a.addIdr(idrs[j], vks[j])
    a.keys_settle()
    reqs, signers, sers = [], [], []
    total = 0
    while total < _C3_SIGS:
        k = int(rng.integers(1, 6))
        who = rng.choice(S, size=k, replace=False)
        target = int(np.exp(rng.uniform(np.log(64), np.log(4096))))
        req = {"identifier": idrs[int(who[0])], "reqId": 1_700_000_000_000_000 + len(reqs),
               "operation": {"type": "1", "raw": ""}, "protocolVersion": 1}
        base = len(serialize_msg_for_signing(req, topLevelKeysToIgnore=["signature", "signatures"]))
        req["operation"]["raw"] = "".join(map(chr, rng.integers(97, 123, size=max(0, target - base))))
        ser = serialize_msg_for_signing(req, topLevelKeysToIgnore=["signature", "signatures"])
        reqs.append(req)
        signers.append([int(w) for w in who])
        sers.append(ser)
        total += k
    lens = np.array([len(s) for s in sers])
    assert lens.min() <= 100 and lens.max() >= 3500  # the 64 B - 4 KiB spread
    item_req = np.repeat(np.arange(len(reqs)), [len(s) for s in signers])
    item_key = np.concatenate([np.array(s) for s in signers]).astype(np.uint32)
    buf, off = pack_messages(sers)
    starts, ends = off[:-1][item_req], off[1:][item_req]
    ibuf, ioff = pack_messages([bytes(buf[s:e]) for s, e in zip(starts, ends)])
    sig = gpu_engine.sign_batch(sks, item_key, ibuf, ioff)
    n = len(item_key)
    bad = rng.random(n) < 0.05
    for i in np.flatnonzero(bad):
        kind = i % 3
        if kind == 0:
            sig[i, int(rng.integers(0, 32))] ^= 1 << int(rng.integers(0, 8))    # R
        elif kind == 1:
            sig[i, 32 + int(rng.integers(0, 31))] ^= 1 << int(rng.integers(0, 8))  # S
        else:
            sig[i] = sig[(i + 1) % n]                                            # someone else's
    moved = rng.choice(len(reqs), size=len(reqs) // 100, replace=False)          # payload changed after signing
    for r in moved:
        reqs[r]["reqId"] += 1
    texts = _hostpack.b58encode_rows(np.ascontiguousarray(sig).tobytes(), 64)
    batch, pos = [], 0
    thresholds = []
    for r, req in enumerate(reqs):
        k = len(signers[r])
        sigs = {idrs[w]: texts[pos + j] for j, w in enumerate(signers[r])}
        pos += k
        thr = [None, 1, k, k + 1, int(rng.integers(1, k + 1))][r % 5]
        thresholds.append(thr)
        batch.append((req, sigs, thr))
    # the oracle's verdict of every signature, over the bytes each request now serializes to
    now = [serialize_msg_for_signing(q, topLevelKeysToIgnore=["signature", "signatures"]) for q in reqs]
    want = _oracle_verdicts(sig, pks[item_key], [now[r] for r in item_req])
    assert 0.85 < want.mean() < 0.97, want.mean()
    # and libsodium 1.0.18 itself on every signature (the requests' messages shared through spans)
    nbuf, noff = pack_messages(now)
    lib = sodium_verdicts(sig, pks[item_key], nbuf, noff[:-1][item_req], noff[1:][item_req])
    assert (lib == want).all(), np.flatnonzero(lib != want)[:10]
    # per-signature verdicts on the GPU path, through the same preparation authenticate_multi uses
    items = []
    for req, sigs, thr in batch:
        _, steps = a._prepare_multi(req, sigs, None)
        items += steps
    assert len(items) == n
    got = np.array(a._verify_many(items), bool)
    bad_i = np.flatnonzero(got != want)[:10]
    assert (got == want).all(), [(int(i), bool(got[i]), bool(want[i]), int(item_key[i]), bool(bad[i]), int(item_req[i]),
                                  int(item_req[i]) in set(moved.tolist()), len(now[item_req[i]])) for i in bad_i]
    assert a.stats["keyed_items"] > 0 and a.stats["batch_items"] > a.stats["keyed_items"]  # both paths ran
    # every request's outcome
    res = a.authenticate_multi_batch(batch)
    pos = 0
    for r, out in enumerate(res):
        k = len(signers[r])
        v = want[pos:pos + k]
        ids = [idrs[w] for w in signers[r]]
        pos += k
        thr = thresholds[r] if thresholds[r] is not None else k
        if k < thr:
            assert isinstance(out, InsufficientSignatures), r
            continue
        good = [i for i, ok in zip(ids, v) if ok]
        if len(good) >= thr:
            assert out == good[:thr], r
        else:
            assert isinstance(out, InsufficientCorrectSignatures) and out.args == (len(good), thr), (r, out)


def test_large_batch_staged_and_streamed_on_gpu(gpu_engine):
    """The two large-batch paths on the device over one 300,000-request batch
    (above 2^18, so the streamed path submits several chunks; staged by
    default): every 10th request forged, a missing signature, an unknown
    identifier -- both give the construction's outcome for every request."""
    import copy
    n = 300_000
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=n, n_nodes=1, n_signers=32)
    batch = [copy.deepcopy(r) for r in reqs]
    del batch[1234]["signature"]
    batch[4321]["identifier"] = "UnknownIdentifier11111111"
    want = []
    for i, r in enumerate(batch):
        want.append("MissingSignature" if i == 1234 else "UnknownIdentifier" if i == 4321 else
                    "InvalidSignature" if i % 10 == 3 else r["identifier"])
    outs = {}
    for mode in ("stage", "stream"):
        a = GpuAuthNr(engine=gpu_engine, stage=(mode == "stage"))
        for idr, vk in zip(idrs, vks):
            a.addIdr(idr, vk)
        a.keys_settle()
        clean = [copy.deepcopy(r) for i, r in enumerate(batch) if i not in (1234, 4321)]
        a.authenticate_batch(clean)  # sizes the pinned buffers, then the steady-state batch
        res = a.authenticate_batch(batch)
        outs[mode] = [r if isinstance(r, str) else type(r).__name__ for r in res]
        assert outs[mode] == want, mode
        ok = a.authenticate_batch(clean)  # the steady state (every item scanned, every key built)
        assert [r if isinstance(r, str) else type(r).__name__ for r in ok] == \
               [w for i, w in enumerate(want) if i not in (1234, 4321)], mode
        assert a._g.last_breakdown is not None, mode


def test_authenticate_batches_pipeline_on_gpu(gpu_engine):
    """authenticate_batches on the device: 3 batches of 70,000 requests (above
    the staging threshold) in flight two at a time over the engine's staging
    sets, plus a batch that leaves the steady state in the middle: every
    outcome equals the synchronous authenticate_batch's."""
    import copy
    n = 70000
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=n, n_nodes=1, n_signers=16)
    a = GpuAuthNr(engine=gpu_engine)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()
    odd = [copy.deepcopy(r) for r in reqs]
    odd[99]["identifier"] = "UnknownIdentifier11111111"
    batches = [reqs, reqs, odd, reqs]
    want = [[r if isinstance(r, str) else type(r).__name__ for r in a.authenticate_batch(b)] for b in batches]
    for rep in range(2):
        got = [[r if isinstance(r, str) else type(r).__name__ for r in res] for res in a.authenticate_batches(batches)]
        assert got == want, rep
    assert want[0].count("InvalidSignature") == n // 10 and want[2][99] == "UnknownIdentifier"


def test_speculative_staged_batches_on_gpu(gpu_engine):
    """A synchronous staged batch's kernels under its own scan on the device
    (edv_verify_staged_part from the scan's copier, key ids from kid_map): a
    300,000-request batch (several 2^16-request parts, a ragged last one)
    with every 7th request forged (and _drain's every 10th), three times -- the first builds the map,
    the next two speculate -- then a batch in which one signer's key was
    replaced in the store (the ids differ: the ordinary verify) and the
    speculation after it; every outcome is the construction's."""
    import copy
    n = 300_001
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=n, n_nodes=1, n_signers=32)
    batch = [copy.deepcopy(r) for r in reqs]
    for i in range(0, n, 7):
        batch[i]["reqId"] += 1
    want = ["InvalidSignature" if i % 7 == 0 or i % 10 == 3 else r["identifier"] for i, r in enumerate(batch)]
    with _own_key_store(gpu_engine):
        _speculate_on_gpu(gpu_engine, batch, want, idrs, vks)


def _speculate_on_gpu(gpu_engine, batch, want, idrs, vks):
    a = GpuAuthNr(engine=gpu_engine, max_keys=32)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()
    spec = []
    for rep in range(3):
        res = a.authenticate_batch(batch)
        assert [r if isinstance(r, str) else type(r).__name__ for r in res] == want, rep
        spec.append(bool(a._g.last_breakdown.get("speculated")))
    assert spec == [False, True, True], spec
    # a signer whose key moves: the store evicts the LRU key for a new one (version bump)
    ks = a._key_store()
    v0 = ks.version
    ks.register([bytes(range(32))])  # any valid-length key: takes a slot by evicting one
    ks.settle()
    assert ks.version > v0
    a._g.last_breakdown = None
    res = a.authenticate_batch(batch)
    assert not (a._g.last_breakdown or {}).get("speculated")  # (an evicted signer: the ordinary path)
    assert [r if isinstance(r, str) else type(r).__name__ for r in res] == want
    a.keys_settle()
    res = a.authenticate_batch(batch)
    assert [r if isinstance(r, str) else type(r).__name__ for r in res] == want


def test_staged_subset_on_gpu(gpu_engine, sodium_verdicts):
    """edv_verify_staged_subset: after a staged batch of 70,000 requests, a subset of its items
    (every 7th, in a scrambled order, some twice) verified again by its own key bytes -- the
    true keys, then a wrong key for every 3rd -- equals libsodium's verdicts on the same bytes;
    refused once the set is reserved again, and for an index outside the batch."""
    import copy
    from plenum_amd import pack_messages
    from plenum_amd._lib import EdVerifyError
    from plenum_amd.base58 import b58decode
    from plenum_amd.serialization import serialize_msg_for_signing
    n = 70000
    reqs, rx, idrs, vks, pks, sers, sig = _drain(gpu_engine, n_req=n, n_nodes=1)
    with _own_key_store(gpu_engine):
        a = GpuAuthNr(engine=gpu_engine, stage=True)
        for idr, vk in zip(idrs, vks):
            a.addIdr(idr, vk)
        a.keys_settle()
        batch = [copy.deepcopy(r) for r in reqs]
        a.authenticate_batch(batch)  # the staged batch (set 0)
        rng = np.random.default_rng(5)
        idx = rng.permutation(np.arange(0, n, 7))
        idx = np.concatenate([idx, idx[:100]]).astype(np.uint32)
        key_of = {i: a._key_for(i) for i in set(r["identifier"] for r in batch)}
        pk = np.stack([np.frombuffer(key_of[batch[i]["identifier"]], np.uint8) for i in idx])
        sm = [b58decode(batch[i]["signature"]) + serialize_msg_for_signing(batch[i], topLevelKeysToIgnore=["signature"])
              for i in idx]
        sig64 = np.stack([np.frombuffer(x[:64], np.uint8) for x in sm])
        buf, off = pack_messages([x[64:] for x in sm])
        for wrong in (False, True):
            k = pk.copy()
            if wrong:
                k[::3] = np.roll(pk, 1, axis=0)[::3]  # another request's key (mostly another signer)
            got = np.asarray(gpu_engine.verify_staged_subset(idx, k), bool)
            want = sodium_verdicts(sig64, k, buf, off[:-1], off[1:])
            assert (got == want).all(), wrong
            assert want.any() and (not wrong or not want.all())
        with pytest.raises(EdVerifyError):
            gpu_engine.verify_staged_subset(np.array([n], np.uint32), pk[:1])
        gpu_engine.stage_select(0)
        gpu_engine.stage_reserve(1 << 20)
        with pytest.raises(EdVerifyError):
            gpu_engine.verify_staged_subset(idx[:1], pk[:1])


def test_key_churn_zipf_on_gpu(gpu_engine, sodium_verdicts):
    """VERDICT r4 'measure key churn': 100,000 signers registered with addIdr
    (more than the store's 16,384 slots), 300,000 json-decoded requests whose
    signers follow Zipf(1.1), in 3 batches, 0.5 % forged after signing.  Keys
    earn slots by verified use and evict the least-recently-used while the
    batches run (asynchronous builds); both paths carry items; every outcome
    is libsodium 1.0.18's verdict on the bytes each request serializes to."""
    import json
    from plenum_amd import _hostpack, pack_messages, synth
    from plenum_amd.base58 import b58encode
    from plenum_amd.serialization import serialize_msg_for_signing
    signers, n, batches = 100_000, 300_000, 3
    pks, sks = gpu_engine.seed_keypair_batch(synth.signer_seeds((1 << 20) + signers)[1 << 20:])
    idrs = [b58encode(bytes(pk[:16])) for pk in pks]
    vks = ["~" + b58encode(bytes(pk[16:])) for pk in pks]
    kidx = synth.zipf_signers(n, signers, 1.1, seed=23)
    msgs, spec = synth.churn_messages(kidx, idrs, alias_len=43)
    buf, off = pack_messages(msgs)
    sig = gpu_engine.sign_batch(sks, kidx, buf, off)
    texts = _hostpack.b58encode_rows(np.ascontiguousarray(sig).tobytes(), 64)
    reqs = []
    for i in range(n):
        r = synth.churn_request_dict(spec, i)
        if i % 200 == 7:
            r["reqId"] += 1
            msgs[i] = serialize_msg_for_signing(r, topLevelKeysToIgnore=["signature"])
        r["signature"] = texts[i]
        reqs.append(json.loads(json.dumps(r)))
    nbuf, noff = pack_messages(msgs)
    want = sodium_verdicts(sig, pks[kidx], nbuf, noff[:-1], noff[1:])
    assert not want[7::200].any() and want.sum() == n - len(range(7, n, 200))
    with _own_key_store(gpu_engine):
        a = GpuAuthNr(engine=gpu_engine)
        for idr, vk in zip(idrs, vks):
            a.addIdr(idr, vk)
        a.keys_settle()
        per = n // batches
        shares, regs = [], []
        for b in range(batches):
            st0 = dict(a.stats)
            res = a.authenticate_batch(reqs[b * per:(b + 1) * per])
            got = np.array([r == q["identifier"] for r, q in zip(res, reqs[b * per:(b + 1) * per])])
            assert all(type(r).__name__ == "InvalidSignature" for r, w in zip(res, want[b * per:]) if not w)
            assert (got == want[b * per:(b + 1) * per]).all(), b
            st1 = dict(a.stats)
            shares.append((st1["keyed_items"] - st0["keyed_items"]) / (st1["batch_items"] - st0["batch_items"]))
            regs.append(st1["keys_registered"] - st0["keys_registered"])
        assert len(a._key_store()) == a._key_store().capacity  # the store stays full
        assert all(0.0 < s < 1.0 for s in shares), shares  # both paths carry items in every batch
        assert sum(regs) > 0, regs  # keys earned slots (evicting others) while batches ran
