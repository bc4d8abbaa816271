"""The native host packer (indy-plenum_amd/csrc/hostpack.cpp, plenum_amd._hostpack)
against the Python restatements that the reference pins (serializer_kat.json from
the reference's own signing_serializer.py; base58 0.2.4 semantics): every fast-path
result is byte-identical, and every case the reference would treat differently
(tuples, non-str keys, subclasses, unencodable text, characters outside the
alphabet) returns None so the Python path -- and its exact exception -- runs."""
import json
import math
import os
import random
import struct

import pytest

from conftest import GOLDEN
from plenum_amd import _hostpack as H
from plenum_amd import client_authn
from plenum_amd.base58 import b58decode_py, b58encode
from plenum_amd.serialization import signing_serializer


def py_ser(obj, ignore=None):
    return signing_serializer.serialize(obj, topLevelKeysToIgnore=ignore)


def test_native_is_loaded():
    assert client_authn._pack_sm is H.pack_sm and client_authn._pack_split64 is H.pack_split64


def test_serializer_reference_kats_native():
    n = 0
    for case in json.load(open(os.path.join(GOLDEN, "serializer_kat.json"))):
        if "bytes_hex" not in case:
            continue
        got = H.serialize_for_signing(case["msg"], case["ignore"])
        if got is not None:  # fast path: must be the reference's bytes
            assert got.hex() == case["bytes_hex"], case["msg"]
            n += 1
    assert n >= 35


def _rand_scalar(r):
    k = r.randrange(8)
    if k == 0:
        return r.choice(["", "abc", "ключ", "值|:,", "é́", "x" * r.randrange(50)])
    if k == 1:
        return r.randrange(-10**30, 10**30)
    if k == 2:
        return r.choice([0.0, -0.0, 1e16, 1e-5, 1.5e15, 123456789012345678.0, 0.1, 1 / 3, 2.5e-300, math.inf, -math.inf])
    if k == 3:
        return struct.unpack("<d", struct.pack("<Q", r.getrandbits(64)))[0]
    if k == 4:
        return r.choice([True, False])
    if k == 5:
        return None
    if k == 6:
        return r.randrange(-5, 5)
    return r.random() * 10 ** r.randrange(-20, 20)


def _rand_obj(r, depth=0):
    k = r.randrange(10)
    if depth > 4 or k < 5:
        return _rand_scalar(r)
    if k < 7:
        return [_rand_obj(r, depth + 1) for _ in range(r.randrange(5))]
    keys = ["".join(r.choice("abcXYZ_é1") for _ in range(r.randrange(1, 5))) for _ in range(r.randrange(6))]
    return {k_: _rand_obj(r, depth + 1) for k_ in keys}


def test_serializer_fuzz_native_equals_python():
    r = random.Random(12)
    fast = 0
    for _ in range(3000):
        obj = _rand_obj(r)
        ignore = r.choice([None, ["signature"], ["a", "b"], []])
        got = H.serialize_for_signing(obj, ignore)
        want = py_ser(obj, ignore) if isinstance(obj, dict) else py_ser(obj)
        assert got is not None, obj
        assert got == want, obj
        fast += 1
    assert fast == 3000


@pytest.mark.parametrize("obj", [
    {"t": (1, 2)}, {"b": b"x"}, {"s": {1, 2}}, {1: "a"}, {"a": {2: "b"}}, {"x": "\ud800"},
    {"e": __import__("enum").IntEnum("E", "A").A}, (1, 2), {"l": [1, (2,)]},
])
def test_serializer_unusual_types_take_python_path(obj):
    assert H.serialize_for_signing(obj, None) is None


def test_b58decode_native():
    r = random.Random(3)
    for _ in range(5000):
        v = b"\0" * r.randrange(3) + bytes(r.getrandbits(8) for _ in range(r.randrange(0, 90)))
        s = b58encode(v)
        assert H.b58decode(s) == b58decode_py(s) == v
        assert H.b58decode(s.encode()) == v
    for bad in ["0OIl", "abc0", "é", "1 1", b"\xff", 17, None, bytearray(b"11")]:
        assert H.b58decode(bad) is None


def test_b58decode_every_length():
    """Random base58 strings of every length 0..130 (the native decoder takes
    its independent-products path up to 90 digits, Horner passes beyond),
    with and without leading '1's (zero bytes), against the Python decoder."""
    from plenum_amd.base58 import alphabet as ALPHABET
    r = random.Random(8)
    for n in range(131):
        for lead in (0, 1, 3):
            s = "1" * lead + "".join(r.choice(ALPHABET) for _ in range(n))
            assert H.b58decode(s) == b58decode_py(s), s
        assert H.b58decode("z" * n) == b58decode_py("z" * n)  # the largest value of each length


def test_pack_split64_is_crypto_sign_open_split():
    r = random.Random(4)
    for _ in range(200):
        n = r.randrange(0, 12)
        sigs = [bytes(r.getrandbits(8) for _ in range(r.choice([0, 10, 63, 64, 65, 100]))) for _ in range(n)]
        sers = [bytes(r.getrandbits(8) for _ in range(r.randrange(0, 70))) for _ in range(n)]
        sig64, msgs, off, short = H.pack_split64(sigs, sers)
        offs = struct.unpack("<%dQ" % (n + 1), off)
        for i in range(n):
            sm = sigs[i] + sers[i]
            if len(sm) < 64:
                assert short[i] == 1 and offs[i + 1] == offs[i]
            else:
                assert short[i] == 0
                assert sig64[64 * i:64 * i + 64] == sm[:64]
                assert msgs[offs[i]:offs[i + 1]] == sm[64:]


def test_pack_sm_layout():
    sigs, sers, keys = [b"s" * 64, b"t" * 3], [b"m", b""], [b"k" * 32, b"q" * 32]
    sm, off, pk = H.pack_sm(sigs, sers, keys)
    assert sm == b"s" * 64 + b"m" + b"t" * 3
    assert struct.unpack("<3Q", off) == (0, 65, 68)
    assert pk == b"k" * 32 + b"q" * 32
    with pytest.raises(ValueError):
        H.pack_sm([b"a"], [b"b"], [b"short"])


_EDGE_INTS = [0, 1, -1, 2**30 - 1, 2**30, -(2**30 - 1), -(2**30), 2**60 - 1, 2**60, -(2**60 - 1), -(2**60),
              2**63 - 1, -(2**63), 2**63, -(2**63) - 1, 2**64, 10**18, -(10**18)]


def _scan_pool(r, n):
    """Request-shaped dicts over the fuzz scalars/objects: every item kind the
    scan must get exactly right (fast, deferred to the GIL, Python path)."""
    msgs = []
    idrs = ["idr%d" % k for k in range(7)] + ["ключ", "é"]
    for i in range(n):
        k = r.randrange(12)
        sig = b58encode(bytes(r.getrandbits(8) for _ in range(r.choice([64, 64, 64, 0, 10, 63, 65, 100]))))
        m = {"identifier": r.choice(idrs), "reqId": r.randrange(10**18), "operation": _rand_obj(r),
             "signature": sig}
        if k == 0:
            m["signature"] = r.choice(["", "0OIl", "é", 17, None])
        elif k == 1:
            del m["identifier"]
        elif k == 2:
            m["identifier"] = r.choice(["", 5, None])
        elif k == 3:
            m = [m]
        elif k == 4:
            m[r.choice(["ключ", "z中"])] = r.random()  # wider-kind keys: ordered under the GIL
        elif k == 5:
            m[3] = "non-str key"
        elif k == 6:  # ints at CPython's digit boundaries (the workers read 1- and 2-digit ints inline)
            m["operation"] = {"n": r.choice(_EDGE_INTS), "x": [r.choice(_EDGE_INTS), r.choice(_EDGE_INTS)]}
            m["reqId"] = r.choice(_EDGE_INTS)
        msgs.append(m)
    return msgs


@pytest.mark.parametrize("threads", [2, 3, 7])
def test_scan_batch_threads_equal_serial(threads):
    """The worker-thread scan (csrc/hostpack.cpp scan_impl: wser_obj on the
    workers, deferred items by ser_obj under the GIL) returns exactly the
    single-threaded result, and the single-threaded result is the Python
    restatement's split of b58decode(sig) || serialize(msg)."""
    r = random.Random(21)
    msgs = _scan_pool(r, 3000)
    one = H.scan_batch(msgs, ["signature"], 1)
    many = H.scan_batch(msgs, ["signature"], threads)
    assert one == many
    fast, idrs, sig64, mbuf, off, short = one
    offs = struct.unpack("<%dQ" % (len(msgs) + 1), off)
    nfast = 0
    for i, m in enumerate(msgs):
        if not fast[i]:
            assert idrs[i] is None and offs[i + 1] == offs[i]
            continue
        nfast += 1
        sm = b58decode_py(m["signature"]) + py_ser(m, ["signature"])
        assert idrs[i] == m["identifier"]
        if len(sm) < 64:
            assert short[i] == 1 and offs[i + 1] == offs[i]
        else:
            assert sig64[64 * i:64 * i + 64] == sm[:64] and mbuf[offs[i]:offs[i + 1]] == sm[64:]
    assert nfast > 1000
    fu, uidx, uniq, *rest = H.scan_batch_u(msgs, ["signature"], threads)
    assert fu == fast and tuple(rest) == (sig64, mbuf, off, short)
    # distinct identifiers in order of first occurrence, whichever worker took which chunk
    assert H.scan_batch_u(msgs, ["signature"], 1) == (fu, uidx, uniq, *rest)
    u = struct.unpack("<%dI" % len(msgs), uidx)
    for i in range(len(msgs)):
        assert (uniq[u[i]] == idrs[i]) if fast[i] else u[i] == 0xffffffff
    assert len(set(uniq)) == len(uniq)


def test_scan_batch_out_buffers_reused():
    """scan_batch(..., out=[bytearray, bytearray]) (the authenticator's reused
    output buffers): the same bytes as fresh output in the first n * 64 /
    off[n] bytes, buffers grown and never shrunk across a large then a small
    batch, and a buffer with a live export falls back to fresh bytes."""
    r = random.Random(5)
    big, small = _scan_pool(r, 2000), _scan_pool(r, 300)
    out = [bytearray(), bytearray()]
    for msgs in (big, small, big):
        want = H.scan_batch_u(msgs, ["signature"], 3)
        got = H.scan_batch_u(msgs, ["signature"], 3, out)
        n = len(msgs)
        end = struct.unpack_from("<Q", want[5], 8 * n)[0]
        assert got[3] is out[0] and got[4] is out[1]
        assert bytes(got[3][:64 * n]) == want[3] and bytes(got[4][:end]) == want[4]
        assert got[:3] == want[:3] and got[5:] == want[5:]
    assert len(out[0]) >= 64 * len(big)
    held = memoryview(out[0])  # a live export: out[0] cannot be resized
    bigger = _scan_pool(r, 2500)
    got = H.scan_batch_u(bigger, ["signature"], 2, out)
    assert isinstance(got[3], bytes) and got[3] == H.scan_batch_u(bigger, ["signature"], 2)[3]
    held.release()


def test_results_from():
    codes = bytes([1, 0, 1, 2])
    got = H.results_from(codes, struct.pack("<4I", 1, 0xffffffff, 0, 0), ["a", "b"])
    assert got == ["b", None, "a", None]
    with pytest.raises(ValueError):
        H.results_from(bytes([1]), struct.pack("<I", 5), ["a"])


def test_gather_u32():
    """gather_u32 (the per-request key ids from the per-identifier ones): table[idx[i]], and
    ValueError past the table."""
    t = struct.pack("<3I", 7, 8, 9)
    assert struct.unpack("<5I", bytes(H.gather_u32(t, struct.pack("<5I", 2, 0, 1, 2, 0)))) == (9, 7, 8, 9, 7)
    assert bytes(H.gather_u32(t, b"")) == b""
    with pytest.raises(ValueError):
        H.gather_u32(t, struct.pack("<I", 3))


def test_results_ok():
    """results_ok: identifiers where ok and not short, None elsewhere, with the failed indices."""
    ok, short = bytes([1, 0, 1, 1]), bytes([0, 0, 1, 0])
    res, failed = H.results_ok(ok, short, struct.pack("<4I", 1, 9, 0, 0), ["a", "b"])
    assert res == ["b", None, None, "a"] and failed == [1, 2]
    with pytest.raises(ValueError):
        H.results_ok(bytes([1]), bytes([0]), struct.pack("<I", 5), ["a"])
    with pytest.raises(ValueError):
        H.results_ok(bytes([1, 1]), bytes([0]), struct.pack("<2I", 0, 0), ["a"])


def test_results_ok_parallel_matches_serial_and_refcounts():
    """results_ok fills the result list on the scan's worker threads and adds
    the reference counts per identifier afterwards: same list as the serial
    definition, failures in index order, and exact reference counts."""
    import sys

    import numpy as np
    from plenum_amd import _hostpack
    rng = np.random.default_rng(5)
    n = 200_000
    uniq = ["idr%d" % i + "x" * i for i in range(7)]
    ok = (rng.random(n) < 0.9).astype(np.uint8)
    short = (rng.random(n) < 0.01).astype(np.uint8)
    uidx = rng.integers(0, len(uniq), n).astype(np.uint32)
    before = [sys.getrefcount(u) for u in uniq]
    none_before = sys.getrefcount(None)
    res, failed = _hostpack.results_ok(ok.tobytes(), short.tobytes(), uidx.tobytes(), uniq)
    want_pass = (ok == 1) & (short == 0)
    assert failed == np.flatnonzero(~want_pass).tolist()
    assert res == [uniq[u] if p else None for u, p in zip(uidx.tolist(), want_pass.tolist())]
    per = np.bincount(uidx[want_pass], minlength=len(uniq))
    after = [sys.getrefcount(u) for u in uniq]
    assert [x - b for x, b in zip(after, before)] == per.tolist()
    assert sys.getrefcount(None) - none_before >= int((~want_pass).sum()) - 10
    del res
    assert [sys.getrefcount(u) for u in uniq] == before
    with pytest.raises(ValueError):
        _hostpack.results_ok(b"\x01", b"\x00", np.array([9], np.uint32).tobytes(), uniq)


def _shape_pool(r, n):
    """Request dicts that mostly share one shape (the scan workers' remembered
    dict shapes) with near misses: keys in another insertion order, a key of
    the same length with other text, an extra or a missing key, a deleted
    entry (a dict with a hole in its entry table), nested dicts of the same
    shape holding other value types, non-ASCII and wider-kind text, long keys,
    ints at the digit boundaries, str subclasses, floats."""
    class S(str):
        pass
    msgs = []
    for i in range(n):
        op = {"type": "1", "dest": "Dest%05d" % (i % 97), "verkey": "~Vk%05d" % (i % 13), "alias": "a" * (i % 40)}
        m = {"identifier": "idr%d" % (i % 9), "reqId": 1500000000000000 + i, "operation": op,
             "protocolVersion": 1, "signature": b58encode(bytes(r.getrandbits(8) for _ in range(64)))}
        k = r.randrange(40)
        if k == 0:
            m = dict(reversed(list(m.items())))
        elif k == 1:
            op["typf"] = op.pop("type")           # same length, other text
        elif k == 2:
            op["extra"] = [1, "x", None]
        elif k == 3:
            del op["alias"]
        elif k == 4:
            m["zz"] = 1
            del m["zz"]                            # a deleted entry in the table
        elif k == 5:
            op["dest"] = {"type": 2, "dest": "x", "verkey": 3.5, "alias": True}   # same shape nested
        elif k == 6:
            op["alias"] = "é" * 3                   # non-ASCII value: deferred to the GIL
        elif k == 7:
            op["ключ"] = "v"                        # wider-kind key
        elif k == 8:
            op["k" * 50] = "long key"
        elif k == 9:
            m["reqId"] = r.choice(_EDGE_INTS)
        elif k == 10:
            op["dest"] = S("subclass")
        elif k == 11:
            m[S("identifier2")] = "x"
        elif k == 12:
            op["alias"] = 0.1
        elif k == 13:
            m["operation"] = {"type": "1", "dest": "D", "verkey": "V", "alias": "x", "a": 1, "b": 2, "c": 3,
                              "d": 4, "e": 5, "f": 6, "g": 7, "h": 8, "i": 9}   # more keys than a shape holds
        elif k == 14:
            del m["signature"]
        elif k == 15:
            m["signature"] = 5
        elif k == 16:
            op["dest"] = [{"type": "1"}, {"type": 1}]
        msgs.append(m)
    return msgs


@pytest.mark.parametrize("threads", [1, 4])
def test_scan_shapes_equal_generic_and_python(monkeypatch, threads):
    """shaped_dict (remembered dict shapes) gives byte for byte what wser_dict
    gives (EDV_SCAN_SHAPES=0), and both the Python restatement's bytes."""
    r = random.Random(5)
    msgs = _shape_pool(r, 4000)
    monkeypatch.setenv("EDV_SCAN_SHAPES", "1")
    on = H.scan_batch_u(msgs, ["signature"], threads)
    monkeypatch.setenv("EDV_SCAN_SHAPES", "0")
    off = H.scan_batch_u(msgs, ["signature"], threads)
    assert on == off
    fast, uidx, uniq, sig64, mbuf, off_b, short = on
    offs = struct.unpack("<%dQ" % (len(msgs) + 1), off_b)
    nfast = 0
    for i, m in enumerate(msgs):
        if not fast[i]:
            continue
        nfast += 1
        sm = b58decode_py(m["signature"]) + py_ser(m, ["signature"])
        assert sig64[64 * i:64 * i + 64] == sm[:64] and mbuf[offs[i]:offs[i + 1]] == sm[64:], (i, m)
    assert nfast > 3000


def _keys_known_py(clients, fk, idrs, field):
    """keys_known restated: the key bytes when clients[idr] is an exact non-empty dict whose
    `field` entry is the very object fast_keys[idr] = (verkey, key bytes) remembers."""
    missing = object()
    keys, holes = [], []
    for j, idr in enumerate(idrs):
        key = None
        if type(idr) is str:
            nym = clients.get(idr)
            if type(nym) is dict and nym:
                vk = nym.get(field, missing)
                e = fk.get(idr) if vk is not missing else None
                if type(e) is tuple and len(e) == 2 and e[0] is vk and type(e[1]) is bytes:
                    key = e[1]
        keys.append(key)
        if key is None:
            holes.append(j)
    return keys, holes


@pytest.mark.parametrize("seed", [0, 1])
def test_keys_known_many_identifiers(seed):
    """keys_known over thousands of identifiers (its prefetch chain runs 8-32 identifiers
    ahead) equals the restatement, with deleted dict entries, non-str and str-subclass
    identifiers, non-ASCII text, nym values that are not exact dicts or are empty, a changed
    verkey object, malformed fast-key entries, and duplicates."""
    rng = random.Random(seed)

    class S(str):
        pass

    class D(dict):
        pass

    clients, fk, idrs = {}, {}, []
    for i in range(3000):
        idr = "%022x" % rng.getrandbits(88) if i % 97 else "idé%d" % i
        vk = "~vk%d" % i
        kind = rng.randrange(12)
        clients[idr] = ({"verkey": vk, "role": None} if kind < 7 else {} if kind == 7 else
                        D(verkey=vk) if kind == 8 else [vk] if kind == 9 else {"role": None})
        fk[idr] = ((vk, os.urandom(32)) if kind != 10 else (vk, "not bytes") if i % 2 else (vk,))
        if kind == 11:
            clients[idr] = {"verkey": "~vk%d" % i}  # an equal verkey, another object
        idrs.append(idr)
    for idr in rng.sample(idrs, 300):  # dummy slots in both dicts
        del clients[idr]
        if rng.random() < 0.5:
            del fk[idr]
    q = [(i + ".")[:-1] for i in rng.sample(idrs, 2500)]  # fresh str objects, as from a scan
    q += [q[5], 12345, None, S(idrs[0]), "unknown", b"bytes"] + [(i + ".")[:-1] for i in rng.sample(idrs, 200)]
    rng.shuffle(q)
    got = H.keys_known(clients, fk, q, "verkey")
    want = _keys_known_py(clients, fk, q, "verkey")
    assert got[1] == want[1]
    assert all(a is b for a, b in zip(got[0], want[0]))
    assert 0 < len(got[1]) < len(q)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_keys_known_flat_matches_keys_known(seed):
    """keys_known_flat (the same lookups on the scan's worker pool, CPython 3.10's dict probe
    restated) answers what keys_known does on every identifier of the adversarial pool above --
    deleted entries, non-str and str-subclass identifiers, non-ASCII text, odd nym values,
    changed verkey objects, malformed fast-key entries, duplicates -- except that keys which are
    not 32 bytes are holes too (the Python path); flat holds each key's bytes, zeros at holes;
    the key objects' reference counts are the serial path's."""
    import sys
    rng = random.Random(seed)

    class S(str):
        pass
    clients, fk, idrs = {}, {}, []
    for i in range(6000):
        idr = "%022x" % rng.getrandbits(88) if i % 97 else "idé%d" % i
        vk = "~vk%d" % i
        kind = rng.randrange(13)
        clients[idr] = ({"verkey": vk, "role": None} if kind < 7 else {} if kind == 7 else
                        [vk] if kind == 9 else {"role": None})
        fk[idr] = ((vk, os.urandom(32)) if kind not in (10, 12) else (vk, os.urandom(31)) if kind == 12 else
                   (vk, "not bytes") if i % 2 else (vk,))
        if kind == 11:
            clients[idr] = {"verkey": "~vk%d" % i}
        idrs.append(idr)
    for idr in rng.sample(idrs, 600):
        del clients[idr]
        if rng.random() < 0.5:
            del fk[idr]
    q = [(i + ".")[:-1] for i in rng.sample(idrs, 5000)]  # fresh str objects: hashes not cached yet
    q += [q[5], 12345, None, S(idrs[0]), "unknown", b"bytes"] + [(i + ".")[:-1] for i in rng.sample(idrs, 400)]
    rng.shuffle(q)
    want_keys, _ = H.keys_known(clients, fk, q, "verkey")
    want_holes = [j for j, k in enumerate(want_keys) if not (type(k) is bytes and len(k) == 32)]
    distinct = list({id(k): k for k in want_keys if k is not None}.values())

    def refs():
        out = []
        for k in distinct:
            out.append(sys.getrefcount(k))
        return out
    before = refs()
    keys, holes, flat = H.keys_known_flat(clients, fk, q, "verkey")
    assert holes == want_holes
    assert all((k is w) if j not in set(holes) else k is None for j, (k, w) in enumerate(zip(keys, want_keys)))
    assert len(flat) == 32 * len(q)
    for j in range(len(q)):
        k = keys[j]
        assert flat[32 * j:32 * j + 32] == (k if k is not None else bytes(32))
    del k
    after = refs()
    assert sum(after) - sum(before) == sum(1 for k in keys if k is not None)  # one reference per entry of keys
    del keys
    assert refs() == before


def test_key_index_matches_a_dict():
    """The key store's native index (KeyIndex: 32-byte keys -> int64, tombstones, growth) answers
    as a dict does over thousands of sets, overwrites, deletes and clears."""
    rng = random.Random(5)
    ki, ref = H.key_index(), {}
    pool = [os.urandom(32) for _ in range(5000)]
    for step in range(40000):
        k = rng.choice(pool)
        r = rng.random()
        if r < 0.5:
            v = rng.randrange(-5, 1 << 40)
            H.key_index_set(ki, k, struct.pack("<q", v))
            ref[k] = v
        elif r < 0.8:
            H.key_index_del(ki, k)
            ref.pop(k, None)
        elif r < 0.8005:
            H.key_index_clear(ki)
            ref.clear()
        if step % 4000 == 0 or step == 39999:
            got = struct.unpack("<%dq" % len(pool), H.key_index_get(ki, b"".join(pool)))
            assert list(got) == [ref.get(k, -1) for k in pool]
            assert H.key_index_len(ki) == len(ref)
    # many keys at once
    ks = [os.urandom(32) for _ in range(3000)]
    H.key_index_set(ki, b"".join(ks), struct.pack("<3000q", *range(3000)))
    assert list(struct.unpack("<3000q", H.key_index_get(ki, b"".join(ks)))) == list(range(3000))
    with pytest.raises(ValueError):
        H.key_index_get(ki, b"x" * 33)


def test_general_items_matches_numpy():
    """general_items: the positions whose identifier is flagged general, ascending, and each one's
    32-byte key -- numpy's mask / flatnonzero / row gather, on the worker pool; ids out of range
    raise."""
    import numpy as np
    from plenum_amd._hostpack import general_items
    rng = np.random.default_rng(3)
    for n, nu in ((0, 4), (7, 3), (5000, 200), (120000, 9000)):
        uidx = rng.integers(0, nu, n).astype(np.uint32)
        isg = (rng.random(nu) < 0.3).astype(np.uint8)
        flat = rng.integers(0, 256, 32 * nu, dtype=np.uint8).tobytes()
        g, k = general_items(uidx, isg, flat)
        gen = np.flatnonzero(isg[uidx])
        assert np.array_equal(np.frombuffer(g, np.uint32), gen)
        assert k == np.frombuffer(flat, np.uint8).reshape(-1, 32)[uidx[gen]].tobytes()
    with pytest.raises(ValueError):
        general_items(np.array([5], np.uint32), np.zeros(3, np.uint8), bytes(96))
    with pytest.raises(ValueError):
        general_items(np.array([0], np.uint32), np.zeros(3, np.uint8), bytes(95))


def test_scan_many_distinct_identifiers_first_occurrence_order():
    """A churning batch's shape: ~15k distinct identifiers in 40k requests (the merge's hash
    partitions on the workers, the first occurrences ordered through the position bitmap): uniq
    is the identifiers in order of first occurrence and uidx maps every request to its own --
    equal to the one-thread scan and to Python's dict.fromkeys order."""
    r = random.Random(5)
    n, distinct = 40000, 15000
    msgs = []
    for i in range(n):
        k = i if i < distinct else r.randrange(distinct)
        msgs.append({"identifier": "D%07d" % ((k * 7919) % 1000003), "reqId": i,
                     "operation": {"type": "1", "alias": "a" * (i % 5)},
                     "signature": b58encode(bytes(r.getrandbits(8) for _ in range(64)))})
    r.shuffle(msgs)
    fu, uidx, uniq, *rest = H.scan_batch_u(msgs, ["signature"], 8)
    assert H.scan_batch_u(msgs, ["signature"], 1) == (fu, uidx, uniq, *rest)
    assert uniq == list(dict.fromkeys(m["identifier"] for m in msgs))
    u = struct.unpack("<%dI" % n, uidx)
    assert all(uniq[u[i]] == msgs[i]["identifier"] for i in range(n))
