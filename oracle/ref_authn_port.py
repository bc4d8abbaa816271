"""TEST/BENCH INFRASTRUCTURE ONLY: a plain-Python port of the reference's
per-request authentication path, timed as bench.py's configs[0] CPU leg
("Plenum CoreAuthNr verifying 10k synthetic signed NYM requests via libsodium
on CPU", BASELINE.json configs[0]).  The reference itself cannot travel to the
GPU box, so this restates its call chain step for step, in Python, over the
same libsodium the reference reaches through libnacl:

  NaclAuthNr.authenticate          plenum/server/client_authn.py:67-107
    base58.b58decode(signature)    :89            (base58 0.2.4 algorithm)
    serializeForSig(msg, ['signature'])  :92 -> SigningSerializer.serialize
                                   common/serializers/signing_serializer.py:35-91
    SimpleAuthNr.getVerkey         :142-154       (dict hit)
    DidVerifier(verkey, identifier) plenum/common/verifier.py:21-46
                                   ('~' expansion: b58encode(b58decode(idr) +
                                   b58decode(vk[1:])), then b58decode -> 32 B)
    vr.verify(sig, ser)            verifier.py:48-49 -> nacl_wrappers.py:232-242
      VerifyKey.verify(sig + msg)  nacl_wrappers.py:100-108
        libnacl.crypto_sign_open   -> libsodium crypto_sign_open (ctypes)

No product code (plenum_amd) is imported.  Usage (a child process of bench.py,
so the GPU process never forks):
    python oracle/ref_authn_port.py INPUT.json [--procs K]
    python oracle/ref_authn_port.py DRAINS.json --drain   (the node's receive loop, run_drains)
INPUT.json: {"requests": [...], "verkeys": {identifier: verkey}}; prints one
JSON line {"value": requests/s, "procs": K, "accepted": A, ...}.
"""
import ctypes
import json
import os
import sys
import time
from collections.abc import Iterable

_ALPH = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def b58encode(v):
    nz = len(v) - len(v.lstrip(b"\0"))
    p, acc = 1, 0
    for c in reversed(v):  # base58 0.2.4: big-endian integer, then digits
        acc += p * c
        p <<= 8
    out = ""
    while acc:
        acc, idx = divmod(acc, 58)
        out = _ALPH[idx] + out
    return _ALPH[0] * nz + out


def b58decode(v):
    if not isinstance(v, str):
        v = v.decode("ascii")
    nz = len(v) - len(v.lstrip(_ALPH[0]))
    p, acc = 1, 0
    for c in reversed(v[nz:]):
        acc += p * _ALPH.index(c)
        p *= 58
    out = []
    while acc > 0:
        acc, mod = divmod(acc, 256)
        out.append(mod)
    return b"\0" * nz + bytes(reversed(out))


ACCEPTABLE = (str, int, float, list, dict, type(None))


def serialize(obj, level=0, ignore=None):
    if not isinstance(obj, ACCEPTABLE):
        raise Exception("invalid type found: {}".format(obj))
    if isinstance(obj, str):
        res = obj
    elif isinstance(obj, dict):
        keys = list(obj.keys()) if level > 0 else [k for k in obj.keys() if k not in (ignore or [])]
        keys.sort()
        res = "|".join(str(k) + ":" + serialize(obj[k], level + 1).decode() for k in keys)
    elif isinstance(obj, Iterable):
        res = ",".join(serialize(o, level + 1).decode() for o in obj)
    elif obj is None:
        res = ""
    else:
        res = str(obj)
    return res.encode("utf-8")


class Sodium:
    def __init__(self):
        for cand in ("libsodium.so.23", "/opt/conda/lib/libsodium.so.23"):
            try:
                self.lib = ctypes.CDLL(cand)
                break
            except OSError:
                continue
        else:
            raise OSError("libsodium not found")
        self.lib.sodium_init()
        self.lib.sodium_version_string.restype = ctypes.c_char_p
        self.version = self.lib.sodium_version_string().decode()

    def crypto_sign_open(self, sm, pk):
        m = ctypes.create_string_buffer(len(sm))
        mlen = ctypes.c_ulonglong()
        if self.lib.crypto_sign_open(m, ctypes.byref(mlen), sm, ctypes.c_ulonglong(len(sm)), pk):
            raise ValueError("Failed to validate message")
        return m.raw[:mlen.value]


def authenticate(sodium, verkeys, msg):
    """-> identifier, or an exception class name (reference check order)."""
    signature = msg.get("signature")
    if not signature:
        return "EmptySignature" if "signature" in msg else "MissingSignature"
    identifier = msg.get("identifier")
    if not identifier:
        return "EmptyIdentifier" if "identifier" in msg else "MissingIdentifier"
    try:
        sig = b58decode(signature)
    except Exception:
        return "InvalidSignatureFormat"
    try:
        ser = serialize(msg, ignore=["signature"])
    except Exception:
        return "CouldNotAuthenticate"
    if identifier not in verkeys:
        return "UnknownIdentifier"
    verkey = verkeys[identifier]
    if verkey is None:
        return "CouldNotAuthenticate"
    try:
        raw_idr = b58decode(identifier)
        vk = verkey
        if len(raw_idr) == 32 and not vk:
            vk = identifier
        if vk[0] == "~":
            vk = b58encode(raw_idr + b58decode(vk[1:]))
        pk = b58decode(vk)
        if len(pk) != 32:  # nacl_wrappers.py:216-230: anything else is hex (HexEncoder)
            pk = bytes.fromhex(pk.decode())
        if len(pk) != 32:
            return "CouldNotAuthenticate"
        try:
            sodium.crypto_sign_open(sig + ser, pk)
        except ValueError:
            return "InvalidSignature"
    except Exception:
        return "CouldNotAuthenticate"
    return identifier


def run_slice(path, lo, hi, out_q=None):
    spec = json.load(open(path))
    reqs, verkeys = spec["requests"][lo:hi], spec["verkeys"]
    sodium = Sodium()
    t0 = time.perf_counter()
    res = [authenticate(sodium, verkeys, m) for m in reqs]
    dt = time.perf_counter() - t0
    acc = sum(1 for r, m in zip(res, reqs) if r == m.get("identifier"))
    return {"n": len(reqs), "seconds": dt, "accepted": acc, "version": sodium.version}


def run_drains(path):
    """--drain: the node's receive loop over recorded drains, the reference way
    (zstack.py:528-549 processReceived: json-decode each entry; node.py:1270-1337
    handleOneNodeMsg: a PROPAGATE authenticates msg.request, a BATCH re-decodes
    and re-enters for every entry; node.py:1399-1451 validateClientMsg: a
    request authenticates SafeRequest(**msg).as_dict, request.py:27-39), every
    authenticate() the reference chain above over libsodium.
    INPUT.json: {"drains": [{"node": [text, ...], "client": [text, ...]}, ...],
    "verkeys": {...}}; the node stack is drained first, as bench.py's leg does."""
    spec = json.load(open(path))
    verkeys = spec["verkeys"]
    sodium = Sodium()
    stats = {"authenticate": 0, "accepted": 0, "entries": 0}

    def auth(req):
        stats["authenticate"] += 1
        r = authenticate(sodium, verkeys, req)
        stats["accepted"] += r == req.get("identifier")

    def node_msg(m):
        if not isinstance(m, dict):
            return
        op = m.get("op")
        if op == "PROPAGATE" and isinstance(m.get("request"), dict):
            auth(m["request"])
        elif op == "BATCH":
            for t in m.get("messages") or ():
                try:
                    node_msg(json.loads(t))
                except ValueError:
                    continue

    def client_msg(m):
        if isinstance(m, dict) and all(k in m for k in ("operation", "identifier", "reqId")):
            req = {"identifier": m["identifier"], "reqId": m["reqId"], "operation": m["operation"]}
            if m.get("signature") is not None:
                req["signature"] = m["signature"]
            if m.get("protocolVersion") is not None:
                req["protocolVersion"] = m["protocolVersion"]
            auth(req)

    t0 = time.perf_counter()
    for d in spec["drains"]:
        for handler, texts in ((node_msg, d["node"]), (client_msg, d["client"])):
            for t in texts:
                stats["entries"] += 1
                try:
                    m = json.loads(t)
                except ValueError:
                    continue
                handler(m)
    dt = time.perf_counter() - t0
    return {"seconds": dt, "drains": len(spec["drains"]), "rx_entries": stats["entries"],
            "authenticate_calls": stats["authenticate"], "accepted": stats["accepted"],
            "authenticate_per_s": stats["authenticate"] / dt, "us_per_authenticate": dt / stats["authenticate"] * 1e6,
            "procs": 1, "libsodium": sodium.version}


def main():
    path = sys.argv[1]
    if "--drain" in sys.argv:
        print(json.dumps(run_drains(path)))
        return
    procs = int(sys.argv[sys.argv.index("--procs") + 1]) if "--procs" in sys.argv else 1
    n = len(json.load(open(path))["requests"])
    if procs == 1:
        r = run_slice(path, 0, n)
        print(json.dumps({"value": r["n"] / r["seconds"], "procs": 1, "n": n, "accepted": r["accepted"],
                          "libsodium": r["version"]}))
        return
    import multiprocessing as mp
    bounds = [(n * i // procs, n * (i + 1) // procs) for i in range(procs)]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(procs) as pool:  # this process never touches a GPU
        parts = pool.starmap(run_slice, [(path, lo, hi) for lo, hi in bounds])
    wall = time.perf_counter() - t0
    slowest = max(p["seconds"] for p in parts)
    print(json.dumps({"value": n / slowest, "value_wall_incl_startup": n / wall, "procs": procs, "n": n,
                      "accepted": sum(p["accepted"] for p in parts), "libsodium": parts[0]["version"]}))


if __name__ == "__main__":
    main()
