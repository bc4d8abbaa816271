"""Stand-ins that let the reference's own Python (/root/reference,
hariexcel/indy-plenum v1.2) import and run in THIS container, for the
fixture generators and drop-in checks under tests/golden/.  Container-side
only: nothing here runs on the GPU box, and no reference source is copied --
the reference modules are imported from /root/reference as they are.

Run the scripts that use this with the conda interpreter (the reference needs
Python < 3.10 for `from collections import Iterable`, signing_serializer.py:23).

Stand-ins (written for these generators; only third-party packages that are
not installed, and modules whose import chain is a SyntaxError on Python >= 3.7):
  libnacl          ctypes over libsodium 1.0.18 (/opt/conda/lib/libsodium.so.23);
                   counts crypto_sign_open calls in CALLS["crypto_sign_open"]
  base58           the 0.2.4 API (b58encode -> str, b58decode -> bytes)
  stp_core.common.log, plenum.common.jsonpickle_util   logging / no-op stubs
  plenum.server.domain_req_handler   getNymDetails looks up NYMS (default empty)
  plenum.common.util                 ONLY getMaxFailures, taken from the text of
                                     the reference's util.py (the module itself is
                                     a SyntaxError at util.py:337 `asyncio.async`)
                                     and executed as written
  plenum.common.messages.node_messages  Prepare / Commit as plain records (models.py
                                     only reads .viewNo / .ppSeqNo; the real module
                                     pulls in the message-validation stack)
"""
import collections
import ctypes
import logging
import os
import re
import sys
import types

REF = "/root/reference"
CALLS = collections.Counter()
NYMS = {}

_sodium = None


def sodium():
    global _sodium
    if _sodium is None:
        _sodium = ctypes.CDLL("/opt/conda/lib/libsodium.so.23")
        _sodium.sodium_init()
    return _sodium


def crypto_sign_open(sm, pk):
    CALLS["crypto_sign_open"] += 1
    m = ctypes.create_string_buffer(len(sm) + 1)
    mlen = ctypes.c_ulonglong()
    if sodium().crypto_sign_open(m, ctypes.byref(mlen), sm, ctypes.c_ulonglong(len(sm)), pk):
        raise ValueError("Failed to validate message")
    return m.raw[:mlen.value]


def crypto_sign_seed_keypair(seed):
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    sodium().crypto_sign_seed_keypair(pk, sk, seed)
    return pk.raw, sk.raw


def crypto_sign(msg, sk):
    sm = ctypes.create_string_buffer(len(msg) + 64)
    smlen = ctypes.c_ulonglong()
    sodium().crypto_sign(sm, ctypes.byref(smlen), msg, ctypes.c_ulonglong(len(msg)), sk)
    return sm.raw[:smlen.value]


_ALPH = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def b58encode(v):
    if not isinstance(v, bytes):
        raise TypeError("a bytes-like object is required")
    nz = len(v) - len(v.lstrip(b"\0"))
    acc, out = int.from_bytes(v, "big"), ""
    while acc:
        acc, r = divmod(acc, 58)
        out = _ALPH[r] + out
    return _ALPH[0] * nz + out


def b58decode(v):
    if not isinstance(v, str):
        v = v.decode("ascii")
    nz = len(v) - len(v.lstrip(_ALPH[0]))
    acc = 0
    for c in v[nz:]:
        acc = acc * 58 + _ALPH.index(c)
    return b"\0" * nz + (acc.to_bytes((acc.bit_length() + 7) // 8, "big") if acc else b"")


def _unused(*a, **k):
    raise NotImplementedError("not needed for signature verification")


def _module(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def reference_function(relpath, name, extra_globals=None):
    """Execute one top-level function of a reference file as written (its text
    up to the next top-level statement) and return it."""
    src = open(os.path.join(REF, relpath)).read()
    m = re.search(r"^def %s\(.*?(?=^\S)" % re.escape(name), src, re.S | re.M)
    if m is None:
        raise LookupError("%s not found in %s" % (name, relpath))
    g = dict(extra_globals or {})
    exec(compile(m.group(0), os.path.join(REF, relpath), "exec"), g)
    return g[name]


def install():
    """Register the stand-ins and put /root/reference on sys.path (idempotent)."""
    if "libnacl" in sys.modules and getattr(sys.modules["libnacl"], "_edv_standin", False):
        return
    libnacl = _module("libnacl", _edv_standin=True, crypto_sign_PUBLICKEYBYTES=32, crypto_sign_SECRETKEYBYTES=64,
                      crypto_sign_BYTES=64, crypto_box_PUBLICKEYBYTES=32, crypto_box_SECRETKEYBYTES=32,
                      crypto_box_NONCEBYTES=24, crypto_sign_SEEDBYTES=32,
                      crypto_box_afternm=_unused, crypto_box_beforenm=_unused, crypto_box_open_afternm=_unused,
                      crypto_scalarmult_base=_unused, crypto_sign_open=crypto_sign_open,
                      crypto_sign_seed_keypair=crypto_sign_seed_keypair, crypto_sign=crypto_sign,
                      randombytes=lambda n: os.urandom(n), crypto_box_keypair=lambda: (None, None))
    libnacl.secret = _module("libnacl.secret")
    _module("base58", b58encode=b58encode, b58decode=b58decode, alphabet=_ALPH)
    log_mod = _module("stp_core.common.log", getlogger=lambda name=None: logging.getLogger("ref"))

    class DomainRequestHandler:
        @staticmethod
        def getNymDetails(state, nym, isCommitted=True):
            return dict(NYMS.get(nym, {}))

    _module("plenum.server.domain_req_handler", DomainRequestHandler=DomainRequestHandler)
    _module("plenum.common.jsonpickle_util", setUpJsonpickle=lambda: None)
    from math import floor
    _module("plenum.common.util",
            getMaxFailures=reference_function("plenum/common/util.py", "getMaxFailures", {"floor": floor}))
    Prepare = collections.namedtuple("Prepare", "instId viewNo ppSeqNo ppTime digest stateRootHash txnRootHash")
    Commit = collections.namedtuple("Commit", "instId viewNo ppSeqNo")
    _module("plenum.common.messages.node_messages", Prepare=Prepare, Commit=Commit)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import stp_core.common  # noqa: F401  (package __init__ only)
    sys.modules["stp_core.common"].log = log_mod
