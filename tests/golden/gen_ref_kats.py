"""Generate reference-pinned KATs by importing the reference's own Python
(/root/reference, hariexcel/indy-plenum v1.2) in THIS container.

Run with the conda interpreter (the reference needs Python < 3.10 for
`from collections import Iterable`, signing_serializer.py:23):
    /opt/conda/bin/python3.9 tests/golden/gen_ref_kats.py

What is imported and run for real: common/serializers/signing_serializer.py,
common/serializers/serialization.py, plenum/common/exceptions.py,
plenum/common/verifier.py, plenum/server/client_authn.py,
stp_core/crypto/nacl_wrappers.py.  Third-party packages the reference needs
that are not installed here are replaced by the stand-ins of ref_standins.py
(libnacl over libsodium 1.0.18, the base58 0.2.4 API, logging stubs, and a
domain_req_handler whose getNymDetails answers from an empty state).
Outputs (pure data, committed): serializer_kat.json, authn_kat.json.  The
quorum / vote-set fixture is gen_ref_quorums.py.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_standins as R  # noqa: E402

R.install()
_b58encode, _b58decode = R.b58encode, R.b58decode
_crypto_sign_seed_keypair, _crypto_sign = R.crypto_sign_seed_keypair, R.crypto_sign

from common.serializers.serialization import serialize_msg_for_signing  # noqa: E402
from plenum.server.client_authn import SimpleAuthNr  # noqa: E402
from plenum.common.verifier import DidVerifier  # noqa: E402


# ------------------------------------------------------------------- KATs
def serializer_kats():
    cases = [
        {"a": 1}, {"b": "x", "a": "y"}, {"k": [1, 2, 3]}, {"k": None}, {"k": True}, {"k": False},
        {"k": 1.5}, {"k": 1e16}, {"k": 0.1}, {"k": -3}, {"k": 12345678901234567890},
        {"nested": {"z": 1, "a": {"q": [1, {"w": "e"}]}}}, {"u": "héllo 世界"},
        {"signature": "drop-me", "identifier": "idr", "reqId": 1},
        {"l": []}, {"d": {}}, {"s": ""}, {"mixed": [None, "a", 1, 2.5, [3, 4], {"x": "y"}]},
        {"identifier": "L5AD5g65TDQr1PPHHRoiGf", "reqId": 1513945121191691,
         "operation": {"type": "1", "dest": "Bf9Z1tKWpcJAvKJVhZhvVZ", "verkey": "~8zH9ZSyZTFPGJ4ZPL5Rvxx"},
         "protocolVersion": 1, "signature": "x"},
        {"myMsg": "42 (forty-two) is the natural number that succeeds 41 and precedes 43."},
        {"1": "a", "2": "b", "3": [1, {"2": "k"}]},
        {"": {"k": "v"}}, {"a": {"": {"q": 1}}}, {"l": [[1, [2]], None, True, 1.5e300, -0.0]},
    ]
    out = []
    for c in cases:
        for ignore in (None, ["signature"]):
            out.append({"msg": c, "ignore": ignore,
                        "bytes_hex": serialize_msg_for_signing(c, topLevelKeysToIgnore=ignore).hex()})
    # non-acceptable types raise
    for bad in ({"t": (1, 2)}, {"b": b"x"}, {"s": {1, 2}},
                {"a": {1: "x"}}, {"a": [{"b": {2: 1}}]}):  # a non-str key below the top: the key-path join raises
        try:
            serialize_msg_for_signing(bad)
            res = "ok"
        except Exception as ex:
            res = type(ex).__name__
        out.append({"msg_repr": repr(bad), "raises": res})
    return out


def authn_kats():
    seed = b"Falcon00000000000000000000000000"
    pk, sk = _crypto_sign_seed_keypair(seed)
    full_vk = _b58encode(pk)
    did_idr = _b58encode(pk[:16])
    abbr_vk = "~" + _b58encode(pk[16:])
    cases = []

    def sign(msg):
        ser = serialize_msg_for_signing(msg, topLevelKeysToIgnore=["signature"])
        return _b58encode(_crypto_sign(ser, sk)[:64])

    def run(name, msg, verkey, identifier=None, signature=None, register=True):
        a = SimpleAuthNr()
        if register:
            a.addIdr(msg.get("identifier") if identifier is None else identifier, verkey)
        try:
            res = {"result": a.authenticate(msg, identifier, signature)}
        except Exception as ex:
            res = {"raises": type(ex).__name__,
                   "cause": type(ex.__cause__).__name__ if ex.__cause__ is not None else None}
        cases.append(dict(name=name, msg=msg, verkey=verkey, identifier=identifier, signature=signature,
                          register=register, **res))

    base = {"identifier": did_idr, "reqId": 1513945121191691, "protocolVersion": 1,
            "operation": {"type": "1", "dest": "Bf9Z1tKWpcJAvKJVhZhvVZ", "verkey": "~8zH9ZSyZTFPGJ4ZPL5Rvxx"}}
    good = dict(base, signature=sign(base))
    run("valid-abbreviated-verkey", good, abbr_vk)
    run("valid-full-verkey", good, full_vk)
    cryp = dict(base, identifier=full_vk)
    cryp = dict(cryp, signature=sign(cryp))
    run("valid-cryptonym-no-verkey", cryp, "", register=True)
    run("tampered-reqId", dict(good, reqId=good["reqId"] + 1), abbr_vk)
    run("tampered-operation", dict(good, operation=dict(good["operation"], dest="x")), abbr_vk)
    run("extra-top-level-key", dict(good, extra="1"), abbr_vk)
    sigb = _b58decode(good["signature"])
    run("sig-63-bytes", dict(good, signature=_b58encode(sigb[:63])), abbr_vk)
    run("sig-65-bytes", dict(good, signature=_b58encode(sigb + b"\x01")), abbr_vk)
    run("sig-leading-zeros", dict(good, signature=_b58encode(b"\0" * 10 + sigb)), abbr_vk)
    run("sig-non-base58", dict(good, signature="0OIl" + good["signature"][4:]), abbr_vk)
    run("sig-empty", dict(good, signature=""), abbr_vk)
    run("sig-missing", dict(base), abbr_vk)
    run("sig-not-str", dict(good, signature=12345), abbr_vk)
    run("idr-empty", dict(good, identifier=""), abbr_vk, identifier=None, register=False)
    nid = dict(good)
    del nid["identifier"]
    run("idr-missing", nid, abbr_vk, register=False)
    run("verkey-31-bytes", good, _b58encode(pk[:31]))
    run("verkey-abbrev-15-bytes", good, "~" + _b58encode(pk[16:31]))
    run("verkey-hex-encoded", good, _b58encode(pk.hex().encode()))
    run("verkey-none", good, None)
    run("verkey-non-base58", good, "~0OIl")
    run("unknown-identifier", good, abbr_vk, register=False)
    run("explicit-identifier-and-signature", dict(base), abbr_vk, identifier=did_idr, signature=good["signature"])
    run("explicit-signature-wrong", dict(base), abbr_vk, identifier=did_idr, signature=sign(dict(base, reqId=2)))
    run("float-field", dict(base, reqId=1.5, signature=sign(dict(base, reqId=1.5))), abbr_vk)
    run("tuple-field", dict(good, operation=(1, 2)), abbr_vk)
    # A signed request the reference itself holds: the PROPAGATE payload of
    # plenum/test/node_request/message_request/test_valid_message_request.py:60-64
    # (data only).  Its identifier is a 32-byte cryptonym, so with an empty
    # verkey on record DidVerifier uses the identifier as the key
    # (plenum/common/verifier.py:26-28).
    prop = {"identifier": "5rArie7XKukPCaEwq5XGQJnM9Fc5aZE3M9HAPVfMU2xC",
            "signature": "ZbZG68WiaK67eU3CsgpVi85jpgCztW9Yqe7D5ezDUfWbKdiPPVbWq4Tb5m4Ur3jcR5wJ8zmBUZXZudjvMN63Aa9",
            "operation": {"amount": 62, "type": "buy"},
            "reqId": 1499782864169193}
    psig = _b58decode(prop["signature"])
    run("ref-propagate-cryptonym", prop, "")
    run("ref-propagate-full-verkey", prop, prop["identifier"])
    run("ref-propagate-tampered-reqId", dict(prop, reqId=prop["reqId"] + 1), "")
    run("ref-propagate-tampered-amount", dict(prop, operation=dict(prop["operation"], amount=63)), "")
    run("ref-propagate-tampered-S", dict(prop, signature=_b58encode(psig[:40] + bytes([psig[40] ^ 1]) + psig[41:])), "")
    run("ref-propagate-sig-63-bytes", dict(prop, signature=_b58encode(psig[:63])), "")
    run("ref-propagate-unregistered", prop, "", register=False)
    # DidVerifier KATs from plenum/test/common/test_verifier.py
    dv = DidVerifier("~8zH9ZSyZTFPGJ4ZPL5Rvxx", identifier="99BgFBg35BehzfSADV5nM4")
    return {"cases": cases, "did_expand": [{"verkey": "~8zH9ZSyZTFPGJ4ZPL5Rvxx", "identifier": "99BgFBg35BehzfSADV5nM4",
                                            "expanded": dv.verkey}],
            "seed_hex": seed.hex(), "pk_hex": pk.hex()}


def main():
    with open(os.path.join(HERE, "serializer_kat.json"), "w") as f:
        json.dump(serializer_kats(), f, indent=0, ensure_ascii=True)
    with open(os.path.join(HERE, "authn_kat.json"), "w") as f:
        json.dump(authn_kats(), f, indent=0, ensure_ascii=True)
    print("ok")


if __name__ == "__main__":
    main()
