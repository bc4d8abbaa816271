"""serialize_msg_for_signing and base58 pinned by the reference itself:
tests/golden/serializer_kat.json was produced by importing the reference's
common/serializers/signing_serializer.py (tests/golden/gen_ref_kats.py); the
base58 / DID KATs are the reference's own test constants
(plenum/test/common/test_verifier.py:6-9, test_signers.py:27-33)."""
import json
import os

import pytest

from conftest import GOLDEN
from plenum_amd.base58 import b58decode, b58encode
from plenum_amd.serialization import serialize_msg_for_signing


def kats():
    return json.load(open(os.path.join(GOLDEN, "serializer_kat.json")))


def test_serializer_matches_reference_kats():
    n = 0
    for case in kats():
        if "bytes_hex" not in case:
            continue
        got = serialize_msg_for_signing(case["msg"], topLevelKeysToIgnore=case["ignore"])
        assert got.hex() == case["bytes_hex"], case["msg"]
        n += 1
    assert n >= 40


@pytest.mark.parametrize("bad", [{"t": (1, 2)}, {"b": b"x"}, {"s": {1, 2}}])
def test_serializer_rejects_non_primitive_types(bad):
    assert any(c.get("raises") == "Exception" for c in kats() if "msg_repr" in c)
    with pytest.raises(Exception, match="invalid type found"):
        serialize_msg_for_signing(bad)


def test_serializer_raises_what_the_reference_raised():
    """Every failing case of the reference-run KATs raises the same exception
    class here (a non-str key below the top level: the reference's key-path
    join raises TypeError; non-primitive values: Exception)."""
    import ast
    raising = [c for c in kats() if "raises" in c]
    assert {c["raises"] for c in raising} == {"Exception", "TypeError"}
    for c in raising:
        with pytest.raises(Exception) as ei:
            serialize_msg_for_signing(ast.literal_eval(c["msg_repr"]))
        assert type(ei.value).__name__ == c["raises"], c


def test_base58_reference_kats():
    cryptonym = 'BPtrqHo3WyjmTNpVchEhWxp3qfDdssdFUNoM8kmKoEWw'
    did_id, did_verkey = 'L5AD5g65TDQr1PPHHRoiGf', 'Bf9Z1tKWpcJAvKJVhZhvVZ'
    assert b58encode(b58decode(did_id) + b58decode(did_verkey)) == cryptonym
    assert b58decode("1112") == b"\0\0\0\x01"
    assert b58encode(b"\0\0\x01") == "112"
    assert b58encode(b"") == "" and b58decode("") == b""
    with pytest.raises(ValueError):
        b58decode("0OIl")
    with pytest.raises(TypeError):
        b58encode("str")


def test_base58_roundtrip_random():
    import random
    rng = random.Random(1)
    for _ in range(500):
        v = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 70)))
        v = b"\0" * rng.randrange(3) + v
        assert b58decode(b58encode(v)) == v
