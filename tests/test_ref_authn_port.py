"""oracle/ref_authn_port.py (the configs[0] CPU leg of bench.py: the
reference's authenticate() chain restated in plain Python over libsodium)
against the reference-produced authn_kat.json outcomes."""
import json
import os
import sys

import pytest

from conftest import GOLDEN, ROOT, sodium

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ref_authn_port as P  # noqa: E402


@pytest.mark.skipif(sodium() is None, reason="needs libsodium")
def test_port_matches_reference_kats():
    s = P.Sodium()
    n = 0
    for c in json.load(open(os.path.join(GOLDEN, "authn_kat.json")))["cases"]:
        if c["identifier"] or c["signature"] or not c["register"]:
            continue
        msg = dict(c["msg"])
        if c["name"] == "tuple-field":
            msg["operation"] = tuple(msg["operation"])
        got = P.authenticate(s, {msg.get("identifier"): c["verkey"]}, msg)
        assert got == c.get("result", c.get("raises")), c["name"]
        n += 1
    assert n >= 19
    assert P.b58decode(P.b58encode(b"\0\0abc")) == b"\0\0abc"
