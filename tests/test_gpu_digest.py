"""Request digests on the GPU (plenum/common/request.py:51-52) against the
reference formula sha256(serialize_msg_for_signing(signingState)).hexdigest()."""
import hashlib

import numpy as np
import pytest

from plenum_amd import pack_messages, synth
from plenum_amd.request_digest import request_digests, signing_state
from plenum_amd.serialization import serialize_msg_for_signing

pytestmark = pytest.mark.gpu


def test_sha256_lengths(gpu_engine):
    rng = np.random.default_rng(5)
    msgs = [bytes(rng.integers(0, 256, int(n), dtype=np.uint8)) for n in
            list(range(0, 300)) + [447, 448, 511, 512, 4095, 4096, 10000]]
    buf, off = pack_messages(msgs)
    got = gpu_engine.sha256_batch(buf, off)
    for i, m in enumerate(msgs):
        assert bytes(got[i]) == hashlib.sha256(m).digest(), len(m)


def test_request_digests_match_reference_formula(gpu_engine):
    pks = [bytes(range(i, i + 32)) for i in range(7)]
    _, _, spec = synth.nym_messages(500, pks, alias_len=20)
    reqs = [synth.nym_request_dict(spec, i, 7) for i in range(500)]
    for i, r in enumerate(reqs):
        r["signature"] = "sig%d" % i
        if i % 5 == 0:
            r["protocolVersion"] = None
        if i % 7 == 0:
            r["extra"] = {"k": i}  # not part of signingState
    got = request_digests(reqs, gpu_engine)
    want = [hashlib.sha256(serialize_msg_for_signing(signing_state(r))).hexdigest() for r in reqs]
    assert got == want
