"""Request digests on the GPU.

Reference: plenum/common/request.py
  :24      self.digest = self.getDigest()            (every request, at construction)
  :51-52   getDigest = sha256(serialize_msg_for_signing(self.signingState)).hexdigest()
  :61-71   signingState = {identifier, reqId, operation[, protocolVersion if not None]}
The signing bytes come from the same serializer as the verify path (native
fast path, plenum_amd/_hostpack); the SHA-256 runs one lane per request in
edv_sha256_kernel (csrc/sha256.h).  For a request whose only top-level keys
are identifier / reqId / operation / protocolVersion / signature, the
signingState bytes equal the bytes the signature covers, so a verify batch's
device message buffer can be hashed in place (edv_sha256_spans_device)."""
import numpy as np

from .serialization import serialize_msg_for_signing

IDENTIFIER, REQ_ID, OPERATION, PROTOCOL_VERSION = "identifier", "reqId", "operation", "protocolVersion"


def signing_state(req):
    """request.py:61-71 for a request given as its dict (Request.as_dict)."""
    dct = {IDENTIFIER: req.get(IDENTIFIER), REQ_ID: req.get(REQ_ID), OPERATION: req.get(OPERATION)}
    if req.get(PROTOCOL_VERSION) is not None:
        dct[PROTOCOL_VERSION] = req[PROTOCOL_VERSION]
    return dct


def request_digests(reqs, engine):
    """Request.digest (hex str) of every request dict, hashed on the GPU."""
    sers = [serialize_msg_for_signing(signing_state(r)) for r in reqs]
    off = np.zeros(len(sers) + 1, np.uint64)
    if sers:
        off[1:] = np.cumsum([len(s) for s in sers])
    out = engine.sha256_batch(np.frombuffer(b"".join(sers), np.uint8), off)
    return [bytes(row).hex() for row in out]
