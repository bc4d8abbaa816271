"""Synthetic signed-request batches shaped like Plenum NYM writes.

Request shape follows the reference's client signing path
(plenum/client/wallet.py:181-217 -> plenum/common/signer_did.py:114-121):
  {identifier: b58(pk[:16]), reqId: int, protocolVersion: 1,
   operation: {type: '1', dest: b58(16 B), verkey: '~' + b58(16 B)[, alias: ...]}}
signed over serialize_msg_for_signing(req, ['signature']).  Signer seeds are
i.to_bytes(2, 'little') + 30 zero bytes.

`nym_messages` builds the signing bytes with one format string per request;
tests/test_synth.py checks it byte-for-byte against serialize_msg_for_signing.
"""
import numpy as np

from .base58 import b58encode
from .serialization import serialize_msg_for_signing

REQ_ID_BASE = 1_500_000_000_000_000


def signer_seeds(n_signers):
    """Seed i = i little-endian in the first bytes, zeros after (i < 2^16: the
    C0 seeds; larger counts -- distinct-key batches -- use 4 bytes)."""
    seeds = np.zeros((n_signers, 32), np.uint8)
    seeds[:, :4] = np.arange(n_signers, dtype="<u4").view(np.uint8).reshape(-1, 4)
    return seeds


def _pool(rng, n, nbytes):
    raw = rng.integers(0, 256, size=(n, nbytes), dtype=np.uint8)
    return [b58encode(bytes(r)) for r in raw]


def nym_request(identifier, req_id, dest, verkey, alias=None, protocol_version=1):
    op = {"type": "1", "dest": dest, "verkey": verkey}
    if alias is not None:
        op["alias"] = alias
    return {"identifier": identifier, "reqId": req_id, "operation": op, "protocolVersion": protocol_version}


def nym_messages(n, signer_pks, alias_len=0, seed=1, req_id_base=REQ_ID_BASE, pool=4096):
    """n NYM requests from len(signer_pks) signers (request i signed by signer
    i % n_signers).  Returns (messages: list[bytes], key_idx: uint32[n],
    spec) where spec lets tests rebuild request i as a dict."""
    rng = np.random.default_rng(seed)
    n_signers = len(signer_pks)
    idrs = [b58encode(bytes(pk[:16])) for pk in signer_pks]
    dests = _pool(rng, pool, 16)
    vks = ["~" + v for v in _pool(rng, pool, 16)]
    alias = None
    if alias_len:
        alias = "".join(rng.choice(list("abcdefghijklmnopqrstuvwxyz0123456789"), size=alias_len))
    key_idx = (np.arange(n) % n_signers).astype(np.uint32)
    op_prefix = "operation:alias:%s|" % alias if alias is not None else "operation:"
    msgs = []
    for i in range(n):
        s = i % n_signers
        msgs.append(("identifier:%s|%sdest:%s|type:1|verkey:%s|protocolVersion:1|reqId:%d" % (
            idrs[s], op_prefix, dests[i % pool], vks[(i * 7) % pool], req_id_base + i)).encode())
    spec = dict(idrs=idrs, dests=dests, vks=vks, alias=alias, pool=pool, req_id_base=req_id_base)
    return msgs, key_idx, spec


def zipf_signers(n, n_signers, s=1.1, seed=17):
    """The signer of each of n requests under a Zipf(s) popularity law over
    n_signers (the signer of rank r drawn with weight r^-s; ranks assigned
    to signers in a random order): a domain ledger's long tail of NYM
    owners, a few of them very active."""
    rng = np.random.default_rng(seed)
    w = np.arange(1, n_signers + 1, dtype=np.float64) ** -s
    ranks = rng.choice(n_signers, size=n, p=w / w.sum())
    return rng.permutation(n_signers).astype(np.uint32)[ranks]


def churn_messages(key_idx, idrs, alias_len=43, seed=1, req_id_base=REQ_ID_BASE, pool=4096):
    """NYM requests signed by signers key_idx[i] (identifiers idrs[k]): the
    signing bytes of each (nym_messages' format) and a spec for its dict
    (churn_request_dict)."""
    rng = np.random.default_rng(seed)
    dests = _pool(rng, pool, 16)
    vks = ["~" + v for v in _pool(rng, pool, 16)]
    alias = "".join(rng.choice(list("abcdefghijklmnopqrstuvwxyz0123456789"), size=alias_len)) if alias_len else None
    op_prefix = "operation:alias:%s|" % alias if alias is not None else "operation:"
    msgs = [("identifier:%s|%sdest:%s|type:1|verkey:%s|protocolVersion:1|reqId:%d" % (
        idrs[k], op_prefix, dests[i % pool], vks[(i * 7) % pool], req_id_base + i)).encode()
        for i, k in enumerate(key_idx.tolist())]
    spec = dict(idrs=idrs, key_idx=key_idx, dests=dests, vks=vks, alias=alias, pool=pool, req_id_base=req_id_base)
    return msgs, spec


def churn_request_dict(spec, i):
    return nym_request(spec["idrs"][int(spec["key_idx"][i])], spec["req_id_base"] + i,
                       spec["dests"][i % spec["pool"]], spec["vks"][(i * 7) % spec["pool"]], spec["alias"])


def nym_request_dict(spec, i, n_signers):
    return nym_request(spec["idrs"][i % n_signers], spec["req_id_base"] + i, spec["dests"][i % spec["pool"]],
                       spec["vks"][(i * 7) % spec["pool"]], spec["alias"])


def check_nym_message(spec, i, n_signers, msg):
    return serialize_msg_for_signing(nym_request_dict(spec, i, n_signers), topLevelKeysToIgnore=["signature"]) == msg


# --- exact-integer helper for the configs[2] "R + T8" corruption ----------
_P = 2**255 - 19
_D = (-121665 * pow(121666, _P - 2, _P)) % _P
_SQRTM1 = pow(2, (_P - 1) // 4, _P)
# an order-8 point (x, y); its y is libsodium's blacklist entry 26e8958f...
_T8_ENC = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")


def _decode(enc):
    v = int.from_bytes(enc, "little")
    y = v & ((1 << 255) - 1)
    sign = v >> 255
    if y >= _P:
        return None
    x2 = (y * y - 1) * pow(_D * y * y + 1, _P - 2, _P) % _P
    x = pow(x2, (_P + 3) // 8, _P)
    if (x * x - x2) % _P:
        x = x * _SQRTM1 % _P
    if (x * x - x2) % _P:
        return None
    if x & 1 != sign:
        x = (_P - x) % _P
    return x, y


def _add(a, b):
    (x1, y1), (x2, y2) = a, b
    t = _D * x1 * x2 * y1 * y2 % _P
    return ((x1 * y2 + x2 * y1) * pow(1 + t, _P - 2, _P) % _P,
            (y1 * y2 + x1 * x2) * pow(1 - t, _P - 2, _P) % _P)


def add_torsion(r_enc):
    """encode(R + T8): a signature R that only the cofactored equation accepts."""
    R = _decode(r_enc)
    if R is None:
        return r_enc
    x, y = _add(R, _decode(_T8_ENC))
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def corrupt_configs2(sig, pk, msgs, off, rng):
    """configs[2] in place on host arrays: 10% rejects, split equally over bit
    flips in R/S/M, S+L, S|2^255, small-order A, non-canonical A, R =
    identity, R + T8.  Returns the expected verdicts."""
    n = sig.shape[0]
    bad = rng.choice(n, size=n // 10, replace=False)
    kinds = bad % 9
    L = 2**252 + 27742317777372353535851937790883648493
    small_A = bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05")
    noncanon_A = (2**255 - 19 + 3).to_bytes(32, "little")
    ident = (1).to_bytes(32, "little")
    for i, k in zip(bad, kinds):
        if k == 0:
            sig[i, rng.integers(0, 32)] ^= 1 << int(rng.integers(0, 8))
        elif k == 1:
            sig[i, 32 + rng.integers(0, 31)] ^= 1 << int(rng.integers(0, 8))
        elif k == 2:
            a, b = int(off[i]), int(off[i + 1])
            msgs[a + int(rng.integers(0, b - a))] ^= 1 << int(rng.integers(0, 8))
        elif k == 3:
            s = int.from_bytes(sig[i, 32:].tobytes(), "little") + L
            sig[i, 32:] = np.frombuffer(s.to_bytes(32, "little"), np.uint8)
        elif k == 4:
            sig[i, 63] |= 0x80
        elif k == 5:
            pk[i] = np.frombuffer(small_A, np.uint8)
        elif k == 6:
            pk[i] = np.frombuffer(noncanon_A, np.uint8)
        elif k == 7:
            sig[i, :32] = np.frombuffer(ident, np.uint8)
        else:
            sig[i, :32] = np.frombuffer(add_torsion(sig[i, :32].tobytes()), np.uint8)
    expect = np.ones(n, dtype=bool)
    expect[bad] = False
    return expect


# ---- configs[4] votes -------------------------------------------------------
def _mix64(x):
    """splitmix64 finalizer over uint64 arrays (a deterministic per-vote hash,
    the same on every rank)."""
    x = np.asarray(x, np.uint64)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


C4_CLASSES = ("random", "random", "random", "random", "prepare_below", "prepare_at", "commit_below", "commit_at")


def c4_votes(g, n_validators, view_len=1000):
    """configs[4] vote g (global index over all ranks): key g // (2V), phase
    (g % 2V) // V (0 PREPARE, 1 COMMIT), voter g % V; the primary of the key's
    view (view = key // view_len, primary = view % V) -- its PREPARE never
    counts (replica.py:1289-1291).  Which votes are present is decided per key
    class (hash of the key, C4_CLASSES) so the tally has decisions to make at
    full size (n = 25: prepare quorum 16, commit quorum 17, quorums.py:15-32):
      random         each vote present with p = 0.95;
      prepare_below  15 non-primary PREPAREs + the primary's (16 if the
                     primary were counted: the rule decides the quorum);
      prepare_at     16 non-primary PREPAREs + the primary's;
      commit_below   16 COMMITs;  commit_at  17 COMMITs;
    (the other phase of those keys random).  Returns (key, phase, voter,
    present, primary_of_key_fn) as arrays over g."""
    V = n_validators
    g = np.asarray(g, np.int64)
    key = g // (2 * V)
    phase = (g % (2 * V)) // V
    voter = g % V
    prim = (key // view_len) % V
    cls = (_mix64(key.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)) % np.uint64(8)).astype(np.int64)
    u = (_mix64(g.astype(np.uint64) + np.uint64(0x51ED2701)) >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    present = u >= 0.05
    o_prep = (voter - prim - 1) % V                      # 0..V-2 for the other voters, V-1 for the primary
    o_com = (voter - (key * 7) % V) % V                  # a window of committers per key
    is_p, is_c = phase == 0, phase == 1
    for c, name in enumerate(C4_CLASSES):
        sel = cls == c
        if name == "prepare_below":
            present = np.where(sel & is_p, (o_prep < 15) | (voter == prim), present)
        elif name == "prepare_at":
            present = np.where(sel & is_p, (o_prep < 16) | (voter == prim), present)
        elif name == "commit_below":
            present = np.where(sel & is_c, o_com < 16, present)
        elif name == "commit_at":
            present = np.where(sel & is_c, o_com < 17, present)
    return key, phase, voter, present, cls


def c4_primary(n_keys, n_validators, view_len=1000):
    return ((np.arange(n_keys) // view_len) % n_validators).astype(np.uint8)
