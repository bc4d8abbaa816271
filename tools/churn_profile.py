"""CPU profile of authenticate_batch under key churn (many distinct signers, few key slots) over
the tests' engine double: where the node thread's per-identifier work goes (keys_and_ids).
usage: python tools/churn_profile.py [signers] [requests] [max_keys]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
from conftest import sodium  # noqa: E402
from engine_double import StagingOracleEngine  # noqa: E402
from plenum_amd import synth  # noqa: E402
from plenum_amd.base58 import b58encode  # noqa: E402
from plenum_amd.client_authn import GpuAuthNr  # noqa: E402
from plenum_amd.serialization import serialize_msg_for_signing  # noqa: E402

signers = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60000
max_keys = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
s = sodium()
keys = []
for i in range(signers):
    pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
    s.crypto_sign_seed_keypair(pk, sk, i.to_bytes(4, "little") + b"\x07" * 28)
    keys.append((b58encode(pk.raw[:16]), "~" + b58encode(pk.raw[16:]), sk))
kidx = synth.zipf_signers(n, signers, 1.1)
reqs = []
for j in range(n):
    idr, _, sk = keys[int(kidx[j])]
    m = {"identifier": idr, "reqId": 1000 + j, "operation": {"type": "1", "dest": "d%d" % j}}
    ser = serialize_msg_for_signing(m, topLevelKeysToIgnore=["signature"])
    sig = ctypes.create_string_buffer(64)
    s.crypto_sign_detached(sig, None, ser, ctypes.c_ulonglong(len(ser)), sk)
    reqs.append(json.loads(json.dumps(dict(m, signature=b58encode(sig.raw)))))
from plenum_amd import client_authn as CA  # noqa: E402
from plenum_amd import keystore as KS  # noqa: E402
CA._STAGE_MIN_BATCH = CA._PINNED_MIN_BATCH = 1000
spent = {}


def timed(owner, name):
    f = getattr(owner, name)

    def w(*args, **kw):
        t = time.perf_counter()
        try:
            return f(*args, **kw)
        finally:
            spent[name] = spent.get(name, 0.0) + time.perf_counter() - t
    setattr(owner, name, w)


for owner, name in ((GpuAuthNr, "_keys_for"), (GpuAuthNr, "_keys_for_py"), (GpuAuthNr, "_resolve_key"),
                    (GpuAuthNr, "_register_waiting"), (KS.KeyStore, "lookup"),
                    (KS.KeyStore, "register"), (GpuAuthNr, "_count_verified_keys"), (GpuAuthNr, "_staged_mixed")):
    timed(owner, name)
a = GpuAuthNr(engine=StagingOracleEngine(), max_keys=max_keys)
for idr, vk, _ in keys:
    a.addIdr(idr, vk)
a.keys_settle()
per = int(os.environ.get("CHURN_BATCH", n))
for b in range(0, n, per):
    spent.clear()
    t0 = time.perf_counter()
    res = a.authenticate_batch(reqs[b:b + per])
    print("batch %d: %.1f ms" % (b // per, (time.perf_counter() - t0) * 1e3),
          {k: round(v * 1e3, 2) for k, v in spent.items()}, "fast_keys", len(a._g.fast_keys),
          {k: round(v, 2) if isinstance(v, float) else v for k, v in (a._g.last_breakdown or {}).items()})
reqs = reqs[n - per:]
res = a.authenticate_batch(reqs)
print("batch %.1f ms, %d distinct signers, breakdown %s" % ((time.perf_counter() - t0) * 1e3,
      len(np.unique(kidx)), {k: round(v, 2) if isinstance(v, float) else v
                             for k, v in (a._g.last_breakdown or {}).items()}))
assert res == [m["identifier"] for m in reqs]
if os.environ.get("CHURN_MICRO"):
    uniq = list(dict.fromkeys(m["identifier"] for m in reqs))
    for rep in range(3):
        t = time.perf_counter()
        ks_ = a._keys_for(uniq)
        t1 = time.perf_counter()
        [a.getVerkey(i) for i in uniq]
        t2 = time.perf_counter()
        fk = a._g.fast_keys
        [fk.get(i) for i in uniq]
        t3 = time.perf_counter()
        print("keys_for %.2f ms, getVerkey alone %.2f ms, fast_keys.get alone %.2f ms, %d identifiers, %d in fast_keys"
              % ((t1 - t) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, len(uniq), sum(1 for i in uniq if i in fk)))
