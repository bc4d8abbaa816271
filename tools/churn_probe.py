"""Key-churn probe on the GPU box: bench.time_key_churn's workload (100k signers, Zipf(1.1),
250k-request batches) with the native scan's phase split on stderr (EDV_SCAN_PROFILE=1) and a
cProfile of one steady-state batch's Python side.  usage: python tools/churn_probe.py [batches]"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

os.environ.setdefault("EDV_SCAN_PROFILE", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from plenum_amd import EdVerifyEngine, _hostpack, pack_messages, synth  # noqa: E402
from plenum_amd.base58 import b58encode  # noqa: E402
from plenum_amd.client_authn import GpuAuthNr  # noqa: E402

batches = int(sys.argv[1]) if len(sys.argv) > 1 else 6
signers, per = 100_000, 250_000
eng = EdVerifyEngine(0)
pks, sks = eng.seed_keypair_batch(synth.signer_seeds((1 << 20) + signers)[1 << 20:])
idrs = [b58encode(bytes(pk[:16])) for pk in pks]
vks = ["~" + b58encode(bytes(pk[16:])) for pk in pks]
n = per * batches
kidx = synth.zipf_signers(n, signers, 1.1)
msgs, spec = synth.churn_messages(kidx, idrs, alias_len=43, req_id_base=synth.REQ_ID_BASE + (1 << 40))
buf, off = pack_messages(msgs)
del msgs
sig = eng.sign_batch(sks, kidx, buf, off)
sig_b58 = _hostpack.b58encode_rows(np.ascontiguousarray(sig).tobytes(), 64)
reqs = []
for i in range(n):
    r = synth.churn_request_dict(spec, i)
    r["signature"] = sig_b58[i]
    reqs.append(json.loads(json.dumps(r)))
a = GpuAuthNr(engine=eng)
for idr, vk in zip(idrs, vks):
    a.addIdr(idr, vk)
a.keys_settle()
chunks = [reqs[b * per:(b + 1) * per] for b in range(batches)]
for b in range(batches):
    prof = b == batches - 1
    pr = cProfile.Profile() if prof else None
    sys.stderr.write("batch %d\n" % b)
    t0 = time.perf_counter()
    if pr:
        pr.enable()
    a.authenticate_batch(chunks[b])
    if pr:
        pr.disable()
    el = time.perf_counter() - t0
    print(json.dumps({"batch": b, "ms": round(el * 1e3, 2), "profiled": prof,
                      "in_batch_ms": a._g.last_breakdown}, default=str), flush=True)
    if pr:
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(s.getvalue(), flush=True)
