"""A/B of the streamed path's chunk size (client_authn._STREAM_CHUNK) in one process:
configs[1]-shaped 1M-request batches, each json-decoded on its own, chunk sizes alternating.
usage: python tools/stream_ab.py [n] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
import bench  # noqa: E402
from plenum_amd import EdVerifyEngine  # noqa: E402
from plenum_amd import client_authn as CA  # noqa: E402
from plenum_amd.client_authn import GpuAuthNr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
eng = EdVerifyEngine(0)
reqs, idrs, vks = bench.e2e_requests(eng, n, 1000, 43)
a = GpuAuthNr(engine=eng)
for idr, vk in zip(idrs, vks):
    a.addIdr(idr, vk)
a.keys_settle()
a.authenticate_batch(reqs[:2048])
a.authenticate_batch(reqs)
sizes = [1 << 18, 1 << 17, 1 << 16]
for rep in range(reps):
    for c in sizes:
        CA._STREAM_CHUNK = c
        t0 = time.perf_counter()
        a.authenticate_batch(reqs)
        el = time.perf_counter() - t0
        print("chunk 2^%d: %.2f ms = %.2f M requests/s  %s" % (
            c.bit_length() - 1, el * 1e3, n / el / 1e6,
            {k: round(v, 2) for k, v in (a._g.last_breakdown or {}).items()}), flush=True)
