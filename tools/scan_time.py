"""Host-only timing of authenticate_batch's native scan (no GPU): configs[1]-shaped
request dicts, each json-decoded on its own, random signatures (the scan does not
verify).  usage: python tools/scan_time.py [n] [threads,...] [slot] [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
from plenum_amd import _hostpack, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
threads = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,8").split(",")]
slot = int(sys.argv[3]) if len(sys.argv) > 3 else 64
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
rng = np.random.default_rng(5)
pks = rng.integers(0, 256, (1000, 32), dtype=np.uint8)
_, _, spec = synth.nym_messages(min(n, 4096), pks, alias_len=43, seed=1)
sig = _hostpack.b58encode_rows(rng.integers(0, 256, (n, 64), dtype=np.uint8).tobytes(), 64)
reqs = []
for i in range(n):
    r = synth.nym_request_dict(spec, i % 4096, 1000)
    r["reqId"] = 1_700_000_000_000_000 + i
    r["signature"] = sig[i]
    reqs.append(json.loads(json.dumps(r)))
out = [bytearray(), bytearray()]
for t in threads:
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        s = _hostpack.scan_batch_u(reqs, ["signature"], t, out, slot)
        best = min(best, time.perf_counter() - t0)
        del s
    print("threads %2d slot %d: %.2f ms / %d = %.0f ns per request (x threads: %.0f ns)" % (
        t, slot, best * 1e3, n, best / n * 1e9, best / n * 1e9 * t), flush=True)
