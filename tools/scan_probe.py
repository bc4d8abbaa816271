"""Host-only A/B of the native scan's switches on configs[1]-shaped requests (each json-decoded on
its own, as bench.py's end_to_end leg builds them), alternating in one process so the host's load
affects every variant alike.  usage: python tools/scan_probe.py [n] [threads,...] [reps] [VAR=a/b ...]
e.g. python tools/scan_probe.py 1000000 1,16 5 EDV_SCAN_SHAPES=1/0 EDV_SCAN_PREFETCH=1/0"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
from plenum_amd import _hostpack, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
threads = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,16").split(",")]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
switches = [a.split("=") for a in sys.argv[4:]]  # VAR=v1/v2/...
variants = [{}]
for var, vals in switches:
    variants = [dict(v, **{var: x}) for v in variants for x in vals.split("/")]
rng = np.random.default_rng(3)
pks = rng.integers(0, 256, (1000, 32), dtype=np.uint8)
msgs, kidx, spec = synth.nym_messages(min(n, 1 << 16), pks, alias_len=43, seed=1)
sig = _hostpack.b58encode_rows(rng.integers(0, 256, (n, 64), dtype=np.uint8).tobytes(), 64)
reqs = []
for i in range(n):
    r = synth.nym_request_dict(spec, i % len(msgs), 1000)
    r["reqId"] = synth.REQ_ID_BASE + i
    r["signature"] = sig[i]
    reqs.append(json.loads(json.dumps(r)))
out = [bytearray(), bytearray()]
_hostpack.scan_batch_u(reqs, ["signature"], 0, out, 96)  # buffers grown once
for t in threads:
    times = {i: [] for i in range(len(variants))}
    for _ in range(reps):
        for i, v in enumerate(variants):
            os.environ.update(v)
            t0 = time.perf_counter()
            s = _hostpack.scan_batch_u(reqs, ["signature"], t, out, 96)
            times[i].append(time.perf_counter() - t0)
            del s
    for i, v in enumerate(variants):
        m = float(np.median(times[i]))
        print("threads %2d %-44s median %.2f ms (min %.2f) = %.0f ns per request x threads" % (
            t, " ".join("%s=%s" % kv for kv in v.items()) or "default", m * 1e3, min(times[i]) * 1e3,
            m / n * 1e9 * t), flush=True)
