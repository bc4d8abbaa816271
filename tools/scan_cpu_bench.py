"""CPU-only timing of the native scan (_hostpack.scan_batch_u) over configs[1]-shaped NYM
request dicts, each json round-tripped as the node receives it.  Signatures are random
64-byte strings (the scan does not verify).  For A/B of the scan's worker loop here.
usage: EDV_SCAN_PROFILE=1 python tools/scan_cpu_bench.py [n] [threads] [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from plenum_amd import _hostpack as H  # noqa: E402
if os.environ.get("HOSTPACK_SO"):  # an instrumented build of the same module
    import importlib.util
    _spec = importlib.util.spec_from_file_location("_hostpack", os.environ["HOSTPACK_SO"])
    H = importlib.util.module_from_spec(_spec)
    _spec.loader.exec_module(H)
from plenum_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
rng = np.random.default_rng(3)
pks = rng.integers(0, 256, (1000, 32), dtype=np.uint8)
msgs, kidx, spec = synth.nym_messages(n, pks, alias_len=43, seed=1)
sig_b58 = H.b58encode_rows(rng.integers(0, 256, (n, 64), dtype=np.uint8).tobytes(), 64)
reqs = []
for i in range(n):
    r = synth.nym_request_dict(spec, i, 1000)
    r["signature"] = sig_b58[i]
    reqs.append(json.loads(json.dumps(r)))
out = [bytearray(), bytearray()]
for rep in range(reps):
    ab = os.environ.get("AB")  # alternate a scan switch off / on (AB=1: EDV_SCAN_PREFETCH; else its name)
    if ab:
        os.environ["EDV_SCAN_PREFETCH" if ab == "1" else ab] = "1" if rep % 2 else "0"
    t0 = time.perf_counter()
    H.scan_batch_u(reqs, ["signature"], threads, out, 96)
    flags = "".join(" %s=%s" % (k[9:].lower(), os.environ.get(k, "1")) for k in ("EDV_SCAN_PREFETCH", "EDV_SCAN_DIRECT"))
    print("scan %d requests, %d threads%s: %.2f ms" % (n, threads, flags, (time.perf_counter() - t0) * 1e3), flush=True)
