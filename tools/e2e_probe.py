"""Where the drop-in's end-to-end time goes on the GPU box: GpuAuthNr.authenticate_batch
over configs[1]-shaped request dicts (1M NYMs, 1,000 signers), timed whole for each
pipeline part size (0 = one scan then one GPU call), then under cProfile, with the native
scan's phase times (EDV_SCAN_PROFILE=1).
usage: EDV_SCAN_PROFILE=1 python tools/e2e_probe.py [n] [part,part,...]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
import bench  # noqa: E402
from plenum_amd import EdVerifyEngine  # noqa: E402
from plenum_amd.client_authn import GpuAuthNr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
parts = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1 << 17, 1 << 18]
eng = EdVerifyEngine(0)
t0 = time.perf_counter()
reqs, idrs, vks = bench.e2e_requests(eng, n, 1000, 43)
if os.environ.get("WIRE"):  # every request json-decoded on its own, as the node receives it (own str objects)
    import json
    reqs = [json.loads(json.dumps(r)) for r in reqs]
print("built %d requests in %.1f s (wire=%s)" % (n, time.perf_counter() - t0, bool(os.environ.get("WIRE"))),
      flush=True)
a = GpuAuthNr(engine=eng)
for idr, vk in zip(idrs, vks):
    a.addIdr(idr, vk)
a.keys_settle()
a.authenticate_batch(reqs[:2048])
a.authenticate_batch(reqs)  # buffers grown
runs = [(p, True, True) for p in parts] + ([(0, True, False), (0, False, False)] if 0 in parts else [])
for part, stream, stage in runs:
    a._g.pipeline_part = part
    a._g.stream = stream
    a._g.stage = stage
    for rep in range(3):
        t0 = time.perf_counter()
        res = a.authenticate_batch(reqs)
        el = time.perf_counter() - t0
        print("authenticate_batch part=%d stream=%d stage=%d: %.3f s = %.2f M requests/s, ok %d" % (
            part, stream, stage, el, n / el / 1e6, sum(1 for r in res[:1000] if isinstance(r, str))), flush=True)
        del res
a._g.pipeline_part = parts[-1]
a._g.stream = True
a._g.stage = True
cProfile.run("a.authenticate_batch(reqs)", "/tmp/e2e.prof")
pstats.Stats("/tmp/e2e.prof").sort_stats("tottime").print_stats(15)
eng.close()

# one request not in the verdict cache: authenticate() vs the engine call alone
import numpy as np  # noqa: E402
eng = EdVerifyEngine(0)
a = GpuAuthNr(engine=eng)
for idr, vk in zip(idrs, vks):
    a.addIdr(idr, vk)
a.keys_settle()
a.authenticate_batch(reqs[:4096])
lat, lat_eng, lat_prep = [], [], []
for r in reqs[:330]:
    a.clear_verdicts()
    t0 = time.perf_counter()
    a.authenticate(r)
    lat.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    p = a._prepare(r)
    lat_prep.append(time.perf_counter() - t0)
    ks = a._key_store()
    kid = np.asarray(ks.lookup([p.key]), np.uint32)
    from plenum_amd.client_authn import _pack_split64
    s64, m, off, short = _pack_split64([p.sig], [p.ser])
    t0 = time.perf_counter()
    eng.verify_batch_keyed(np.frombuffer(s64, np.uint8).reshape(-1, 64), kid, np.frombuffer(m, np.uint8),
                           np.frombuffer(off, np.uint64))
    lat_eng.append(time.perf_counter() - t0)
for name, v in (("authenticate", lat), ("_prepare", lat_prep), ("engine call n=1", lat_eng)):
    v = np.array(v[30:]) * 1e6
    print("single %-16s p50 %.1f us  p99 %.1f us" % (name, np.percentile(v, 50), np.percentile(v, 99)))
print("phases of the last n=1 call (ms):", eng.last_phases_ms(), eng.last_host_stats())
# where a single authenticate()'s time goes (Python frames vs the library call)
def _singles():
    for r in reqs[:300]:
        a.clear_verdicts()
        a.authenticate(r)
cProfile.run("_singles()", "/tmp/single.prof")
pstats.Stats("/tmp/single.prof").sort_stats("tottime").print_stats(12)
