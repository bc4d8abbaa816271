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
print("built %d requests in %.1f s" % (n, time.perf_counter() - t0), flush=True)
a = GpuAuthNr(engine=eng)
for idr, vk in zip(idrs, vks):
    a.addIdr(idr, vk)
a.authenticate_batch(reqs[:2048])
a.authenticate_batch(reqs)  # buffers grown
for part in parts:
    a._g.pipeline_part = part
    for rep in range(3):
        t0 = time.perf_counter()
        res = a.authenticate_batch(reqs)
        el = time.perf_counter() - t0
        print("authenticate_batch part=%d: %.3f s = %.2f M requests/s, ok %d" % (
            part, el, n / el / 1e6, sum(1 for r in res[:1000] if isinstance(r, str))), flush=True)
        del res
a._g.pipeline_part = parts[-1]
cProfile.run("a.authenticate_batch(reqs)", "/tmp/e2e.prof")
pstats.Stats("/tmp/e2e.prof").sort_stats("tottime").print_stats(15)
eng.close()
