"""A/B of the end-to-end authenticate_batch paths in one process (configs[1]-shaped
1M-request batches, each request json-decoded on its own, modes alternating):
  stream  the default (scan with the pack deferred, 2^17-request submits)
  stage   stage=True (the scan's workers queue each 4k chunk's DMA while scanning)
  MODE:VAR=VAL   that mode with the environment variable set around each of its calls
                 (e.g. stage:EDV_SCAN_SHAPES=0)
usage: python tools/e2e_ab.py [n] [reps] [mode,mode,...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
import bench  # noqa: E402
from plenum_amd import EdVerifyEngine  # noqa: E402
from plenum_amd.client_authn import GpuAuthNr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
modes = (sys.argv[3] if len(sys.argv) > 3 else "stream,stage").replace("+", ",").split(",")
eng = EdVerifyEngine(0)
reqs, idrs, vks = bench.e2e_requests(eng, n, 1000, 43)
auths = {}
def env_of(m):
    return dict(kv.split("=", 1) for kv in m.split(":")[1:])


def with_env(m, f):
    saved = {k: os.environ.get(k) for k in env_of(m)}
    os.environ.update(env_of(m))
    try:
        return f()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


for m in modes:
    a = GpuAuthNr(engine=eng, stage=(m.split(":")[0] == "stage"))
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()
    a.authenticate_batch(reqs[:2048])
    a.authenticate_batch(reqs)
    auths[m] = a
for rep in range(reps):
    for m in modes:
        a = auths[m]
        a._g.last_breakdown = None
        t0 = time.perf_counter()
        res = with_env(m, lambda: a.authenticate_batch(reqs))
        el = time.perf_counter() - t0
        ok = sum(1 for r, q in zip(res, reqs) if r == q["identifier"])
        del res
        print("%-24s %.2f ms = %.2f M requests/s  accepted %d  %s" % (
            m, el * 1e3, n / el / 1e6, ok, {k: round(v, 2) for k, v in (a._g.last_breakdown or {}).items()}),
            flush=True)
