"""Probe: the speculative staged path on the device, printing each batch's path and any
staging error (tests/test_gpu_authn.py::test_large_batch_staged_and_streamed_on_gpu's flow)."""
import copy
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
import conftest  # noqa
from test_gpu_authn import _drain  # noqa
from plenum_amd import EdVerifyEngine, client_authn as CA  # noqa
from plenum_amd.client_authn import GpuAuthNr  # noqa

eng = EdVerifyEngine(0)
for cls_name in ("stage_reserve", "stage_select", "verify_staged_begin", "verify_staged_end", "verify_staged_collect"):
    f = getattr(eng, cls_name)

    def wrap(*a, _f=f, _n=cls_name):
        try:
            r = _f(*a)
            print("  ", _n, "ok", flush=True)
            return r
        except Exception as ex:
            print("  ", _n, "RAISED", repr(ex), flush=True)
            raise
    setattr(eng, cls_name, wrap)
if "--after-staged-test" in sys.argv:
    import test_gpu_authn
    test_gpu_authn.test_staged_batch_on_gpu(eng)
    print("test_staged_batch_on_gpu done", flush=True)
n = 300_000
reqs, rx, idrs, vks, pks, sers, sig = _drain(eng, n_req=n, n_nodes=1, n_signers=32)
batch = [copy.deepcopy(r) for r in reqs]
del batch[1234]["signature"]
batch[4321]["identifier"] = "UnknownIdentifier11111111"
a = GpuAuthNr(engine=eng, stage=True)
for idr, vk in zip(idrs, vks):
    a.addIdr(idr, vk)
a.keys_settle()
clean = [copy.deepcopy(r) for i, r in enumerate(batch) if i not in (1234, 4321)]
for name, b in (("clean", clean), ("batch", batch), ("clean", clean), ("clean", clean)):
    a._g.last_breakdown = None
    res = a.authenticate_batch(b)
    print(name, a._g.last_breakdown, flush=True)
