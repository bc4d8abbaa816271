"""Host-side cost of GpuAuthNr.authenticate_batch on synthetic NYM requests (a fake
engine answers True, so only the Python/native host work is timed).
usage: python tools/prof_host.py"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "indy-plenum_amd"))
import numpy as np
from plenum_amd import synth
from plenum_amd.client_authn import GpuAuthNr
from plenum_amd.base58 import b58encode
import cProfile, pstats

class FakeEngine:
    def keys_reset(self): pass
    def keys_set_window(self, w): pass
    def keys_add(self, pk): return 0
    def verify_batch_keyed(self, sig, ids, msgs, off): return np.ones(len(ids), bool)
    def sign_open_batch(self, sm, off, pk): return np.ones(len(off) - 1, bool)

n = int(os.environ.get("PROF_N", "20000"))
rng = np.random.default_rng(0)
pks = [bytes(rng.integers(0,256,32,dtype=np.uint8)) for _ in range(100)]
msgs_b, kidx, spec = synth.nym_messages(n, pks, alias_len=43)
reqs = [synth.nym_request_dict(spec, i, 100) for i in range(n)]
for r in reqs:
    r["signature"] = b58encode(bytes(rng.integers(0,256,64,dtype=np.uint8)))
a = GpuAuthNr(engine=FakeEngine())
for i, pk in enumerate(pks):
    a.addIdr(spec["idrs"][i], b58encode(pk))
t0 = time.perf_counter(); res = a.authenticate_batch(reqs); t1 = time.perf_counter()
print("authenticate_batch: %.1f us/request" % ((t1 - t0) / n * 1e6), res[:1])
cProfile.run("a.authenticate_batch(reqs)", "/tmp/prof.out")
pstats.Stats("/tmp/prof.out").sort_stats("tottime").print_stats(12)
