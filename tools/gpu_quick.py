"""Quick GPU parity probe: golden vectors through the HIP library."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "indy-plenum_amd"))
from plenum_amd import EdVerifyEngine
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
eng = EdVerifyEngine(0)
print(eng.version)
for name in ("ed25519_valid.npz", "ed25519_edge.npz"):
    d = np.load(os.path.join(G, name))
    t0 = time.time()
    got = eng.verify_batch(d["sig"], d["pk"], d["msgs"], d["off"])
    exp = d["expect"].astype(bool)
    print(name, "n=%d" % len(exp), "match=%d" % (got == exp).sum(), "accepted=%d/%d" % (got.sum(), exp.sum()), "%.3fs" % (time.time() - t0))
    bad = np.nonzero(got != exp)[0]
    print("mismatch idx", bad[:20])
k = np.load(os.path.join(G, "sign_kat.npz"))
pk, sk = eng.seed_keypair_batch(k["seed"])
print("keypair match", (pk == k["pk"]).all(axis=1).sum(), "/", len(pk))
sig = eng.sign_batch(sk, np.arange(len(pk), dtype=np.uint32), k["msgs"], k["off"])
print("sign match", (sig == k["sig"]).all(axis=1).sum(), "/", len(sig))
# throughput probe: 64k copies of valid vectors
d = np.load(os.path.join(G, "ed25519_valid.npz"))
n = 1 << 16
idx = np.arange(n) % 300
msgs = [bytes(d["msgs"][int(d["off"][i]):int(d["off"][i + 1])]) for i in idx]
from plenum_amd import pack_messages
buf, off = pack_messages(msgs)
for rep in range(3):
    t0 = time.time()
    got = eng.verify_batch(d["sig"][idx], d["pk"][idx], buf, off)
    dt = time.time() - t0
    print("64k verify: %.1f ms wall, all ok=%s, phases(ms)=%s -> %.2f M verifies/s (kernels)" % (
        dt * 1e3, got.all(), ["%.2f" % x for x in eng.last_phase_ms()], n / sum(eng.last_phase_ms()) / 1e3))
