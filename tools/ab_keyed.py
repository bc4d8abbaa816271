"""A/B timing of library variants on the keyed configs[1] workload.
usage: python tools/ab_keyed.py lib1.so lib2.so ...  (each run in a child process)"""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, time
import numpy as np, torch
sys.path.insert(0, os.path.join(%r, "indy-plenum_amd"))
from plenum_amd import EdVerifyEngine, pack_messages, synth
n = 1_000_000
dev = torch.device("cuda", 0); torch.cuda.set_device(0)
eng = EdVerifyEngine(0)
pks, sks = eng.seed_keypair_batch(synth.signer_seeds(1000))
msgs, kidx, _ = synth.nym_messages(n, pks, alias_len=43)
buf, off = pack_messages(msgs)
d_msgs = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
d_off = torch.from_numpy(off.view(np.int64)).to(dev)
d_k = torch.from_numpy(kidx.astype(np.int32)).to(dev)
d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
eng.sign_batch_device(torch.from_numpy(sks).to(dev), d_k, d_msgs, d_off, n, d_sig)
eng.keys_add(pks)
words = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
res = []
for it in range(12):
    eng.verify_batch_keyed_device(d_sig, d_k, d_msgs, d_off, n, words)
    res.append(eng.last_phase_ms())
bits = np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n]
print(json.dumps({"comb_ms": sorted(r[2] for r in res[2:])[len(res[2:])//2], "hash_ms": sorted(r[0] for r in res[2:])[len(res[2:])//2], "all_ok": int(bits.sum()) == n}))
''' % ROOT
for lib in sys.argv[1:]:
    env = dict(os.environ, PLENUM_EDVERIFY_LIB=os.path.abspath(lib))
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    print(os.path.basename(lib), line[-1] if line else out.stderr[-2000:], flush=True)
