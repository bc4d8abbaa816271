"""A/B timing of library variants on the keyed configs[1] workload.
usage: python tools/ab_keyed.py lib1.so[:W] lib2.so[:W] ...  (each run in a child process;
W = key window, default 8; also times the general path once per library)"""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, time
import numpy as np, torch
sys.path.insert(0, os.path.join(%r, "indy-plenum_amd"))
from plenum_amd import EdVerifyEngine, pack_messages, synth
n = 1_000_000
dev = torch.device("cuda", 0); torch.cuda.set_device(0)
torch.zeros(1, device=dev); torch.cuda.synchronize()
t0 = time.perf_counter(); eng = EdVerifyEngine(0); create_ms = (time.perf_counter() - t0) * 1e3
pks, sks = eng.seed_keypair_batch(synth.signer_seeds(1000))
msgs, kidx, _ = synth.nym_messages(n, pks, alias_len=43)
buf, off = pack_messages(msgs)
d_msgs = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
d_off = torch.from_numpy(off.view(np.int64)).to(dev)
d_k = torch.from_numpy(kidx.astype(np.int32)).to(dev)
d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
eng.sign_batch_device(torch.from_numpy(sks).to(dev), d_k, d_msgs, d_off, n, d_sig)
eng.keys_set_window(int(os.environ.get("AB_KEY_WINDOW", "8")))
if hasattr(eng._lib, "edv_set_pipeline"):
    eng.set_pipeline(int(os.environ.get("AB_PIPELINE", "1")))
t0 = time.perf_counter(); eng.keys_add(pks); kb = (time.perf_counter() - t0) * 1e3
words = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
def med(res):
    a = np.median(np.array(res[2:]), axis=0)
    return dict(zip(("hash", "table", "core", "encode"), [round(float(x), 4) for x in a]))
def wall(fn, reps=10):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / reps * 1e3, 4)
res = []
for it in range(10):
    eng.verify_batch_keyed_device(d_sig, d_k, d_msgs, d_off, n, words)
    res.append(eng.last_phases_ms())
wall_keyed = wall(lambda: eng.verify_batch_keyed_device(d_sig, d_k, d_msgs, d_off, n, words))
bits = np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n]
t0 = time.perf_counter(); eng.keys_reset(); eng.keys_add(pks); kb2 = (time.perf_counter() - t0) * 1e3
out = {"keyed_wall_ms": wall_keyed, "keyed": med(res), "keyed_ok": int(bits.sum()) == n, "key_build_ms": [round(kb, 2), round(kb2, 2)],
       "create_ms": round(create_ms, 1)}
if os.environ.get("AB_GENERAL", "1") == "1":
    d_pk = torch.from_numpy(pks).to(dev)[d_k.long()].contiguous()
    words.zero_()
    res = []
    for it in range(5):
        eng.verify_batch_device(d_sig, d_pk, d_msgs, d_off, n, words)
        res.append(eng.last_phases_ms())
    bits = np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n]
    out.update({"general_wall_ms": wall(lambda: eng.verify_batch_device(d_sig, d_pk, d_msgs, d_off, n, words), 3),
                "general": med(res), "general_ok": int(bits.sum()) == n})
print(json.dumps(out))
''' % ROOT
for spec in sys.argv[1:]:
    lib, _, w = spec.partition(":")
    env = dict(os.environ, PLENUM_EDVERIFY_LIB=os.path.abspath(lib), AB_KEY_WINDOW=w or "8", PLENUM_EDVERIFY_LENIENT="1")
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    print(os.path.basename(lib), "W=%s" % (w or "8"), line[-1] if line else out.stderr[-2000:], flush=True)
