"""A/B timing of libplenum_edverify.so build variants on the keyed configs[1]
workload (1M NYM requests, 1,000 signers), alternating variants in child
processes on one box so every variant sees the same device and clock regime.

usage: python tools/ab_libs.py [--rounds R] [--window W] [--config c1|c2|distinct] [--path keyed|general] lib_a.so ...
(distinct: every request signed by its own key)
Per run: wall ms per 1M-request keyed step with 4 sub-batches (the bench
step), the comb phase alone with 1 sub-batch, correctness vs construction.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, time
import numpy as np, torch
sys.path.insert(0, os.path.join(%r, "indy-plenum_amd"))
from plenum_amd import EdVerifyEngine, pack_messages, synth
n = 1_000_000
W = int(os.environ["AB_W"]); cfg = os.environ["AB_CONFIG"]
dev = torch.device("cuda", 0); torch.cuda.set_device(0)
eng = EdVerifyEngine(0)
pks, sks = eng.seed_keypair_batch(synth.signer_seeds(n if cfg == "distinct" else 1000))
msgs, kidx, _ = synth.nym_messages(n, pks, alias_len=43)
buf, off = pack_messages(msgs)
d_msgs = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
d_off = torch.from_numpy(off.view(np.int64)).to(dev)
d_k = torch.from_numpy(kidx.astype(np.int32)).to(dev)
d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
eng.sign_batch_device(torch.from_numpy(sks).to(dev), d_k, d_msgs, d_off, n, d_sig)
torch.cuda.synchronize()
expect = np.ones(n, bool)
reg = pks
if cfg == "c2":
    sig, pk, b2 = d_sig.cpu().numpy(), pks[kidx].copy(), buf.copy()
    expect = synth.corrupt_configs2(sig, pk, b2, off, np.random.default_rng(2))
    reg, inv = np.unique(pk, axis=0, return_inverse=True)
    d_sig = torch.from_numpy(sig).to(dev)
    d_msgs = torch.from_numpy(np.concatenate([b2, np.zeros(16, np.uint8)])).to(dev)
    d_k = torch.from_numpy(inv.reshape(-1).astype(np.int32)).to(dev)
if os.environ.get("AB_PATH") != "general":
    eng.keys_set_window(W)
    eng.keys_add(reg)
words = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
if os.environ.get("AB_PATH") == "general":
    d_pk = torch.from_numpy(pks[kidx] if cfg != "c2" else pk).to(dev)
    step = lambda: eng.verify_batch_device(d_sig, d_pk, d_msgs, d_off, n, words)
    reps = 5
else:
    step = lambda: eng.verify_batch_keyed_device(d_sig, d_k, d_msgs, d_off, n, words)
    reps = 30
eng.set_pipeline(4)
for _ in range(3): step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps): step()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / reps * 1e3
ph4 = eng.last_phases_ms()
bits = np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
walls = {}
for p in (1, 2):
    eng.set_pipeline(p)
    step(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps): step()
    torch.cuda.synchronize()
    walls[p] = round((time.perf_counter() - t0) / reps * 1e3, 4)
eng.set_pipeline(1)
solo = []
for _ in range(5):
    step(); solo.append(eng.last_phases_ms())
solo = np.median(np.array(solo), axis=0)
print(json.dumps({"wall_ms": round(wall, 4), "rate_M": round(n / wall / 1e3, 1),
                  "wall_p1": walls[1], "wall_p2": walls[2], "phases4": [round(x, 3) for x in ph4], "solo": [round(float(x), 4) for x in solo],
                  "ok": bool((bits == expect).all())}))
''' % ROOT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--window", type=int, default=14)
    ap.add_argument("--config", default="c1")
    ap.add_argument("--path", default="keyed", choices=["keyed", "general"])
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, PLENUM_EDVERIFY_LIB=os.path.abspath(lib), PLENUM_EDVERIFY_LENIENT="1",
                       AB_W=str(a.window), AB_CONFIG=a.config, AB_PATH=a.path)
            out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in out.stdout.splitlines() if x.startswith("{")]
            print("round %d %s W=%d %s: %s" % (r, os.path.basename(lib), a.window, a.config,
                                               line[-1] if line else out.stderr[-2000:]), flush=True)
            if not line:
                sys.exit(1)


if __name__ == "__main__":
    main()
