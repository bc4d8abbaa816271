"""Probe: configs[1] steps (1M keyed verifies, inputs in HBM) issued back to back through two
engines (two library contexts, each with its own scratch, key store and base table) on two
streams of one GPU, against one engine stepping alone -- whether the encode's latency-bound tail
and the kernels' wave tails of one batch fill with the next batch's hash and comb.
usage: python tools/two_streams.py [steps] [key_window]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from plenum_amd import EdVerifyEngine, pack_messages, synth  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
window = int(sys.argv[2]) if len(sys.argv) > 2 else 14
n = 1_000_000
dev = torch.device("cuda", 0)
engs = [EdVerifyEngine(0), EdVerifyEngine(0)]
pks, sks = engs[0].seed_keypair_batch(synth.signer_seeds(1000))
msgs_l, key_idx, _ = synth.nym_messages(n, pks, alias_len=43, seed=1, req_id_base=synth.REQ_ID_BASE)
buf, off = pack_messages(msgs_l)
del msgs_l
d_kidx = torch.from_numpy(key_idx.astype(np.int32)).to(dev)
d_msgs = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
d_ms = torch.from_numpy(off[:-1].astype(np.int64)).to(dev)
d_me = torch.from_numpy(off[1:].astype(np.int64)).to(dev)
d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
engs[0].sign_spans_device(torch.from_numpy(sks).to(dev), d_kidx, d_msgs, d_ms, d_me, n, d_sig)
for e in engs:
    e.keys_reset()
    e.keys_set_window(window)
    e.keys_add(pks)
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
words = [torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev) for _ in engs]
torch.cuda.synchronize()


def run(k, which):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(k):
        j = which[s % len(which)]
        engs[j].verify_spans_device(d_sig, d_kidx, True, d_msgs, d_ms, d_me, n, words[j], stream=streams[j])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


for rep in range(3):
    for name, which in (("one engine", [0]), ("two engines, two streams", [0, 1])):
        for w in words:
            w.zero_()
        run(4, which)  # warm
        ms = run(steps, which)
        ok = all(bool((w == -1).all()) for w in (words[:1] if len(which) == 1 else words))
        print("%-26s %d steps: %.3f ms per 1M-request step = %.1f M verifies/s  all accepted: %s" % (
            name, steps, ms, n / ms / 1e3, ok), flush=True)
