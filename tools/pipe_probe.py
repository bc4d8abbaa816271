"""Whole-node A/B probe: the same GpuAuthNr timing K batches of 1M configs[1] requests through
authenticate_batch (sync), authenticate_batches (pipe) and a plain generator around
authenticate_batch (gen), in alternating rounds, with each form's scan time per batch -- whether
the pipelined form's slower batches follow the form or the time they run at.
usage: python tools/pipe_probe.py [rounds] [K]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
import bench  # noqa: E402
from plenum_amd import EdVerifyEngine, synth  # noqa: E402
from plenum_amd.client_authn import GpuAuthNr  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
eng = EdVerifyEngine(0)
pks, sks = eng.seed_keypair_batch(synth.signer_seeds(1000))
sets, idrs, vks = bench.whole_node_sets(eng, 1_000_000, pks, sks, 43, 0)
a = GpuAuthNr(engine=eng)
for idr, vk in zip(idrs, vks):
    a.addIdr(idr, vk)
a.keys_settle()
for k in range(3):
    a.authenticate_batch(sets[k % 2])
order = [sets[k % 2] for k in range(K)]


def gen(batches):
    for b in batches:
        yield a.authenticate_batch(b)


def run(form):
    per, scan = [], []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tb = t0
    if form == "sync":
        for b in order:
            a.authenticate_batch(b)
            tn = time.perf_counter()
            per.append(tn - tb)
            scan.append(a._g.last_breakdown["scan_and_copies"])
            tb = tn
    else:
        it = a.authenticate_batches(order) if form == "pipe" else gen(order)
        for _ in it:
            tn = time.perf_counter()
            per.append(tn - tb)
            scan.append(a._g.last_breakdown["scan_and_copies"])
            tb = tn
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print("%-4s %.2f M/s  batch p50 %.2f ms  scan p50 %.2f ms  each %s" % (
        form, K * 1e6 / el / 1e6, np.median(per) * 1e3, np.median(scan),
        " ".join("%.1f" % (x * 1e3) for x in per)), flush=True)


for r in range(rounds):
    for form in ("sync", "pipe", "gen"):
        run(form)
