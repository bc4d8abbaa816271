"""Whole-node A/B of the scan's worker count in one process (EDV_SCAN_THREADS is read per call):
rounds of 6 synchronous 1M-request batches at each count, the counts interleaved, so drift over
the run weighs on each alike.  usage: python tools/threads_probe.py [rounds]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
import bench  # noqa: E402
from plenum_amd import EdVerifyEngine, synth  # noqa: E402
from plenum_amd.client_authn import GpuAuthNr  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
eng = EdVerifyEngine(0)
pks, sks = eng.seed_keypair_batch(synth.signer_seeds(1000))
sets, idrs, vks = bench.whole_node_sets(eng, 1_000_000, pks, sks, 43, 0)
a = GpuAuthNr(engine=eng)
for idr, vk in zip(idrs, vks):
    a.addIdr(idr, vk)
a.keys_settle()
for k in range(3):
    a.authenticate_batch(sets[k % 2])
res = {}
for r in range(rounds):
    for T in (16, 15, 14, 17):
        os.environ["EDV_SCAN_THREADS"] = str(T)
        for k in range(6):
            t = time.perf_counter()
            a.authenticate_batch(sets[k % 2])
            res.setdefault(T, []).append(time.perf_counter() - t)
for T, v in sorted(res.items()):
    print("threads %d: batch p50 %.2f ms, mean %.2f ms (%d batches)" % (T, np.median(v) * 1e3, np.mean(v) * 1e3,
                                                                        len(v)), flush=True)
