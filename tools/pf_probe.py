"""Whole-node A/B of the scan's prefetch distances in one process (EDV_SCAN_PF, read per call):
rounds of 6 synchronous 1M-request batches at each scale, interleaved.  usage: python
tools/pf_probe.py [rounds]"""
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

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
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
    for pf in ("1", "2", "3"):
        os.environ["EDV_SCAN_PF"] = pf
        for k in range(6):
            t = time.perf_counter()
            a.authenticate_batch(sets[k % 2])
            res.setdefault(pf, []).append(time.perf_counter() - t)
for pf, v in sorted(res.items()):
    print("prefetch scale %s: batch p50 %.2f ms, mean %.2f ms (%d batches)" % (pf, np.median(v) * 1e3,
                                                                             np.mean(v) * 1e3, len(v)), flush=True)
