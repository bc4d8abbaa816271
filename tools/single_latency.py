"""Engine-call latency of one keyed request (edv_verify_one): the resident kernel against a
kernel launch per request (EDV_RESIDENT=0 context), p50 / p99 of N back-to-back calls, plus the
resident kernel's launch / served counters.  usage: python tools/single_latency.py [N]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "indy-plenum_amd"))
from plenum_amd import EdVerifyEngine, pack_messages  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
eng = EdVerifyEngine(0)
rng = np.random.default_rng(5)
pk, sk = eng.seed_keypair_batch(rng.integers(0, 256, (4, 32), dtype=np.uint8))
msg = bytes(rng.integers(0, 256, 200, dtype=np.uint8))
b, o = pack_messages([msg])
sig = bytes(eng.sign_batch(sk, np.zeros(1, np.uint32), b, o)[0])
os.environ["EDV_RESIDENT"] = "0"
launch = EdVerifyEngine(0)
del os.environ["EDV_RESIDENT"]
for w in (10, 14):
    for name, e in (("resident", eng), ("launch", launch)):
        e.keys_reset()
        e.keys_set_window(w)
        e.keys_add(pk)
        lat, svc = [], []
        for _ in range(n):
            t = time.perf_counter()
            assert e.verify_one_keyed(sig, 0, msg)
            lat.append((time.perf_counter() - t) * 1e6)
            if name == "resident":
                svc.append(e.stats()["resident_service_us"])
        lat = np.array(lat[50:])
        st = e.stats()
        print("W=%d %-8s p50 %.1f us  p10 %.1f  p99 %.1f  resident launches %d served %d%s" % (
            w, name, np.percentile(lat, 50), np.percentile(lat, 10), np.percentile(lat, 99),
            st["resident_launches"], st["resident_served"],
            ("  in-kernel p50 %.1f us" % np.percentile(svc[50:], 50)) if svc else ""), flush=True)
launch.close()
eng.close()
