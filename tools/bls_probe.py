"""Throughput probe of the GPU BLS verify (edv_bls_verify_batch): n signed
items (distinct keys and messages), one call, wall time incl. H2D.
usage: python tools/bls_probe.py [FORM [n n ...]]  (FORM: wave / quad / pair / one)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "indy-plenum_amd"))
from plenum_amd import EdVerifyEngine, pack_messages  # noqa: E402
from plenum_amd.bls import GENERATOR, ORDER  # noqa: E402
from plenum_amd.base58 import b58decode  # noqa: E402

eng = EdVerifyEngine(0)
if os.environ.get("BLS_PAIR") is not None:  # batches up to this many checks: two lanes per check
    eng.bls_set_pair_lanes(int(os.environ["BLS_PAIR"]))
FORM = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("BLS_FORM")  # wave / quad / pair / one: that verify form at every size
gen = np.frombuffer(b58decode(GENERATOR), np.uint8)
rng = np.random.default_rng(1)
SIZES = ",".join(sys.argv[2:]) if len(sys.argv) > 2 else os.environ.get("BLS_SIZES", "64,1024,16384,65536,262144")
for n in [int(x) for x in SIZES.split(",")]:
    sks = np.frombuffer(b"".join((int.from_bytes(rng.bytes(32), "big") % ORDER).to_bytes(32, "big")
                                 for _ in range(n)), np.uint8).reshape(n, 32)
    t = time.time()
    vks = eng.bls_keygen_batch(sks, gen)
    tk = time.time() - t
    msgs = [rng.bytes(96) for _ in range(n)]
    buf, off = pack_messages(msgs)
    t = time.time()
    sigs = eng.bls_sign_batch(sks, buf, off)
    ts = time.time() - t
    if FORM:
        eng.bls_set_wave_checks(n if FORM == "wave" else 0)
        eng.bls_set_pair_lanes({"wave": 0, "quad": 2 * n, "pair": n, "one": 0}[FORM])
    t = time.time()
    ok = eng.bls_verify_batch(sigs, buf, off, vks, gen)
    tv = time.time() - t
    print("%s n=%6d keygen %.3f s  sign %.3f s  verify %.2f ms = %.0f verifies/s  all_ok=%s" % (
        FORM or "default", n, tk, ts, tv * 1e3, n / tv, bool(ok.all())), flush=True)
    if tv > 60:
        break
