"""Where one request's time goes in edv_verify_small_kernel (the authenticate() cache-miss
path): phase timestamps from a probe build (EDV_SMALL_PROFILE=1, wall clock at 100 MHz) and
the engine call's latency.  usage: PLENUM_EDVERIFY_LIB=tools/variants/lib_sprof.so
python tools/small_probe.py [key_window]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from plenum_amd import EdVerifyEngine, synth  # noqa: E402
from plenum_amd._lib import LIB_PATH  # noqa: E402

kw = int(sys.argv[1]) if len(sys.argv) > 1 else 14
eng = EdVerifyEngine(0)
eng.keys_set_window(kw)
pks, sks = eng.seed_keypair_batch(synth.signer_seeds(16))
eng.keys_add(pks)
msgs, kidx, spec = synth.nym_messages(400, pks, alias_len=43, seed=1)
off = np.zeros(len(msgs) + 1, np.uint64)
off[1:] = np.cumsum([len(m) for m in msgs])
buf = np.frombuffer(b"".join(msgs), np.uint8)
sig = eng.sign_batch(sks, kidx, buf, off)
lib = ctypes.CDLL(os.environ.get("PLENUM_EDVERIFY_LIB", LIB_PATH))
prof = getattr(lib, "edv_small_profile", None)
names = ["hash", "base tree", "decode part 1", "(barrier)", "decode total", "key tree (after barrier)", "end",
         "shader clock (MHz)"]
rows, lat = [], []
for i in range(len(msgs)):
    t0 = time.perf_counter()
    ok = eng.verify_one_keyed(bytes(sig[i]), int(kidx[i]), msgs[i])
    lat.append(time.perf_counter() - t0)
    assert ok
    if prof is not None:
        out = (ctypes.c_uint64 * 10)()
        assert prof(out) == 0
        t = [out[k] - out[0] for k in range(8)]
        clk = (out[9] - out[8]) / max(1, t[7]) * 100.0  # shader clock over the kernel, MHz
        rows.append([t[1], t[2], t[3], t[4], t[5], t[6] - t[4], t[7], clk * 100.0])
lat = np.array(lat[50:]) * 1e6
try:
    comb_us = eng.last_phases_ms()[2] * 1e3
except Exception:  # EDV_SMALL_NOEV=1: the small path records no phase events
    comb_us = float("nan")
print("key window %d: engine call n=1 p50 %.1f us p99 %.1f us; phases (comb) %.1f us" % (
    kw, np.percentile(lat, 50), np.percentile(lat, 99), comb_us))
if rows:
    med = np.median(np.array(rows[50:], dtype=np.float64), axis=0) / 100.0  # 100 MHz ticks -> us
    for n_, v in zip(names, med):
        print("  %-26s %7.1f us (from kernel start)" % (n_, v) if n_ not in (names[5], names[7]) else
              "  %-26s %7.1f" % (n_, v))
eng.close()
