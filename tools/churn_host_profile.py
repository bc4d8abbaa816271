"""The key-churn batches' host steps on the CPU (no GPU): bench.py's
time_key_churn workload through GpuAuthNr over the staging test double with
its verify answered instantly (all True), so the breakdown's scan /
keys_and_ids / verdicts are the host's alone.  A profiling probe, not a
result: signatures are random (nothing is checked).

  python tools/churn_host_profile.py [batches] [signers] [per_batch]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from engine_double import StagingOracleEngine  # noqa: E402
from plenum_amd import _hostpack, synth  # noqa: E402
from plenum_amd.base58 import b58encode  # noqa: E402
from plenum_amd.client_authn import GpuAuthNr  # noqa: E402


class InstantEngine(StagingOracleEngine):
    def _verify(self, sig64, pk32, msgs, msg_off):
        return np.ones(len(msg_off) - 1, bool)

    def verify_batch_keyed(self, sig64, key_idx, msgs, msg_off, sig_slot=64):
        self.calls += 1
        return np.ones(len(key_idx), bool)


def main():
    batches = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    signers = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 250_000
    rng = np.random.default_rng(3)
    pks = rng.integers(0, 256, size=(signers, 32), dtype=np.uint8)
    idrs = [b58encode(bytes(pk[:16])) for pk in pks]
    vks = ["~" + b58encode(bytes(pk[16:])) for pk in pks]
    n = per * batches
    kidx = synth.zipf_signers(n, signers, 1.1)
    msgs, spec = synth.churn_messages(kidx, idrs, alias_len=43)
    del msgs
    sig_b58 = _hostpack.b58encode_rows(rng.integers(0, 256, size=(n, 64), dtype=np.uint8).tobytes(), 64)
    reqs = []
    for i in range(n):
        r = synth.churn_request_dict(spec, i)
        r["signature"] = sig_b58[i]
        reqs.append(json.loads(json.dumps(r)))
    eng = InstantEngine()
    a = GpuAuthNr(engine=eng)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()
    chunks = [reqs[b * per:(b + 1) * per] for b in range(batches)]
    for b in range(batches):
        t0 = time.perf_counter()
        a.authenticate_batch(chunks[b])
        el = time.perf_counter() - t0
        print(json.dumps({"batch": b, "ms": round(el * 1e3, 2),
                          "in_batch_ms": {k: (round(v, 3) if isinstance(v, float) else v)
                                          for k, v in (a._g.last_breakdown or {}).items()}}), flush=True)


if __name__ == "__main__":
    main()
