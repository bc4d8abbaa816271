"""A/B of _hostpack.keys_known's prefetch chain (EDV_KEYS_PREFETCH=0 turns it off): a churning
batch's ~31k distinct identifiers resolved against 100k addIdr signers (clients nym dicts and the
fast-key map), caches flushed between repetitions by writing 512 MiB, as a batch's scan does.
usage: python tools/keys_known_ab.py [signers] [identifiers] [reps]  (CPU only)"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(signers, m, reps):
    sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))
    import numpy as np
    from plenum_amd._hostpack import keys_known
    rng = np.random.default_rng(0)
    idrs = [os.urandom(16).hex()[:22] for _ in range(signers)]
    clients, fk = {}, {}
    for i in idrs:
        vk = "~" + os.urandom(16).hex()[:22]
        clients[i] = {"verkey": vk, "role": None}
        fk[i] = (vk, os.urandom(32))
    flush = np.zeros(512 << 20, np.uint8)
    out = []
    for _ in range(reps):
        q = [(idrs[j] + ".")[:-1] for j in rng.choice(signers, m, replace=False)]  # fresh str objects
        flush += 1
        t = time.perf_counter()
        keys, holes = keys_known(clients, fk, q, "verkey")
        out.append((time.perf_counter() - t) * 1e3)
        assert not holes
    print("%.2f" % float(np.median(out)))


def main():
    signers = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 31_000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    if os.environ.get("KK_CHILD"):
        return child(signers, m, reps)
    for rnd in range(3):
        for pf in ("1", "0"):
            env = dict(os.environ, KK_CHILD="1", EDV_KEYS_PREFETCH=pf)
            r = subprocess.run([sys.executable, __file__, str(signers), str(m), str(reps)], env=env,
                               capture_output=True, text=True, check=True)
            print("round %d prefetch %s: keys_known median %s ms for %d identifiers of %d signers"
                  % (rnd, pf, r.stdout.strip(), m, signers), flush=True)


if __name__ == "__main__":
    main()
