"""The oracle (oracle/ed25519_oracle.c) pinned against libsodium 1.0.18's own
outputs: the committed golden vectors (tests/golden/gen_golden.py) and, where
libsodium is loadable, a differential run on fresh random/adversarial inputs."""
import ctypes
import hashlib
import random

import pytest

from conftest import items_of, load_npz, sodium

L = 2**252 + 27742317777372353535851937790883648493


@pytest.mark.parametrize("name", ["ed25519_valid.npz", "ed25519_edge.npz"])
def test_oracle_matches_golden(oracle, name):
    items = items_of(load_npz(name))
    for i, (sig, pk, msg, expect) in enumerate(items):
        assert (oracle.oracle_verify_detached(sig, msg, len(msg), pk) == 0) == expect, i


def test_oracle_sign_open_split(oracle):
    # crypto_sign_open: < 64 bytes rejects; else split at 64 (nacl_wrappers.py:108)
    d = items_of(load_npz("ed25519_valid.npz"))
    sig, pk, msg, _ = d[5]
    assert oracle.oracle_sign_open(sig + msg, len(sig) + len(msg), pk) == 0
    assert oracle.oracle_sign_open(sig[:63], 63, pk) == -1
    assert oracle.oracle_sign_open(sig[:63] + msg, 63 + len(msg), pk) == -1
    assert oracle.oracle_sign_open(b"", 0, pk) == -1


def test_oracle_sign_kat(oracle):
    k = load_npz("sign_kat.npz")
    for i in range(len(k["seed"])):
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        oracle.oracle_seed_keypair(pk, sk, k["seed"][i].tobytes())
        assert pk.raw == k["pk"][i].tobytes()
        msg = k["msgs"][int(k["off"][i]):int(k["off"][i + 1])].tobytes()
        sig = ctypes.create_string_buffer(64)
        oracle.oracle_sign_detached(sig, msg, ctypes.c_uint64(len(msg)), sk)
        assert sig.raw == k["sig"][i].tobytes()


def test_oracle_sha512_and_reduce(oracle):
    rng = random.Random(3)
    for n in list(range(0, 300)) + [1000, 4096]:
        m = bytes(rng.getrandbits(8) for _ in range(n))
        out = ctypes.create_string_buffer(64)
        oracle.oracle_sha512(out, m, ctypes.c_uint64(n))
        assert out.raw == hashlib.sha512(m).digest()
    for t in range(300):
        x = bytes(rng.getrandbits(8) for _ in range(64)) if t > 2 else [b"\xff" * 64, L.to_bytes(64, "little"),
                                                                      b"\0" * 64][t]
        out = ctypes.create_string_buffer(32)
        oracle.oracle_sc_reduce(out, x)
        assert int.from_bytes(out.raw, "little") == int.from_bytes(x, "little") % L


def test_oracle_small_order_blacklist_is_the_8_torsion_points(oracle):
    import edwards as E
    for P in E.order8_points():
        enc = bytearray(E.encode(P))
        assert oracle.oracle_has_small_order(bytes(enc))
        enc[31] ^= 0x80
        assert oracle.oracle_has_small_order(bytes(enc))


def test_oracle_differential_vs_libsodium(oracle):
    s = sodium()
    if s is None:
        pytest.skip("libsodium not loadable here; golden vectors still pin the oracle")
    assert s.sodium_version_string() == b"1.0.18"
    rng = random.Random(11)
    for t in range(300):
        seed = bytes(rng.getrandbits(8) for _ in range(32))
        pk, sk = ctypes.create_string_buffer(32), ctypes.create_string_buffer(64)
        s.crypto_sign_seed_keypair(pk, sk, seed)
        m = bytes(rng.getrandbits(8) for _ in range(rng.randrange(400)))
        sig = ctypes.create_string_buffer(64)
        s.crypto_sign_detached(sig, None, m, ctypes.c_ulonglong(len(m)), sk)
        sg, pkk = bytearray(sig.raw), bytearray(pk.raw)
        mode = t % 5
        if mode == 1:
            sg[rng.randrange(64)] ^= 1 << rng.randrange(8)
        elif mode == 2:
            pkk[rng.randrange(32)] ^= 1 << rng.randrange(8)
        elif mode == 3:
            sg[63] |= 0x80
        elif mode == 4:
            sg = bytearray(rng.getrandbits(8) for _ in range(64))
        want = s.crypto_sign_verify_detached(bytes(sg), m, ctypes.c_ulonglong(len(m)), bytes(pkk))
        assert oracle.oracle_verify_detached(bytes(sg), m, len(m), bytes(pkk)) == want, t


@pytest.mark.parametrize("name", ["ed25519_valid.npz", "ed25519_edge.npz"])
def test_full_batch_sodium_harness_matches_golden(sodium_verdicts, name):
    """The -m gpu tests' full-batch check (conftest.sodium_verdicts: libsodium on
    every host CPU over message spans) gives the golden verdicts, with items
    sharing one message copy too."""
    import numpy as np
    d = load_npz(name)
    off = d["off"].astype(np.uint64)
    got = sodium_verdicts(d["sig"], d["pk"], d["msgs"], off[:-1], off[1:])
    assert (got == d["expect"].astype(bool)).all()
    rev = np.arange(len(off) - 1)[::-1]  # the same messages through reordered spans
    got = sodium_verdicts(d["sig"][rev], d["pk"][rev], d["msgs"], off[:-1][rev], off[1:][rev])
    assert (got == d["expect"].astype(bool)[rev]).all()
