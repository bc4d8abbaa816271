"""Generate the Ed25519 golden vectors under tests/golden/ from libsodium 1.0.18.

libsodium is the third-party library the reference's hot path ends in
(stp_core/crypto/nacl_wrappers.py:108 -> libnacl.crypto_sign_open ->
crypto_sign_verify_detached); it is not part of /root/reference.  The version
pinned here is the one in this image (/opt/conda/lib/libsodium.so.23 ->
sodium_version_string() == "1.0.18").  Every verdict below is libsodium's own
return value; edwards.py only constructs adversarial inputs.

Outputs (numpy .npz, loaded with allow_pickle=False):
  ed25519_valid.npz  libsodium-signed vectors, message lengths 0..300 plus
                     every SHA-512 block boundary up to 4096 bytes.
  ed25519_edge.npz   the libsodium 1.0.18 acceptance-edge table (labels in
                     ed25519_edge_labels.json), plus random corruptions.
  sign_kat.npz       seeds -> (pk, sig) for the signer kernels.

Run:  python3 tests/golden/gen_golden.py   (needs libsodium; not run by tests)
"""
import ctypes
import json
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import edwards as E  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def load_sodium():
    for cand in ("/opt/conda/lib/libsodium.so.23", "libsodium.so.23", "libsodium.so"):
        try:
            lib = ctypes.CDLL(cand)
        except OSError:
            continue
        lib.sodium_init()
        lib.sodium_version_string.restype = ctypes.c_char_p
        return lib
    raise SystemExit("libsodium not found")


S = load_sodium()
assert S.sodium_version_string() == b"1.0.18", S.sodium_version_string()


def keypair(seed):
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    S.crypto_sign_seed_keypair(pk, sk, seed)
    return pk.raw, sk.raw


def sign(msg, sk):
    sig = ctypes.create_string_buffer(64)
    S.crypto_sign_detached(sig, None, msg, ctypes.c_ulonglong(len(msg)), sk)
    return sig.raw


def verify(sig, msg, pk):
    return S.crypto_sign_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0


def pack(items):
    sig = np.frombuffer(b"".join(i[0] for i in items), dtype=np.uint8).reshape(-1, 64)
    pk = np.frombuffer(b"".join(i[1] for i in items), dtype=np.uint8).reshape(-1, 32)
    msgs = b"".join(i[2] for i in items)
    off = np.zeros(len(items) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(i[2]) for i in items])
    expect = np.array([verify(i[0], i[2], i[1]) for i in items], dtype=np.uint8)
    return dict(sig=sig, pk=pk, msgs=np.frombuffer(msgs, dtype=np.uint8), off=off, expect=expect)


def gen_valid(rng):
    lens = list(range(0, 301))
    for blk in range(1, 34):  # SHA-512 stream = 64 + mlen; boundaries at 111/112 mod 128
        for delta in (-2, -1, 0, 1):
            m = 128 * blk - 64 - 17 + delta
            if 300 < m <= 4096:
                lens.append(m)
    lens.append(4096)
    items = []
    for n, ml in enumerate(lens):
        seed = bytes(rng.getrandbits(8) for _ in range(32))
        pk, sk = keypair(seed)
        msg = bytes(rng.getrandbits(8) for _ in range(ml))
        items.append((sign(msg, sk), pk, msg))
    d = pack(items)
    assert d["expect"].all()
    return d


def gen_edge(rng):
    items, labels = [], []

    def add(label, sig, pk, msg):
        items.append((sig, pk, msg))
        labels.append(label)

    seed = bytes(range(32))
    pk, sk = keypair(seed)
    a, prefix = E.secret_expand(seed)
    msg = b"plenum request"
    sig = sign(msg, sk)
    add("valid", sig, pk, msg)
    add("valid-empty-msg", sign(b"", sk), pk, b"")
    Sint = int.from_bytes(sig[32:], "little")
    # --- S canonicity (sc25519_is_canonical)
    if Sint + E.L < 2**256:
        add("S+L", sig[:32] + (Sint + E.L).to_bytes(32, "little"), pk, msg)
    add("S|2^255", sig[:32] + (Sint | (1 << 255)).to_bytes(32, "little"), pk, msg)
    add("S=L", sig[:32] + E.L.to_bytes(32, "little"), pk, msg)
    add("S=L-1", sig[:32] + (E.L - 1).to_bytes(32, "little"), pk, msg)
    add("S=2^256-1", sig[:32] + b"\xff" * 32, pk, msg)
    add("S=0", sig[:32] + b"\x00" * 32, pk, msg)
    # --- R small order (blacklist, sign bit masked) and non-canonical R
    small = [E.encode(P) for P in E.order8_points()]
    noncanon_y = [(E.p + k) for k in range(0, 19)]
    bl = set()
    for enc in small:
        for sbit in (0, 1):
            e = bytearray(enc)
            e[31] = (e[31] & 0x7F) | (sbit << 7)
            bl.add(bytes(e))
    for y in noncanon_y:
        for sbit in (0, 1):
            bl.add((y | (sbit << 255)).to_bytes(32, "little"))
    for enc in sorted(bl):
        add("R=" + enc.hex(), enc + sig[32:], pk, msg)
    # R = identity with an equation that holds: S = k*a with nonce r = 0
    r0_sig, _, _ = E.sign_with(a, prefix, pk, msg, r=0)
    add("R=identity,eq-holds", r0_sig, pk, msg)
    # --- A small order / non-canonical / off-curve
    for enc in sorted(bl):
        add("A=" + enc.hex(), sig, enc, msg)
    # A small-order with a signature whose equation holds for that A:
    # A = identity, R = [S]B
    s_rand = rng.randrange(E.L)
    Rb = E.encode(E.mul(s_rand, E.B))
    add("A=identity,eq-holds", Rb + s_rand.to_bytes(32, "little"), E.encode(E.IDENTITY), msg)
    for t in range(8):
        while True:
            y = rng.randrange(E.p)
            if E.recover_x(y, 0) is None:
                break
        add("A=off-curve-%d" % t, sig, y.to_bytes(32, "little"), msg)
    # --- mixed-order A (A0 + T8), cofactorless-valid (k = 0 mod 8) and not
    T8 = [P for P in E.order8_points() if E.mul(4, P) != E.IDENTITY]
    A0 = E.mul(a, E.B)
    for ti, T in enumerate(T8):
        A_mixed = E.encode(E.add(A0, T))
        got_valid = got_invalid = 0
        while not (got_valid and got_invalid):
            r = rng.randrange(E.L)
            s2, _, k = E.sign_with(a, prefix, A_mixed, msg, r=r)
            if k % 8 == 0 and not got_valid:
                add("A=mixed-order-%d,k%%8==0" % ti, s2, A_mixed, msg)
                got_valid = 1
            elif k % 8 != 0 and not got_invalid:
                add("A=mixed-order-%d,k%%8!=0" % ti, s2, A_mixed, msg)
                got_invalid = 1
    # A with torsion of order 2/4 too
    for T in E.order8_points():
        if T == E.IDENTITY:
            continue
        A_mixed = E.encode(E.add(A0, T))
        r = rng.randrange(E.L)
        s2, _, k = E.sign_with(a, prefix, A_mixed, msg, r=r)
        add("A=A0+T(order%d)" % min(o for o in (2, 4, 8) if E.mul(o, T) == E.IDENTITY), s2, A_mixed, msg)
    # --- R + T8: valid only under the cofactored equation
    for ti, T in enumerate(T8):
        r = rng.randrange(E.L)
        R = E.mul(r, E.B)
        Rt = E.encode(E.add(R, T))
        k = E.sha512_int(Rt, pk, msg) % E.L
        Sx = (r + k * a) % E.L
        add("R=R+T8-%d" % ti, Rt + Sx.to_bytes(32, "little"), pk, msg)
    # --- pk encodings with x = 0 and sign bit 1 (y = 1, y = -1)
    for y in (1, E.p - 1):
        add("A=x0-sign1-y%s" % ("1" if y == 1 else "-1"), sig, (y | (1 << 255)).to_bytes(32, "little"), msg)
    # --- pk with the sign bit flipped (valid point -A'): equation fails
    pkf = bytearray(pk)
    pkf[31] ^= 0x80
    add("A=sign-flipped", sig, bytes(pkf), msg)
    # --- single bit flips in R, S, pk, msg
    for t in range(48):
        sg = bytearray(sig)
        pkk = bytearray(pk)
        mm = bytearray(msg)
        where = t % 4
        if where == 0:
            sg[rng.randrange(32)] ^= 1 << rng.randrange(8)
        elif where == 1:
            sg[32 + rng.randrange(32)] ^= 1 << rng.randrange(8)
        elif where == 2:
            pkk[rng.randrange(32)] ^= 1 << rng.randrange(8)
        else:
            mm[rng.randrange(len(mm))] ^= 1 << rng.randrange(8)
        add("flip-%s-%d" % ("RSAM"[where], t), bytes(sg), bytes(pkk), bytes(mm))
    # --- random garbage
    for t in range(32):
        add("garbage-%d" % t, bytes(rng.getrandbits(8) for _ in range(64)),
            bytes(rng.getrandbits(8) for _ in range(32)), bytes(rng.getrandbits(8) for _ in range(rng.randrange(200))))
    d = pack(items)
    return d, labels


def gen_sign_kat(rng):
    seeds, pks, sigs, msgs = [], [], [], []
    for t in range(64):
        seed = bytes(rng.getrandbits(8) for _ in range(32))
        pk, sk = keypair(seed)
        msg = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 400)))
        seeds.append(seed)
        pks.append(pk)
        sigs.append(sign(msg, sk))
        msgs.append(msg)
    off = np.zeros(len(msgs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return dict(seed=np.frombuffer(b"".join(seeds), dtype=np.uint8).reshape(-1, 32),
                pk=np.frombuffer(b"".join(pks), dtype=np.uint8).reshape(-1, 32),
                sig=np.frombuffer(b"".join(sigs), dtype=np.uint8).reshape(-1, 64),
                msgs=np.frombuffer(b"".join(msgs), dtype=np.uint8), off=off)


def main():
    rng = random.Random(20171015)
    np.savez_compressed(os.path.join(HERE, "ed25519_valid.npz"), **gen_valid(rng))
    edge, labels = gen_edge(rng)
    np.savez_compressed(os.path.join(HERE, "ed25519_edge.npz"), **edge)
    with open(os.path.join(HERE, "ed25519_edge_labels.json"), "w") as f:
        json.dump({"libsodium": S.sodium_version_string().decode(), "labels": labels,
                   "expect": [int(x) for x in edge["expect"]]}, f, indent=0)
    np.savez_compressed(os.path.join(HERE, "sign_kat.npz"), **gen_sign_kat(rng))
    print("valid:", len(gen_valid(random.Random(1))["expect"]), "edge:", len(labels),
          "accepted edge:", int(edge["expect"].sum()))


if __name__ == "__main__":
    main()
