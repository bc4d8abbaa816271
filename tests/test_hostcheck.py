"""The exact kernel arithmetic (indy-plenum_amd/csrc/*.h, compiled for the CPU
with EDV_BOUND_CHECK limb-bound assertions) against the golden vectors and the
oracle -- catches arithmetic bugs without a GPU."""
import ctypes
import hashlib
import random

import pytest

from conftest import items_of, load_npz

p = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493


@pytest.mark.parametrize("name", ["ed25519_edge.npz", "ed25519_valid.npz"])
def test_kernel_verify_on_cpu_matches_golden(hostcheck, name):
    items = items_of(load_npz(name))
    if name == "ed25519_valid.npz":
        items = items[::7]  # the host build is slow (-O1, assertions)
    for i, (sig, pk, msg, expect) in enumerate(items):
        assert (hostcheck.edv_host_verify(sig, pk, msg, ctypes.c_uint64(len(msg))) == 0) == expect, i


def test_kernel_sha512_any_alignment(hostcheck):
    rng = random.Random(5)
    for t in range(200):
        pre = bytes(rng.getrandbits(8) for _ in range(64))
        m = bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 600)))
        off = rng.randrange(0, 16)
        buf = ctypes.create_string_buffer(b"\0" * off + m + b"\0" * 16)
        out = ctypes.create_string_buffer(64)
        hostcheck.edv_host_sha512_prefixed(out, pre, ctypes.byref(buf, off), ctypes.c_uint64(len(m)))
        assert out.raw == hashlib.sha512(pre + m).digest()


def test_kernel_sha512_packed_units(hostcheck):
    """Length-bucketed SoA layout (sha512.h pack_lane_units /
    sha512_prefixed_units): every SHA-512 block boundary of R||A||M around
    0..4 KiB, any alignment, lane stride 1 and 64; the units are the padded
    big-endian stream words after the 64-byte prefix, bit length last."""
    hostcheck.edv_host_sha512_units_count.restype = ctypes.c_uint64
    rng = random.Random(8)
    lens = sorted({k for b in range(34) for k in (128 * b - 81, 128 * b - 80, 128 * b - 79, 128 * b - 65,
                                                   128 * b - 64, 128 * b - 63) if 0 <= k <= 4200} | {0, 1, 15, 16, 17})
    for t, mlen in enumerate(lens + [rng.randrange(0, 4200) for _ in range(60)]):
        pre = bytes(rng.getrandbits(8) for _ in range(64))
        m = bytes(rng.getrandbits(8) for _ in range(mlen))
        off = rng.randrange(0, 16)
        buf = ctypes.create_string_buffer(b"\0" * off + m + b"\0" * 16)
        stride = 64 if t % 2 else 1
        nu = hostcheck.edv_host_sha512_units_count(ctypes.c_uint64(mlen))
        units = ctypes.create_string_buffer(16 * nu)
        out = ctypes.create_string_buffer(64)
        hostcheck.edv_host_sha512_units(out, pre, ctypes.byref(buf, off), ctypes.c_uint64(mlen),
                                        ctypes.c_uint64(stride), units)
        assert out.raw == hashlib.sha512(pre + m).digest(), (mlen, off)
        # the units are the stream after the prefix: M || 0x80 || 0.. || 128-bit length, as u64 words
        total = 64 + mlen
        nblocks = (total + 16) // 128 + 1
        assert nu == 8 * nblocks - 4
        stream = m + b"\x80" + b"\0" * (128 * nblocks - total - 17) + (8 * total).to_bytes(16, "big")
        words = [int.from_bytes(stream[8 * k:8 * k + 8], "big") for k in range(2 * nu)]
        got = [int.from_bytes(units.raw[8 * k:8 * k + 8], "little") for k in range(2 * nu)]
        assert got == words, (mlen, off)


def test_kernel_sc_reduce_and_canonical(hostcheck):
    rng = random.Random(6)
    specials = [0, 1, L - 1, L, L + 1, 2 * L, 2**512 - 1, 2**512 - 1 - L, 2**252, 2**253 - 1, (2**256 - 1) * L % 2**512]
    for t in range(3000):
        x = specials[t] if t < len(specials) else rng.getrandbits(512)
        out = ctypes.create_string_buffer(32)
        hostcheck.edv_host_sc_reduce(out, x.to_bytes(64, "little"))
        assert int.from_bytes(out.raw, "little") == x % L, hex(x)
    for s in [0, L - 1, L, L + 1, 2**256 - 1, 2**255, L | 2**255]:
        assert hostcheck.edv_host_sc_is_canonical(s.to_bytes(32, "little")) == (s < L)


def test_kernel_field_ops(hostcheck):
    rng = random.Random(7)
    edge = [0, 1, 2, p - 1, p, p + 1, 2**255 - 1, 19, 2**254, (1 << 26) - 1]
    for t in range(4000):
        a = edge[t % len(edge)] if t < 100 else rng.getrandbits(255)
        b = edge[(t // len(edge)) % len(edge)] if t < 100 else rng.getrandbits(255)
        out = ctypes.create_string_buffer(32)
        hostcheck.edv_host_fe_mul(out, a.to_bytes(32, "little"), b.to_bytes(32, "little"), 0)
        assert int.from_bytes(out.raw, "little") == a * b % p
        hostcheck.edv_host_fe_mul(out, a.to_bytes(32, "little"), b.to_bytes(32, "little"), 1)
        assert int.from_bytes(out.raw, "little") == a * a % p
        if a % p and t % 8 == 0:
            hostcheck.edv_host_fe_invert(out, a.to_bytes(32, "little"))
            assert int.from_bytes(out.raw, "little") == pow(a, p - 2, p)


_LIMB_AT = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]  # radix 2^25.5 limb positions


@pytest.mark.parametrize("order", [1, 2, 3])
def test_kernel_product_orders_at_class_bounds(hostcheck, order):
    """fe_mul_o / fe_sq_o in every product order (3: the small kernel's two half-chains)
    on limbs up to the class bounds their callers may pass (f in W = 5 x 2^26 / 5 x 2^25 +
    2^18, g in L = 3 x 2^26 / 3 x 2^25 + 2^18): the value mod p, output limbs in class C
    (asserted inside the -DEDV_BOUND_CHECK build)."""
    rng = random.Random(40 + order)
    W = [(5 << 26) if k % 2 == 0 else (5 << 25) + (1 << 18) for k in range(10)]
    L = [(3 << 26) if k % 2 == 0 else (3 << 25) + (1 << 18) for k in range(10)]
    val = lambda v: sum(x << s for x, s in zip(v, _LIMB_AT)) % p  # noqa: E731
    arr = ctypes.c_uint32 * 10
    for t in range(400):
        if t < 4:
            a = W if t % 2 == 0 else [x - 1 for x in W]
            b = L
        else:
            a = [rng.randrange(m + 1) for m in W]
            b = [rng.randrange(m + 1) for m in L]
        out = arr()
        hostcheck.edv_host_fe_mul_limbs(out, arr(*a), arr(*b), 2 * order)
        assert val(list(out)) == val(a) * val(b) % p
        sq_in = [min(x, m) for x, m in zip(a, L)]
        hostcheck.edv_host_fe_mul_limbs(out, arr(*sq_in), arr(*sq_in), 2 * order + 1)
        assert val(list(out)) == val(sq_in) ** 2 % p


def test_kernel_point_roundtrip_and_blacklist(hostcheck, oracle):
    import edwards as E
    rng = random.Random(8)
    for t in range(200):
        y = rng.randrange(p) if t else 1
        enc = (y | (rng.getrandbits(1) << 255)).to_bytes(32, "little")
        o1, o2 = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
        r1 = hostcheck.edv_host_point_roundtrip(o1, enc)
        r2 = oracle.oracle_point_roundtrip(o2, enc)
        assert r1 == r2
        if r1 == 0:
            assert o1.raw == o2.raw
    for P in E.order8_points():
        enc = E.encode(P)
        assert hostcheck.edv_host_has_small_order(enc)
    for y in range(p, 2**255):
        for s in (0, 1):
            enc = (y | (s << 255)).to_bytes(32, "little")
            assert hostcheck.edv_host_is_canonical_point(enc) == oracle.oracle_is_canonical_point(enc) == 0
            assert hostcheck.edv_host_has_small_order(enc) == oracle.oracle_has_small_order(enc)


def test_kernel_comb_path_on_cpu_matches_golden(hostcheck):
    """The key-table path's arithmetic (comb.h: W=4 key tables, W=8 base
    table, signed-digit recoding, mixed additions) on the CPU."""
    items = items_of(load_npz("ed25519_edge.npz"))[::3] + items_of(load_npz("ed25519_valid.npz"))[::41]
    for i, (sig, pk, msg, expect) in enumerate(items):
        assert (hostcheck.edv_host_verify_comb(sig, pk, msg, ctypes.c_uint64(len(msg))) == 0) == expect, i


@pytest.mark.parametrize("k", [1, 2, 4, 8])
def test_kernel_split_ladder(hostcheck, k):
    """The general path's split-table ladder (verify_core.h
    verify_phase_table_split / verify_phase_dsm_split_point: K tables of
    2^(256t/K)(-A), 256/K - 4 doublings) on the CPU, edge + valid vectors."""
    items = items_of(load_npz("ed25519_edge.npz"))[::7] + items_of(load_npz("ed25519_valid.npz"))[::61]
    for i, (sig, pk, msg, expect) in enumerate(items):
        got = hostcheck.edv_host_verify_split(sig, pk, msg, ctypes.c_uint64(len(msg)), k) == 0
        assert got == expect, (k, i)


@pytest.mark.parametrize("w", [4, 5, 6, 7, 8, 9, 10, 11, 12])
def test_kernel_comb_windows(hostcheck, w):
    """comb.h's generic signed radix-2^W recoding (9-word bias; W = 5, 6, 7
    digits straddle 32-bit words) at every window the key store can use."""
    items = items_of(load_npz("ed25519_edge.npz"))[::23] + items_of(load_npz("ed25519_valid.npz"))[::97]
    for i, (sig, pk, msg, expect) in enumerate(items):
        got = hostcheck.edv_host_verify_comb_w(sig, pk, msg, ctypes.c_uint64(len(msg)), w) == 0
        assert got == expect, (w, i)


def test_kernel_batch_encode(hostcheck):
    """batch_encode.h (Montgomery's trick over 16 results, the edv_encode_kernel
    code) gives per-item verdicts: mixed accept/reject groups, a ragged last
    group, and a poisoned Z = 0 that must reject only its own item."""
    import numpy as np
    items = items_of(load_npz("ed25519_valid.npz"))[:23] + items_of(load_npz("ed25519_edge.npz"))[::9]
    n = len(items)
    sig = b"".join(s for s, _, _, _ in items)
    pk = b"".join(k for _, k, _, _ in items)
    msgs = b"".join(m for _, _, m, _ in items) + b"\0" * 8
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum([len(m) for _, _, m, _ in items])
    expect = np.array([e for _, _, _, e in items], bool)
    for zero_at in (None, 5, n - 1):
        zz = np.zeros(n, np.uint8)
        if zero_at is not None:
            zz[zero_at] = 1
        bits = ctypes.create_string_buffer((n + 7) // 8)
        hostcheck.edv_host_verify_batch_comb(sig, pk, msgs, off.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint64(n), 8,
                                             zz.ctypes.data_as(ctypes.c_void_p), bits)
        got = np.unpackbits(np.frombuffer(bits.raw, np.uint8), bitorder="little")[:n].astype(bool)
        want = expect.copy()
        if zero_at is not None:
            want[zero_at] = False
        assert (got == want).all(), (zero_at, np.nonzero(got != want))


def test_comb_recoding_exact_up_to_L():
    """Signed radix-2^W digits (comb.h) reconstruct every scalar below L,
    including the top of the range where x + bias needs W*rows >= 254 bits
    (W = 11 with 23 rows would overflow there), and stay in table range."""
    import ctypes as C
    from conftest import PKG
    import os
    lib = C.CDLL(os.path.join(PKG, "libedv_hostcheck.so"))
    rng = random.Random(11)
    xs = [0, 1, L - 1, L - 2, 2**252, 2**252 - 1, L - 2**200] + [rng.randrange(L) for _ in range(300)]
    xs += [L - 1 - rng.randrange(2**128) for _ in range(100)]
    for w in range(4, 15):
        out = (C.c_int * 80)()
        for x in xs:
            rows = lib.edv_host_comb_digits(x.to_bytes(32, "little"), w, out)
            assert rows == -(-254 // w)
            d = list(out[:rows])
            assert all(-(1 << (w - 1)) <= v < (1 << (w - 1)) for v in d), (w, x)
            assert sum(v << (w * i) for i, v in enumerate(d)) == x, (w, hex(x))


def test_kernel_sha256_any_alignment(hostcheck):
    """csrc/sha256.h (request digests) vs hashlib, all block boundaries and 16 alignments."""
    rng = random.Random(21)
    lens = list(range(0, 200)) + [247, 248, 255, 256, 311, 312, 319, 320, 1000, 4095, 4096]
    for t, n in enumerate(lens):
        m = bytes(rng.getrandbits(8) for _ in range(n))
        off = t % 16
        buf = ctypes.create_string_buffer(b"\0" * off + m + b"\0" * 16)
        out = ctypes.create_string_buffer(32)
        hostcheck.edv_host_sha256(out, ctypes.byref(buf, off), ctypes.c_uint64(n))
        assert out.raw == hashlib.sha256(m).digest(), n
