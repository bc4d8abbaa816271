"""Exact-integer edwards25519 helpers used ONLY to construct adversarial test
inputs (small-order / mixed-order keys, R + T8, non-canonical encodings).
Verdicts for every constructed case come from libsodium 1.0.18 itself
(gen_golden.py) or from the oracle, never from this file."""
import hashlib

p = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
d = (-121665 * pow(121666, p - 2, p)) % p
SQRTM1 = pow(2, (p - 1) // 4, p)


def inv(x):
    return pow(x, p - 2, p)


def recover_x(y, sign):
    """x for y (None if y is not a valid y-coordinate)."""
    if y >= p:
        return None
    x2 = (y * y - 1) * inv(d * y * y + 1) % p
    if x2 == 0:
        return None if sign else 0
    x = pow(x2, (p + 3) // 8, p)
    if (x * x - x2) % p:
        x = x * SQRTM1 % p
    if (x * x - x2) % p:
        return None
    if x & 1 != sign:
        x = p - x
    return x


def add(P, Q):
    x1, y1 = P
    x2, y2 = Q
    t = d * x1 * x2 * y1 * y2 % p
    return ((x1 * y2 + x2 * y1) * inv(1 + t) % p, (y1 * y2 + x1 * x2) * inv(1 - t) % p)


def neg(P):
    return ((-P[0]) % p, P[1])


def mul(k, P):
    R = (0, 1)
    while k:
        if k & 1:
            R = add(R, P)
        P = add(P, P)
        k >>= 1
    return R


By = 4 * inv(5) % p
B = (recover_x(By, 0), By)
IDENTITY = (0, 1)


def encode(P):
    x, y = P
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def decode(s):
    v = int.from_bytes(s, "little")
    y = v & ((1 << 255) - 1)
    x = recover_x(y, v >> 255)
    return None if x is None else (x, y)


def order8_points():
    """All 8 points of the small-order subgroup."""
    pts = set()
    # y^2 = (-1 +- sqrt(1+d)) / d gives the order-8 points; plus order 1,2,4.
    for P in [(0, 1), (0, p - 1), (SQRTM1, 0), (p - SQRTM1, 0)]:
        pts.add(P)
    s = pow(1 + d, (p + 3) // 8, p)
    if (s * s - (1 + d)) % p:
        s = s * SQRTM1 % p
    for sq in (s, p - s):
        y2 = (p - 1 + sq) * inv(d) % p
        y = pow(y2, (p + 3) // 8, p)
        if (y * y - y2) % p:
            y = y * SQRTM1 % p
        if (y * y - y2) % p:
            continue
        for yy in (y, p - y):
            for sign in (0, 1):
                x = recover_x(yy, sign)
                if x is not None and mul(8, (x, yy)) == IDENTITY:
                    pts.add((x, yy))
    return sorted(pts)


def sha512_int(*parts):
    return int.from_bytes(hashlib.sha512(b"".join(parts)).digest(), "little")


def secret_expand(seed):
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]


def sign_with(a, prefix, A_enc, msg, r=None):
    """Ed25519 signature with explicit secret scalar / optional fixed nonce r;
    A_enc is the (possibly adversarial) public-key encoding hashed into k."""
    if r is None:
        r = sha512_int(prefix, msg) % L
    R = mul(r, B)
    R_enc = encode(R)
    k = sha512_int(R_enc, A_enc, msg) % L
    S = (r + k * a) % L
    return R_enc + S.to_bytes(32, "little"), r, k
