"""TEST INFRASTRUCTURE ONLY: CPU restatement of the BLS signature check the
GPU edv_bls_* kernels implement.

The reference verifies COMMIT BLS signatures through indy-crypto 0.1.6
(setup.py:57) -- crypto/bls/indy_crypto/bls_crypto_indy_crypto.py:59-90:
  verify_sig(sig, msg, pk)        Bls.verify: e(sig, g) == e(H(msg), vk)
  verify_multi_sig(sig, msg, pks) Bls.verify_multi_sig: vk = sum(pks) first
  create_multi_sig(sigs)          MultiSignature.new: the sum of the points
indy-crypto (Rust) and the AMCL library under it are absent from this
machine, so their published algorithm is restated here:
  * curve AMCL "BN254": x = -0x4080000000000001, p = 36x^4+36x^3+24x^2+6x+1,
    r = 36x^4+36x^3+18x^2+6x+1, E: y^2 = x^3 + 2 over Fp (G1, signatures and
    H(m)); D-type sextic twist E': y^2 = x^3 + 2/(1+i) over Fp2 = Fp[i]/(i^2+1)
    (G2, generator and verkeys).
  * H(m) = Bls::_hash: SHA-256(m) as a big-endian integer h, then AMCL
    ECP::new_big: x = h mod p, y = (x^3+2)^((p+1)/4) when x^3+2 is a square,
    else h += 1 and retry.
  * G2 bytes (128): x.a | x.b | y.a | y.b, 32-byte big-endian each (AMCL
    ECP2::tobytes); a decoding that is not on the curve is the point at
    infinity.  G1 bytes (128): 0x04 | x | y | 63 zero bytes (ECP::tobytes
    into indy-crypto's 128-byte buffer); a first byte other than 0x04 takes
    y = sqrt(x^3+2) (ECP::new_big); off-curve or x, y >= p is infinity.
  * the pairing: the reduced optimal ate pairing of BN curves, loop |6x+2|,
    conjugation for x < 0, then the lines through pi(Q) and -pi^2(Q).
PINNING: only the curve, twist and G2 encoding are pinned, by the one
literal the reference holds (the generator, bls_crypto_indy_crypto.py:14-15:
it decodes to a point of order r on exactly this twist, test_bls_oracle.py).
The G1 encoding and H(m) are restated from indy-crypto/AMCL as described
above and are PARITY UNPINNED (no reference vector exists; the reference's
tests generate keys and signatures at run time).

Arithmetic here is deliberately different from the device code (bn254.h):
Fp12 is Fp[w]/(w^12 - 2 w^6 + 2) (w^6 = 1 + i) with schoolbook polynomial
products, points are affine, every line is evaluated in Fp12 from the
affine twist slope (psi(x', y') = (x' w^2, y' w^3)) without scaling, and the
final exponentiation is one plain power; the device's reduced pairing must
equal this one bit for bit (tests/test_bls.py).
Only tests/ and bench.py's checker may import this."""
import hashlib

BN_X = -0x4080000000000001
P = 36 * BN_X**4 + 36 * BN_X**3 + 24 * BN_X**2 + 6 * BN_X + 1
R = 36 * BN_X**4 + 36 * BN_X**3 + 18 * BN_X**2 + 6 * BN_X + 1
ATE_LOOP = abs(6 * BN_X + 2)
FINAL_EXP = (P**12 - 1) // R

G2_GEN_B58 = ("3LHpUjiyFC2q2hD7MnwwNmVXiuaFbQx2XkAFJWzswCjgN1utjsCeLzHsKk1nJvFEaS4fcrUmVAkdhtPCYbrVyATZcmzwJReTcJqwqBCPTmTQ9"
              "uWPwz6rEncKb2pYYYFcdHa8N17HzVyTqKfgPi4X9pMetfT3A5xCHq54R2pDNYWVLDX")


# ---------------------------------------------------------------- Fp2 = Fp[i]/(i^2 + 1)
class F2:
    __slots__ = ("a", "b")

    def __init__(self, a, b=0):
        self.a, self.b = a % P, b % P

    def __add__(s, o):
        return F2(s.a + o.a, s.b + o.b)

    def __sub__(s, o):
        return F2(s.a - o.a, s.b - o.b)

    def __neg__(s):
        return F2(-s.a, -s.b)

    def __mul__(s, o):
        if isinstance(o, int):
            return F2(s.a * o, s.b * o)
        return F2(s.a * o.a - s.b * o.b, s.a * o.b + s.b * o.a)

    def __eq__(s, o):
        return s.a == o.a and s.b == o.b

    def inv(s):
        d = pow(s.a * s.a + s.b * s.b, P - 2, P)
        return F2(s.a * d, -s.b * d)

    def iszero(s):
        return s.a == 0 and s.b == 0

    def __repr__(s):
        return "F2(%#x, %#x)" % (s.a, s.b)


B1 = 2
B2 = F2(2) * F2(1, 1).inv()  # 2 / (1 + i)


# ---------------------------------------------------------------- Fp12 = Fp[w]/(w^12 - 2 w^6 + 2)
# (w^6 = 1 + i; i = w^6 - 1)
class F12:
    __slots__ = ("c",)

    def __init__(self, c):
        self.c = [v % P for v in c]

    @staticmethod
    def one():
        return F12([1] + [0] * 11)

    def __mul__(s, o):
        t = [0] * 23
        for i, x in enumerate(s.c):
            if x:
                for j, y in enumerate(o.c):
                    t[i + j] += x * y
        for k in range(22, 11, -1):  # w^k = 2 w^(k-6) - 2 w^(k-12)
            v = t[k]
            if v:
                t[k - 6] += 2 * v
                t[k - 12] -= 2 * v
        return F12(t[:12])

    def __add__(s, o):
        return F12([x + y for x, y in zip(s.c, o.c)])

    def __sub__(s, o):
        return F12([x - y for x, y in zip(s.c, o.c)])

    def __neg__(s):
        return F12([-x for x in s.c])

    def __eq__(s, o):
        return s.c == o.c

    def __pow__(s, e):
        r, b = F12.one(), s
        while e:
            if e & 1:
                r = r * b
            b = b * b
            e >>= 1
        return r

    def inv(s):
        return s ** (P**12 - 2)

    def isone(s):
        return s.c == [1] + [0] * 11


def f12_from_fp(v):
    return F12([v] + [0] * 11)


def f12_from_f2(z):  # a + b i = a + b (w^6 - 1)
    c = [0] * 12
    c[0] = z.a - z.b
    c[6] = z.b
    return F12(c)


W = F12([0, 1] + [0] * 10)
W2, W3 = W * W, W * W * W


# ---------------------------------------------------------------- groups (affine; None = infinity)
def g1_on_curve(pt):
    return pt is None or (pt[1] * pt[1] - pt[0] ** 3 - B1) % P == 0


def g2_on_curve(pt):
    return pt is None or pt[1] * pt[1] == pt[0] * pt[0] * pt[0] + B2


def _add(pt, qt, field_inv, zero, three, two):
    if pt is None:
        return qt
    if qt is None:
        return pt
    (x1, y1), (x2, y2) = pt, qt
    if x1 == x2:
        if y1 == y2 and not (y1 == zero):
            lam = (x1 * x1 * three) * field_inv(y1 * two)
        else:
            return None
    else:
        lam = (y2 - y1) * field_inv(x2 - x1)
    x3 = lam * lam - x1 - x2
    return (x3, lam * (x1 - x3) - y1)


def g1_add(pt, qt):
    if pt is None:
        return qt
    if qt is None:
        return pt
    (x1, y1), (x2, y2) = pt, qt
    if x1 == x2:
        if y1 != y2 or y1 == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, P - 2, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, P - 2, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def g1_neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def g1_mul(pt, k):
    acc = None
    for bit in bin(k % R if pt is not None else 0)[2:] if k else "":
        acc = g1_add(acc, acc)
        if bit == "1":
            acc = g1_add(acc, pt)
    return acc


def g2_add(pt, qt):
    return _add(pt, qt, lambda z: z.inv(), F2(0), 3, 2)


def g2_neg(pt):
    return None if pt is None else (pt[0], -pt[1])


def g2_mul(pt, k):
    acc = None
    if pt is None:
        return None
    for bit in bin(k)[2:]:
        acc = g2_add(acc, acc)
        if bit == "1":
            acc = g2_add(acc, pt)
    return acc


# ---------------------------------------------------------------- encodings
_B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def b58decode(s):
    n = 0
    for ch in s:
        n = n * 58 + _B58.index(ch)
    body = n.to_bytes((n.bit_length() + 7) // 8, "big") if n else b""
    return b"\0" * (len(s) - len(s.lstrip("1"))) + body


def b58encode(b):
    n = int.from_bytes(b, "big")
    out = ""
    while n:
        n, rem = divmod(n, 58)
        out = _B58[rem] + out
    return "1" * (len(b) - len(b.lstrip(b"\0"))) + out


def g2_from_bytes(b):
    """AMCL ECP2::frombytes: x.a | x.b | y.a | y.b big-endian; off curve -> infinity."""
    assert len(b) == 128
    v = [int.from_bytes(b[32 * k:32 * k + 32], "big") for k in range(4)]
    pt = (F2(v[0], v[1]), F2(v[2], v[3]))
    return pt if g2_on_curve(pt) else None


def g2_to_bytes(pt):
    if pt is None:
        return b"\0" * 128
    x, y = pt
    return b"".join(v.to_bytes(32, "big") for v in (x.a, x.b, y.a, y.b))


def _sqrt_p(v):
    """AMCL FP::sqrt for p = 3 mod 4: v^((p+1)/4) (no sign normalisation)."""
    return pow(v, (P + 1) // 4, P)


def _is_square(v):
    return v % P != 0 and pow(v, (P - 1) // 2, P) == 1


def g1_from_bytes(b):
    """ECP::frombytes as described in the header (parity unpinned)."""
    assert len(b) >= 65
    x = int.from_bytes(b[1:33], "big")
    if x >= P:
        return None
    if b[0] == 4:
        y = int.from_bytes(b[33:65], "big")
        if y >= P:
            return None
        pt = (x, y)
        return pt if g1_on_curve(pt) else None
    rhs = (x**3 + B1) % P
    if not _is_square(rhs):
        return None
    return (x, _sqrt_p(rhs))


def g1_to_bytes(pt):
    if pt is None:
        return b"\0" * 128
    return b"\x04" + pt[0].to_bytes(32, "big") + pt[1].to_bytes(32, "big") + b"\0" * 63


def hash_to_g1(msg):
    """indy-crypto Bls::_hash -> PointG1::from_hash -> ECP::new_big (try and increment)."""
    h = int.from_bytes(hashlib.sha256(msg).digest(), "big")
    while True:
        x = h % P
        rhs = (x**3 + B1) % P
        if _is_square(rhs):
            return (x, _sqrt_p(rhs))
        h += 1


# ---------------------------------------------------------------- pairing
# Q stays on the twist: for psi(x', y') = (x' w^2, y' w^3) a slope of E(Fp12)
# is lambda' w with lambda' the twist's own slope, so every line value is a
# product in Fp12 and no Fp12 inversion is needed.
GAMMA2 = None  # xi^((p-1)/3), xi^((p-1)/2): pi(x', y') = (conj(x') g2, conj(y') g3)
GAMMA3 = None


def _xi_pow(e):
    r, b = F2(1), F2(1, 1)
    while e:
        if e & 1:
            r = r * b
        b = b * b
        e >>= 1
    return r


GAMMA2 = _xi_pow((P - 1) // 3)
GAMMA3 = _xi_pow((P - 1) // 2)


def twist_frobenius(q):
    """pi on the twist: psi^-1(Frob(psi(q)))."""
    x, y = q
    return (F2(x.a, -x.b) * GAMMA2, F2(y.a, -y.b) * GAMMA3)


def _slope(a, b):
    (x1, y1), (x2, y2) = a, b
    if x1 == x2 and y1 == y2:
        return (x1 * x1 * 3) * (y1 * 2).inv()
    return (y2 - y1) * (x2 - x1).inv()


def _line(a, b, px, py):
    """The line through psi(a) and psi(b) (tangent if a == b) at P, in Fp12:
    (yP - y1 w^3) - lambda' w (xP - x1 w^2)."""
    lam = f12_from_f2(_slope(a, b)) * W
    return (py - f12_from_f2(a[1]) * W3) - lam * (px - f12_from_f2(a[0]) * W2)


def miller_loop(p1, q2):
    """f_{|6x+2|,Q}(P), conjugated for x < 0, times the two R-ate lines."""
    if p1 is None or q2 is None:
        return F12.one()
    px, py = f12_from_fp(p1[0]), f12_from_fp(p1[1])
    t, f = q2, F12.one()
    for bit in bin(ATE_LOOP)[3:]:
        f = f * f * _line(t, t, px, py)
        t = g2_add(t, t)
        if bit == "1":
            f = f * _line(t, q2, px, py)
            t = g2_add(t, q2)
    if BN_X < 0:
        f = f ** (P**6)  # conjugation: the inverse up to the final exponentiation
        t = g2_neg(t)
    q1 = twist_frobenius(q2)
    qm2 = g2_neg(twist_frobenius(q1))
    f = f * _line(t, q1, px, py)
    t = g2_add(t, q1)
    f = f * _line(t, qm2, px, py)
    return f


def final_exp(f):
    return f ** FINAL_EXP


def pairing(p1, q2):
    return final_exp(miller_loop(p1, q2))


# ---------------------------------------------------------------- BLS (indy-crypto Bls)
def generator():
    return g2_from_bytes(b58decode(G2_GEN_B58))


def keygen(sk, gen=None):
    return g2_mul(gen or generator(), sk % R)


def sign(msg, sk):
    return g1_mul(hash_to_g1(msg), sk % R)


def aggregate(sigs):
    acc = None
    for s in sigs:
        acc = g1_add(acc, s)
    return acc


def verify(sig, msg, vk, gen=None):
    """Bls.verify: e(sig, g) == e(H(m), vk).  A signature, verkey (sum) or
    generator at infinity is rejected (the product's policy, bn254.h
    bls_check: 1 == 1 would accept a forged multi-signature with no
    participants; AMCL's own answer for these inputs is unpinned)."""
    gen = gen or generator()
    if sig is None or vk is None or gen is None:
        return False
    lhs = final_exp(miller_loop(sig, gen) * miller_loop(g1_neg(hash_to_g1(msg)), vk))
    return lhs.isone()


def verify_multi(msig, msg, vks, gen=None):
    """Bls.verify_multi_sig: the verkeys are summed, then verify."""
    acc = None
    for v in vks:
        acc = g2_add(acc, v)
    return verify(msig, msg, acc, gen)


def verify_bytes(sig128, msg, vk128, gen128=None):
    """verify_sig over the wire bytes (the reference's bls_from_str has already
    checked the lengths: 32 or 128)."""
    gen = g2_from_bytes(gen128) if gen128 else generator()
    return verify(g1_from_bytes(sig128), msg, g2_from_bytes(vk128), gen)


def f12_to_tower(f):
    """Fp12 (w-polynomial) -> the device's tower coefficients: f = sum over
    (k in {0,1}, j in {0,1,2}) of (x + y i) v^j w^k with v = w^2, i = w^6 - 1;
    returned as [c0.a0.x, c0.a0.y, c0.a1.x, ..., c1.a2.y] (12 ints)."""
    # coefficient of w^(2j+k) and w^(2j+k+6): x - y and y
    out = []
    for k in range(2):
        for j in range(3):
            e = 2 * j + k
            y = f.c[e + 6]
            x = (f.c[e] + y) % P
            out += [x, y]
    return out
