"""Generate indy-plenum_amd/csrc/bls_program.h: the BLS pairing check as one
straight-line program of Fp operations, scheduled over the 64 lanes of a wave.

Why: a BN254 pairing check is ~50k Fp operations with no data-dependent branch
between the decoded points and the final "== 1" (the loop |6x + 2| and the
exponent are constants).  The one- / two- / four-lane kernels (bls.hip) run
those operations one after another on a lane or a few; a COMMIT round's ~25
checks then take 18-19 ms although the GPU is nearly idle.  Here the whole
check -- the shared Miller loop of e(sig, g) * e(-H(m), vk) and the final
exponentiation -- is traced once into a dependency graph, list-scheduled into
steps of at most 64 independent operations (one per lane), and register-
allocated into LDS slots.  edv_bls_verify_wave_kernel (bls.hip) runs one wave
per check: each step, every lane executes its operation (a Montgomery product,
a sum or difference, an inversion, or a degenerate-case test) on LDS slots.

What is traced (bn254.h is the per-lane form of the same algorithm, and the
oracle the reference of the result):
  * inputs: P1 = sig and P2 = H(m) affine in G1 (decode and hash stay per-lane
    code in the kernel's prologue); Q1 = generator, Q2 = the verkeys' sum,
    Jacobian on the twist (no inversion before the loop: lines through a
    Jacobian Q are scaled by Fp2 factors of Q's Z, which the final
    exponentiation removes, like bn254.h's own line scalings);
  * one accumulator for both Miller loops: f <- f^2 * l1 * l2 per bit (the
    two lines multiplied together first), conjugation for x < 0, the lines
    through pi(Q) and -pi^2(Q) -- the product of bn254.h's two
    miller_loop_acc values;
  * final_exp as in bn254.h (easy part with one Fp inversion -- a binary
    extended gcd on one lane --, hard part through t^x, t^(x^2), t^(x^3));
  * degenerate cases bn254.h's general Jacobian addition handles with
    branches (T at infinity before a step, T = +-Q at an addition) are
    flagged (ZCHK), and the kernel re-runs a flagged check on the four-lane
    kernel -- so every verdict is bn254.h's.  They need a verkey sum outside
    the order-r subgroup; valid inputs never flag.

Self-check (python tools/gen_bls_program.py --check): the scheduled, slot-
allocated program is simulated step by step (every lane's operands read
before any lane writes, as on the device) and its result compared with the
oracle's reduced pairing product e(P1, Q1) e(-P2, Q2).  tests/test_bls_program.py
runs the same comparison.

usage: python3 tools/gen_bls_program.py [--out PATH] [--check N] [--stats]
"""
import argparse
import os
import random
import sys

BN_X = -0x4080000000000001
P = 36 * BN_X ** 4 + 36 * BN_X ** 3 + 24 * BN_X ** 2 + 6 * BN_X + 1
R_ORDER = 36 * BN_X ** 4 + 36 * BN_X ** 3 + 18 * BN_X ** 2 + 6 * BN_X + 1
ATE = abs(6 * BN_X + 2)
MONT = 1 << 256
LANES = 64

# operation kinds (bls.hip kBlsOp*)
NOP, MUL, ADD, SUB, INV, ZCHK = 0, 1, 2, 3, 4, 5
IN, CONST = 100, 101
HEAVY = (MUL, INV)


class Graph:
    """Hash-consed dependency graph of Fp operations with constant folding.
    With concrete input values bound, every node also carries its value (the
    structure never depends on them)."""

    def __init__(self, values=None):
        self.kind, self.args, self.val = [], [], []
        self.memo, self.consts, self.inputs = {}, {}, {}
        self.checks = []
        self.values = values  # input name -> int, or None

    def _node(self, kind, args, v):
        key = (kind, tuple(sorted(args)) if kind in (MUL, ADD) else tuple(args))
        n = self.memo.get(key)
        if n is None:
            n = len(self.kind)
            self.kind.append(kind)
            self.args.append(tuple(args))
            self.val.append(v)
            self.memo[key] = n
        return n

    def const(self, v):
        v %= P
        n = self.consts.get(v)
        if n is None:
            n = len(self.kind)
            self.kind.append(CONST)
            self.args.append(())
            self.val.append(v)
            self.consts[v] = n
        return n

    def inp(self, name):
        n = len(self.kind)
        self.kind.append(IN)
        self.args.append(())
        self.val.append(None if self.values is None else self.values[name] % P)
        self.inputs[name] = n
        return n

    def cval(self, n):
        return self.val[n] if self.kind[n] == CONST else None

    def _v(self, f, *ns):
        if self.values is None:
            return None
        return f(*[self.val[n] for n in ns]) % P

    def mul(self, a, b):
        ca, cb = self.cval(a), self.cval(b)
        if ca is not None and cb is not None:
            return self.const(ca * cb)
        if ca == 0 or cb == 0:
            return self.const(0)
        if ca == 1:
            return b
        if cb == 1:
            return a
        return self._node(MUL, (a, b), self._v(lambda x, y: x * y, a, b))

    def add(self, a, b):
        ca, cb = self.cval(a), self.cval(b)
        if ca is not None and cb is not None:
            return self.const(ca + cb)
        if ca == 0:
            return b
        if cb == 0:
            return a
        return self._node(ADD, (a, b), self._v(lambda x, y: x + y, a, b))

    def sub(self, a, b):
        ca, cb = self.cval(a), self.cval(b)
        if ca is not None and cb is not None:
            return self.const(ca - cb)
        if cb == 0:
            return a
        if a == b:
            return self.const(0)
        return self._node(SUB, (a, b), self._v(lambda x, y: x - y, a, b))

    def neg(self, a):
        return self.sub(self.const(0), a)

    def inv(self, a):
        ca = self.cval(a)
        if ca is not None:
            return self.const(pow(ca, P - 2, P))
        return self._node(INV, (a,), self._v(lambda x: pow(x, P - 2, P), a))

    def zchk(self, a, b):
        """Flag the check when a == 0 and b == 0 (an Fp2 value is zero)."""
        n = self._node(ZCHK, (a, b), None)
        if n not in self.checks:
            self.checks.append(n)


# ---------------------------------------------------------------- tower (bn254.h's, traced)
class F2:
    __slots__ = ("a", "b")

    def __init__(self, a, b):
        self.a, self.b = a, b

    def __add__(s, o):
        return F2(G.add(s.a, o.a), G.add(s.b, o.b))

    def __sub__(s, o):
        return F2(G.sub(s.a, o.a), G.sub(s.b, o.b))

    def neg(s):
        return F2(G.neg(s.a), G.neg(s.b))

    def dbl(s):
        return s + s

    def conj(s):
        return F2(s.a, G.neg(s.b))

    def __mul__(s, o):  # schoolbook: 4 products, no pre-sums on the critical path
        return F2(G.sub(G.mul(s.a, o.a), G.mul(s.b, o.b)), G.add(G.mul(s.a, o.b), G.mul(s.b, o.a)))

    def sqr(s):  # a^2 - b^2, 2ab
        ab = G.mul(s.a, s.b)
        return F2(G.sub(G.mul(s.a, s.a), G.mul(s.b, s.b)), G.add(ab, ab))

    def mul_fp(s, k):
        return F2(G.mul(s.a, k), G.mul(s.b, k))

    def mul_xi(s):  # (a + b i)(1 + i)
        return F2(G.sub(s.a, s.b), G.add(s.a, s.b))

    def iszero_check(s):
        G.zchk(s.a, s.b)


def f2c(v):
    return F2(G.const(v[0]), G.const(v[1]))


def F2ZERO():
    return F2(G.const(0), G.const(0))


def F2ONE():
    return F2(G.const(1), G.const(0))


class F6:
    __slots__ = ("c0", "c1", "c2")

    def __init__(self, c0, c1, c2):
        self.c0, self.c1, self.c2 = c0, c1, c2

    def __add__(s, o):
        return F6(s.c0 + o.c0, s.c1 + o.c1, s.c2 + o.c2)

    def __sub__(s, o):
        return F6(s.c0 - o.c0, s.c1 - o.c1, s.c2 - o.c2)

    def neg(s):
        return F6(s.c0.neg(), s.c1.neg(), s.c2.neg())

    def mul_v(s):
        return F6(s.c2.mul_xi(), s.c0, s.c1)

    def __mul__(x, y):  # Karatsuba over v^3 = xi: 6 Fp2 products (bn254.h fp6_mul)
        t0, t1, t2 = x.c0 * y.c0, x.c1 * y.c1, x.c2 * y.c2
        c0 = ((x.c1 + x.c2) * (y.c1 + y.c2) - t1 - t2).mul_xi() + t0
        c1 = (x.c0 + x.c1) * (y.c0 + y.c1) - t0 - t1 + t2.mul_xi()
        c2 = (x.c0 + x.c2) * (y.c0 + y.c2) - t0 - t2 + t1
        return F6(c0, c1, c2)

    def mul_01(a, b0, b1):  # a * (b0 + b1 v) (bn254.h fp6_mul_01)
        t0, t1 = a.c0 * b0, a.c1 * b1
        c0 = t0 + (a.c2 * b1).mul_xi()
        c1 = (a.c0 + a.c1) * (b0 + b1) - t0 - t1
        c2 = a.c2 * b0 + t1
        return F6(c0, c1, c2)

    def inv(x):  # bn254.h fp6_inv
        t0 = x.c0.sqr() - (x.c1 * x.c2).mul_xi()
        t1 = x.c2.sqr().mul_xi() - x.c0 * x.c1
        t2 = x.c1.sqr() - x.c0 * x.c2
        d = (x.c2 * t1 + x.c1 * t2).mul_xi() + x.c0 * t0
        # Fp2 inverse: (a - b i) / (a^2 + b^2)
        n = G.add(G.mul(d.a, d.a), G.mul(d.b, d.b))
        ni = G.inv(n)
        di = F2(G.mul(d.a, ni), G.neg(G.mul(d.b, ni)))
        return F6(t0 * di, t1 * di, t2 * di)


def F6ZERO():
    return F6(F2ZERO(), F2ZERO(), F2ZERO())


class F12:
    __slots__ = ("c0", "c1")

    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    @staticmethod
    def one():
        return F12(F6(F2ONE(), F2ZERO(), F2ZERO()), F6ZERO())

    def __mul__(x, y):  # 3 Fp6 products (bn254.h fp12_mul)
        t0, t1 = x.c0 * y.c0, x.c1 * y.c1
        c1 = (x.c0 + x.c1) * (y.c0 + y.c1) - t0 - t1
        return F12(t0 + t1.mul_v(), c1)

    def sqr(x):  # complex squaring (bn254.h fp12_sqr)
        ab = x.c0 * x.c1
        s = (x.c0 + x.c1) * (x.c0 + x.c1.mul_v())
        return F12(s - ab - ab.mul_v(), ab + ab)

    def conj(x):
        return F12(x.c0, x.c1.neg())

    def inv(x):  # (a - b w) / (a^2 - v b^2)
        t = (x.c0 * x.c0 - (x.c1 * x.c1).mul_v()).inv()
        return F12(x.c0 * t, (x.c1 * t).neg())

    def frob(x):  # bn254.h fp12_frob
        return F12(F6(x.c0.c0.conj(), x.c0.c1.conj() * f2c(GAMMA[2]), x.c0.c2.conj() * f2c(GAMMA[4])),
                   F6(x.c1.c0.conj() * f2c(GAMMA[1]), x.c1.c1.conj() * f2c(GAMMA[3]),
                      x.c1.c2.conj() * f2c(GAMMA[5])))

    def cyclo_sqr(x):  # Granger-Scott (bn254.h fp12_cyclo_sqr)
        def fp4_sqr(a, b):
            a2, b2, ab = a.sqr(), b.sqr(), a * b
            return a2 + b2.mul_xi(), ab + ab

        def m2z(t, z):  # 3t - 2z
            d = t - z
            return d + d + t

        def p2z(t, z):  # 3t + 2z
            d = t + z
            return d + d + t
        t0, t1 = fp4_sqr(x.c0.c0, x.c1.c1)
        t2, t3 = fp4_sqr(x.c1.c0, x.c0.c2)
        t4, t5 = fp4_sqr(x.c0.c1, x.c1.c2)
        return F12(F6(m2z(t0, x.c0.c0), m2z(t2, x.c0.c1), m2z(t4, x.c0.c2)),
                   F6(p2z(t5.mul_xi(), x.c1.c0), p2z(t1, x.c1.c1), p2z(t3, x.c1.c2)))

    def mul_line(f, l0, l1, l2):  # f * (l0 + (l1 + l2 v) w) (bn254.h fp12_mul_line)
        aA = F6(f.c0.c0 * l0, f.c0.c1 * l0, f.c0.c2 * l0)
        bB = f.c1.mul_01(l1, l2)
        s = (f.c0 + f.c1).mul_01(l0 + l1, l2)
        return F12(aA + bB.mul_v(), s - aA - bB)


def line_product(l, m):
    """(l0 + (l1 + l2 v) w)(m0 + (m1 + m2 v) w) as a full Fp12 (8 Fp2 products)."""
    l0, l1, l2 = l
    m0, m1, m2 = m
    # w^2 = v: (l1 + l2 v)(m1 + m2 v) v = (xi l2 m2) + (l1 m1) v + (l1 m2 + l2 m1) v^2 ... times v
    p11, p22 = l1 * m1, l2 * m2
    p12 = l1 * m2 + l2 * m1
    c0 = F6(l0 * m0 + p22.mul_xi(), p11, p12)
    c1 = F6(l0 * m1 + m0 * l1, l0 * m2 + m0 * l2, F2ZERO())
    return F12(c0, c1)


def xi_pow(e):
    r, b = (1, 0), (1, 1)

    def m(x, y):
        return ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)
    while e:
        if e & 1:
            r = m(r, b)
        b = m(b, b)
        e >>= 1
    return r


GAMMA = [xi_pow(e * (P - 1) // 6) for e in range(6)]


# ---------------------------------------------------------------- the pairing check
class Jac:
    def __init__(self, X, Y, Z):
        self.X, self.Y, self.Z = X, Y, Z


def line_dbl(T, xP, yP):
    """bn254.h miller_dbl: the tangent line at T (scaled) and T <- 2T."""
    T.Z.iszero_check()  # T at infinity: bn254.h keeps T (branch) -- the four-lane kernel redoes the check
    A, B, ZZ, YZ = T.X.sqr(), T.Y.sqr(), T.Z.sqr(), T.Y * T.Z
    l0 = (YZ * ZZ).dbl().mul_fp(yP)
    E = A.dbl() + A
    l1 = (E * ZZ).mul_fp(xP).neg()
    l2 = E * T.X - B.dbl()
    C = B.sqr()
    t = (T.X + B).sqr() - A - C
    D = t.dbl()
    F = E.sqr()
    Z3 = YZ.dbl()
    X3 = F - D - D
    C8 = C.dbl().dbl().dbl()
    Y3 = E * (D - X3) - C8
    return (l0, l1, l2), Jac(X3, Y3, Z3)


def line_add(T, Q, Qzz, Qzzz, xP, yP):
    """bn254.h miller_add for a Jacobian Q = (Xq, Yq, Zq): the line through T
    and Q scaled by Zq^2 (Zq = 1 gives bn254.h's line) and T <- T + Q by the
    general Jacobian addition (its non-degenerate branch)."""
    T.Z.iszero_check()
    ZZ = T.Z.sqr()
    ZZZ = ZZ * T.Z
    U1, U2 = T.X * Qzz, Q.X * ZZ
    S1, S2 = T.Y * Qzzz, Q.Y * ZZZ
    H = U2 - U1    # eps' = (xQ Z^2 - X) Zq^2
    Rr = S2 - S1   # theta' = (yQ Z^3 - Y) Zq^3
    H.iszero_check()  # T = +-Q: bn254.h doubles or returns infinity (branch)
    k = T.Z * H
    l0 = (k * Qzzz).mul_fp(yP)
    l1 = (Rr * Qzz).mul_fp(xP).neg()
    l2 = Rr * Q.X - k * Q.Y
    HH = H.sqr()
    HHH = HH * H
    V = U1 * HH
    X3 = Rr.sqr() - HHH - V - V
    Y3 = Rr * (V - X3) - S1 * HHH
    Z3 = k * Q.Z
    return (l0, l1, l2), Jac(X3, Y3, Z3)


def twist_frob(Q):
    """pi on the twist, Jacobian: (conj(X) gamma_2, conj(Y) gamma_3, conj(Z))."""
    return Jac(Q.X.conj() * f2c(GAMMA[2]), Q.Y.conj() * f2c(GAMMA[3]), Q.Z.conj())


def miller_shared(pairs):
    """prod over (xP, yP, Q) of bn254.h's miller_loop_acc, one accumulator."""
    f = F12.one()
    Ts = [Jac(Q.X, Q.Y, Q.Z) for _, _, Q in pairs]
    pre = [(Q.Z.sqr(), None) for _, _, Q in pairs]
    pre = [(zz, zz * Q.Z) for (zz, _), (_, _, Q) in zip(pre, pairs)]

    def mul_lines(f, lines):
        acc = line_product(lines[0], lines[1]) if len(lines) == 2 else None
        if acc is None:
            return f.mul_line(*lines[0])
        return f * acc
    for bit in bin(ATE)[3:]:
        f = f.sqr()
        lines = []
        for k, (xP, yP, Q) in enumerate(pairs):
            l, Ts[k] = line_dbl(Ts[k], xP, yP)
            lines.append(l)
        f = mul_lines(f, lines)
        if bit == "1":
            lines = []
            for k, (xP, yP, Q) in enumerate(pairs):
                l, Ts[k] = line_add(Ts[k], Q, pre[k][0], pre[k][1], xP, yP)
                lines.append(l)
            f = mul_lines(f, lines)
    f = f.conj()  # x < 0
    Ts = [Jac(T.X, T.Y.neg(), T.Z) for T in Ts]
    for step in range(2):
        lines = []
        for k, (xP, yP, Q) in enumerate(pairs):
            Q1 = twist_frob(Q)
            Qs = Q1 if step == 0 else twist_frob(Q1)
            if step == 1:
                Qs = Jac(Qs.X, Qs.Y.neg(), Qs.Z)
            zz = Qs.Z.sqr()
            l, Ts[k] = line_add(Ts[k], Qs, zz, zz * Qs.Z, xP, yP)
            lines.append(l)
        f = mul_lines(f, lines)
    return f


def pow_x(f):  # bn254.h fp12_pow_x: |x| = 2^62 + 2^55 + 1, conjugated (x < 0)
    acc = f
    for bit in range(61, -1, -1):
        acc = acc.cyclo_sqr()
        if bit in (55, 0):
            acc = acc * f
    return acc.conj()


def pow_small(f, k):
    acc = f
    for bit in range(k.bit_length() - 2, -1, -1):
        acc = acc.cyclo_sqr()
        if (k >> bit) & 1:
            acc = acc * f
    return acc


def final_exp(f):  # bn254.h final_exp, the same chain
    t = f.conj() * f.inv()
    t = t.frob().frob() * t
    a = pow_x(t)
    b = pow_x(a)
    c = pow_x(b)
    c36 = pow_small(c, 36)
    b6 = (b.cyclo_sqr() * b).cyclo_sqr()
    b12 = b6.cyclo_sqr()
    b18 = b12 * b6
    a6 = (a.cyclo_sqr() * a).cyclo_sqr()
    a12 = a6.cyclo_sqr()
    y = b18 * b12 * c36 * (a12 * a6) * t.cyclo_sqr()
    res = y.conj()
    y = (b18 * c36 * a12).conj() * t
    res = res * y.frob()
    y = b6 * t
    res = res * y.frob().frob()
    y = t.frob().frob().frob()
    return res * y


INPUTS = ["xP1", "yP1", "xP2", "yP2"] + ["Q%d%s%s" % (q, c, h) for q in (1, 2) for c in "XYZ" for h in "ab"]


def build(values=None):
    """The check's graph: e = FE(ML(P1, Q1) ML(-P2, Q2)); returns (graph, the 12 output nodes)."""
    global G
    G = Graph(values)
    n = {k: G.inp(k) for k in INPUTS}
    Qs = [Jac(F2(n["Q%dXa" % q], n["Q%dXb" % q]), F2(n["Q%dYa" % q], n["Q%dYb" % q]),
              F2(n["Q%dZa" % q], n["Q%dZb" % q])) for q in (1, 2)]
    pairs = [(n["xP1"], n["yP1"], Qs[0]), (n["xP2"], G.neg(n["yP2"]), Qs[1])]
    e = final_exp(miller_shared(pairs))
    outs = []
    for c6 in (e.c0, e.c1):
        for c2 in (c6.c0, c6.c1, c6.c2):
            outs += [c2.a, c2.b]
    return G, outs


# ---------------------------------------------------------------- fuse, schedule, slots
LIN = 6        # signed sum of up to MAX_TERMS slots (device kind kLin)
MAX_TERMS = 12  # terms per operation (signed sums; a product: two sums of at most 2)


class Op:
    """A device operation: MUL = (sum A) * (sum B); LIN = sum A; INV = A[0]^-1;
    ZCHK = flag if A[0] == A[1] == 0.  A, B: lists of (node, negated)."""
    __slots__ = ("kind", "A", "B")

    def __init__(self, kind, A, B=()):
        self.kind, self.A, self.B = kind, list(A), list(B)

    def args(self):
        return [t for t, _ in self.A] + [t for t, _ in self.B]


def fuse(g, outs, mul_terms=2, dup=True):
    """Collapse sums and differences into LIN operations of up to MAX_TERMS
    signed terms: an operand that is itself a sum is expanded in place when
    the terms fit (dup: even when other operations read it too -- the lanes
    are mostly idle, the steps are not); one- or two-term sums are folded into
    a product's operands (Karatsuba's pre-sums) when mul_terms >= 2.  Only
    what the outputs and zero tests reach through the final terms is kept.
    Returns (ops: node -> Op in topological order, outs with aliases resolved)."""
    need, stack = set(), list(outs) + list(g.checks)
    while stack:
        x = stack.pop()
        if x in need or g.kind[x] in (IN, CONST):
            continue
        need.add(x)
        stack.extend(g.args[x])
    order = sorted(need)
    fan = {}
    for x in order:
        for a in g.args[x]:
            fan[a] = fan.get(a, 0) + 1
    out_set = set(outs)
    zero = g.consts.get(0)
    expr, alias, sides = {}, {}, {}

    def res(y):
        while y in alias:
            y = alias[y]
        return y

    def size(e):
        return sum(abs(c) for c in e.values())

    def operand(y, limit):
        y = res(y)
        if y in expr and (dup or fan.get(y, 0) == 1) and size(expr[y]) <= limit:
            return dict(expr[y])
        return {y: 1}

    def combine(ea, eb, sign):
        e = dict(ea)
        for t, c in eb.items():
            e[t] = e.get(t, 0) + sign * c
        return {t: c for t, c in e.items() if c != 0 and t != zero}

    for x in order:
        k = g.kind[x]
        if k in (ADD, SUB):
            a, b = g.args[x]
            sign = 1 if k == ADD else -1
            e = None
            for ta, tb in ((True, True), (True, False), (False, True), (False, False)):
                ea = operand(a, MAX_TERMS) if ta else {res(a): 1}
                eb = operand(b, MAX_TERMS) if tb else {res(b): 1}
                e = combine(ea, eb, sign)
                if size(e) <= MAX_TERMS:
                    break
            if not e:
                alias[x] = zero if zero is not None else g.const(0)
            elif len(e) == 1 and list(e.values())[0] == 1:
                alias[x] = list(e)[0]
            else:
                expr[x] = e
        elif k == MUL:
            sides[x] = [operand(y, mul_terms) if mul_terms >= 2 else {res(y): 1} for y in g.args[x]]

    def terms(e):
        t = []
        for n, c in sorted(e.items()):
            t += [(n, c < 0)] * abs(c)
        return t

    def op_of(x):
        if x in expr:
            return Op(LIN, terms(expr[x]))
        k = g.kind[x]
        if k == MUL:
            return Op(MUL, terms(sides[x][0]), terms(sides[x][1]))
        if k == INV:
            return Op(INV, [(res(g.args[x][0]), False)])
        if k == ZCHK:
            return Op(ZCHK, [(res(g.args[x][0]), False), (res(g.args[x][1]), False)])
        raise AssertionError(k)
    outs = [res(o) for o in outs]
    keep, stack = {}, list(outs) + list(g.checks)
    while stack:
        x = stack.pop()
        if x in keep or g.kind[x] in (IN, CONST):
            continue
        keep[x] = op_of(x)
        stack.extend(keep[x].args())
    return {x: keep[x] for x in sorted(keep)}, outs


def _is_heavy(op):
    return op.kind in HEAVY


RIDERS = True  # heavy steps also take ready sums (--no-riders: products only)
MUL_WEIGHT = 6.0  # a product's cost in light steps, for the critical-path priorities (--mul-weight)


def schedule(ops, outs):
    """List scheduling into steps of <= LANES operations.  A step whose best
    ready operation is a product (or inversion) is a heavy step and takes
    every kind of ready operation (RIDERS) or only products; otherwise only
    light ones (sums, zero tests) -- a product costs ~2 light steps."""
    w = {MUL: MUL_WEIGHT, INV: 40.0, LIN: 1.0, ZCHK: 1.0}
    order = list(ops)  # topological
    users = {x: [] for x in order}
    for x in order:
        for a in set(ops[x].args()):
            if a in users:
                users[a].append(x)
    prio = {}
    for x in reversed(order):
        op = ops[x]
        c = w[op.kind] + (0.05 * len(op.A) if op.kind == LIN else 0)
        prio[x] = c + max((prio[u] for u in users[x]), default=0)
    pending = {x: len([a for a in set(ops[x].args()) if a in users]) for x in order}
    import heapq
    heap_h, heap_l = [], []
    for x in order:
        if pending[x] == 0:
            heapq.heappush(heap_h if _is_heavy(ops[x]) else heap_l, (-prio[x], x))
    steps = []
    while heap_h or heap_l:
        best_h = -heap_h[0][0] if heap_h else -1
        best_l = -heap_l[0][0] if heap_l else -1
        take = []
        heavy = best_h >= best_l
        if heavy:
            while heap_h and len(take) < LANES:
                take.append(heapq.heappop(heap_h)[1])
        if RIDERS or not heavy:
            while heap_l and len(take) < LANES:
                take.append(heapq.heappop(heap_l)[1])
        steps.append(take)
        for x in take:
            for u in users[x]:
                pending[u] -= 1
                if pending[u] == 0:
                    heapq.heappush(heap_h if _is_heavy(ops[u]) else heap_l, (-prio[u], u))
    return steps


def allocate(g, ops, outs, steps):
    """LDS slots: inputs and constants pinned; an operation's result lives from
    its step to its last reader's step, and its slot is reused from the step
    after that (never within a step)."""
    last = {}
    for s, st in enumerate(steps):
        for x in st:
            for a in ops[x].args():
                last[a] = max(last.get(a, -1), s)
    for o in outs:
        last[o] = len(steps)
    slot = {}
    nxt = 0
    pinned = [x for x in range(len(g.kind)) if g.kind[x] in (IN, CONST) and
              (x in last or x in g.inputs.values() or x == ZERO_NODE)]
    for x in pinned:
        slot[x] = nxt
        nxt += 1
    import heapq
    free = []
    release_at = {}
    for x, s in last.items():
        if x in ops:
            release_at.setdefault(s, []).append(x)
    for s, st in enumerate(steps):
        for x in st:
            if ops[x].kind == ZCHK:
                continue
            slot[x] = heapq.heappop(free) if free else nxt
            if slot[x] == nxt:
                nxt += 1
        for x in release_at.get(s, ()):
            if x in slot:
                heapq.heappush(free, slot[x])
        for x in st:
            if ops[x].kind != ZCHK and x not in last:
                heapq.heappush(free, slot[x])
    return slot, nxt, pinned


def op_words():
    """32-bit words per operation: the header, then 16-bit fields dst, t0 .. t(MAX_TERMS-1); a
    multiple of 4 (16-byte loads)."""
    return -(-(1 + (MAX_TERMS + 2) // 2) // 4) * 4


def encode(ops, steps, slot):
    """Per operation: kind | nA << 4 | nB << 8 | negated-term mask << 12 (terms A then B),
    then dst and the term slots, two 16-bit fields a word."""
    words, starts = [], [0]
    for st in steps:
        for x in st:
            op = ops[x]
            # a product's two sums sit at fixed fields (terms 0-1 and 2-3), so the device reads every
            # field at a compile-time position (a run-time index into the words would put them in
            # scratch memory)
            # unused term fields name the constant-zero slot: the device sums every field of a sum
            # unconditionally (all operand loads issued at once, no branch per term)
            if op.kind == MUL:
                t = op.A + [(ZERO_NODE, False)] * (2 - len(op.A)) + op.B + [(ZERO_NODE, False)] * (2 - len(op.B))
            elif op.kind == LIN:
                t = op.A + [(ZERO_NODE, False)] * (MAX_TERMS - len(op.A))
            else:
                t = op.A + op.B
            assert len(t) <= MAX_TERMS and len(op.A) < 16 and len(op.B) < 16
            neg = 0
            for i, (_, ng) in enumerate(t):
                neg |= int(ng) << i
            halves = [slot.get(x, 0) if op.kind != ZCHK else 0] + [slot[n] for n, _ in t]
            halves += [0] * (2 * (op_words() - 1) - len(halves))
            w = [op.kind | (len(op.A) << 4) | (len(op.B) << 8) | (neg << 12)]
            w += [halves[2 * i] | (halves[2 * i + 1] << 16) for i in range(op_words() - 1)]
            words.append(tuple(w))
        starts.append(len(words))
    return words, starts


def simulate(g, ops, steps, slot, nslots, values):
    """The allocated program on concrete values (plain integers mod p; the
    device's Montgomery form maps onto it exactly).  Returns (slots, flag)."""
    mem = [None] * nslots
    for name, x in g.inputs.items():
        mem[slot[x]] = values[name] % P
    for v, x in g.consts.items():
        if x in slot:
            mem[slot[x]] = v

    def lsum(terms):
        acc = 0
        for n, ng in terms:
            v = mem[slot[n]]
            if v is None:
                raise AssertionError("read of an unwritten slot")
            acc += -v if ng else v
        return acc % P
    flag = False
    for st in steps:
        writes = []
        for x in st:
            op = ops[x]
            if op.kind == MUL:
                writes.append((slot[x], lsum(op.A) * lsum(op.B) % P))
            elif op.kind == LIN:
                writes.append((slot[x], lsum(op.A)))
            elif op.kind == INV:
                writes.append((slot[x], pow(lsum(op.A), P - 2, P)))
            elif op.kind == ZCHK:
                flag = flag or (lsum(op.A[:1]) == 0 and lsum(op.A[1:]) == 0)
        for s_, v in writes:
            mem[s_] = v
    return mem, flag


def estimate_us(ops, steps, clock_ghz=2.1):
    """Rough device time: a heavy step ~2,900 cycles (+250 when a lane sums a
    product's operands), a light one ~450 + 60 per term of its longest sum."""
    cyc = 0
    for st in steps:
        if any(ops[x].kind == INV for x in st):
            cyc += 150000
        elif any(ops[x].kind == MUL for x in st):
            cyc += 2900 + (250 if any(len(ops[x].A) + len(ops[x].B) > 2 for x in st if ops[x].kind == MUL) else 0)
        else:
            cyc += 450 + 60 * max(len(ops[x].A) for x in st)
    return cyc / clock_ghz / 1e3


ZERO_NODE = None


def compile_program(mul_terms=2, dup=True):
    global ZERO_NODE
    g, outs = build()
    ZERO_NODE = g.const(0)
    ops, outs = fuse(g, outs, mul_terms, dup)
    steps = schedule(ops, outs)
    slot, nslots, pinned = allocate(g, ops, outs, steps)
    return g, ops, outs, steps, slot, nslots, pinned


# ---------------------------------------------------------------- emit
def limbs(v):
    return [(v >> (32 * k)) & 0xffffffff for k in range(8)]


def mont(v):
    return v * MONT % P


def emit(prog):
    g, ops, outs, steps, slot, nslots, pinned = prog
    words, starts = encode(ops, steps, slot)
    heavy = sum(1 for st in steps if any(_is_heavy(ops[x]) for x in st))
    n_ops = len(words)
    consts = [(slot[x], g.val[x]) for x in pinned if g.kind[x] == CONST]
    lines = ["// Generated by tools/gen_bls_program.py -- do not edit.",
             "// The BLS pairing check FE(ML(sig, g) * ML(-H(m), vk)) as a straight-line program of Fp",
             "// operations over the 64 lanes of a wave (edv_bls_verify_wave_kernel, bls.hip).",
             "// %d steps (%d with products), %d operations, %d LDS slots." % (len(steps), heavy, n_ops, nslots),
             "#pragma once", "#include <stdint.h>",
             "#if defined(__HIPCC__)", "#define EDV_BLSP_CONST __device__ static const", "#else",
             "#define EDV_BLSP_CONST static const", "#endif",
             "namespace edv {", "namespace blsp {",
             "enum : uint32_t { kNop = %d, kMul = %d, kInv = %d, kZchk = %d, kLin = %d };" % (NOP, MUL, INV, ZCHK, LIN),
             "constexpr int kMaxTerms = %d;" % MAX_TERMS,
             "constexpr int kOpWords = %d;" % op_words(),
             "constexpr int kSteps = %d;" % len(steps),
             "constexpr int kOps = %d;" % n_ops,
             "constexpr int kSlots = %d;" % nslots,
             "constexpr int kConsts = %d;" % len(consts)]
    for name in INPUTS:
        lines.append("constexpr int kIn_%s = %d;" % (name, slot[g.inputs[name]]))
    lines.append("EDV_BLSP_CONST uint16_t kOut[12] = {%s};" % ", ".join(str(slot[o]) for o in outs))
    lines.append("// 8p, 4p, 2p, p as 9 limbs: a signed sum's reduction (sums < 16p)")
    pm = []
    for k in (8, 4, 2, 1):
        pm += [((k * P) >> (32 * j)) & 0xffffffff for j in range(9)]
    lines.append("EDV_BLSP_CONST uint32_t kPMul[36] = {%s};" % ", ".join("0x%08xu" % w for w in pm))
    kp = []
    for k in range(MAX_TERMS + 1):
        kp += [((k * (P + 1)) >> (32 * j)) & 0xffffffff for j in range(9)]
    lines.append("// k (p + 1), k = 0 .. kMaxTerms, as 9 limbs: a signed sum's correction for its k negated terms")
    lines.append("EDV_BLSP_CONST uint32_t kKP1[%d] = {%s};" % (len(kp), ", ".join("0x%08xu" % w for w in kp)))
    lines.append("// R^3 mod p (plain): Montgomery inverse = plain inverse * R^3 / R")
    lines.append("EDV_BLSP_CONST uint32_t kR3[8] = {%s};" % ", ".join("0x%08xu" % w for w in limbs(MONT ** 3 % P)))
    lines.append("EDV_BLSP_CONST uint16_t kConstSlot[%d] = {%s};" % (max(1, len(consts)),
                                                                    ", ".join(str(s) for s, _ in consts) or "0"))
    cv = []
    for _, v in consts:
        cv += limbs(mont(v))
    lines.append("EDV_BLSP_CONST uint32_t kConstVal[%d] = {" % max(8, len(cv)))
    for i in range(0, len(cv), 8):
        lines.append("    " + ", ".join("0x%08xu" % w for w in cv[i:i + 8]) + ",")
    lines.append("};")
    lines.append("// operations [kStep[s], kStep[s + 1]) of step s, lane = index - kStep[s]")
    lines.append("EDV_BLSP_CONST uint32_t kStep[%d] = {" % (len(starts)))
    for i in range(0, len(starts), 16):
        lines.append("    " + ", ".join(str(v) for v in starts[i:i + 16]) + ",")
    lines.append("};")
    lines.append("// per operation (kOpWords words): kind | nA << 4 | nB << 8 | negated-term mask << 12; then")
    lines.append("// dst, t0, t1, ... two 16-bit fields a word -- LIN: the signed sum of terms 0..nA-1; MUL:")
    lines.append("// (sum of terms 0..nA-1) * (sum of terms 2..2+nB-1); INV: t0^-1; ZCHK: flag if t0 == t1 == 0")
    lines.append("EDV_BLSP_CONST uint32_t kOp[%d] __attribute__((aligned(16))) = {" % (op_words() * n_ops))
    flat = [w for pair in words for w in pair]
    for i in range(0, len(flat), 18):
        lines.append("    " + ",".join("0x%x" % v for v in flat[i:i + 18]) + ",")
    lines.append("};")
    lines += ["}  // namespace blsp", "}  // namespace edv", ""]
    return "\n".join(lines)


# ---------------------------------------------------------------- self-check against the oracle
def _oracle():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import bls_bn254_oracle as o
    return o


def check(prog, trials=2, seed=1):
    """Simulate the allocated program on random inputs (Q2 a sum of two keys:
    Jacobian with Z != 1) and compare with the oracle's reduced pairings."""
    o = _oracle()
    g, ops, outs, steps, slot, nslots, pinned = prog
    rng = random.Random(seed)
    gen = o.generator()
    for t in range(trials):
        p1 = o.g1_mul(o.hash_to_g1(b"p1 %d" % t), rng.randrange(1, R_ORDER))
        p2 = o.hash_to_g1(b"p2 %d" % t)
        q1 = o.g2_mul(gen, rng.randrange(1, R_ORDER))
        # Q2 = k1 g + k2 g in Jacobian coordinates with a random Z
        q2 = o.g2_mul(gen, rng.randrange(1, R_ORDER))
        z = (rng.randrange(1, P), rng.randrange(P))
        vals = {"xP1": p1[0], "yP1": p1[1], "xP2": p2[0], "yP2": p2[1]}
        for q, pt, zz in ((1, q1, (1, 0)), (2, q2, z)):
            X, Y = _jac2(pt, zz)
            vals.update({"Q%dXa" % q: X[0], "Q%dXb" % q: X[1], "Q%dYa" % q: Y[0], "Q%dYb" % q: Y[1],
                         "Q%dZa" % q: zz[0], "Q%dZb" % q: zz[1]})
        mem, flag = simulate(g, ops, steps, slot, nslots, vals)
        got = [mem[slot[x]] for x in outs]
        want = o.f12_to_tower(o.pairing(p1, q1) * o.pairing(o.g1_neg(p2), q2))
        assert not flag, "valid inputs flagged"
        assert got == want, "program result != oracle pairing product (trial %d)" % t
    return True


def _jac2(pt, z):
    """Affine twist point -> Jacobian (x z^2, y z^3, z) over Fp2."""
    def m(x, y):
        return ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)
    z2 = m(z, z)
    z3 = m(z2, z)
    return m((pt[0].a, pt[0].b), z2), m((pt[1].a, pt[1].b), z3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--check", type=int, default=0)
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--mul-terms", type=int, default=2)
    ap.add_argument("--max-terms", type=int, default=MAX_TERMS)
    ap.add_argument("--no-riders", action="store_true")
    ap.add_argument("--mul-weight", type=float, default=MUL_WEIGHT)
    a = ap.parse_args()
    globals()["MUL_WEIGHT"] = a.mul_weight
    globals()["MAX_TERMS"] = a.max_terms
    globals()["RIDERS"] = not a.no_riders
    prog = compile_program(a.mul_terms)
    g, ops, outs, steps, slot, nslots, pinned = prog
    if a.stats or not a.out:
        kinds = {}
        for st in steps:
            for x in st:
                kinds[ops[x].kind] = kinds.get(ops[x].kind, 0) + 1
        heavy = sum(1 for st in steps if any(_is_heavy(ops[x]) for x in st))
        print("steps %d (heavy %d, light %d), ops %s, slots %d, estimate %.0f us" % (
            len(steps), heavy, len(steps) - heavy, kinds, nslots, estimate_us(ops, steps)), file=sys.stderr)
    if a.check:
        check(prog, a.check)
        print("check: %d random pairings == oracle" % a.check, file=sys.stderr)
    if a.out:
        text = emit(prog)
        old = open(a.out).read() if os.path.exists(a.out) else None
        if old != text:
            with open(a.out, "w") as f:
                f.write(text)


if __name__ == "__main__":
    main()
