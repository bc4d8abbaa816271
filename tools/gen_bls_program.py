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


# ---------------------------------------------------------------- schedule + slots
def schedule(g, outs, weights=None):
    """List scheduling into steps of <= LANES operations.  A step whose best
    ready operation is a product (or inversion) is a heavy step and takes
    every kind of ready operation; otherwise only light ones (sums,
    differences, zero tests) -- a product costs ~6 light steps."""
    w = weights or {MUL: 6, INV: 40, ADD: 1, SUB: 1, ZCHK: 1}
    need = set()
    stack = list(outs) + list(g.checks)
    while stack:
        x = stack.pop()
        if x in need or g.kind[x] in (IN, CONST):
            continue
        need.add(x)
        stack.extend(g.args[x])
    order = sorted(need)  # node ids are topological (args precede)
    users = {x: [] for x in order}
    for x in order:
        for a in g.args[x]:
            if a in users:
                users[a].append(x)
    prio = {}
    for x in reversed(order):
        prio[x] = w[g.kind[x]] + max((prio[u] for u in users[x]), default=0)
    pending = {x: sum(1 for a in g.args[x] if a in users) for x in order}
    ready = [x for x in order if pending[x] == 0]
    steps = []
    import heapq
    heap_h, heap_l = [], []
    for x in ready:
        heapq.heappush(heap_h if g.kind[x] in HEAVY else heap_l, (-prio[x], x))
    while heap_h or heap_l:
        best_h = -heap_h[0][0] if heap_h else -1
        best_l = -heap_l[0][0] if heap_l else -1
        take = []
        if best_h >= best_l:
            while heap_h and len(take) < LANES:
                take.append(heapq.heappop(heap_h)[1])
        while heap_l and len(take) < LANES:
            take.append(heapq.heappop(heap_l)[1])
        steps.append(take)
        for x in take:
            for u in users[x]:
                pending[u] -= 1
                if pending[u] == 0:
                    heapq.heappush(heap_h if g.kind[u] in HEAVY else heap_l, (-prio[u], u))
    return steps


def allocate(g, outs, steps):
    """LDS slots: inputs and constants pinned; an operation's result lives from
    its step to its last reader's step, and its slot is reused from the step
    after that (never within a step)."""
    step_of = {}
    for s, ops in enumerate(steps):
        for x in ops:
            step_of[x] = s
    last = {}
    for s, ops in enumerate(steps):
        for x in ops:
            for a in g.args[x]:
                last[a] = max(last.get(a, -1), s)
    for o in outs:
        last[o] = len(steps)
    slot = {}
    nxt = 0
    pinned = [x for x in range(len(g.kind)) if g.kind[x] in (IN, CONST) and (x in last or x in g.inputs.values())]
    for x in pinned:
        slot[x] = nxt
        nxt += 1
    free = []
    import heapq
    release_at = {}  # step -> slots freed after it
    for x, s in last.items():
        if x in step_of:
            release_at.setdefault(s, []).append(x)
    for s, ops in enumerate(steps):
        for x in ops:
            if g.kind[x] == ZCHK:
                continue
            if free:
                slot[x] = heapq.heappop(free)
            else:
                slot[x] = nxt
                nxt += 1
        for x in release_at.get(s, ()):
            if x in slot:
                heapq.heappush(free, slot[x])
        # a result nobody reads (none expected) would leak its slot: free it
        for x in ops:
            if g.kind[x] != ZCHK and x not in last:
                heapq.heappush(free, slot[x])
    return slot, nxt, pinned


def encode(g, steps, slot):
    words, starts = [], [0]
    for ops in steps:
        for x in ops:
            k = g.kind[x]
            a = g.args[x]
            dst = slot.get(x, 0) if k != ZCHK else 0
            sa = slot[a[0]]
            sb = slot[a[1]] if len(a) > 1 else 0
            words.append((k | (dst << 8), sa | (sb << 16)))
        starts.append(len(words))
    return words, starts


def simulate(g, steps, slot, nslots, values):
    """The allocated program on concrete values (plain integers mod p; the
    device's Montgomery form maps onto it exactly).  Returns (slots, flag)."""
    mem = [None] * nslots
    for name, x in g.inputs.items():
        mem[slot[x]] = values[name] % P
    for v, x in g.consts.items():
        if x in slot:
            mem[slot[x]] = v
    flag = False
    for ops in steps:
        reads = [[mem[slot[a]] for a in g.args[x]] for x in ops]
        writes = []
        for x, r in zip(ops, reads):
            k = g.kind[x]
            if any(v is None for v in r):
                raise AssertionError("read of an unwritten slot")
            if k == MUL:
                writes.append((slot[x], r[0] * r[1] % P))
            elif k == ADD:
                writes.append((slot[x], (r[0] + r[1]) % P))
            elif k == SUB:
                writes.append((slot[x], (r[0] - r[1]) % P))
            elif k == INV:
                writes.append((slot[x], pow(r[0], P - 2, P)))
            elif k == ZCHK:
                flag = flag or (r[0] == 0 and r[1] == 0)
        for s, v in writes:
            mem[s] = v
    return mem, flag


def compile_program():
    g, outs = build()
    steps = schedule(g, outs)
    slot, nslots, pinned = allocate(g, outs, steps)
    return g, outs, steps, slot, nslots, pinned


# ---------------------------------------------------------------- emit
def limbs(v):
    return [(v >> (32 * k)) & 0xffffffff for k in range(8)]


def mont(v):
    return v * MONT % P


def emit(prog):
    g, outs, steps, slot, nslots, pinned = prog
    words, starts = encode(g, steps, slot)
    heavy = sum(1 for ops in steps if any(g.kind[x] in HEAVY for x in ops))
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
             "enum : uint32_t { kNop = %d, kMul = %d, kAdd = %d, kSub = %d, kInv = %d, kZchk = %d };" % (
                 NOP, MUL, ADD, SUB, INV, ZCHK),
             "constexpr int kSteps = %d;" % len(steps),
             "constexpr int kOps = %d;" % n_ops,
             "constexpr int kSlots = %d;" % nslots,
             "constexpr int kConsts = %d;" % len(consts)]
    for name in INPUTS:
        lines.append("constexpr int kIn_%s = %d;" % (name, slot[g.inputs[name]]))
    lines.append("EDV_BLSP_CONST uint16_t kOut[12] = {%s};" % ", ".join(str(slot[o]) for o in outs))
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
    lines.append("// per operation: kind | dst << 8, a | b << 16")
    lines.append("EDV_BLSP_CONST uint32_t kOp[%d] = {" % (2 * n_ops))
    flat = [w for pair in words for w in pair]
    for i in range(0, len(flat), 12):
        lines.append("    " + ",".join("0x%x" % v for v in flat[i:i + 12]) + ",")
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
    g, outs, steps, slot, nslots, pinned = prog
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
        mem, flag = simulate(g, steps, slot, nslots, vals)
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
    a = ap.parse_args()
    prog = compile_program()
    g, outs, steps, slot, nslots, pinned = prog
    if a.stats or not a.out:
        kinds = {}
        for ops in steps:
            for x in ops:
                kinds[g.kind[x]] = kinds.get(g.kind[x], 0) + 1
        heavy = sum(1 for ops in steps if any(g.kind[x] in HEAVY for x in ops))
        inv = sum(1 for ops in steps if any(g.kind[x] == INV for x in ops))
        print("steps %d (heavy %d, inv %d, light %d), ops %s, slots %d" % (
            len(steps), heavy, inv, len(steps) - heavy, kinds, nslots), file=sys.stderr)
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
