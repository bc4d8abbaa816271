"""csrc/fe_lanes.h's lane-distributed GF(2^255 - 19) square and product (edv_verify_small_kernel
and edv_resident_kernel decode R with them) modelled on the CPU lane by lane: the per-lane term
table (make_lane_tab), the 32-bit operand scalings, the 64-bit column sums of the four rows, and
lane_cols_carry's one-exchange carry (EDV_LANE_CARRY 1 and 2 -- ds_bpermute or DPP row moves, the
same arithmetic: a_k + b_{k-1} + d_{k-2}, x19 past 2^255, limb 0's excess into limb 1).  Every intermediate is checked against the machine width it lives
in, and every result against exact arithmetic mod p, over long chains that start from limbs at
the stated output bounds -- the bound argument of fe_lanes.h, executed."""
import random

P = 2 ** 255 - 19
W = [26 if k % 2 == 0 else 25 for k in range(10)]
POS = [sum(W[:k]) for k in range(10)]


def lane_tab(square):
    """fe_lanes.h make_lane_tab: lane 16 r + k holds terms (ia, ib, ma, mb) of column k."""
    tab = [[] for _ in range(64)]
    for k in range(10):
        q = 0
        for i in range(10):
            for j in range(i if square else 0, 10):
                if (i + j) % 10 != k:
                    continue
                per = 2 if square else 3
                lane = (q // per) * 16 + k
                odd2 = (i & 1) and (j & 1)
                ma = (2 if square and i != j else 1) * (2 if odd2 else 1)
                mb = 19 if i + j >= 10 else 1
                tab[lane].append((i, j, ma, mb))
                q += 1
    return tab


SQ, MU = lane_tab(True), lane_tab(False)


def value(limbs):
    return sum(v << POS[k] for k, v in enumerate(limbs)) % P


def columns(f, g, tab):
    p = [0] * 64
    for lane in range(64):
        for i, j, ma, mb in tab[lane]:
            a, b = f[i] * ma, g[j] * mb
            assert a < 2 ** 32 and b < 2 ** 32, (a, b)
            p[lane] += a * b
            assert p[lane] < 2 ** 64
    cols = []
    for k in range(10):
        s = p[k] + p[32 + k] + p[16 + k] + p[48 + k]
        assert s < 2 ** 64
        cols.append(s)
    return cols


def carry(cols):
    a = [c & ((1 << W[k]) - 1) for k, c in enumerate(cols)]
    b = [(c >> W[k]) & ((1 << W[(k + 1) % 10]) - 1) for k, c in enumerate(cols)]
    d = [c >> 51 for c in cols]
    r = []
    for k in range(10):
        s1, s2 = (9 if k == 0 else k - 1), (k - 2 if k >= 2 else k + 8)
        m1, m2 = (19 if k == 0 else 1), (19 if k <= 1 else 1)
        assert b[s1] * m1 < 2 ** 32 and d[s2] * m2 < 2 ** 32
        v = a[k] + b[s1] * m1 + d[s2] * m2
        assert v < 2 ** 32
        r.append(v)
    c0 = r[0] >> 26
    r[0] &= (1 << 26) - 1
    r[1] += c0
    return r


BOUND_EVEN, BOUND_ODD, BOUND_1 = 2 ** 27 + 2 ** 12, 2 ** 26 + 2 ** 12, 2 ** 26 + 2 ** 16


def in_bounds(r):
    return r[0] < 2 ** 26 and r[1] < BOUND_1 and all(r[k] < (BOUND_EVEN if k % 2 == 0 else BOUND_ODD)
                                                    for k in range(2, 10))


def extreme(rng):
    """Limbs at (or just under) the output bounds, or random within them."""
    out = []
    for k in range(10):
        top = 2 ** 26 if k == 0 else BOUND_1 if k == 1 else BOUND_EVEN if k % 2 == 0 else BOUND_ODD
        out.append(top - 1 - (rng.randrange(16) if rng.random() < 0.7 else rng.randrange(top)))
    return out


def test_distributed_square_and_product_exact_within_bounds():
    rng = random.Random(7)
    for trial in range(40):
        f, g = extreme(rng), extreme(rng)
        for step in range(60):
            if rng.random() < 0.8:
                r = carry(columns(f, f, SQ))
                assert value(r) == value(f) * value(f) % P
            else:
                r = carry(columns(f, g, MU))
                assert value(r) == value(f) * value(g) % P
            assert in_bounds(r), r
            f = r if rng.random() < 0.7 else extreme(rng)


def test_distributed_ops_on_canonical_inputs():
    """Class-C inputs (what dist_from_lane0 hands in) and small values."""
    rng = random.Random(11)
    for x in [0, 1, 2, 19, P - 1, P - 2, 2 ** 255 - 20] + [rng.randrange(P) for _ in range(200)]:
        f = [(x >> POS[k]) & ((1 << W[k]) - 1) for k in range(10)]
        r = carry(columns(f, f, SQ))
        assert value(r) == x * x % P and in_bounds(r)
