"""Static bound analysis of the radix-2^25.5 field arithmetic (fe25519.h):
for the operand classes the group formulas feed it (C, L, W), every 32-bit
multiplier operand fits in 32 bits and every 64-bit accumulator stays below
2^64 (including the carries added during fe_carry64)."""
C = [2**26 - 1 if k % 2 == 0 else 2**25 + 2**18 for k in range(10)]
L = [3 * 2**26 if k % 2 == 0 else 3 * 2**25 + 3 * 2**18 for k in range(10)]
W = [5 * 2**26 if k % 2 == 0 else 5 * 2**25 + 5 * 2**18 for k in range(10)]


def mul_worst(F, G):
    worst = 0
    for k in range(10):
        acc = 0
        for i in range(10):
            j = k - i
            fi = F[i] * (2 if (i % 2 and j % 2) else 1)
            gj = G[j] if j >= 0 else 19 * G[j + 10]
            assert fi < 2**32 and gj < 2**32
            acc += fi * gj
        worst = max(worst, acc)
    return worst


def sq_worst(F):
    worst = 0
    for k in range(10):
        acc = 0
        for i in range(10):
            for j in range(i, 10):
                if (i + j) % 10 != k:
                    continue
                fi = F[i] * (2 if i != j else 1)
                fj = F[j] * (2 if (i % 2 and j % 2) else 1) * (19 if i + j >= 10 else 1)
                assert fi < 2**32 and fj < 2**32
                acc += fi * fj
        worst = max(worst, acc)
    return worst


def test_mul_bounds():
    carry_headroom = 2**40  # carries folded into an accumulator before it is shifted
    for F, G in ((W, L), (L, L), (W, C), (C, C)):
        assert mul_worst(F, G) + carry_headroom < 2**64


def test_sq_bounds():
    assert sq_worst(L) + 2**40 < 2**64


def test_sub_bias_covers_subtrahend():
    two_p = [2**27 - 38] + [(2**26 - 2) if k % 2 else (2**27 - 2) for k in range(1, 10)]
    four_p = [2**28 - 76] + [(2**27 - 4) if k % 2 else (2**28 - 4) for k in range(1, 10)]
    assert all(two_p[k] >= C[k] for k in range(10))            # fe_sub: g in C
    L2 = [2 * c for c in C]
    assert all(four_p[k] >= L2[k] for k in range(10))          # fe_sub4: g = C + C
    # results land in the classes the formulas assume
    assert all(C[k] + two_p[k] <= L[k] for k in range(10))     # C - C -> L
    assert all(C[k] + four_p[k] <= W[k] for k in range(10))    # C - L -> W
    assert all(3 * C[k] + two_p[k] <= W[k] for k in range(10))  # 3C - C -> W (dbl's T)
