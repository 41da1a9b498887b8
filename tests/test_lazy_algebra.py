"""CPU checks of the lazy radix-2^28 field layer (coconut-rust_amd/csrc/lazy.h) the pairing kernels use.

Restates lz_mont (signed product scanning, Montgomery R' = 2^392), squeeze and canon limb for limb in
Python with explicit signed 64-bit overflow checks, and drives them at the limits of the bounds the
header's types enforce (sum A_a A_b <= 533,000 in units of 2^40; B in units of p/16): every column
fits a signed 64-bit accumulator, the result is congruent to (ab + cd) / R' mod p, and its value
stays inside the B_out = 16 + ceil(sum B_a B_b / 40,304) the types claim.
"""
import random

import pytest

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
LN = 14
M28 = (1 << 28) - 1
RP = 1 << 392
N0 = (-pow(P, -1, 1 << 28)) % (1 << 28)
PL = [(P >> (28 * k)) & M28 for k in range(LN)]
I64 = 1 << 63


def value(v):
    return sum(x << (28 * k) for k, x in enumerate(v))


def chk(acc):
    assert -I64 <= acc < I64, "signed 64-bit accumulator overflow"
    return acc


def mont(a, b, c=None, d=None):
    """lazy.h lz_mont<NP>: limbs 0..12 of the result in [0, 2^28), the signed top limb last."""
    m = [0] * LN
    r = [0] * LN
    acc = 0
    for k in range(2 * LN - 1):
        acc2 = 0
        for i in range(LN):
            j = k - i
            if 0 <= j < LN:
                acc = chk(acc + a[i] * b[j])
                if c is not None:
                    acc2 = chk(acc2 + c[i] * d[j])
        acc = chk(acc + acc2)
        for i in range(min(k, LN)):
            j = k - i
            if 0 <= j < LN:
                acc = chk(acc + m[i] * PL[j])
        if k < LN:
            m[k] = ((acc & 0xFFFFFFFF) * N0) & M28
            acc = chk(acc + m[k] * PL[0])
        else:
            r[k - LN] = acc & M28
        assert acc & M28 == 0 or k >= LN
        acc >>= 28
    r[LN - 1] = acc
    assert -(1 << 31) <= acc < (1 << 31)
    return r


def squeeze(v):
    r, hi = [], 0
    for k in range(LN - 1):
        r.append((v[k] & M28) + hi)
        hi = v[k] >> 28
    r.append(v[LN - 1] + hi)
    return r


def rand_lz(a_bound, b_bound, rng, extreme=True):
    """Random signed limbs with |limb| < a_bound * 2^20 and |value| < b_bound * p / 16 (rejection)."""
    lim = a_bound << 20
    vmax = b_bound * P // 16
    while True:
        if extreme:
            v = [rng.choice([-1, 1]) * (lim - 1 - rng.randrange(4)) for _ in range(LN - 1)]
        else:
            v = [rng.randrange(-lim + 1, lim) for _ in range(LN - 1)]
        low = value(v)
        top = rng.randrange(-((vmax + low) >> 364), ((vmax - low) >> 364) + 1)
        v.append(top)
        if abs(value(v)) < vmax and all(abs(x) < lim for x in v):
            return v


@pytest.mark.parametrize("a1,a2,b1,b2", [(514, 514, 16, 16), (256, 1027, 100, 30), (1040, 256, 18, 18)])
def test_mont2_at_the_limb_bound(a1, a2, b1, b2):
    assert 2 * a1 * a2 <= 533000
    rng = random.Random(a1 * 7 + a2)
    bout = 16 + (2 * b1 * b2 + 40303) // 40304
    for _ in range(60):
        x, y = rand_lz(a1, b1, rng), rand_lz(a2, b2, rng)
        xs, ys = rand_lz(a1, b1, rng), rand_lz(a2, b2, rng)
        r = mont(x, y, xs, [-t for t in ys])
        want = (value(x) * value(y) - value(xs) * value(ys)) * pow(RP, -1, P) % P
        assert value(r) % P == want
        assert abs(value(r)) < bout * P // 16
        assert all(0 <= t <= M28 for t in r[:-1])


def test_mont_single_product_and_squeeze():
    rng = random.Random(5)
    for _ in range(60):
        x = rand_lz(1030, 200, rng, extreme=False)
        sq = squeeze(x)
        assert value(sq) == value(x)
        assert all(abs(t) < 257 << 20 for t in sq)
        y = rand_lz(517, 200, rng)
        r = mont(x, y)
        assert value(r) % P == value(x) * value(y) * pow(RP, -1, P) % P
        assert abs(value(r)) < (16 + (200 * 200 + 40303) // 40304) * P // 16


def test_column_bound_is_tight():
    """Just past the bound (every limb at the maximum, same signs) the accumulator overflows."""
    big = [(1 << 30) - 1] * LN  # A = 1024: 2 * 1024 * 1024 > 533,000
    with pytest.raises(AssertionError):
        mont(big, big, big, big)


def canon(v):
    """lazy.h lz_canon_call: carry, estimate floor(V / p) from the top 56 bits, fix up."""
    u, c = list(v), 0
    for k in range(LN - 1):
        t = u[k] + c
        u[k], c = t & M28, t >> 28
    u[LN - 1] += c
    h = (u[LN - 1] << 28) + u[LN - 2]
    import math
    q = math.floor(float(h) / (P / 2 ** 336))
    w = value(u) - q * P
    assert -P <= w < 2 * P
    while w < 0:
        w += P
    while w >= P:
        w -= P
    return w


def test_canon_range():
    rng = random.Random(9)
    for _ in range(200):
        x = rand_lz(1500, 4000, rng, extreme=False)
        assert canon(x) == value(x) % P


def reduce(v):
    """lazy.h reduce: q = round(top limb * (2^364 / p)) in float32, V - q p carried into normalised limbs."""
    import numpy as np
    q = int(np.rint(np.float32(v[LN - 1]) * (np.float32(1.0) / np.float32(106513.12))))
    r, c = [], 0
    for k in range(LN - 1):
        c += v[k] - q * PL[k]
        r.append(c & M28)
        c >>= 28
    r.append(v[LN - 1] - q * PL[LN - 1] + c)
    return r


def test_reduce_bound():
    """Any input the types allow (A <= 2047, |V| < 2048 p) comes back below 0.5625 p (B = 9)."""
    rng = random.Random(13)
    worst = 0.0
    for _ in range(3000):
        x = rand_lz(2047, 32768, rng, extreme=rng.random() < 0.5)
        r = reduce(x)
        assert value(r) % P == value(x) % P
        assert all(0 <= t <= M28 for t in r[:-1]) and -(1 << 31) <= r[-1] < (1 << 31)
        worst = max(worst, abs(value(r)) / P)
    assert worst < 9 / 16
