"""CPU checks of the identities the fexp kernel relies on (coconut-rust_amd/csrc/fexp_pl.hip),
against the oracle's Fp12 arithmetic (AMCL tower; Fp12 coefficient k multiplies W^k, W^6 = xi, so the
kernel's a0 b0 c0 a1 b1 c1 are coefficients 0 1 2 3 4 5):
  * compressed cyclotomic squaring (b, c) -> (b', c') and the decompression of a from (b, c);
  * the safegcd inversion's range argument, restated with 32/64-bit wrapping (field.h fp_inv).
"""
import random

from oracle import bls12_381 as B

P = B.P


def _cyclotomic(seed):
    rnd = random.Random(seed)
    x = [(rnd.randrange(P), rnd.randrange(P)) for _ in range(6)]
    g = B.f12_mul(B.f12_conj(x), B.f12_inv(x))
    return B.f12_mul(B.f12_pow(g, P * P), g)


def _k(a, n):
    return B.f2_muls(a, n % P)


def comp_sqr(b0, b1, c0, c1):
    s, xi, add, sub = B.f2_sqr, B.f2_mul_xi, B.f2_add, B.f2_sub
    Xb = sub(sub(s(add(b0, b1)), s(b0)), s(b1))
    Tb = add(s(b0), xi(s(b1)))
    Xc = xi(sub(sub(s(add(c0, c1)), s(c0)), s(c1)))
    Tc = add(s(c0), xi(s(c1)))
    return (add(_k(Xc, 3), _k(b0, 2)), sub(_k(Tc, 3), _k(b1, 2)),
            sub(_k(Tb, 3), _k(c0, 2)), add(_k(Xb, 3), _k(c1, 2)))


def decompress(b0, b1, c0, c1):
    s, m, xi, add, sub = B.f2_sqr, B.f2_mul, B.f2_mul_xi, B.f2_add, B.f2_sub
    Nb = sub(s(b0), xi(s(b1)))
    Nc = sub(s(c0), xi(s(c1)))
    D = _k(sub(m(b0, c0), xi(m(b1, c1))), 2)
    Di = B.f2_inv(D)
    return [m(add(m(b0, Nb), xi(m(c1, Nc))), Di), b0, c0, m(add(m(c0, Nc), m(b1, Nb)), Di), b1, c1]


def test_compressed_squaring_and_decompression():
    cur = _cyclotomic(5)
    st = (cur[1], cur[4], cur[2], cur[5])
    for _ in range(12):
        cur = B.f12_sqr(cur)
        st = comp_sqr(*st)
        assert st == (cur[1], cur[4], cur[2], cur[5])
        assert decompress(*st) == cur


def quad_comp_sqr(V, W):
    """fexp_q.hip qz_sqr as the quad runs it: pair j holds (V_j, W_j) = (c0, b0) | (b1, c1); each pair
    squares S1 = V, S2 = W, S3 = W + V' (primes: the other pair), then X = (S3 - S2)' - S1 (times xi on
    pair 0), T = S1' + S2 + i B with B = S1' | S2, V <- 3T - 2V, W <- 3X + 2W."""
    s, xi, add, sub = B.f2_sqr, B.f2_mul_xi, B.f2_add, B.f2_sub
    mul_i = lambda y: B.f2_mul(y, (0, 1))  # noqa: E731
    S1 = [s(V[j]) for j in (0, 1)]
    S2 = [s(W[j]) for j in (0, 1)]
    S3 = [s(add(W[j], V[1 - j])) for j in (0, 1)]
    E = [sub(S3[j], S2[j]) for j in (0, 1)]
    nV, nW = [None, None], [None, None]
    for j in (0, 1):
        X = sub(E[1 - j], S1[j])
        Xs = add(X, mul_i(X)) if j == 0 else X
        Bv = S1[1 - j] if j == 0 else S2[j]
        T = add(add(S1[1 - j], S2[j]), mul_i(Bv))
        nV[j] = sub(_k(T, 3), _k(V[j], 2))
        nW[j] = add(_k(Xs, 3), _k(W[j], 2))
    assert add(X, mul_i(X)) == xi(X)  # xi = 1 + i
    return nV, nW


def test_quad_compressed_squaring_matches():
    cur = _cyclotomic(7)
    b0, b1, c0, c1 = cur[1], cur[4], cur[2], cur[5]
    V, W = [c0, b1], [b0, c1]
    for _ in range(8):
        cur = B.f12_sqr(cur)
        V, W = quad_comp_sqr(V, W)
        assert (W[0], V[1], V[0], W[1]) == (cur[1], cur[4], cur[2], cur[5])


def test_pow_x_schedule():
    """|x| = 2^63 + 2^62 + 2^60 + 2^57 + 2^48 + 2^16: the kernel's snapshot/Granger-Scott split."""
    x_abs = 0xD201000000010000
    assert [b for b in range(64) if x_abs >> b & 1] == [16, 48, 57, 60, 62, 63]


# ---- safegcd restated with explicit wrapping (mirrors field.h divsteps30 / s30_update_*)
M30 = (1 << 30) - 1
N = 13
P30 = [(P >> (30 * i)) & M30 for i in range(N)]
INV256 = [(-pow(2 * i + 1, -1, 256)) % 256 for i in range(128)]


def _neg_inv256(f):
    """field.h divsteps30: -f^-1 mod 256 by Newton's iteration from (3f) ^ 2 (32-bit wrapping)."""
    fi = _u32(3 * f) ^ 2
    fi = _u32(fi * _u32(2 - f * fi))
    return _u32(-fi)


def _u32(x):
    return x & 0xFFFFFFFF


def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >> 31 else x


def test_newton_inverse_matches_the_table():
    """Every odd 32-bit word's Newton inverse agrees with -f^-1 mod 256 on the low byte."""
    for f in list(range(1, 1 << 12, 2)) + [0xFFFFFFFF, 0x80000001, 0xDEADBEEF]:
        assert _neg_inv256(f) & 255 == INV256[(f >> 1) & 127], f


def _divsteps(eta, f, g):
    u, v, q, r, i = 1, 0, 0, 1, 30
    while True:
        gg = _u32(g | _u32(0xFFFFFFFF << i))
        z = (gg & -gg).bit_length() - 1
        g >>= z
        u, v, eta, i = _u32(u << z), _u32(v << z), eta - z, i - z
        if i == 0:
            break
        if eta < 0:
            eta, f, g = -eta, g, _u32(-f)
            u, q = q, _u32(-u)
            v, r = r, _u32(-v)
        limit = min(eta + 1, i)
        w = _u32(g * _neg_inv256(f)) & (0xFFFFFFFF >> (32 - limit)) & 255
        g, q, r = _u32(g + f * w), _u32(q + u * w), _u32(r + v * w)
    return eta, [_i32(u), _i32(v), _i32(q), _i32(r)]


def _val(a):
    return sum(a[i] << (30 * i) for i in range(N))


def _apply(a, b, t0, t1, md=None):
    c = t0 * a[0] + t1 * b[0] + (P30[0] * md if md is not None else 0)
    assert c % (1 << 30) == 0
    c >>= 30
    out = []
    for i in range(1, N):
        c += t0 * a[i] + t1 * b[i] + (P30[i] * md if md is not None else 0)
        assert -(1 << 63) <= c < (1 << 63)
        out.append(_i32(c) & M30)
        c >>= 30
    return out + [_i32(c)]


def _md(t0, t1, d, e):
    m = _i32((t0 if d[-1] < 0 else 0) + (t1 if e[-1] < 0 else 0))
    cd = t0 * d[0] + t1 * e[0]
    return _i32(m - (_u32(0x30003 * _u32(cd) + _u32(m)) & M30))


def safegcd_inv(x):
    d, e, f, g = [0] * N, [1] + [0] * (N - 1), P30[:], [(x >> (30 * i)) & M30 for i in range(N)]
    eta = -1
    for _ in range(40):
        eta, t = _divsteps(eta, f[0], g[0])
        md, me = _md(t[0], t[1], d, e), _md(t[2], t[3], d, e)
        d, e = _apply(d, e, t[0], t[1], md), _apply(d, e, t[2], t[3], me)
        f, g = _apply(f, g, t[0], t[1]), _apply(f, g, t[2], t[3])
        assert -2 * P < _val(d) < P and -2 * P < _val(e) < P
        if not any(g):
            break
    D = -_val(d) if _val(f) < 0 else _val(d)
    return D % P


def test_safegcd_inversion():
    rnd = random.Random(11)
    for x in [0, 1, 2, P - 1, P - 2, (1 << 380) + 7] + [rnd.randrange(P) for _ in range(200)]:
        r = safegcd_inv(x)
        assert (x == 0 and r == 0) or r * x % P == 1


# ---- the same schedule mod r (fr.h fr_inv_int: 9 limbs, r = 1 mod 2^30 so r^-1 mod 2^30 = 1)
RN = 9
R30 = [(B.R >> (30 * i)) & M30 for i in range(RN)]


def _apply_r(a, b, t0, t1, md=None):
    c = t0 * a[0] + t1 * b[0] + (R30[0] * md if md is not None else 0)
    assert c % (1 << 30) == 0
    c >>= 30
    out = []
    for i in range(1, RN):
        c += t0 * a[i] + t1 * b[i] + (R30[i] * md if md is not None else 0)
        assert -(1 << 63) <= c < (1 << 63)
        out.append(_i32(c) & M30)
        c >>= 30
    return out + [_i32(c)]


def _md_r(t0, t1, d, e):
    m = _i32((t0 if d[-1] < 0 else 0) + (t1 if e[-1] < 0 else 0))
    cd = t0 * d[0] + t1 * e[0]
    return _i32(m - (_u32(_u32(cd) + _u32(m)) & M30))


def safegcd_inv_r(x):
    val = lambda a: sum(a[i] << (30 * i) for i in range(RN))  # noqa: E731
    d, e, f, g = [0] * RN, [1] + [0] * (RN - 1), R30[:], [(x >> (30 * i)) & M30 for i in range(RN)]
    eta, batches = -1, 0
    for _ in range(30):
        batches += 1
        eta, t = _divsteps(eta, f[0], g[0])
        md, me = _md_r(t[0], t[1], d, e), _md_r(t[2], t[3], d, e)
        d, e = _apply_r(d, e, t[0], t[1], md), _apply_r(d, e, t[2], t[3], me)
        f, g = _apply_r(f, g, t[0], t[1]), _apply_r(f, g, t[2], t[3])
        assert -2 * B.R < val(d) < B.R and -2 * B.R < val(e) < B.R
        if not any(g):
            break
    assert not any(g), "the loop bound of fr_inv_int must suffice"
    D = -val(d) if val(f) < 0 else val(d)
    return D % B.R, batches


def test_safegcd_inversion_mod_r():
    """fr.h fr_inv_int (the Lagrange kernel's inversion) restated: exact inverses mod r, intermediates in
    the signed 64-bit accumulators, d and e in (-2r, r), and g = 0 within the kernel's 30 batches."""
    rnd = random.Random(12)
    worst = 0
    for x in [0, 1, 2, B.R - 1, B.R - 2, (1 << 254) + 5] + [rnd.randrange(B.R) for _ in range(300)]:
        r, nb = safegcd_inv_r(x)
        worst = max(worst, nb)
        assert (x == 0 and r == 0) or r * x % B.R == 1
    assert worst <= 30


# ---- RLC signed-digit coefficient (fr.h rlc_delta_signed) restated word by word
R_ORDER = B.R


def _delta_words(blk):
    h = [(w >> 7) & 0x01010101 for w in blk]
    m = [(h[0] << 8) & 0xFFFFFFFF, ((h[1] << 8) | (h[0] >> 24)) & 0xFFFFFFFF,
         ((h[2] << 8) | (h[1] >> 24)) & 0xFFFFFFFF, ((h[3] << 8) | (h[2] >> 24)) & 0xFFFFFFFF, h[3] >> 24]
    u = sum(blk[k] << (32 * k) for k in range(4))
    mm = sum(m[k] << (32 * k) for k in range(5))
    t = (u - mm) % (1 << 256)
    if u < mm:
        t = (t + R_ORDER) % (1 << 256)
    return t


def test_rlc_signed_digits():
    """delta = sum int8(b_w) 256^w; the kernel's U - 256 H (+ r when negative) is delta mod r."""
    rnd = random.Random(7)
    cases = [[0, 0, 0, 0], [0xFFFFFFFF] * 4, [0x80808080] * 4, [0x7F7F7F7F] * 4]
    cases += [[rnd.getrandbits(32) for _ in range(4)] for _ in range(500)]
    for blk in cases:
        b = b"".join(w.to_bytes(4, "little") for w in blk)
        delta = sum((x - 256 if x >= 128 else x) << (8 * w) for w, x in enumerate(b))
        S = ((1 << 128) - 1) // 255  # 2^128 consecutive values: [-128 S, 127 S]
        assert -128 * S <= delta <= 127 * S
        assert _delta_words(blk) == delta % R_ORDER
