// Fp4 / Fp12 layers, Miller-loop line functions and cyclotomic operations on the lazy pair-lane field
// (lazy.h) — device code (the product path).  Same tower and formulas as tower.inc / pairing.inc
// (AMCL's Fp2 -> Fp4 -> Fp12), written over bound-typed values: every
// multiplication squeezes an operand only when the column bound demands it (mulr / sqrr below decide
// at compile time), and sums are squeezed where a limb would leave int32.
#pragma once
#include "lazy.h"

namespace cc {
namespace lz {

// ---------------------------------------------------------------- bound-driven helpers
// x squeezed iff its limbs exceed L
template <int L, int A, int B>
DEV auto lim(const F2<A, B>& x) {
    if constexpr (A > L) return squeeze(x);
    else return x;
}
template <int A, int B>
DEV auto norm(const F2<A, B>& x) { return lim<AS>(x); }

// x * y, squeezing the wider operand(s) as the column bound requires
template <int A1, int B1, int A2, int B2>
DEV auto mulr(const F2<A1, B1>& x, const F2<A2, B2>& y) {
    if constexpr (2LL * A1 * A2 <= AMAX) return mul(x, y);
    else if constexpr (A1 >= A2 && 2LL * AS * A2 <= AMAX) return mul(squeeze(x), y);
    else if constexpr (A2 > A1 && 2LL * A1 * AS <= AMAX) return mul(x, squeeze(y));
    else return mul(squeeze(x), squeeze(y));
}
template <int A, int B>
DEV auto sqrr(const F2<A, B>& x) {
    if constexpr (4LL * A * A <= AMAX) return sqr(x);
    else return sqr(squeeze(x));
}
template <int A, int B>
DEV auto sqrr_in(const F2<A, B>& x) {
    if constexpr (4LL * A * A <= AMAX) return sqr_in(x);
    else return sqr_in(squeeze(x));
}
template <int A1, int B1, int A2, int B2>
DEV auto mul_fpr(const F2<A1, B1>& x, const Fq<A2, B2>& k) {
    if constexpr ((long long)A1 * A2 <= AMAX) return mul_fp(x, k);
    else return mul_fp(squeeze(x), k);
}

// ============================== Fp4 = Fp2[s]/(s^2 - xi)
template <int A, int B>
struct F4 {
    static constexpr int AV = A, BV = B;
    F2<A, B> a, b;  // a + b s
};
template <int A1, int B1, int A2, int B2>
DEV F4<cmax(A1, A2), cmax(B1, B2)> mk4(const F2<A1, B1>& a, const F2<A2, B2>& b) {
    constexpr int A = cmax(A1, A2), B = cmax(B1, B2);
    return {fit<A, B>(a), fit<A, B>(b)};
}
template <int A2, int B2, int A, int B>
DEV F4<A2, B2> fit(const F4<A, B>& x) { return {fit<A2, B2>(x.a), fit<A2, B2>(x.b)}; }

template <int A1, int B1, int A2, int B2>
DEV auto add(const F4<A1, B1>& x, const F4<A2, B2>& y) { return mk4(add(x.a, y.a), add(x.b, y.b)); }
template <int A1, int B1, int A2, int B2>
DEV auto sub(const F4<A1, B1>& x, const F4<A2, B2>& y) { return mk4(sub(x.a, y.a), sub(x.b, y.b)); }
template <int A, int B>
DEV auto dbl(const F4<A, B>& x) { return mk4(dbl(x.a), dbl(x.b)); }
template <int A, int B>
DEV auto norm(const F4<A, B>& x) { return mk4(norm(x.a), norm(x.b)); }
template <int L, int A, int B>
DEV auto lim(const F4<A, B>& x) { return mk4(lim<L>(x.a), lim<L>(x.b)); }
// a - b s
template <int A, int B>
DEV F4<A, B> f4_conj(const F4<A, B>& x) { return {x.a, neg(x.b)}; }
// x s = xi b + a s
template <int A, int B>
DEV auto mul_s(const F4<A, B>& x) { return mk4(xi(x.b), x.a); }

// Karatsuba: t0 = a a', t1 = b b', (a + b)(a' + b') - t0 - t1, a a' + xi b b'
template <int A1, int B1, int A2, int B2>
DEV auto mul(const F4<A1, B1>& x, const F4<A2, B2>& y) {
    const auto t0 = mulr(x.a, y.a);
    const auto t1 = mulr(x.b, y.b);
    const auto s = mulr(add(x.a, x.b), add(y.a, y.b));
    return mk4(add(t0, xi(t1)), sub(sub(s, t0), t1));
}
// (a + b s)^2 = (a + b)(a + xi b) - ab (1 + xi)  +  2 ab s
template <int A, int B>
DEV auto sqr(const F4<A, B>& x) {
    const auto ab = mulr(x.a, x.b);
    const auto s = mulr(add(x.a, x.b), add(xi(x.b), x.a));
    return mk4(sub(sub(s, ab), xi(ab)), dbl(ab));
}
template <int A1, int B1, int A2, int B2>
DEV auto mul_f2(const F4<A1, B1>& x, const F2<A2, B2>& c) { return mk4(mulr(x.a, c), mulr(x.b, c)); }

// ============================== Fp12 = Fp4[w]/(w^3 - s)
template <int A, int B>
struct F12 {
    static constexpr int AV = A, BV = B;
    F4<A, B> a, b, c;  // a + b w + c w^2
};
template <class X, class Y, class Z>
DEV auto mk12(const X& a, const Y& b, const Z& c) {
    constexpr int A = cmax(cmax(X::AV, Y::AV), Z::AV), B = cmax(cmax(X::BV, Y::BV), Z::BV);
    return F12<A, B>{fit<A, B>(a), fit<A, B>(b), fit<A, B>(c)};
}
template <int A2, int B2, int A, int B>
DEV F12<A2, B2> fit(const F12<A, B>& x) { return {fit<A2, B2>(x.a), fit<A2, B2>(x.b), fit<A2, B2>(x.c)}; }
template <int A, int B>
DEV auto norm(const F12<A, B>& x) { return mk12(norm(x.a), norm(x.b), norm(x.c)); }

DEV F12<AN, BC> f12_one() {
    const F4<AN, BC> o{f2_one(), f2_zero()}, z{f2_zero(), f2_zero()};
    return {o, z, z};
}
// conj = x^(p^6): w -> -w, s -> -s
template <int A, int B>
DEV F12<A, B> f12_conj(const F12<A, B>& x) {
    F12<A, B> r;
    r.a = f4_conj(x.a);
    r.b = {neg(x.b.a), x.b.b};
    r.c = f4_conj(x.c);
    return r;
}

// Chung-Hasan SQR2 (tower.inc f12_sqr): s0 = a^2, s1 = 2ab, s2 = (a - b + c)^2, s3 = 2bc, s4 = c^2;
// r.a = s0 + s s3, r.b = s1 + s s4, r.c = s1 + s2 + s3 - s0 - s4
template <int A, int B>
DEV auto f12_sqr(const F12<A, B>& x) {
    const auto s2 = norm(sqr(norm(add(sub(x.a, x.b), x.c))));
    const auto s0 = norm(sqr(x.a));
    const auto s1 = norm(dbl(mul(x.a, x.b)));
    const auto s3 = norm(dbl(mul(x.b, x.c)));
    const auto s4 = norm(sqr(x.c));
    return norm(mk12(add(s0, mul_s(s3)), add(s1, mul_s(s4)), sub(sub(add(add(s1, s2), s3), s0), s4)));
}

// f * (A + C w^2), A = (l0, l3), C = (l2, 0) (tower.inc f12_mul_line): 13 Fp2 products
template <int A, int B, class L0, class L2, class L3>
DEV auto f12_mul_line(const F12<A, B>& f, const L0& l0, const L2& l2, const L3& l3) {
    const auto la = mk4(l0, l3);
    const auto t0 = mul(f.a, la);                                  // a A
    const auto t2 = mul_f2(f.c, l2);                               // c C
    const auto s = mul(add(f.a, f.c), mk4(add(l0, l2), l3));              // (a + c)(A + C), squeezed by mulr
    const auto rc = sub(sub(s, t0), t2);                           // c A + a C
    const auto ra = add(t0, mul_s(mul_f2(f.b, l2)));               // a A + s (b C)
    const auto rb = add(mul(f.b, la), mul_s(t2));                  // b A + s (c C)
    return norm(mk12(ra, rb, rc));
}


// ---------------------------------------------------------------- Frobenius (pairing.inc), R' constants
// gamma_k = xi^(k(p-1)/6) (a, b) and gamma2_k = xi^(k(p^2-1)/6) in Fp (tools/gen_lz_constants.py)
struct F2cz {
    int32_t a[LN], b[LN];
};
__constant__ static const F2cz kGammaZ1[6] = {
    {{0x347fcb8, 0xd800000, 0x002b119, 0x0cde6d2, 0xc7212e0, 0x83a2090, 0x037669f, 0xda0f73e, 0x9b09b42, 0x1297bb0, 0x515d98f, 0x012ca7c, 0x659fcfa, 0x000577a},
     {0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000}},
    {{0x9f1ba38, 0xed52b31, 0x3131f18, 0x932815a, 0x35bde3f, 0x7c4a4df, 0xc6f7465, 0x266b7cc, 0x2acd4ff, 0xcae398d, 0x243b688, 0xa613121, 0x72d376f, 0x0001c3e},
     {0x60df073, 0x11ad4ce, 0x0ece0a1, 0x6cd69bb, 0x2c8406c, 0x24ac630, 0x2f7bc6d, 0xcd1995f, 0x1ca7685, 0x80c93e9, 0x963ffba, 0x4087390, 0xabd0210, 0x00183d2}},
    {{0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000},
     {0x2421b59, 0xbee4867, 0x1d31002, 0x4760184, 0x4cc5086, 0xc76dc00, 0xaae891b, 0xac70ad2, 0xfe377c4, 0xe4686b8, 0x5ed1568, 0x8f5a180, 0x02b5c1f, 0x000d1a4}},
    {{0x33e2f27, 0x32a25aa, 0x27ca1d2, 0xc1e049e, 0xc3f707a, 0x055ca94, 0x2010b7b, 0x3b93794, 0xd5a86aa, 0xa544de3, 0x556a044, 0x9c66da5, 0x38ec515, 0x000cea3},
     {0x33e2f27, 0x32a25aa, 0x27ca1d2, 0xc1e049e, 0xc3f707a, 0x055ca94, 0x2010b7b, 0x3b93794, 0xd5a86aa, 0xa544de3, 0x556a044, 0x9c66da5, 0x38ec515, 0x000cea3}},
    {{0x58a1811, 0x96e4867, 0x1d5c11c, 0x543e856, 0x13e6366, 0x4b0fc91, 0xae5efbb, 0x8680210, 0x9941307, 0xf700269, 0xb02eef7, 0x9086bfc, 0x6855919, 0x001291e},
     {0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000, 0x0000000}},
    {{0xd2fe95f, 0x1ff50db, 0x58fc0eb, 0x55085f8, 0xf9b4eba, 0x81a6f73, 0xe707fe0, 0x61fef60, 0x0075ba9, 0x7028771, 0x79a56cd, 0x4279ec6, 0xabbfc85, 0x000eae1},
     {0x2cfc14c, 0xdf0af24, 0xe703ece, 0xaaf651c, 0x688cff1, 0x1f4fb9b, 0x0f6b0f2, 0x91861cb, 0x46fefdb, 0xdb84605, 0x40d5f75, 0xa4205eb, 0x72e3cfa, 0x000b52f}},
};
__constant__ static const int32_t kGammaZ2[6][LN] = {
    {0x347fcb8, 0xd800000, 0x002b119, 0x0cde6d2, 0xc7212e0, 0x83a2090, 0x037669f, 0xda0f73e, 0x9b09b42, 0x1297bb0, 0x515d98f, 0x012ca7c, 0x659fcfa, 0x000577a},
    {0xdbd8f52, 0x401b798, 0x22cefb7, 0xb89e991, 0x157ce25, 0xd988f0f, 0x4b8a7b6, 0x4714659, 0x493d3c0, 0x67446bd, 0x5baa0da, 0x5740331, 0x1bedd60, 0x000ce6d},
    {0xa75929a, 0x681b798, 0x22a3e9d, 0xabc02bf, 0x4e5bb45, 0x55e6e7e, 0x4814117, 0x6d04f1b, 0xae3387d, 0x54acb0c, 0x0a4c74b, 0x56138b5, 0xb64e066, 0x00076f2},
    {0xcb7adf3, 0x26fffff, 0x3fd4ea0, 0xf320443, 0x9b20bcb, 0x1d54a7e, 0xf2fca33, 0x19759ed, 0xac6b042, 0x39151c5, 0x691dcb4, 0xe56da35, 0xb903c85, 0x0014896},
    {0x2421b59, 0xbee4867, 0x1d31002, 0x4760184, 0x4cc5086, 0xc76dc00, 0xaae891b, 0xac70ad2, 0xfe377c4, 0xe4686b8, 0x5ed1568, 0x8f5a180, 0x02b5c1f, 0x000d1a4},
    {0x58a1811, 0x96e4867, 0x1d5c11c, 0x543e856, 0x13e6366, 0x4b0fc91, 0xae5efbb, 0x8680210, 0x9941307, 0xf700269, 0xb02eef7, 0x9086bfc, 0x6855919, 0x001291e},
};
DEV F2<AN, BC> ld_gamma1(int k) {
    const bool im = half_id() != 0;
    F2<AN, BC> r;
#pragma unroll
    for (int j = 0; j < LN; j++) r.c.v[j] = im ? kGammaZ1[k].b[j] : kGammaZ1[k].a[j];
    return r;
}
DEV Fq<AN, BC> ld_gamma2(int k) {
    Fq<AN, BC> r;
#pragma unroll
    for (int j = 0; j < LN; j++) r.v[j] = kGammaZ2[k][j];
    return r;
}
// x^p coefficient-wise: conj(c) gamma_k for the coefficient of W^k (AMCL slots: a.a 0, a.b 3, b.a 1,
// b.b 4, c.a 2, c.b 5)
template <int A, int B>
DEV auto f12_frob(const F12<A, B>& x) {
    const auto z = [&](const F2<A, B>& c, int k) { return mulr(conj(c), ld_gamma1(k)); };
    return mk12(mk4(conj(x.a.a), z(x.a.b, 3)), mk4(z(x.b.a, 1), z(x.b.b, 4)), mk4(z(x.c.a, 2), z(x.c.b, 5)));
}
template <int A, int B>
DEV auto f12_frob2(const F12<A, B>& x) {
    const auto z = [&](const F2<A, B>& c, int k) { return mul_fpr(c, ld_gamma2(k)); };
    return mk12(mk4(x.a.a, z(x.a.b, 3)), mk4(z(x.b.a, 1), z(x.b.b, 4)), mk4(z(x.c.a, 2), z(x.c.b, 5)));
}

// Karatsuba over the cubic extension (tower.inc f12_mul)
template <int A1, int B1, int A2, int B2>
DEV auto f12_mul(const F12<A1, B1>& x, const F12<A2, B2>& y) {
    const auto t0 = norm(mul(x.a, y.a));
    const auto t1 = norm(mul(x.b, y.b));
    const auto t2 = norm(mul(x.c, y.c));
    const auto ra = add(mul_s(norm(sub(sub(mul(norm(add(x.b, x.c)), norm(add(y.b, y.c))), t1), t2))), t0);
    const auto rb = add(sub(sub(mul(norm(add(x.a, x.b)), norm(add(y.a, y.b))), t0), t1), mul_s(t2));
    const auto rc = add(sub(sub(mul(norm(add(x.a, x.c)), norm(add(y.a, y.c))), t0), t2), t1);
    return norm(mk12(ra, rb, rc));
}

// Granger-Scott squaring in the cyclotomic subgroup (tower.inc f12_cyc_sqr):
// a' = 3a^2 - 2 conj(a), b' = 3 s c^2 + 2 conj(b), c' = 3 b^2 - 2 conj(c)
template <int A, int B>
DEV auto f12_cyc_sqr(const F12<A, B>& x) {
    const auto a2 = norm(sqr(x.a));
    const auto c2s = norm(mul_s(norm(sqr(x.c))));
    const auto b2 = norm(sqr(x.b));
    // 3u - 2 conj(v) = u + 2 (u - conj(v));  3u + 2 conj(v) = u + 2 (u + conj(v))
    const auto ra = add(a2, dbl(sub(a2, f4_conj(x.a))));
    const auto rb = add(c2s, dbl(add(c2s, f4_conj(x.b))));
    const auto rc = add(b2, dbl(sub(b2, f4_conj(x.c))));
    return norm(mk12(ra, rb, rc));
}

// (a + b s)^-1 = (a - b s) / (a^2 - xi b^2)
template <int A, int B>
DEV auto f4_inv(const F4<A, B>& x) {
    const auto n = norm(sub(sqrr(x.a), xi(sqrr(x.b))));
    const auto ni = inv(n);
    return mk4(mulr(x.a, ni), neg(mulr(x.b, ni)));
}
// tower.inc f12_inv
template <int A, int B>
DEV auto f12_inv(const F12<A, B>& x) {
    const auto A0 = norm(sub(sqr(x.a), mul_s(norm(mul(x.b, x.c)))));   // a^2 - s bc
    const auto B0 = norm(sub(mul_s(norm(sqr(x.c))), mul(x.a, x.b)));  // s c^2 - ab
    const auto C0 = norm(sub(sqr(x.b), mul(x.a, x.c)));               // b^2 - ac
    const auto F = norm(add(mul_s(norm(add(mul(x.c, B0), mul(x.b, C0)))), mul(x.a, A0)));
    const auto Fi = norm(f4_inv(F));
    return norm(mk12(mul(A0, Fi), mul(B0, Fi), mul(C0, Fi)));
}

// ---------------------------------------------------------------- line functions (pairing.inc)
template <int BX, int BY, int BZ>
struct G2P {
    F2<AS, BX> x;
    F2<AS, BY> y;
    F2<AS, BZ> z;  // homogeneous projective on the twist
};

// Doubling step, T <- 4 (2T) (the scale keeps the halvings of pairing.inc's formula out; T is
// projective):  B = Y^2, C = Z^2, E = 3 b' C = 12 xi C, F = 3E, H = (Y + Z)^2 - B - C,
//   X' = 2 XY (B - F),  Y' = (B + F)^2 - 12 E^2,  Z' = 4 B H;
// line before evaluation at P: l0 = E - B, l2c = 3 X^2, l3c = -H.
template <class L0, class L2, class L3>
struct Line {
    L0 l0;
    L2 l2;
    L3 l3;
};
template <class L0, class L2, class L3>
DEV Line<L0, L2, L3> mk_line(const L0& l0, const L2& l2, const L3& l3) { return {l0, l2, l3}; }

template <int BX, int BY, int BZ>
DEV auto line_dbl(G2P<BX, BY, BZ>& T) {
    const auto a = mulr(T.x, T.y);
    const auto b = sqrr(T.y);
    const auto c = sqrr(T.z);
    const auto e3 = norm(smul<3>(xi(c)));             // 3 xi C
    const auto e = smul<4>(e3);                        // E = 12 xi C
    const auto f = dbl(norm(smul<6>(e3)));            // F = 3 E = 2 (6 e3)
    const auto ln = mk_line(norm(sub(e, b)), norm(smul<3>(sqrr(T.x))), norm(neg(sub(sub(sqrr(add(T.y, T.z)), b), c))));
    const auto h = neg(ln.l3);                         // H (squeezed)
    const auto t = sqrr(norm(e));
    T.x = fit<AS, BX>(norm(dbl(mulr(a, sub(b, f)))));
    T.y = fit<AS, BY>(norm(sub(sqrr(add(b, f)), smul<3>(norm(smul<4>(t))))));
    T.z = fit<AS, BZ>(norm(smul<4>(mulr(b, h))));
    return ln;
}

// Addition step with affine Q: T <- T + Q (pairing.inc line_add);
//   l0 = theta x_Q - lambda y_Q, l2c = -theta, l3c = lambda.
template <int BX, int BY, int BZ, class Q>
DEV auto line_add(G2P<BX, BY, BZ>& T, const Q& qx, const Q& qy) {
    const auto theta = norm(sub(T.y, mulr(qy, T.z)));
    const auto lambda = norm(sub(T.x, mulr(qx, T.z)));
    const auto c = sqrr(theta);
    const auto d = sqrr(lambda);
    const auto e = mulr(lambda, d);
    const auto f = mulr(T.z, c);
    const auto g = mulr(T.x, d);
    const auto h = sub(add(e, f), dbl(g));
    const auto ln = mk_line(norm(sub(mulr(theta, qx), mulr(lambda, qy))), neg(theta), lambda);
    const auto ey = mulr(e, T.y);
    T.x = fit<AS, BX>(norm(mulr(lambda, h)));
    T.y = fit<AS, BY>(norm(sub(mulr(theta, sub(g, h)), ey)));
    T.z = fit<AS, BZ>(norm(mulr(T.z, e)));
    return ln;
}

}  // namespace lz
}  // namespace cc
