// Quad-lane Fp4 / Fp12 on the lazy field (lazy.h, tower_lz.h) — device code (the product path).
// Same tower, formulas and bound types as tower_lz.h (AMCL's Fp2 -> Fp4 -> Fp12, SURVEY.md §8a
// rows T3, V6); different lane mapping: ONE credential per QUAD of adjacent lanes.
//
//   lane 4i + 2j + h holds half h (re / im) of component j of every Fp4 value u + v s of credential i
//   (j = 0: u, j = 1: v).  An Fp12 = a + b w + c w^2 is then 3 Fp a lane (42 words, against 84 in the
//   pair layout of tower_lz.h), and each pair of the quad is an ordinary pair-lane Fp2 (lazy.h: the
//   partner half over DPP quad_perm [1,0,3,2]); the two pairs exchange components over DPP
//   quad_perm [2,3,0,1] (qx below).
//
// Work is split so the two pairs always run the same instructions on different data:
//   Fp4 product  (u + v s)(u' + v' s):  T0 = u u' (pair 0), T1 = v v' (pair 1), S = (u + v)(u' + v');
//                two products share one call so that pair 0 forms S of the first and pair 1 S of the
//                second: 3 Fp2 products a lane for two Fp4 products (the pair layout: 6).
//   Fp4 square   (u + v s)^2 = (u + v)(u + xi v) - uv (1 + xi) + 2 uv s: pair 0 forms uv, pair 1 the
//                other product: 1 Fp2 product a lane (the pair layout: 2).
// so every Fp12 operation costs each lane half the products of the pair layout, on twice the lanes.
// Control flow is quad-uniform (every predicate agrees on the four lanes).
#pragma once
#include "tower_lz.h"

namespace cc {
namespace lz {

// component index j of this lane (bit 1 of the lane id)
DEV bool qhi() { return ((__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) >> 1) & 1u) != 0; }
DEV int32_t qswp(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true); }
// the other pair's value (lane 4i + 2j + h <-> 4i + 2(1 - j) + h)
template <int A, int B>
DEV F2<A, B> qx(const F2<A, B>& x) {
    F2<A, B> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.c.v[k] = qswp(x.c.v[k]);
    return r;
}
template <int A1, int B1, int A2, int B2>
DEV F2<cmax(A1, A2), cmax(B1, B2)> qsel(bool c, const F2<A1, B1>& x, const F2<A2, B2>& y) {
    F2<cmax(A1, A2), cmax(B1, B2)> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.c.v[k] = c ? x.c.v[k] : y.c.v[k];
    return r;
}
// all four lanes of the quad
DEV bool quad_all(bool own) {
    uint32_t o = own ? 1u : 0u;
    o &= (uint32_t)swp((int32_t)o);
    o &= (uint32_t)qswp((int32_t)o);
    return o != 0;
}

// ---------------------------------------------------------------- masked half operations
// lane 4i + 2j + h: pair j, half h.  Masks of the lanes an operation runs on (exec narrowed inside one asm
// statement and restored, as lazy.h neg_re14: the other lanes keep their values).
constexpr uint64_t kP0Re = 0x1111111111111111ull, kP0Im = 0x2222222222222222ull;  // pair 0, re / im half
constexpr uint64_t kRe = 0x5555555555555555ull, kIm = 0xAAAAAAAAAAAAAAAAull;      // every re / im half
// 7 limbs: x <- x - s on the lanes of mre, x + s on the lanes of mim
DEV void addsub_ops7(int32_t* x, const int32_t* s, uint64_t mre, uint64_t mim) {
    uint64_t save;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_and_b64 exec, %0, %15\n\t"
        "v_sub_u32 %1, %1, %8\n\tv_sub_u32 %2, %2, %9\n\tv_sub_u32 %3, %3, %10\n\tv_sub_u32 %4, %4, %11\n\t"
        "v_sub_u32 %5, %5, %12\n\tv_sub_u32 %6, %6, %13\n\tv_sub_u32 %7, %7, %14\n\t"
        "s_and_b64 exec, %0, %16\n\t"
        "v_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %9\n\tv_add_u32 %3, %3, %10\n\tv_add_u32 %4, %4, %11\n\t"
        "v_add_u32 %5, %5, %12\n\tv_add_u32 %6, %6, %13\n\tv_add_u32 %7, %7, %14\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(save), "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6])
        : "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]), "v"(s[4]), "v"(s[5]), "v"(s[6]), "s"(mre), "s"(mim));
}
// x + i y (i y = -y_im + y_re i: the partner's half of y, negated on the re half)
template <int A1, int B1, int A2, int B2>
DEV F2<A1 + A2, B1 + B2> add_i(const F2<A1, B1>& x, const F2<A2, B2>& y) {
    F2<A1 + A2, B1 + B2> r;
    int32_t s[LN];
#pragma unroll
    for (int k = 0; k < LN; k++) {
        r.c.v[k] = x.c.v[k];
        s[k] = swp(y.c.v[k]);
    }
    addsub_ops7(r.c.v, s, kRe, kIm);
    addsub_ops7(r.c.v + 7, s + 7, kRe, kIm);
    return r;
}
// xi x = x + i x on pair 0, x on pair 1 (this lane's half)
template <int A, int B>
DEV F2<2 * A, 2 * B> xi_pair0(const F2<A, B>& x) {
    F2<2 * A, 2 * B> r;
    int32_t s[LN];
#pragma unroll
    for (int k = 0; k < LN; k++) {
        r.c.v[k] = x.c.v[k];
        s[k] = swp(x.c.v[k]);
    }
    addsub_ops7(r.c.v, s, kP0Re, kP0Im);
    addsub_ops7(r.c.v + 7, s + 7, kP0Re, kP0Im);
    return r;
}

// ---------------------------------------------------------------- inversion, one per quad
// field.h fp_inv_int with the quad's four lanes holding the same input: the divstep iteration's four
// vectors f, g, d, e sit one per lane (lane & 3 = 0 f, 1 g, 2 d, 3 e; partners f/g and d/e over DPP
// quad_perm [1,0,3,2]), so a batch's matrix update is ONE signed carry chain a lane (3 mads a limb, the
// p multiple zero on the f/g lanes) instead of four; the divsteps on the low words (f0, g0 broadcast)
// run on every lane.
DEV int32_t qbcast(int32_t x, int src) {
    switch (src) {
        case 0: return __builtin_amdgcn_mov_dpp(x, 0x00, 0xF, 0xF, true);
        case 1: return __builtin_amdgcn_mov_dpp(x, 0x55, 0xF, 0xF, true);
        case 2: return __builtin_amdgcn_mov_dpp(x, 0xAA, 0xF, 0xF, true);
        default: return __builtin_amdgcn_mov_dpp(x, 0xFF, 0xF, 0xF, true);
    }
}
DEV void fp_inv_int_quad(Fp& out, const Fp& a) {
    const uint32_t role = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 3u;
    const bool de = role >= 2, odd = (role & 1u) != 0;
    S30 X, Y;  // this lane's vector and its partner's
    {
        S30 g;
        s30_from_fp(g, a);
#pragma unroll
        for (int i = 0; i < S30N; i++) {
            const int32_t f = p30_limb(i), d = 0, e = i == 0 ? 1 : 0;
            const int32_t own = role == 0 ? f : role == 1 ? g.v[i] : role == 2 ? d : e;
            const int32_t par = role == 0 ? g.v[i] : role == 1 ? f : role == 2 ? e : d;
            X.v[i] = own;
            Y.v[i] = par;
        }
    }
    int32_t eta = -1;
    for (int it = 0; it < 40; it++) {
        int32_t t[4];
        eta = divsteps30(eta, (uint32_t)qbcast(X.v[0], 0), (uint32_t)qbcast(X.v[0], 1), t);
        // f' = t0 f + t1 g, g' = t2 f + t3 g, d' = t0 d + t1 e + p md, e' = t2 d + t3 e + p me (all / 2^30)
        const int32_t ta = odd ? t[3] : t[0], tb = odd ? t[2] : t[1];
        int64_t c = smad(tb, Y.v[0], smad(ta, X.v[0], 0));
        int32_t m = (ta & (X.v[S30N - 1] >> 31)) + (tb & (Y.v[S30N - 1] >> 31));
        m -= (int32_t)((PINV30 * (uint32_t)c + (uint32_t)m) & (uint32_t)M30);
        m = de ? m : 0;
        c = smad(p30_limb(0), m, c);
        c >>= 30;
#pragma unroll
        for (int i = 1; i < S30N; i++) {
            c = smad(p30_limb(i), m, smad(tb, Y.v[i], smad(ta, X.v[i], c)));
            X.v[i - 1] = (int32_t)c & M30;
            c >>= 30;
        }
        X.v[S30N - 1] = (int32_t)c;
        int32_t o = 0;
#pragma unroll
        for (int i = 0; i < S30N; i++) {
            Y.v[i] = __builtin_amdgcn_mov_dpp(X.v[i], 0xB1, 0xF, 0xF, true);
            o |= X.v[i];
        }
        if (qbcast(o, 1) == 0) break;  // g = 0 (quad-uniform)
    }
    // f = +-1 (or p when a = 0, where d = 0): x = sign(f) d mod p, d in (-2p, p) (fp_inv_int)
    const int32_t fsign = qbcast(X.v[S30N - 1], 0);
    S30 d;
#pragma unroll
    for (int i = 0; i < S30N; i++) d.v[i] = qbcast(X.v[i], 2);
    if (fsign < 0) {
#pragma unroll
        for (int i = 0; i < S30N; i++) d.v[i] = -d.v[i];
        s30_carry(d);
    }
    s30_add_kp(d, d.v[S30N - 1] < 0 ? 1 : 0);
    s30_add_kp(d, d.v[S30N - 1] < 0 ? 1 : 0);
    S30 tt = d;
    s30_add_kp(tt, -1);
    if (tt.v[S30N - 1] >= 0) d = tt;
    fp_from_s30(out, d);
}
// lazy.h inv() for values the four lanes of a quad hold alike
template <int A, int B>
DEV auto qinv(const Fq<A, B>& x) {
    constexpr int32_t C[LN] = {LZ_R3_LIMBS};
    Fp a = canon(x), ai;
    fp_inv_int_quad(ai, a);  // (x R')^-1
    return mul(from_fp(ai), fq_const(C));
}
template <int A, int B>
DEV auto qinv(const F2<A, B>& x) {
    static_assert(2LL * A * A <= AMAX, "f2 inv: limb bound");
    int32_t xs[LN];
#pragma unroll
    for (int k = 0; k < LN; k++) xs[k] = swp(x.c.v[k]);
    const W14 n = lz_mont<2>(x.c.v, x.c.v, xs, xs);  // a^2 + b^2 on both lanes
    const auto ni = qinv(fq<bprod(2LL * B * B)>(n));
    const auto r = mul(x.c, ni);
    return conj(F2<AN, decltype(r)::BV>{r});
}

template <class T>
struct Two {
    T a, b;
};
template <class X, class Y>
DEV auto two(const X& a, const Y& b) {
    constexpr int A = cmax(X::AV, Y::AV), B = cmax(X::BV, Y::BV);
    return Two<F2<A, B>>{fit<A, B>(a), fit<A, B>(b)};
}

// ---------------------------------------------------------------- Fp4 (this lane's component)
// x s = xi v + u s
template <class X>
DEV auto q_mul_s(const X& x) {
    const auto p = qx(x);
    return qsel(qhi(), p, xi(p));
}
// u - v s
template <class X>
DEV auto q_conj4(const X& x) { return qsel(qhi(), neg(x), x); }

// two Fp4 products (header): returns this lane's component of x_A y_A and x_B y_B
template <class XA, class YA, class XB, class YB>
DEV auto q4_mul2(const XA& xA, const YA& yA, const XB& xB, const YB& yB) {
    const bool j = qhi();
    const auto TA = mulr(xA, yA);  // pair 0: u u', pair 1: v v' (of A)
    const auto TB = mulr(xB, yB);
    // pair 0 forms S_A = (uA + vA)(uA' + vA'), pair 1 S_B: each receives the component it lacks
    const auto sx = add(qsel(j, xB, xA), qx(qsel(j, xA, xB)));
    const auto sy = add(qsel(j, yB, yA), qx(qsel(j, yA, yB)));
    const auto S = mulr(sx, sy);
    const auto pTA = qx(TA), pTB = qx(TB), pS = qx(S);
    // u = T0 + xi T1 (pair 0), v = S - T0 - T1 (pair 1)
    const auto rA = qsel(j, sub(sub(pS, pTA), TA), add(TA, xi(pTA)));
    const auto rB = qsel(j, sub(sub(S, pTB), TB), add(TB, xi(pTB)));
    return two(norm(rA), norm(rB));
}
// one Fp4 product: both pairs form S (2 Fp2 products a lane)
template <class X, class Y>
DEV auto q4_mul1(const X& x, const Y& y) {
    const bool j = qhi();
    const auto T = mulr(x, y);
    const auto S = mulr(add(x, qx(x)), add(y, qx(y)));
    const auto pT = qx(T);
    return norm(qsel(j, sub(sub(S, T), pT), add(T, xi(pT))));
}
// Fp4 square (header)
template <class X>
DEV auto q4_sqr(const X& x) {
    const bool j = qhi();
    const auto p = qx(x);
    const auto u = qsel(j, p, x), v = qsel(j, x, p);
    const auto M = mulr(qsel(j, add(u, v), u), qsel(j, add(u, xi(v)), v));  // pair 0: u v; pair 1: (u + v)(u + xi v)
    const auto pM = qx(M);
    return norm(qsel(j, dbl(pM), sub(sub(pM, M), xi(M))));
}

// ---------------------------------------------------------------- Fp12 = Fp4[w]/(w^3 - s)
template <int A, int B>
struct Q12 {
    static constexpr int AV = A, BV = B;
    F2<A, B> a, b, c;  // this lane's component of the Fp4 coefficients a + b w + c w^2
};
template <class X, class Y, class Z>
DEV auto mkq(const X& a, const Y& b, const Z& c) {
    constexpr int A = cmax(cmax(X::AV, Y::AV), Z::AV), B = cmax(cmax(X::BV, Y::BV), Z::BV);
    return Q12<A, B>{fit<A, B>(a), fit<A, B>(b), fit<A, B>(c)};
}
template <int A, int B>
DEV auto norm(const Q12<A, B>& x) { return mkq(norm(x.a), norm(x.b), norm(x.c)); }
using QR = Q12<AN, 9>;  // at rest: reduced
template <int A, int B>
DEV QR rest(const Q12<A, B>& x) { return {reduce(x.a), reduce(x.b), reduce(x.c)}; }

// x^(p^6): w -> -w, s -> -s  (tower_lz.h f12_conj)
template <int A, int B>
DEV Q12<A, B> q12_conj(const Q12<A, B>& x) {
    const bool j = qhi();
    return {qsel(j, neg(x.a), x.a), qsel(j, x.b, neg(x.b)), qsel(j, neg(x.c), x.c)};
}
// Karatsuba over the cubic extension (tower_lz.h f12_mul): 6 Fp4 products as 3 balanced pairs
template <int A1, int B1, int A2, int B2>
DEV auto q12_mul(const Q12<A1, B1>& x, const Q12<A2, B2>& y) {
    const auto m0 = q4_mul2(x.a, y.a, x.b, y.b);                                      // t0, t1
    const auto m1 = q4_mul2(x.c, y.c, add(x.b, x.c), add(y.b, y.c));                  // t2, (b + c)(b' + c')
    const auto m2 = q4_mul2(add(x.a, x.b), add(y.a, y.b), add(x.a, x.c), add(y.a, y.c));  // (a + b)(..), (a + c)(..)
    const auto ra = add(q_mul_s(norm(sub(sub(m1.b, m0.b), m1.a))), m0.a);
    const auto rb = add(sub(sub(m2.a, m0.a), m0.b), q_mul_s(m1.a));
    const auto rc = add(sub(sub(m2.b, m0.a), m1.a), m0.b);
    return norm(mkq(ra, rb, rc));
}
// Granger-Scott squaring in the cyclotomic subgroup (tower_lz.h f12_cyc_sqr)
template <int A, int B>
DEV auto q12_cyc_sqr(const Q12<A, B>& x) {
    const auto a2 = q4_sqr(x.a);
    const auto c2s = norm(q_mul_s(q4_sqr(x.c)));
    const auto b2 = q4_sqr(x.b);
    const auto ra = add(a2, dbl(sub(a2, q_conj4(x.a))));
    const auto rb = add(c2s, dbl(add(c2s, q_conj4(x.b))));
    const auto rc = add(b2, dbl(sub(b2, q_conj4(x.c))));
    return norm(mkq(ra, rb, rc));
}
// x^p, x^(p^2) coefficient-wise (tower_lz.h f12_frob / f12_frob2): the coefficient held by component j
// of a, b, c is AMCL slot 3j, 3j + 1, 3j + 2 (gamma_0 = 1: pair 0 multiplies a by one, quad-uniform)
template <int A, int B>
DEV auto q12_frob(const Q12<A, B>& x) {
    const bool j = qhi();
    const auto z = [&](const F2<A, B>& c, int k) { return mulr(conj(c), qsel(j, ld_gamma1(k + 3), ld_gamma1(k))); };
    return mkq(z(x.a, 0), z(x.b, 1), z(x.c, 2));
}
template <int A, int B>
DEV auto q12_frob2(const Q12<A, B>& x) {
    const bool j = qhi();
    const auto z = [&](const F2<A, B>& c, int k) { return mul_fpr(c, sel(j, ld_gamma2(k + 3), ld_gamma2(k))); };
    return mkq(z(x.a, 0), z(x.b, 1), z(x.c, 2));
}
// (u + v s)^-1 = (u - v s) / (u^2 - xi v^2)
template <int A, int B>
DEV auto q4_inv(const F2<A, B>& x) {
    const bool j = qhi();
    const auto sq = sqrr(x);
    const auto psq = qx(sq);
    const auto nrm = norm(qsel(j, sub(psq, xi(sq)), sub(sq, xi(psq))));  // u^2 - xi v^2 on both pairs
    const auto ni = qinv(nrm);
    const auto r = mulr(x, ni);
    return qsel(j, neg(r), r);
}
// tower_lz.h f12_inv
template <int A, int B>
DEV auto q12_inv(const Q12<A, B>& x) {
    const auto m0 = q4_mul2(x.b, x.c, x.a, x.b);  // bc, ab
    const auto A0 = norm(sub(q4_sqr(x.a), q_mul_s(m0.a)));            // a^2 - s bc
    const auto B0 = norm(sub(q_mul_s(q4_sqr(x.c)), m0.b));            // s c^2 - ab
    const auto C0 = norm(sub(q4_sqr(x.b), q4_mul1(x.a, x.c)));        // b^2 - ac
    const auto m1 = q4_mul2(x.c, B0, x.b, C0);                         // c B0, b C0
    const auto F = norm(add(q_mul_s(norm(add(m1.a, m1.b))), q4_mul1(x.a, A0)));
    const auto Fi = norm(q4_inv(F));
    const auto m2 = q4_mul2(A0, Fi, B0, Fi);
    return norm(mkq(m2.a, m2.b, q4_mul1(C0, Fi)));
}

}  // namespace lz
}  // namespace cc
