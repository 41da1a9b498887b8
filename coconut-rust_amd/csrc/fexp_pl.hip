// Final-exponentiation kernel for gfx950 (AMCL `pair::fexp` via amcl_wrapper `GT::ate_2_pairing`,
// reference src/lib.rs:13), pair-lane form (tower_pl.h): one credential per
// pair of adjacent lanes, each lane holding one half of every Fp2 value.
//
// CC_FP_INLINE: the multiplications are inlined inside each step function; the steps themselves are
// out of line and exchange Fp12 values through a per-lane SoA scratch (one load/store per step,
// against thousands of Fp multiplications per step), so each step's code exists once.
#ifdef CC_HOT_INLINE  // build option (Makefile HOT_INLINE=1): inline every Fp multiplication
#define CC_FP_INLINE 1
#endif
#include <cstdlib>
#include <cstring>
#include "codec.h"
#include "lazy.h"  // LZ_ONE_LIMBS (k_wide_pairs)
#include "tower_q.h"  // lz::fp_inv_int_quad (the wide forms' inversions)
#include "tower_pl.h"

namespace cc {
namespace pl {

// ================================================================ final exponentiation
// f^((p^6-1)(p^2+1)) then the hard part 3 + (x-1)^2 [p^3 + x p^2 + (x^2-1) p + x^3 - x]
// (= 3*Phi_12(p)/r, AMCL's exponent).  Each step below is one out-of-line function reading its
// Fp12 operands from, and writing its result to, a per-lane SoA slot (12 Fp slots each).
enum FxOp { OP_ID = 0, OP_CONJ = 1, OP_FROB = 2, OP_FROB2 = 3 };
template <bool W>
DEV void m12(Fp12& r, const Fp12& x, const Fp12& y);  // f12_mul, wide when W (below)
template <bool W>
DEV void cs12(Fp12& r, const Fp12& x);  // f12_cyc_sqr, wide when W (below)
DEV void f12_inv_wide(Fp12& r, const Fp12& x);  // f12_inv, wide (below)

DEV void fx_apply(Fp12& x, int op) {
    if (op == OP_CONJ) {
        f12_conj(x, x);
    } else if (op == OP_FROB) {
        Fp12 t = x;
        f12_frob(x, t);
    } else if (op == OP_FROB2) {
        Fp12 t = x;
        f12_frob2(x, t);
    }
}
DEV void f12_frobs_wide(Fp12& x, int op);  // the Frobenius maps spread over the lane pairs (below)
template <bool W>
DEV void fx_apply_w(Fp12& x, int op) {
    if (W && (op == OP_FROB || op == OP_FROB2)) f12_frobs_wide(x, op);
    else fx_apply(x, op);
}

// dst <- src^-1 (templated like every step: the one-wave kernel's looser register bound must not
// reach k_fexp through a shared out-of-line function)
template <bool W>
static __device__ __noinline__ void fx_inv(Soa src, Soa dst, size_t i) {
    Fp12 f, t;
    ld_f12(f, src, i);
    if (W) f12_inv_wide(t, f);
    else f12_inv(t, f);
    st_f12(dst, i, t);
}

// dst <- src^3 (cyclotomic)
template <bool W>
static __device__ __noinline__ void fx_cube(Soa src, Soa dst, size_t i) {
    Fp12 f, r;
    ld_f12(f, src, i);
    cs12<W>(r, f);
    m12<W>(r, r, f);
    st_f12(dst, i, r);
}

// dst <- src^x, x = -|x| (cyclotomic square-and-multiply, then conj).  The base is re-read from src at
// each of the 5 multiplications instead of being held in registers across the 63 squarings.
// Fallback of fx_pow_x below for the (never honestly reached) case of a zero decompression
// denominator.
template <bool W>
static __device__ __noinline__ void fx_pow_x_gs(Soa src, Soa dst, size_t i) {
    Fp12 acc;
    ld_f12(acc, src, i);
    for (int b = 62; b >= 0; b--) {
        cs12<W>(acc, acc);
        if ((X_ABS >> b) & 1ull) {
            asm volatile("" ::: "memory");  // keep the reload inside the loop
            Fp12 y;
            ld_f12(y, src, i);
            m12<W>(acc, acc, y);
        }
    }
    f12_conj(acc, acc);
    st_f12(dst, i, acc);
}

// ---------------------------------------------------------------- compressed cyclotomic squaring
// Karabina's compression (eprint 2010/542) restated for this tower.  For x = a + b w + c w^2 in the
// cyclotomic subgroup (a = a0 + a1 s, b = b0 + b1 s, c = c0 + c1 s), Granger-Scott's b', c' depend on
// b and c only:
//     b0' = 6 xi c0 c1 + 2 b0      b1' = 3 (c0^2 + xi c1^2) - 2 b1
//     c0' = 3 (b0^2 + xi b1^2) - 2 c0      c1' = 6 b0 b1 + 2 c1
// with 2 uv = (u + v)^2 - u^2 - v^2: six Fp2 squarings (392 mads a lane each) against Granger-Scott's
// six Fp2 multiplications (588).  a is recovered from x conj(x) = 1 (its w and w^2 coefficients are
// linear in a0, a1):
//     a0 = (b0 Nb + xi c1 Nc) / D,  a1 = (c0 Nc + b1 Nb) / D,
//     Nb = b0^2 - xi b1^2,  Nc = c0^2 - xi c1^2,  D = 2 (b0 c0 - xi b1 c1).
// (tests/test_fexp_algebra.py checks both against the oracle's Fp12 arithmetic.)
struct Cyc4 {
    Fp2 b0, b1, c0, c1;
};

// r = 3 u + 2 v  /  3 u - 2 v   (u + 2 (u +- v))
DEV void f2_3u_p2v(Fp2& r, const Fp2& u, const Fp2& v) {
    Fp2 t;
    f2_add(t, u, v);
    f2_dbl(t, t);
    f2_add(r, t, u);
}
DEV void f2_3u_m2v(Fp2& r, const Fp2& u, const Fp2& v) {
    Fp2 t;
    f2_sub(t, u, v);
    f2_dbl(t, t);
    f2_add(r, t, u);
}

DEV void cyc4_sqr(Cyc4& x) {
    Fp2 s0, s1, t, Tb, Xb, Tc, Xc;
    f2_sqr(s0, x.b0);
    f2_sqr(s1, x.b1);
    f2_add_lz(t, x.b0, x.b1);
    f2_sqr(Xb, t);
    f2_sub(Xb, Xb, s0);
    f2_sub(Xb, Xb, s1);  // 2 b0 b1
    f2_mul_xi(s1, s1);
    f2_add(Tb, s0, s1);  // b0^2 + xi b1^2
    f2_sqr(s0, x.c0);
    f2_sqr(s1, x.c1);
    f2_add_lz(t, x.c0, x.c1);
    f2_sqr(Xc, t);
    f2_sub(Xc, Xc, s0);
    f2_sub(Xc, Xc, s1);
    f2_mul_xi(Xc, Xc);   // 2 xi c0 c1
    f2_mul_xi(s1, s1);
    f2_add(Tc, s0, s1);  // c0^2 + xi c1^2
    f2_3u_p2v(x.b0, Xc, x.b0);
    f2_3u_m2v(x.b1, Tc, x.b1);
    f2_3u_m2v(x.c0, Tb, x.c0);
    f2_3u_p2v(x.c1, Xb, x.c1);
}

// numerators (n0, n1) and denominator D of a0, a1
DEV void cyc4_num(Fp2& n0, Fp2& n1, Fp2& den, const Cyc4& x) {
    Fp2 s0, s1, Nb, Nc, t;
    f2_sqr(s0, x.b0);
    f2_sqr(s1, x.b1);
    f2_mul_xi(s1, s1);
    f2_sub(Nb, s0, s1);
    f2_sqr(s0, x.c0);
    f2_sqr(s1, x.c1);
    f2_mul_xi(s1, s1);
    f2_sub(Nc, s0, s1);
    f2_mul(n0, x.b0, Nb);
    f2_mul(t, x.c1, Nc);
    f2_mul_xi(t, t);
    f2_add(n0, n0, t);
    f2_mul(n1, x.c0, Nc);
    f2_mul(t, x.b1, Nb);
    f2_add(n1, n1, t);
    f2_mul(den, x.b0, x.c0);
    f2_mul(t, x.b1, x.c1);
    f2_mul_xi(t, t);
    f2_sub(den, den, t);
    f2_dbl(den, den);
}

DEV void cyc4_expand(Fp12& r, const Cyc4& x, const Fp2& n0, const Fp2& n1, const Fp2& inv) {
    f2_mul(r.a.a, n0, inv);
    f2_mul(r.a.b, n1, inv);
    r.b.a = x.b0;
    r.b.b = x.b1;
    r.c.a = x.c0;
    r.c.b = x.c1;
}

// ---------------------------------------------------------------- wide forms (k_fexp1: one element a wave)
// A latency-bound final exponentiation (the RLC batch mode's one per batch, and every credential of
// a small batch) runs on ONE wave: the 32 lane pairs hold the same element, and the independent Fp2
// products of a step are spread over them — the 6 squarings of cyc4_sqr, the 18 products of
// f12_mul, the 6 of f12_cyc_sqr — as ONE call (same instructions, different data), the results
// gathered with ds_bpermute shuffles.  A step's latency then holds one product instead of 6 or 18.
// The combinations are spread too (round 5): a lone wave's time is its instruction count, so no
// pair redoes what another pair computes (f12w_assemble, cyc4_sqr_dist, f12_cyc_sqr_wide).
DEV int pair_idx() { return (int)(threadIdx.x >> 1); }
// tower_pl.h f2_inv for a value every pair of the wave holds: the norm is then the same on all four
// lanes of each quad, so its divstep inversion runs in the quad form (tower_q.h fp_inv_int_quad: the
// iteration's f, g, d, e one per lane, one update chain a lane instead of four)
DEV void f2_inv_q(Fp2& r, const Fp2& x) {
    const Fp xs = swp(x.c);
    Fp n = fp_mul2_v(x.c, x.c, xs, xs), ni;
    lz::fp_inv_int_quad(ni, n);  // plain integer inverse of the Montgomery residue
    constexpr uint32_t R3[NL] = {CC_R3_LIMBS};
    Fp r3;
#pragma unroll
    for (int j = 0; j < NL; j++) r3.v[j] = R3[j];
    fp_mul(n, ni, r3);  // (n R)^-1 R^3 R^-1 = n^-1 R (field.h fp_inv)
    Fp2 t;
    fp_mul(t.c, x.c, n);
    f2_conj(r, t);
}
DEV Fp2 bcast_f2(const Fp2& v, int src_pair) {
    const int lane = 2 * src_pair + (int)half_id();
    Fp2 r;
#pragma unroll
    for (int k = 0; k < NL; k++) r.c.v[k] = (uint32_t)__shfl((int)v.c.v[k], lane);
    return r;
}
DEV Fp2 f2_pick(int j, const Fp2* opts, int nopt) {
    Fp2 r = opts[0];
    for (int k = 1; k < nopt; k++) r.c = fp_sel(j == k, opts[k].c, r.c);
    return r;
}

DEV void cyc4_sqr_wide(Cyc4& x) {
    const int j = pair_idx() % 6;
    Fp2 opt[6];
    opt[0] = x.b0;
    opt[1] = x.b1;
    f2_add_lz(opt[2], x.b0, x.b1);
    opt[3] = x.c0;
    opt[4] = x.c1;
    f2_add_lz(opt[5], x.c0, x.c1);
    Fp2 in = f2_pick(j, opt, 6), sq;
    f2_sqr(sq, in);
    Fp2 s0 = bcast_f2(sq, 0), s1 = bcast_f2(sq, 1), Xb = bcast_f2(sq, 2);
    Fp2 Tb, Tc, Xc;
    f2_sub(Xb, Xb, s0);
    f2_sub(Xb, Xb, s1);  // 2 b0 b1
    f2_mul_xi(s1, s1);
    f2_add(Tb, s0, s1);  // b0^2 + xi b1^2
    s0 = bcast_f2(sq, 3);
    s1 = bcast_f2(sq, 4);
    Xc = bcast_f2(sq, 5);
    f2_sub(Xc, Xc, s0);
    f2_sub(Xc, Xc, s1);
    f2_mul_xi(Xc, Xc);   // 2 xi c0 c1
    f2_mul_xi(s1, s1);
    f2_add(Tc, s0, s1);  // c0^2 + xi c1^2
    f2_3u_p2v(x.b0, Xc, x.b0);
    f2_3u_m2v(x.b1, Tc, x.b1);
    f2_3u_m2v(x.c0, Tb, x.c0);
    f2_3u_p2v(x.c1, Xb, x.c1);
}

// cyc4_sqr with the state spread: pair q (mod 4) holds component q of (b0, b1, c0, c1).  Pair t (mod 6)
// squares b0, b1, b0 + b1, c0, c1, c0 + c1 (its inputs gathered from pairs 0..3), then pair q forms its
// new component from three gathered squares S_t:
//     b0' = 3 xi (S5 - S3 - S4) + 2 b0     b1' = 3 (S3 + xi S4) - 2 b1
//     c0' = 3 (S0 + xi S1) - 2 c0          c1' = 3 (S2 - S0 - S1) + 2 c1
// — the same values as cyc4_sqr_wide without every pair redoing all four.
DEV void cyc4_sqr_dist(Fp2& V) {
    const int j = pair_idx(), t = j % 6, q = j & 3;
    Fp2 a = bcast_f2(V, (0x232010 >> (4 * t)) & 15), b = bcast_f2(V, (0x300100 >> (4 * t)) & 15), s, sq;
    f2_add_lz(s, a, b);
    a.c = fp_sel(t == 2 || t == 5, s.c, a.c);
    f2_sqr(sq, a);
    const Fp2 G1 = bcast_f2(sq, (0x2035 >> (4 * q)) & 15), G2 = bcast_f2(sq, (0x0143 >> (4 * q)) & 15),
              G3 = bcast_f2(sq, (0x1004 >> (4 * q)) & 15);
    const bool xf = q == 0 || q == 3;  // X family: G1 - G2 - G3 (times xi for b0'); else T: G1 + xi G2
    Fp2 x, u, w;
    f2_sub(x, G1, G2);
    f2_sub(x, x, G3);
    f2_mul_xi(u, x);
    x.c = fp_sel(q == 0, u.c, x.c);
    f2_mul_xi(u, G2);
    f2_add(w, G1, u);
    u = w;
    u.c = fp_sel(xf, x.c, w.c);
    f2_neg(w, V);  // 3u + 2V = u + 2 (u + V) (X family), 3u - 2V = u + 2 (u - V) (T family)
    w.c = fp_sel(xf, V.c, w.c);
    f2_add(w, u, w);
    f2_dbl(w, w);
    f2_add(V, w, u);
}
DEV void st_cyc4_dist(const Soa& K, int base, size_t i, const Fp2& V) {
    Cyc4 c{bcast_f2(V, 0), bcast_f2(V, 1), bcast_f2(V, 2), bcast_f2(V, 3)};
    st_f2(K, base + 0, i, c.b0);
    st_f2(K, base + 2, i, c.b1);
    st_f2(K, base + 4, i, c.c0);
    st_f2(K, base + 6, i, c.c1);
}
// cyc4_sqr_dist on the lazy field (lazy.h: 14 signed 28-bit limbs, R' form, bounds in the types): the
// same values, with the squaring's Montgomery product and the combination's additions in the lazy
// form (carry-free additions, one reduction a step) instead of the storage form's canonical ones.
using LzF2 = lz::F2<lz::AN, 9>;
DEV LzF2 bcast_lz(const LzF2& v, int src_pair) {
    const int lane = 2 * src_pair + (int)half_id();
    LzF2 r;
#pragma unroll
    for (int k = 0; k < lz::LN; k++) r.c.v[k] = __shfl(v.c.v[k], lane);
    return r;
}
template <int A, int B>
DEV lz::F2<A, B> sel2(bool c, const lz::F2<A, B>& x, const lz::F2<A, B>& y) { return {lz::sel(c, x.c, y.c)}; }
DEV void cyc4_sqr_dist_lz(LzF2& V) {
    using namespace lz;
    const int j = pair_idx(), t = j % 6, q = j & 3;
    const LzF2 a = bcast_lz(V, (0x232010 >> (4 * t)) & 15), b = bcast_lz(V, (0x300100 >> (4 * t)) & 15);
    const auto s = add(a, b);
    const auto in = sel2(t == 2 || t == 5, s, fit<decltype(s)::AV, decltype(s)::BV>(a));
    const LzF2 sq = reduce(sqrr_in(in));
    const LzF2 G1 = bcast_lz(sq, (0x2035 >> (4 * q)) & 15), G2 = bcast_lz(sq, (0x0143 >> (4 * q)) & 15),
               G3 = bcast_lz(sq, (0x1004 >> (4 * q)) & 15);
    const bool xf = q == 0 || q == 3;  // X family: G1 - G2 - G3 (times xi for b0'); else T: G1 + xi G2
    const auto x = sub(sub(G1, G2), G3);
    const auto xx = xi(x);
    const auto w = add(G1, xi(G2));
    using U = F2<decltype(xx)::AV, decltype(xx)::BV>;
    const U u0 = sel2(q == 0, xx, fit<U::AV, U::BV>(x));
    const auto u = squeeze(sel2(xf, u0, fit<U::AV, U::BV>(w)));
    const auto y = sel2(xf, V, neg(V));  // 3u + 2V = u + 2 (u + V) (X family), 3u - 2V = u + 2 (u - V) (T)
    V = reduce(add(u, dbl(add(u, y))));
}
// the full compressed state (b0, b1, c0, c1) in the storage form at K slots base.. (each pair converts
// its own component, then four broadcasts)
DEV void st_cyc4_dist_lz(const Soa& K, int base, size_t i, const LzF2& V) {
    const Fp2 own = lz::out_r2(V);
    st_cyc4_dist(K, base, i, own);
}

// f4_mul's three products of operand set m, spread: pair 3m + p computes product p
DEV void f4_from_products(Fp4& r, const Fp2& p0, const Fp2& p1, const Fp2& p2) {
    Fp2 t;
    f2_mul_xi(t, p1);
    f2_add(r.a, p0, t);
    f2_sub(t, p2, p0);
    f2_sub(r.b, t, p1);
}

// = f12_mul (tower.inc): the six f4 products (t0, t1, t2 and the three cross terms) as 18 Fp2
// products on pairs 0..17 — f12w_operands picks pair j's two factors, f12w_assemble combines the
// products (so a caller can run other independent products on pairs 18..31 in the same call).
// Operand m of the six (a, b, c, b + c, a + b, a + c) is formed by each pair for its own m only: one
// pick of its first term, one of its second (zero for m < 3), one f4 addition.
DEV Fp4 f4_pick3(int k, const Fp4& a, const Fp4& b, const Fp4& c) {  // k in {0, 1, 2}
    Fp4 r = a;
    r.a.c = fp_sel(k == 1, b.a.c, r.a.c);
    r.b.c = fp_sel(k == 1, b.b.c, r.b.c);
    r.a.c = fp_sel(k == 2, c.a.c, r.a.c);
    r.b.c = fp_sel(k == 2, c.b.c, r.b.c);
    return r;
}
DEV Fp4 f12w_term(int m, const Fp12& x) {
    // first term a b c b a a, second - - - c b c (m = 0..5)
    Fp4 u = f4_pick3((0x001210 >> (4 * m)) & 15, x.a, x.b, x.c);
    Fp4 v = f4_pick3((0x212000 >> (4 * m)) & 15, x.a, x.b, x.c);
    Fp4 r;
    f4_add(r, u, v);
    r.a.c = fp_sel(m < 3, u.a.c, r.a.c);
    r.b.c = fp_sel(m < 3, u.b.c, r.b.c);
    return r;
}
DEV void f12w_operands(Fp2& o1, Fp2& o2, int j, const Fp12& x, const Fp12& y) {
    j %= 18;
    const int m = j / 3, p = j % 3;
    const Fp4 U = f12w_term(m, x), V = f12w_term(m, y);
    Fp2 s1, s2;
    o1 = U.a;
    o2 = V.a;
    f2_add_lz(s1, U.a, U.b);
    f2_add_lz(s2, V.a, V.b);
    o1.c = fp_sel(p == 1, U.b.c, o1.c);
    o2.c = fp_sel(p == 1, V.b.c, o2.c);
    o1.c = fp_sel(p == 2, s1.c, o1.c);
    o2.c = fp_sel(p == 2, s2.c, o2.c);
}
// The combination, spread: (1) pair k < 12 forms component k & 1 of Fp4 result k / 2 (t0, t1, t2 and
// the three cross products, f4_mul's (p0 + xi p1, p2 - p0 - p1)) from its three products, gathered
// with one shuffle each; (2) pair q < 6 forms Fp12 coefficient q (a.a, a.b, b.a, b.b, c.a, c.b) as
// xi^[q = 0] (G1 - G2 - G3) + xi^[q = 2] G4 from four components of step 1:
//     a.a = xi (s_bc.b - t1.b - t2.b) + t0.a     a.b = s_bc.a - t1.a - t2.a + t0.b
//     b.a = s_ab.a - t0.a - t1.a + xi t2.b       b.b = s_ab.b - t0.b - t1.b + t2.a
//     c.a = s_ac.a - t0.a - t2.a + t1.a          c.b = s_ac.b - t0.b - t2.b + t1.b
// (3) the six coefficients broadcast to every pair.  Same field values as the sequential assembly.
DEV void f12w_assemble(Fp12& r, const Fp2& prod, int base = 0) {
    const int j = pair_idx();
    Fp2 C;
    {
        const int k = j % 12, m = k >> 1;
        const Fp2 p0 = bcast_f2(prod, base + 3 * m), p1 = bcast_f2(prod, base + 3 * m + 1),
                  p2 = bcast_f2(prod, base + 3 * m + 2);
        Fp2 t, ca, cb;
        f2_mul_xi(t, p1);
        f2_add(ca, p0, t);
        f2_sub(t, p2, p0);
        f2_sub(cb, t, p1);
        C = ca;
        C.c = fp_sel(k & 1, cb.c, ca.c);
    }
    Fp2 O;
    {
        const int q = j % 6;
        const Fp2 G1 = bcast_f2(C, (0xBA9867 >> (4 * q)) & 15), G2 = bcast_f2(C, (0x101023 >> (4 * q)) & 15),
                  G3 = bcast_f2(C, (0x543245 >> (4 * q)) & 15);
        Fp2 G4 = bcast_f2(C, (0x324510 >> (4 * q)) & 15), u, v;
        f2_sub(u, G1, G2);
        f2_sub(u, u, G3);
        f2_mul_xi(v, u);
        u.c = fp_sel(q == 0, v.c, u.c);
        f2_mul_xi(v, G4);
        G4.c = fp_sel(q == 2, v.c, G4.c);
        f2_add(O, u, G4);
    }
    r.a.a = bcast_f2(O, 0);
    r.a.b = bcast_f2(O, 1);
    r.b.a = bcast_f2(O, 2);
    r.b.b = bcast_f2(O, 3);
    r.c.a = bcast_f2(O, 4);
    r.c.b = bcast_f2(O, 5);
}
DEV void f12_mul_wide(Fp12& r, const Fp12& x, const Fp12& y) {
    Fp2 o1, o2, prod;
    f12w_operands(o1, o2, pair_idx(), x, y);
    f2_mul(prod, o1, o2);
    f12w_assemble(r, prod);
}

// = f12_cyc_sqr (Granger-Scott): f4_sqr of a, b, c as 6 products on pairs 0..5 (pair 2m: ab,
// pair 2m + 1: (a + b)(a + xi b) of operand m)
DEV void f12_cyc_sqr_wide(Fp12& r, const Fp12& x) {
    const int j = pair_idx() % 6;
    const int m = j >> 1;
    Fp2 oa[3] = {x.a.a, x.b.a, x.c.a}, ob[3] = {x.a.b, x.b.b, x.c.b};
    const Fp2 a = f2_pick(m, oa, 3), b = f2_pick(m, ob, 3);
    Fp2 o1 = a, o2 = b, s0, s1, prod;
    f2_add_lz(s0, a, b);
    f2_mul_xi(s1, b);
    f2_add_lz(s1, s1, a);
    o1.c = fp_sel(j & 1, s0.c, o1.c);
    o2.c = fp_sel(j & 1, s1.c, o2.c);
    f2_mul(prod, o1, o2);
    // the combination, spread: pair q < 6 forms coefficient q (a.a, a.b, b.a, b.b, c.a, c.b) of
    //   a' = 3A - 2 conj(a), b' = 3 s C + 2 conj(b), c' = 3 B - 2 conj(c)   (A, B, C the f4 squares:
    //   (t - ab - xi ab, 2ab) from pair 2m's ab and pair 2m + 1's t = (a + b)(a + xi b))
    // as 3u - 2y with u = t - ab - xi ab (a.a, b.b, c.a) or 3u + 2y with u = 2ab (xi 2ab for b.a)
    const int q = pair_idx() % 6;
    const Fp2 Gab = bcast_f2(prod, (0x224400 >> (4 * q)) & 15), Gt = bcast_f2(prod, (0x135111 >> (4 * q)) & 15);
    const bool fa = q == 0 || q == 3 || q == 4;
    Fp2 u, v, w, y;
    f2_sub(u, Gt, Gab);
    f2_mul_xi(v, Gab);
    f2_sub(u, u, v);
    f2_dbl(w, Gab);
    f2_mul_xi(v, w);
    w.c = fp_sel(q == 2, v.c, w.c);
    u.c = fp_sel(fa, u.c, w.c);
    const Fp2 cs[6] = {x.a.a, x.a.b, x.b.a, x.b.b, x.c.a, x.c.b};
    y = f2_pick(q, cs, 6);
    f2_neg(v, y);
    y.c = fp_sel(fa, v.c, y.c);
    f2_add(w, u, y);  // u +- y
    f2_dbl(w, w);
    f2_add(v, w, u);  // 3u +- 2y
    r.a.a = bcast_f2(v, 0);
    r.a.b = bcast_f2(v, 1);
    r.b.a = bcast_f2(v, 2);
    r.b.b = bcast_f2(v, 3);
    r.c.a = bcast_f2(v, 4);
    r.c.b = bcast_f2(v, 5);
}

// acc <- x z (f12_mul_wide, pairs 0..17) and y <- y^2 (f12_cyc_sqr_wide, pairs 18..23) in ONE level:
// pow-by-x's tail multiplies acc by snapshots of y while y keeps squaring (each operand read before
// either result is written, so z may be y)
DEV void f12_mul_cs_wide(Fp12& acc, const Fp12& x, const Fp12& z, Fp12& y) {
    const int j = pair_idx();
    Fp2 o1, o2, prod;
    f12w_operands(o1, o2, j, x, z);
    {
        const int jc = j % 6;  // pairs 18..23: product jc = j - 18
        const int m = jc >> 1;
        Fp2 oa[3] = {y.a.a, y.b.a, y.c.a}, ob[3] = {y.a.b, y.b.b, y.c.b};
        const Fp2 a = f2_pick(m, oa, 3), b = f2_pick(m, ob, 3);
        Fp2 c1 = a, c2 = b, s0, s1;
        f2_add_lz(s0, a, b);
        f2_mul_xi(s1, b);
        f2_add_lz(s1, s1, a);
        c1.c = fp_sel(jc & 1, s0.c, c1.c);
        c2.c = fp_sel(jc & 1, s1.c, c2.c);
        o1.c = fp_sel(j >= 18, c1.c, o1.c);
        o2.c = fp_sel(j >= 18, c2.c, o2.c);
    }
    f2_mul(prod, o1, o2);
    Fp2 v;
    {  // f12_cyc_sqr_wide's combination, its products on pairs 18..23
        const int q = j % 6;
        const Fp2 Gab = bcast_f2(prod, 18 + ((0x224400 >> (4 * q)) & 15)),
                  Gt = bcast_f2(prod, 18 + ((0x135111 >> (4 * q)) & 15));
        const bool fa = q == 0 || q == 3 || q == 4;
        Fp2 u, w, t;
        f2_sub(u, Gt, Gab);
        f2_mul_xi(t, Gab);
        f2_sub(u, u, t);
        f2_dbl(w, Gab);
        f2_mul_xi(t, w);
        w.c = fp_sel(q == 2, t.c, w.c);
        u.c = fp_sel(fa, u.c, w.c);
        const Fp2 cs[6] = {y.a.a, y.a.b, y.b.a, y.b.b, y.c.a, y.c.b};
        Fp2 yy = f2_pick(q, cs, 6);
        f2_neg(t, yy);
        yy.c = fp_sel(fa, t.c, yy.c);
        f2_add(w, u, yy);
        f2_dbl(w, w);
        f2_add(v, w, u);
    }
    f12w_assemble(acc, prod);
    y.a.a = bcast_f2(v, 0);
    y.a.b = bcast_f2(v, 1);
    y.b.a = bcast_f2(v, 2);
    y.b.b = bcast_f2(v, 3);
    y.c.a = bcast_f2(v, 4);
    y.c.b = bcast_f2(v, 5);
}

// f12_frob / f12_frob2 (pairing.inc) spread: pair q < 6 maps coefficient q (a.a, a.b, b.a, b.b, c.a,
// c.b; the coefficient of W^k, k = 0 3 1 4 2 5): conj(c) gamma1_k, or c gamma2_k (gamma_0 = 1), then
// the six are broadcast
DEV void f12_frobs_wide(Fp12& x, int op) {
    const int q = pair_idx() % 6, k = (0x524130 >> (4 * q)) & 15;
    const Fp2 cs[6] = {x.a.a, x.a.b, x.b.a, x.b.b, x.c.a, x.c.b};
    Fp2 c = f2_pick(q, cs, 6), r;
    if (op == OP_FROB) {  // wave-uniform
        Fp2 g, t;
        load_f2c(g, kGamma1[k]);
        f2_conj(t, c);
        f2_mul(r, t, g);
    } else {
        Fp g;
#pragma unroll
        for (int j = 0; j < NL; j++) g.v[j] = kGamma2[k][j];
        f2_mul_fp(r, c, g);
    }
    x.a.a = bcast_f2(r, 0);
    x.a.b = bcast_f2(r, 1);
    x.b.a = bcast_f2(r, 2);
    x.b.b = bcast_f2(r, 3);
    x.c.a = bcast_f2(r, 4);
    x.c.b = bcast_f2(r, 5);
}

// k Fp4 products x_m y_m (m < k <= 10) as 3k Fp2 products on pairs 0..3k-1 (f4_mul's Karatsuba: pair
// 3m + p forms x.a y.a, x.b y.b, (x.a + x.b)(y.a + y.b) for p = 0, 1, 2); every pair gets all k results
DEV void f4w_mul(Fp4* r, const Fp4* x, const Fp4* y, int k) {
    const int j = pair_idx() % (3 * k), m = j / 3, p = j % 3;
    Fp2 xa[10], xb[10], ya[10], yb[10];
    for (int t = 0; t < k; t++) {
        xa[t] = x[t].a; xb[t] = x[t].b; ya[t] = y[t].a; yb[t] = y[t].b;
    }
    const Fp2 Xa = f2_pick(m, xa, k), Xb = f2_pick(m, xb, k), Ya = f2_pick(m, ya, k), Yb = f2_pick(m, yb, k);
    Fp2 o1 = Xa, o2 = Ya, s1, s2, pr;
    f2_add_lz(s1, Xa, Xb);
    f2_add_lz(s2, Ya, Yb);
    o1.c = fp_sel(p == 1, Xb.c, o1.c);
    o2.c = fp_sel(p == 1, Yb.c, o2.c);
    o1.c = fp_sel(p == 2, s1.c, o1.c);
    o2.c = fp_sel(p == 2, s2.c, o2.c);
    f2_mul(pr, o1, o2);
    for (int t = 0; t < k; t++) f4_from_products(r[t], bcast_f2(pr, 3 * t), bcast_f2(pr, 3 * t + 1), bcast_f2(pr, 3 * t + 2));
}

// = f12_inv (tower.inc) for the one-element kernel: its 40 Fp2 products as five spread calls and the
// one inversion (a^2, bc, c^2, ab, b^2, ac | c B0, b C0, a A0 | F.a^2, F.b^2 | inverse | A0, B0, C0 by 1/F)
DEV void f12_inv_wide(Fp12& r, const Fp12& x) {
    Fp4 P[6];
    {
        const Fp4 X[6] = {x.a, x.b, x.c, x.a, x.b, x.a}, Y[6] = {x.a, x.c, x.c, x.b, x.b, x.c};
        f4w_mul(P, X, Y, 6);
    }
    Fp4 A0, B0, C0, t;
    f4_mul_s(t, P[1]);
    f4_sub(A0, P[0], t);  // a^2 - s bc
    f4_mul_s(t, P[2]);
    f4_sub(B0, t, P[3]);  // s c^2 - ab
    f4_sub(C0, P[4], P[5]);  // b^2 - ac
    Fp4 F;
    {
        const Fp4 X[3] = {x.c, x.b, x.a}, Y[3] = {B0, C0, A0};
        f4w_mul(P, X, Y, 3);
        f4_add(F, P[0], P[1]);
        f4_mul_s(F, F);
        f4_add(F, F, P[2]);
    }
    Fp2 n, pr, u, v;
    {  // f4_inv: pairs 0, 1 square F.a, F.b
        const int j = pair_idx() & 1;
        Fp2 in = F.a;
        in.c = fp_sel(j == 1, F.b.c, in.c);
        f2_sqr(pr, in);
        f2_mul_xi(u, bcast_f2(pr, 1));
        f2_sub(n, bcast_f2(pr, 0), u);  // a^2 - xi b^2
    }
    f2_inv_q(n, n);
    {
        const int j = pair_idx() & 1;
        Fp2 in = F.a;
        in.c = fp_sel(j == 1, F.b.c, in.c);
        f2_mul(pr, in, n);
        u = bcast_f2(pr, 0);
        v = bcast_f2(pr, 1);
    }
    Fp4 Fi;
    Fi.a = u;
    f2_neg(Fi.b, v);
    {
        const Fp4 X[3] = {A0, B0, C0}, Y[3] = {Fi, Fi, Fi};
        f4w_mul(P, X, Y, 3);
    }
    r.a = P[0];
    r.b = P[1];
    r.c = P[2];
}

template <bool W>
DEV void m12(Fp12& r, const Fp12& x, const Fp12& y) {
    if (W) f12_mul_wide(r, x, y);
    else f12_mul(r, x, y);
}
template <bool W>
DEV void cs12(Fp12& r, const Fp12& x) {
    if (W) f12_cyc_sqr_wide(r, x);
    else f12_cyc_sqr(r, x);
}
template <bool W>
DEV void c4s(Cyc4& x) {
    if (W) cyc4_sqr_wide(x);
    else cyc4_sqr(x);
}

// snapshot slots (Fp2 pairs) in the K region: per snapshot b0 b1 c0 c1 n0 n1
DEV void st_cyc4(const Soa& K, int base, size_t i, const Cyc4& x) {
    st_f2(K, base + 0, i, x.b0);
    st_f2(K, base + 2, i, x.b1);
    st_f2(K, base + 4, i, x.c0);
    st_f2(K, base + 6, i, x.c1);
}
DEV void ld_cyc4(Cyc4& x, const Soa& K, int base, size_t i) {
    ld_f2(x.b0, K, base + 0, i);
    ld_f2(x.b1, K, base + 2, i);
    ld_f2(x.c0, K, base + 4, i);
    ld_f2(x.c1, K, base + 6, i);
}

// dst <- src^x.  |x| = 2^63 + 2^62 + 2^60 + 2^57 + 2^48 + 2^16: 57 compressed squarings with
// snapshots g^(2^16), g^(2^48) stored to K; the three compressed values g^(2^16), g^(2^48), g^(2^57)
// decompressed with ONE inversion (Montgomery's trick); then g^(2^60), g^(2^62), g^(2^63) by six
// Granger-Scott squarings of g^(2^57) (cheaper than three more decompressions).  Five Fp12
// multiplications as before.  A zero denominator (b = c = 0 pattern; never reached by honest inputs,
// e.g. src = 1) sends the lane pair to the Granger-Scott ladder.
// The wide (one-element) form of the decompression: the three snapshots' 12 squarings, then their 18
// products, as two spread calls (pair j loads its operands from the scratch by index), the three
// denominators' pairwise products, ONE inversion, the three inverses and the six a-coefficients —
// six product latencies and the inversion, against the 42 products one after another of the
// per-lane form.  Snapshots (Cyc4, 8 slots each) at K slots 0 (g^(2^16)), 8 (g^(2^48)), 16 (g^(2^57));
// N_b, N_c and then the numerators in the scratch region X (12 slots; the chain's S, free during a
// pow-by-x).  Returns false on a zero denominator (the Granger-Scott fallback).
DEV bool decompress3_wide(Fp12& a16, Fp12& a48, Fp12& a57, const Soa& K, const Soa& X, size_t i) {
    const int j = pair_idx();
    {  // squarings of b0, b1, c0, c1 of each snapshot (pairs 0..11)
        const int jj = j % 12;
        Fp2 in, sq;
        ld_f2(in, K, 8 * (jj >> 2) + 2 * (jj & 3), i);
        f2_sqr(sq, in);
        for (int s = 0; s < 3; s++) {
            Fp2 t, u;
            f2_mul_xi(t, bcast_f2(sq, 4 * s + 1));
            f2_sub(u, bcast_f2(sq, 4 * s), t);  // N_b = b0^2 - xi b1^2
            st_f2(X, 4 * s, i, u);
            f2_mul_xi(t, bcast_f2(sq, 4 * s + 3));
            f2_sub(u, bcast_f2(sq, 4 * s + 2), t);  // N_c = c0^2 - xi c1^2
            st_f2(X, 4 * s + 2, i, u);
        }
    }
    Fp2 d[3];
    {  // per snapshot: b0 N_b, c1 N_c, c0 N_c, b1 N_b, b0 c0, b1 c1 (pairs 0..17)
        const int jj = j % 18, s = jj / 6, t = jj % 6;
        const int c1 = (0x101230 >> (4 * t)) & 15;  // first factor's component: b0 c1 c0 b1 b0 b1
        Fp2 o1, o2, pr;
        ld_f2(o1, K, 8 * s + 2 * c1, i);
        if (t < 4) ld_f2(o2, X, 4 * s + (t == 1 || t == 2 ? 2 : 0), i);
        else ld_f2(o2, K, 8 * s + (t == 4 ? 4 : 6), i);
        f2_mul(pr, o1, o2);
        for (int s2 = 0; s2 < 3; s2++) {
            Fp2 u, v;
            f2_mul_xi(u, bcast_f2(pr, 6 * s2 + 1));
            f2_add(v, bcast_f2(pr, 6 * s2), u);  // a0 numerator: b0 N_b + xi c1 N_c
            st_f2(X, 4 * s2, i, v);
            f2_add(v, bcast_f2(pr, 6 * s2 + 2), bcast_f2(pr, 6 * s2 + 3));  // a1 numerator: c0 N_c + b1 N_b
            st_f2(X, 4 * s2 + 2, i, v);
            f2_mul_xi(u, bcast_f2(pr, 6 * s2 + 5));
            f2_sub(v, bcast_f2(pr, 6 * s2 + 4), u);
            f2_dbl(d[s2], v);  // D = 2 (b0 c0 - xi b1 c1)
        }
    }
    Fp2 e[3], p2, inv;
    {  // pairs 0..2: d16 d48, d48 d57, d16 d57
        const int jj = j % 3;
        Fp2 pr;
        f2_mul(pr, f2_pick(jj == 1 ? 1 : 0, d, 3), f2_pick(jj == 0 ? 1 : 2, d, 3));
        for (int k = 0; k < 3; k++) e[k] = bcast_f2(pr, k);
    }
    f2_mul(p2, e[0], d[2]);
    if (f2_is_zero(p2)) return false;  // wave-uniform: every pair holds the same values
    f2_inv_q(inv, p2);
    Fp2 iv[3];
    {  // pairs 0..2: 1/d16 = inv d48 d57, 1/d48 = inv d16 d57, 1/d57 = inv d16 d48
        const int jj = j % 3;
        Fp2 pr;
        f2_mul(pr, inv, f2_pick(jj == 0 ? 1 : jj == 1 ? 2 : 0, e, 3));
        for (int k = 0; k < 3; k++) iv[k] = bcast_f2(pr, k);
    }
    {  // pairs 0..5: the a-coefficients, numerator (s, h) times 1/d_s
        const int jj = j % 6, s = jj >> 1;
        Fp2 nm, pr;
        ld_f2(nm, X, 4 * s + 2 * (jj & 1), i);
        f2_mul(pr, nm, f2_pick(s, iv, 3));
        Fp12* outs[3] = {&a16, &a48, &a57};
        for (int s2 = 0; s2 < 3; s2++) {
            Fp12& r = *outs[s2];
            r.a.a = bcast_f2(pr, 2 * s2);
            r.a.b = bcast_f2(pr, 2 * s2 + 1);
            ld_f2(r.b.a, K, 8 * s2, i);
            ld_f2(r.b.b, K, 8 * s2 + 2, i);
            ld_f2(r.c.a, K, 8 * s2 + 4, i);
            ld_f2(r.c.b, K, 8 * s2 + 6, i);
        }
    }
    return true;
}

template <bool W>
static __device__ __noinline__ void fx_pow_x(Soa src, Soa dst, Soa K, size_t i, Soa X) {
    Cyc4 c;
    ld_f2(c.b0, src, 4, i);
    ld_f2(c.b1, src, 6, i);
    ld_f2(c.c0, src, 8, i);
    ld_f2(c.c1, src, 10, i);
    if (W) {  // one element a wave (k_fexp1): the squarings' state and the decompression spread over the pairs
        LzF2 V;
        {
            Fp2 v;
            ld_f2(v, src, 4 + 2 * (pair_idx() & 3), i);
            V = lz::reduce(lz::in_r2(v));
        }
        for (int k = 1; k <= 57; k++) {
            cyc4_sqr_dist_lz(V);
            if (k == 16) st_cyc4_dist_lz(K, 0, i, V);
            if (k == 48) st_cyc4_dist_lz(K, 8, i, V);
        }
        st_cyc4_dist_lz(K, 16, i, V);
        Fp12 acc, t, y;
        if (!decompress3_wide(acc, t, y, K, X, i)) {
            fx_pow_x_gs<W>(src, dst, i);
            return;
        }
        // the tail's products of acc and its squarings of y pair up: 7 levels instead of 11
        const Fp12 y57 = y;
        f12_mul_cs_wide(acc, acc, t, y);    // acc = g^(2^16 + 2^48), y = g^(2^58)
        f12_mul_cs_wide(acc, acc, y57, y);  // acc *= g^(2^57), y = g^(2^59)
        f12_cyc_sqr_wide(y, y);             // 2^60
        f12_mul_cs_wide(acc, acc, y, y);    // acc *= g^(2^60), y = g^(2^61)
        f12_cyc_sqr_wide(y, y);             // 2^62
        f12_mul_cs_wide(acc, acc, y, y);    // acc *= g^(2^62), y = g^(2^63)
        f12_mul_wide(acc, acc, y);          // acc *= g^(2^63)
        f12_conj(acc, acc);
        st_f12(dst, i, acc);
        return;
    }
    for (int k = 1; k <= 57; k++) {
        c4s<W>(c);
        if (k == 16) st_cyc4(K, 0, i, c);
        if (k == 48) st_cyc4(K, 12, i, c);
    }
    Fp2 n0, n1, d57, d16, d48, p1, p2, inv;
    {
        Cyc4 s;
        ld_cyc4(s, K, 0, i);
        cyc4_num(n0, n1, d16, s);
        st_f2(K, 8, i, n0);
        st_f2(K, 10, i, n1);
        ld_cyc4(s, K, 12, i);
        cyc4_num(n0, n1, d48, s);
        st_f2(K, 20, i, n0);
        st_f2(K, 22, i, n1);
    }
    cyc4_num(n0, n1, d57, c);
    f2_mul(p1, d16, d48);
    f2_mul(p2, p1, d57);
    if (f2_is_zero(p2)) {  // pair-uniform
        fx_pow_x_gs<W>(src, dst, i);
        return;
    }
    f2_inv(inv, p2);
    Fp12 y, acc, t;
    {
        Fp2 i57;
        f2_mul(i57, inv, p1);
        cyc4_expand(y, c, n0, n1, i57);  // g^(2^57)
    }
    f2_mul(inv, inv, d57);               // (d16 d48)^-1
    {
        Cyc4 s;
        Fp2 ik;
        f2_mul(ik, inv, d48);
        ld_cyc4(s, K, 0, i);
        ld_f2(n0, K, 8, i);
        ld_f2(n1, K, 10, i);
        cyc4_expand(acc, s, n0, n1, ik);  // g^(2^16)
        f2_mul(ik, inv, d16);
        ld_cyc4(s, K, 12, i);
        ld_f2(n0, K, 20, i);
        ld_f2(n1, K, 22, i);
        cyc4_expand(t, s, n0, n1, ik);    // g^(2^48)
    }
    m12<W>(acc, acc, t);
    m12<W>(acc, acc, y);
    for (int k = 0; k < 3; k++) cs12<W>(y, y);
    m12<W>(acc, acc, y);  // 2^60
    for (int k = 0; k < 2; k++) cs12<W>(y, y);
    m12<W>(acc, acc, y);  // 2^62
    cs12<W>(y, y);
    m12<W>(acc, acc, y);  // 2^63
    f12_conj(acc, acc);
    st_f12(dst, i, acc);
}

// dst <- op_a(a) * op_b(b)
template <bool W>
static __device__ __noinline__ void fx_mul(Soa a, int opa, Soa b, int opb, Soa dst, size_t i) {
    Fp12 x, y;
    ld_f12(x, a, i);
    fx_apply_w<W>(x, opa);
    ld_f12(y, b, i);
    fx_apply_w<W>(y, opb);
    m12<W>(x, x, y);
    st_f12(dst, i, x);
}

// the chain (W = false: element i of n, per lane pair; k_fexp1: element i on a whole wave, wide steps)
template <bool W>
DEV void fexp_chain(size_t n, size_t i, uint32_t* fbuf, uint32_t* scratch) {
    const Soa F{fbuf, n};
    const Soa T{scratch, n}, A{scratch + (size_t)12 * NL * n, n}, S{scratch + (size_t)24 * NL * n, n},
        R{scratch + (size_t)36 * NL * n, n}, K{scratch + (size_t)48 * NL * n, n};
    fx_inv<W>(F, T, i);
    fx_mul<W>(F, OP_CONJ, T, OP_ID, F, i);   // f^(p^6 - 1)
    fx_mul<W>(F, OP_FROB2, F, OP_ID, F, i);  // ^(p^2 + 1)
    fx_cube<W>(F, R, i);                     // res = f^3
    fx_pow_x<W>(F, T, K, i, S);
    fx_mul<W>(T, OP_ID, F, OP_CONJ, T, i);   // t = f^(x-1)
    fx_pow_x<W>(T, A, K, i, S);
    fx_mul<W>(A, OP_ID, T, OP_CONJ, A, i);   // a = f^((x-1)^2)
    fx_mul<W>(A, OP_FROB2, A, OP_CONJ, S, i);
    fx_mul<W>(S, OP_FROB, R, OP_ID, R, i);   // res *= (a^(p^2) a^-1)^p
    fx_pow_x<W>(A, T, K, i, S);                 // b = a^x
    fx_mul<W>(T, OP_FROB2, T, OP_CONJ, S, i);
    fx_mul<W>(S, OP_ID, R, OP_ID, R, i);     // res *= b^(p^2) b^-1
    fx_pow_x<W>(T, A, K, i, S);                 // c = b^x
    fx_mul<W>(A, OP_FROB, R, OP_ID, R, i);   // res *= c^p
    fx_pow_x<W>(A, T, K, i, S);                 // d = c^x
    fx_mul<W>(T, OP_ID, R, OP_ID, R, i);     // res *= d
}

DEV void fexp_out(size_t n, size_t i, const uint32_t* scratch, const uint32_t* flags, uint8_t* verdicts,
                  uint8_t* gt_out, bool writer) {
    Fp12 res;
    ld_f12(res, Soa{const_cast<uint32_t*>(scratch) + (size_t)36 * NL * n, n}, i);
    const uint32_t fl = flags ? flags[i] : 0u;
    const bool ok = f12_is_one(res) && (fl & 11u) == 0;  // sigma_1/sigma_2 = O or PoK Schnorr failure
    if (!writer) return;
    if (!half_id()) verdicts[i] = ok ? 1 : 0;
    if (gt_out) {  // each lane writes its halves: Fp slots 2k + h of the AMCL FP12 order
        const Fp2* v = reinterpret_cast<const Fp2*>(&res);
        uint8_t* o = gt_out + i * 576 + 48 * half_id();
        for (int k = 0; k < 6; k++) {
            Fp c;
            fp_from_mont(c, v[k].c);
            store_be48_aligned(o + 96 * k, c);
        }
    }
}

// one element per wave (64 lanes, all pairs holding the same values; pair 0 writes the outputs):
// element blockIdx.x of n, its chain through SoA scratch of stride n.  One wave per SIMD (HIP's second
// bound): the whole register file (every step function is a W = true instantiation).  Latency-bound
// small batches (cck_fexp: n <= kFexpWideMax) and the RLC batch's one product; larger batches run the
// quad-lane lazy-field kernel of fexp_q.hip.
__global__ __launch_bounds__(64, 1) void k_fexp1(size_t n, uint32_t* __restrict__ fbuf, uint32_t* __restrict__ scratch,
                                              const uint32_t* __restrict__ flags, uint8_t* __restrict__ verdicts,
                                              uint8_t* __restrict__ gt_out) {
    const size_t i = blockIdx.x;
    if (i >= n) return;  // wave-uniform
    fexp_chain<true>(n, i, fbuf, scratch);
    fexp_out(n, i, scratch, flags, verdicts, gt_out, threadIdx.x < 2);
}

// ================================================================ wide Miller loop
// The RLC fold's 16 window pairs (fold.hip): few, so each runs alone on a wave in the wide form of
// k_fexp1 — the 32 lane pairs hold the same values and a step's independent Fp2 products (pairing.inc
// line_dbl / line_add / eval_line / f12_mul_line, the same formulas) are spread over them, one
// product a pair, results gathered with shuffles.  The point T's chain and f's chain are independent
// until f takes a line, so the loop runs them as a pipeline of LEVELS, one Fp2 product a pair each:
// pairs 18.. take T's next level — a doubling is two (A: X Y, Y^2, Z^2, (Y + Z)^2, X^2; B: T's a (b -
// 3e), e^2, g^2, b h with the line's evaluation at P), an addition four (Q_y Z, Q_x Z | theta^2,
// lambda^2, theta Q_x, lambda Q_y | lambda d, Z c, X d and the evaluation | T's four products) — and
// pairs 0..17 the oldest of f's pending operations (f^2, or f times a finished line as a full Fp12
// A + C w^2).  f's operations keep their order, so the result is the sequential loop's, in 147 levels
// instead of 209 (a doubling iteration 2 instead of 3): X = T's A | f times the previous doubling's
// line (f^2 after an addition step), Y = T's B | f^2; an addition step's first level takes the
// doubling's line, its last the addition's.
// P (slots S_P1..+2) is in evaluation form (X Z, Y, Z^3); an Fp factor multiplies as the Fp2 (k, 0).
DEV Fp2 f2_of_fp(const Fp& k) {
    Fp z;
    fp_zero(z);
    Fp2 r;
    r.c = fp_sel(half_id() != 0, z, k);
    return r;
}
// pair j's operands: opts1[j], opts2[j] for j < n (pair-uniform j)
DEV void pick2(Fp2& o1, Fp2& o2, int j, const Fp2* a, const Fp2* b, int n) {
    for (int k = 0; k < n; k++) {
        o1.c = fp_sel(j == k, a[k].c, o1.c);
        o2.c = fp_sel(j == k, b[k].c, o2.c);
    }
}
DEV void line_fp12(Fp12& L, const Fp2& a0, const Fp2& a2, const Fp2& a3) {  // A + C w^2 (pairing.inc)
    L.a.a = a0;
    L.a.b = a3;
    f2_zero(L.b.a);
    f2_zero(L.b.b);
    L.c.a = a2;
    f2_zero(L.c.b);
}

__global__ __launch_bounds__(64, 1) void k_miller_wide(size_t n, const uint32_t* __restrict__ prep,
                                                    const uint32_t* __restrict__ flags, uint32_t* __restrict__ fout,
                                                    size_t fstride, size_t foff) {
    const size_t i = blockIdx.x;  // the pair of this wave (wave-uniform)
    if (i >= n) return;
    const int j = pair_idx();
    const Soa S{const_cast<uint32_t*>(prep), n};
    Fp12 f;
    f12_one(f);
    if (!(flags[i] & 5u)) {
        Aff<Fp2> Q;
        ld_f2(Q.x, S, S_Q1, i);
        ld_f2(Q.y, S, S_Q1 + 2, i);
        Fp px, py, pz;
        cc::ld_fp(px, S, S_P1, i);
        cc::ld_fp(py, S, S_P1 + 1, i);
        cc::ld_fp(pz, S, S_P1 + 2, i);
        const Fp2 PX = f2_of_fp(px), PY = f2_of_fp(py), PZ = f2_of_fp(pz);
        G2Proj T;
        T.x = Q.x;
        T.y = Q.y;
        f2_one(T.z);
        // the doubling line not yet multiplied into f (taken at the next iteration's first level)
        Fp2 lp0, lp2, lp3;
        bool havep = false;
#pragma unroll 1
        for (int b = 62; b >= 0; b--) {
            Fp2 o1, o2, pr, l0, l2c, l3c;
            {  // X: T's A products (pairs 18..22) | f times the pending line, else f^2 (pairs 0..17)
                if (havep) {
                    Fp12 L;
                    line_fp12(L, lp0, lp2, lp3);
                    f12w_operands(o1, o2, j, f, L);
                } else {
                    f12w_operands(o1, o2, j, f, f);
                }
                Fp2 yz;
                f2_add_lz(yz, T.y, T.z);
                const Fp2 a1[5] = {T.x, T.y, T.z, yz, T.x}, a2[5] = {T.y, T.y, T.z, yz, T.x};
                pick2(o1, o2, j - 18, a1, a2, 5);
                f2_mul(pr, o1, o2);
                f12w_assemble(f, pr);
            }
            Fp2 a = bcast_f2(pr, 18), bb = bcast_f2(pr, 19), c = bcast_f2(pr, 20), h = bcast_f2(pr, 21),
                t = bcast_f2(pr, 22), e, ff, g;
            f2_half(a, a);
            f2_sub(h, h, bb);
            f2_sub(h, h, c);
            f2_mul_xi(e, c);
            f2_mul12(e, e);  // e = 3 b' Z^2
            f2_dbl(ff, e);
            f2_add(ff, ff, e);
            f2_add(g, bb, ff);
            f2_half(g, g);
            f2_sub(l0, e, bb);
            f2_dbl(l2c, t);
            f2_add(l2c, l2c, t);
            f2_neg(l3c, h);
            {  // Y: T's B products and the line's evaluation (pairs 18..24) | f^2 if X took the line
                Fp2 bmf;
                f2_sub(bmf, bb, ff);
                const Fp2 a1[7] = {a, e, g, bb, l0, l2c, l3c}, a2[7] = {bmf, e, g, h, PZ, PX, PY};
                if (havep) {
                    f12w_operands(o1, o2, j, f, f);
                } else {
                    o1 = a1[0];
                    o2 = a2[0];
                }
                pick2(o1, o2, j - 18, a1, a2, 7);
                f2_mul(pr, o1, o2);
                if (havep) f12w_assemble(f, pr);
            }
            T.x = bcast_f2(pr, 18);
            {
                const Fp2 e2 = bcast_f2(pr, 19);
                T.y = bcast_f2(pr, 20);
                f2_sub(T.y, T.y, e2);
                f2_sub(T.y, T.y, e2);
                f2_sub(T.y, T.y, e2);
            }
            T.z = bcast_f2(pr, 21);
            lp0 = bcast_f2(pr, 22);
            lp2 = bcast_f2(pr, 23);
            lp3 = bcast_f2(pr, 24);
            havep = true;
            if (!((X_ABS >> b) & 1ull)) continue;
            // addition step (pairing.inc line_add); its first level also takes the doubling's line
            Fp2 theta, lambda;
            {  // D1: Q_y Z, Q_x Z (pairs 18, 19) | f times the doubling's line (pairs 0..17)
                Fp12 L;
                line_fp12(L, lp0, lp2, lp3);
                f12w_operands(o1, o2, j, f, L);
                const Fp2 a1[2] = {Q.y, Q.x}, a2[2] = {T.z, T.z};
                pick2(o1, o2, j - 18, a1, a2, 2);
                f2_mul(pr, o1, o2);
                f12w_assemble(f, pr);
                havep = false;
                f2_sub(theta, T.y, bcast_f2(pr, 18));
                f2_sub(lambda, T.x, bcast_f2(pr, 19));
            }
            {  // D2
                const Fp2 a1[4] = {theta, lambda, theta, lambda}, a2[4] = {theta, lambda, Q.x, Q.y};
                o1 = a1[0];
                o2 = a2[0];
                pick2(o1, o2, j, a1, a2, 4);
                f2_mul(pr, o1, o2);
            }
            c = bcast_f2(pr, 0);
            const Fp2 d = bcast_f2(pr, 1);
            f2_sub(l0, bcast_f2(pr, 2), bcast_f2(pr, 3));
            f2_neg(l2c, theta);
            l3c = lambda;
            {  // D3
                const Fp2 a1[6] = {lambda, T.z, T.x, l0, l2c, l3c}, a2[6] = {d, c, d, PZ, PX, PY};
                o1 = a1[0];
                o2 = a2[0];
                pick2(o1, o2, j, a1, a2, 6);
                f2_mul(pr, o1, o2);
            }
            e = bcast_f2(pr, 0);
            ff = bcast_f2(pr, 1);
            g = bcast_f2(pr, 2);
            f2_add(h, e, ff);
            f2_sub(h, h, g);
            f2_sub(h, h, g);
            {  // D4: T's four products on pairs 0..3, f times the line on pairs 4..21
                Fp12 L;
                line_fp12(L, bcast_f2(pr, 3), bcast_f2(pr, 4), bcast_f2(pr, 5));
                Fp2 gmh;
                f2_sub(gmh, g, h);
                f12w_operands(o1, o2, j - 4, f, L);
                const Fp2 a1[4] = {lambda, theta, e, T.z}, a2[4] = {h, gmh, T.y, e};
                pick2(o1, o2, j, a1, a2, 4);
                f2_mul(pr, o1, o2);
                T.x = bcast_f2(pr, 0);
                f2_sub(T.y, bcast_f2(pr, 1), bcast_f2(pr, 2));
                T.z = bcast_f2(pr, 3);
                f12w_assemble(f, pr, 4);
            }
        }
        if (havep) {  // the last doubling's line
            Fp2 o1, o2, pr;
            Fp12 L;
            line_fp12(L, lp0, lp2, lp3);
            f12w_operands(o1, o2, j, f, L);
            f2_mul(pr, o1, o2);
            f12w_assemble(f, pr);
        }
        f12_conj(f, f);
    }
    if (threadIdx.x < 2) st_f12(Soa{fout, fstride}, foff + i, f);
}

// The same loop on TWO waves a pair, for launches of up to kWide2Max pairs (fewer waves than the chip
// has SIMDs, so the second wave is free): wave 1 walks T's chain (its A / B levels, the addition's four)
// and leaves each iteration's evaluated lines in LDS; wave 0 squares f and multiplies it by them one
// iteration behind.  A block barrier per iteration hands the lines over (two LDS slots).  Wave 0's
// iteration is then its two or three Fp12 operations alone (no T products or glue in its levels).
constexpr size_t kWide2Max = 256;
__global__ __launch_bounds__(128, 1) void k_miller_wide2(size_t n, const uint32_t* __restrict__ prep,
                                                      const uint32_t* __restrict__ flags, uint32_t* __restrict__ fout,
                                                      size_t fstride, size_t foff) {
    const size_t i = blockIdx.x;
    if (i >= n) return;  // block-uniform
    const bool twave = threadIdx.x >= 64;  // wave-uniform
    const int j = (int)((threadIdx.x & 63) >> 1), h = (int)(threadIdx.x & 1);
    __shared__ uint32_t lbuf[2][2][3][2][NL];  // [slot][doubling / addition line][coefficient][half][word]
    const Soa S{const_cast<uint32_t*>(prep), n};
    Fp12 f;
    f12_one(f);
    if (!(flags[i] & 5u)) {  // block-uniform
        if (twave) {
            Aff<Fp2> Q;
            ld_f2(Q.x, S, S_Q1, i);
            ld_f2(Q.y, S, S_Q1 + 2, i);
            Fp px, py, pz;
            cc::ld_fp(px, S, S_P1, i);
            cc::ld_fp(py, S, S_P1 + 1, i);
            cc::ld_fp(pz, S, S_P1 + 2, i);
            const Fp2 PX = f2_of_fp(px), PY = f2_of_fp(py), PZ = f2_of_fp(pz);
            G2Proj T;
            T.x = Q.x;
            T.y = Q.y;
            f2_one(T.z);
            auto put = [&](int slot, int which, const Fp2& x0, const Fp2& x2, const Fp2& x3) {
                if (j == 0) {
#pragma unroll
                    for (int w = 0; w < NL; w++) {
                        lbuf[slot][which][0][h][w] = x0.c.v[w];
                        lbuf[slot][which][1][h][w] = x2.c.v[w];
                        lbuf[slot][which][2][h][w] = x3.c.v[w];
                    }
                }
            };
#pragma unroll 1
            for (int k = 0; k <= 63; k++) {
                if (k <= 62) {
                    const int b = 62 - k;
                    Fp2 o1, o2, pr, l0, l2c, l3c;
                    {  // A: X Y, Y^2, Z^2, (Y + Z)^2, X^2
                        Fp2 yz;
                        f2_add_lz(yz, T.y, T.z);
                        const Fp2 a1[5] = {T.x, T.y, T.z, yz, T.x}, a2[5] = {T.y, T.y, T.z, yz, T.x};
                        o1 = a1[0];
                        o2 = a2[0];
                        pick2(o1, o2, j, a1, a2, 5);
                        f2_mul(pr, o1, o2);
                    }
                    Fp2 a = bcast_f2(pr, 0), bb = bcast_f2(pr, 1), c = bcast_f2(pr, 2), hh = bcast_f2(pr, 3),
                        t = bcast_f2(pr, 4), e, ff, g;
                    f2_half(a, a);
                    f2_sub(hh, hh, bb);
                    f2_sub(hh, hh, c);
                    f2_mul_xi(e, c);
                    f2_mul12(e, e);  // e = 3 b' Z^2
                    f2_dbl(ff, e);
                    f2_add(ff, ff, e);
                    f2_add(g, bb, ff);
                    f2_half(g, g);
                    f2_sub(l0, e, bb);
                    f2_dbl(l2c, t);
                    f2_add(l2c, l2c, t);
                    f2_neg(l3c, hh);
                    {  // B: T's a (b - 3e), e^2, g^2, b h and the line's evaluation at P
                        Fp2 bmf;
                        f2_sub(bmf, bb, ff);
                        const Fp2 a1[7] = {a, e, g, bb, l0, l2c, l3c}, a2[7] = {bmf, e, g, hh, PZ, PX, PY};
                        o1 = a1[0];
                        o2 = a2[0];
                        pick2(o1, o2, j, a1, a2, 7);
                        f2_mul(pr, o1, o2);
                    }
                    T.x = bcast_f2(pr, 0);
                    {
                        const Fp2 e2 = bcast_f2(pr, 1);
                        T.y = bcast_f2(pr, 2);
                        f2_sub(T.y, T.y, e2);
                        f2_sub(T.y, T.y, e2);
                        f2_sub(T.y, T.y, e2);
                    }
                    T.z = bcast_f2(pr, 3);
                    put(b & 1, 0, bcast_f2(pr, 4), bcast_f2(pr, 5), bcast_f2(pr, 6));
                    if ((X_ABS >> b) & 1ull) {  // addition step (pairing.inc line_add)
                        Fp2 theta, lambda;
                        {
                            const Fp2 a1[2] = {Q.y, Q.x}, a2[2] = {T.z, T.z};
                            o1 = a1[0];
                            o2 = a2[0];
                            pick2(o1, o2, j, a1, a2, 2);
                            f2_mul(pr, o1, o2);
                            f2_sub(theta, T.y, bcast_f2(pr, 0));
                            f2_sub(lambda, T.x, bcast_f2(pr, 1));
                        }
                        {
                            const Fp2 a1[4] = {theta, lambda, theta, lambda}, a2[4] = {theta, lambda, Q.x, Q.y};
                            o1 = a1[0];
                            o2 = a2[0];
                            pick2(o1, o2, j, a1, a2, 4);
                            f2_mul(pr, o1, o2);
                        }
                        c = bcast_f2(pr, 0);
                        const Fp2 d = bcast_f2(pr, 1);
                        f2_sub(l0, bcast_f2(pr, 2), bcast_f2(pr, 3));
                        f2_neg(l2c, theta);
                        l3c = lambda;
                        {
                            const Fp2 a1[6] = {lambda, T.z, T.x, l0, l2c, l3c}, a2[6] = {d, c, d, PZ, PX, PY};
                            o1 = a1[0];
                            o2 = a2[0];
                            pick2(o1, o2, j, a1, a2, 6);
                            f2_mul(pr, o1, o2);
                        }
                        e = bcast_f2(pr, 0);
                        ff = bcast_f2(pr, 1);
                        g = bcast_f2(pr, 2);
                        put(b & 1, 1, bcast_f2(pr, 3), bcast_f2(pr, 4), bcast_f2(pr, 5));
                        f2_add(hh, e, ff);
                        f2_sub(hh, hh, g);
                        f2_sub(hh, hh, g);
                        {
                            Fp2 gmh;
                            f2_sub(gmh, g, hh);
                            const Fp2 a1[4] = {lambda, theta, e, T.z}, a2[4] = {hh, gmh, T.y, e};
                            o1 = a1[0];
                            o2 = a2[0];
                            pick2(o1, o2, j, a1, a2, 4);
                            f2_mul(pr, o1, o2);
                            T.x = bcast_f2(pr, 0);
                            f2_sub(T.y, bcast_f2(pr, 1), bcast_f2(pr, 2));
                            T.z = bcast_f2(pr, 3);
                        }
                    }
                }
                __syncthreads();
            }
        } else {
            auto get = [&](int slot, int which) {
                Fp12 L;
                Fp2 x0, x2, x3;
#pragma unroll
                for (int w = 0; w < NL; w++) {
                    x0.c.v[w] = lbuf[slot][which][0][h][w];
                    x2.c.v[w] = lbuf[slot][which][1][h][w];
                    x3.c.v[w] = lbuf[slot][which][2][h][w];
                }
                line_fp12(L, x0, x2, x3);
                return L;
            };
#pragma unroll 1
            for (int k = 0; k <= 63; k++) {
                if (k >= 1) {  // iteration b = 63 - k, its lines written in round k - 1
                    const int b = 63 - k;
                    f12_mul_wide(f, f, f);
                    f12_mul_wide(f, f, get(b & 1, 0));
                    if ((X_ABS >> b) & 1ull) f12_mul_wide(f, f, get(b & 1, 1));
                }
                __syncthreads();
            }
            f12_conj(f, f);
        }
    }
    if (threadIdx.x < 2) st_f12(Soa{fout, fstride}, foff + i, f);
}

// ================================================================ small batches: one wave per pair
// A batch of n credentials fills 2n lanes of the pair-lane Miller kernel (k_miller): for small n that is
// a handful of waves, each the latency of a 2-pair loop on one lane pair (~7.5 ms alone on its SIMD,
// whatever n up to ~4k).  For n <= kWideMax (capi.cpp) each credential's two pairs run instead as two
// waves of k_miller_wide (one pair a wave, the independent products of a step spread over the lane
// pairs: ~1.8 ms), and k_f12_reduce_wide multiplies each credential's two Miller values.  k_wide_pairs
// lays the pairs out for it: pair 2i = credential i's pair 0, 2i + 1 its pair 1, Q affine (storage R
// form) in slots S_Q1.., P in evaluation form (X Z, Y, Z^3) in S_P1..; wide flag bit 0 = skip.
//   SigG2: pair 0 (sigma_1, pr), pair 1 (-sigma_2, g~);  SigG1: pair 0 (pr, sigma_1), pair 1 (g~, -sigma_2)
// The prep's P are affine in the lazy R' form (kAffRp): words x R' mod p, read by the storage-form tower
// as x 2^-14, so P = (x, y) goes in as (x R', y R', R' mod p) = 2^-14 (x, y, 1), a scaling of the
// evaluation form by an Fp constant (the final exponentiation removes it).  g~ (ctx gtilde_aff, AoS,
// R form) goes in as (x, y, 1) in R form.  Verdict flags stay per credential (the prep's).
DEV Fp one_rprime_words() {  // R' mod p (lazy.h LZ_ONE_LIMBS, 14 x 28 bits) as 12 x 32-bit words
    constexpr uint32_t L[14] = {LZ_ONE_LIMBS};
    Fp r;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        uint64_t w = 0;
#pragma unroll
        for (int k = 0; k < 14; k++) {
            const int sh = 28 * k - 32 * j;
            if (sh >= 32 || sh <= -28) continue;
            w |= sh >= 0 ? (uint64_t)L[k] << sh : (uint64_t)L[k] >> -sh;
        }
        r.v[j] = (uint32_t)w;
    }
    return r;
}
template <int MODE>
__global__ __launch_bounds__(64) void k_wide_pairs(size_t n, size_t ps, const uint32_t* __restrict__ prep,
                                                   const uint32_t* __restrict__ flags,
                                                   const uint32_t* __restrict__ gaff, uint32_t* __restrict__ wprep,
                                                   uint32_t* __restrict__ wflags) {
    const size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (e >= 2 * n) return;
    const size_t i = e >> 1;
    const int k = (int)(e & 1);
    const Soa S{const_cast<uint32_t*>(prep), ps}, W{wprep, 2 * n};
    Fp v;
    const bool q_is_g = MODE == 1 && k == 1, p_is_g = MODE == 0 && k == 1;
#pragma unroll
    for (int j = 0; j < 4; j++) {  // Q: x.a, x.b, y.a, y.b
        if (q_is_g) {
#pragma unroll
            for (int l = 0; l < NL; l++) v.v[l] = gaff[NL * j + l];
        } else {
            ld_fp(v, S, (k ? S_Q2 : S_Q1) + j, i);
        }
        st_fp(W, S_Q1 + j, e, v);
    }
    if (p_is_g) {
#pragma unroll
        for (int j = 0; j < 2; j++) {
#pragma unroll
            for (int l = 0; l < NL; l++) v.v[l] = gaff[NL * j + l];
            st_fp(W, S_P1 + j, e, v);
        }
        fp_one(v);
    } else {
#pragma unroll
        for (int j = 0; j < 2; j++) {
            ld_fp(v, S, (k ? S_P2 : S_P1) + j, i);
            st_fp(W, S_P1 + j, e, v);
        }
        v = one_rprime_words();
    }
    st_fp(W, S_P1 + 2, e, v);
    wflags[e] = (flags[i] & (k ? 18u : 5u)) ? 1u : 0u;
}

// one level of the RLC product tree in the wide form: out[t] = in[2t] in[2t+1] (in[2t] alone for an odd
// tail), one wave per product, the 18 Fp2 products on the wave's lane pairs at once.  The tree's short
// levels are latency-bound (k_f12_reduce: one product on one lane pair, ~45 us a level whatever its
// width); here a level holds about one Fp2 product's latency.
__global__ __launch_bounds__(64, 2) void k_f12_reduce_wide(size_t n_in, const uint32_t* __restrict__ in,
                                                          uint32_t* __restrict__ out) {
    const size_t t = blockIdx.x;
    const size_t n_out = (n_in + 1) / 2;
    if (t >= n_out) return;  // wave-uniform
    const Soa I{const_cast<uint32_t*>(in), n_in}, O{out, n_out};
    Fp12 a;
    ld_f12(a, I, 2 * t);
    if (2 * t + 1 < n_in) {
        Fp12 b;
        ld_f12(b, I, 2 * t + 1);
        f12_mul_wide(a, a, b);
    }
    if (threadIdx.x < 2) st_f12(O, t, a);
}

}  // namespace pl
}  // namespace cc

// one level of the product tree, wide form (k_f12_reduce_wide): (n + 1) / 2 waves
extern "C" int cck_f12_reduce_wide(size_t n, const uint32_t* d_in, uint32_t* d_out, hipStream_t st) {
    if (n < 2) return -1;
    hipLaunchKernelGGL(cc::pl::k_f12_reduce_wide, dim3((unsigned)((n + 1) / 2)), dim3(64), 0, st, n, d_in, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

// the batched kernel: lazy field, one credential per lane quad, the chain in registers (fexp_q.hip)
extern "C" int cck_fexp_q(size_t n, const uint32_t* d_f, const uint32_t* d_flags, uint8_t* d_verdicts, uint8_t* d_gt,
                          hipStream_t st);

// n <= wide_max (the caller's threshold; d_scratch >= 72 x 12 x n words): one wave per element, the
// latency-bound form (k_fexp1); otherwise the quad-lane batch kernel
extern "C" int cck_fexp(size_t n, uint32_t* d_f, uint32_t* d_scratch, const uint32_t* d_flags, uint8_t* d_verdicts,
                        uint8_t* d_gt, size_t wide_max, hipStream_t st) {
    if (!n) return 0;
    if (n > wide_max) return cck_fexp_q(n, d_f, d_flags, d_verdicts, d_gt, st);
    hipLaunchKernelGGL(cc::pl::k_fexp1, dim3((unsigned)n), dim3(64), 0, st, n, d_f, d_scratch, d_flags, d_verdicts, d_gt);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// credential i's two Miller pairs as wide pairs 2i, 2i + 1 (k_wide_pairs above); gaff: g~ affine (AoS,
// R form) of the context
extern "C" int cck_wide_pairs(int mode, size_t n, size_t ps, const uint32_t* d_prep, const uint32_t* d_flags,
                              const uint32_t* d_gaff, uint32_t* d_wprep, uint32_t* d_wflags, hipStream_t st) {
    if (!n) return 0;
    if (ps < n) return -1;
    const unsigned g = nblocks(2 * n, 64);
    if (mode == 0)
        hipLaunchKernelGGL(cc::pl::k_wide_pairs<0>, dim3(g), dim3(64), 0, st, n, ps, d_prep, d_flags, d_gaff, d_wprep,
                           d_wflags);
    else
        hipLaunchKernelGGL(cc::pl::k_wide_pairs<1>, dim3(g), dim3(64), 0, st, n, ps, d_prep, d_flags, d_gaff, d_wprep,
                           d_wflags);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the RLC fold's window pairs: pair i = SoA element i of n (Q: slots S_Q1.., P: S_P1.. in evaluation
// form; flags bit 0 / 2: skip), one wave each; Miller value i to element foff + i of stride fstride
extern "C" int cck_miller_wide(size_t n, const uint32_t* d_prep, const uint32_t* d_flags, uint32_t* d_f,
                               size_t fstride, size_t foff, hipStream_t st) {
    if (!n) return 0;
    if (fstride < foff + n) return -1;
    if (n <= cc::pl::kWide2Max)  // fewer pairs than SIMDs: a second wave a pair takes T's chain
        hipLaunchKernelGGL(cc::pl::k_miller_wide2, dim3((unsigned)n), dim3(128), 0, st, n, d_prep, d_flags, d_f, fstride,
                           foff);
    else
        hipLaunchKernelGGL(cc::pl::k_miller_wide, dim3((unsigned)n), dim3(64), 0, st, n, d_prep, d_flags, d_f, fstride,
                           foff);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
