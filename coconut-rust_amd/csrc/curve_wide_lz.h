// Point doubling and addition with a step's independent products SPREAD over the lanes of one wave —
// device code (the product path, small batches).  Same formulas and exceptional cases as curve_lz.h
// (dbl-2009-l, madd-2007-bl, add-2007-bl: AMCL's group law), for a wave whose lanes all hold the SAME
// point in each GROUP of G lanes (G1, one Fp value a lane) or G lane pairs (G2, one half of an Fp2 a
// lane): product k of a level runs on member k of the group and the products are gathered back to every
// member with ds_bpermute shuffles.  A lone wave's time is its instruction count, so a doubling then
// costs 3 product times instead of 7 and an addition 5 instead of 16 (the one-wave kernels' chains: the
// PoK's chal J, the per-credential-verkey Straus, one base a group).  No level has more than 4 products
// (G = 4); members past a level's last product compute a duplicate that nobody gathers.
#pragma once
#include "curve_lz.h"
#include "curve_pl.h"
#include "tower_q.h"  // qinv: the quad divstep inversion

namespace cc {
namespace lz {
namespace wide {

constexpr int vmax() { return 0; }
template <class... I>
constexpr int vmax(int a, I... b) { return a > vmax(b...) ? a : vmax(b...); }

// ---------------------------------------------------------------- G1: product k on member k of a lane group
constexpr int G = 4;
DEV int lane() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
DEV int member() { return lane() & (G - 1); }
// member src's value of this lane's group
template <int A, int B>
DEV Fq<A, B> gat(const Fq<A, B>& x, int src) {
    const int from = (lane() & ~(G - 1)) + src;
    Fq<A, B> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = __shfl(x.v[k], from);
    return r;
}
// operand k of a level: x_k on members k < N, the last one beyond (fitted to the widest bound)
template <class X0, class... Xs>
DEV auto pick(int k, const X0& x0, const Xs&... xs) {
    constexpr int A = vmax(X0::AV, Xs::AV...), B = vmax(X0::BV, Xs::BV...);
    Fq<A, B> r = fit<A, B>(x0);
    int idx = 1;
    ((r = sel(k >= idx++, fit<A, B>(xs), r)), ...);
    return r;
}

// dbl-2009-l: level 1 X^2, Y^2, Z^2, (Y + Z)^2 (all squarings: Z3 = 2 Y Z = (Y + Z)^2 - Y^2 - Z^2);
// level 2 C = B^2, (X + B)^2, E^2; level 3 E (D - X3)
DEV JG jg_dbl(const JG& p) {
    const int k = member();
    const auto m1 = sqrr1(pick(k, p.x, p.y, p.z, add(p.y, p.z)));
    const auto A = gat(m1, 0), B = gat(m1, 1);
    const auto Z3 = sub(sub(gat(m1, 3), B), gat(m1, 2));
    const auto E = smul<3>(A);
    const auto m2 = sqrr1(pick(k, B, add(p.x, B), E));
    const auto C = gat(m2, 0), XB = gat(m2, 1), E2 = gat(m2, 2);
    const auto t = sub(sub(XB, A), C);
    const auto D = squeeze(add(t, t));  // 2 ((X + B)^2 - A - C)
    const auto X3 = sub(E2, add(D, D));
    const auto Y3 = sub(mulr1(E, sub(D, X3)), smul<2>(squeeze(smul<4>(C))));  // E (D - X3) - 8 C
    return {reduce(X3), reduce(Y3), reduce(Z3)};
}

// madd-2007-bl: p + q (q affine canonical, not the identity)
DEV JG jg_add_aff(const JG& p, const AG& q) {
    if (jg_is_inf(p)) return {reduce(q.x), reduce(q.y), r1_one()};
    const int k = member();
    const auto m1 = mulr1(pick(k, p.z, q.y), p.z);  // Z1^2, y2 Z1
    const auto z1z1 = gat(m1, 0), t = gat(m1, 1);
    const auto m2 = mulr1(pick(k, q.x, t), z1z1);  // u2, s2
    const FR h = reduce(sub(gat(m2, 0), p.x));
    const FR r0 = reduce(sub(gat(m2, 1), p.y));
    if (r1_is_zero(h)) return r1_is_zero(r0) ? wide::jg_dbl(p) : jg_inf();
    const auto rr = add(r0, r0);
    const auto m3 = sqrr1(pick(k, h, rr, add(p.z, h)));  // h^2, rr^2, (Z1 + h)^2
    const auto hh = gat(m3, 0), rr2 = gat(m3, 1), zh = gat(m3, 2);
    const auto i = smul<4>(hh);
    const auto m4 = mulr1(pick(k, h, p.x), i);  // j = h i, v = X1 i
    const auto j = gat(m4, 0), v = gat(m4, 1);
    const FR X3 = reduce(sub(sub(rr2, j), add(v, v)));
    const auto Y3 = smul<2>(mul2(r0, sub(v, X3), neg(p.y), j));  // 2 (r0 (v - X3) - y j)
    const auto Z3 = sub(sub(zh, z1z1), hh);
    return {X3, reduce(Y3), reduce(Z3)};
}

// add-2007-bl: general addition with the exceptional cases; Z3 = 2 Z1 Z2 H (the same value as
// ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H) keeps every level at <= 4 products
DEV JG jg_add(const JG& p, const JG& q) {
    if (jg_is_inf(p)) return q;
    if (jg_is_inf(q)) return p;
    const int k = member();
    const auto m1 = mulr1(pick(k, p.z, q.z, p.y, q.y), pick(k, p.z, q.z, q.z, p.z));
    const auto z1z1 = gat(m1, 0), z2z2 = gat(m1, 1);
    const auto m2 = mulr1(pick(k, p.x, q.x, gat(m1, 2), gat(m1, 3)), pick(k, z2z2, z1z1, z2z2, z1z1));
    const auto u1 = gat(m2, 0), s1 = gat(m2, 2);
    const FR h = reduce(sub(gat(m2, 1), u1));
    const FR r0 = reduce(sub(gat(m2, 3), s1));
    if (r1_is_zero(h)) return r1_is_zero(r0) ? wide::jg_dbl(p) : jg_inf();
    const auto h2 = add(h, h), rr = add(r0, r0);
    const auto m3 = mulr1(pick(k, h2, rr, p.z), pick(k, h2, rr, q.z));  // (2h)^2, rr^2, Z1 Z2
    const auto i = gat(m3, 0), rr2 = gat(m3, 1);
    const auto m4 = mulr1(pick(k, h, u1, gat(m3, 2)), pick(k, i, i, h2));  // j = h i, v = u1 i, Z3
    const auto j = gat(m4, 0), v = gat(m4, 1), Z3 = gat(m4, 2);
    const FR X3 = reduce(sub(sub(rr2, j), add(v, v)));
    const auto Y3 = smul<2>(mul2(r0, sub(v, X3), neg(s1), j));  // 2 (r0 (v - X3) - s1 j)
    return {X3, reduce(Y3), reduce(Z3)};
}

// ---------------------------------------------------------------- G2 (pair-lane): product k on member pair k
DEV int pmember() { return (lane() >> 1) & (G - 1); }
template <int A, int B>
DEV F2<A, B> gat(const F2<A, B>& x, int src_pair) {
    const int from = (lane() & ~(2 * G - 1)) + 2 * src_pair + (lane() & 1);
    F2<A, B> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.c.v[k] = __shfl(x.c.v[k], from);
    return r;
}
template <int A, int B>
DEV F2<A, B> sel(bool c, const F2<A, B>& x, const F2<A, B>& y) {
    return {lz::sel(c, x.c, y.c)};
}
template <class X0, class... Xs>
DEV auto pick2(int k, const X0& x0, const Xs&... xs) {
    constexpr int A = vmax(X0::AV, Xs::AV...), B = vmax(X0::BV, Xs::BV...);
    F2<A, B> r = fit<A, B>(x0);
    int idx = 1;
    ((r = sel(k >= idx++, fit<A, B>(xs), r)), ...);
    return r;
}

DEV JL jl_dbl(const JL& p) {
    const int k = pmember();
    const auto m1 = sqrr(pick2(k, p.x, p.y, p.z, add(p.y, p.z)));
    const auto A = gat(m1, 0), B = gat(m1, 1);
    const auto Z3 = sub(sub(gat(m1, 3), B), gat(m1, 2));
    const auto E = smul<3>(A);
    const auto m2 = sqrr(pick2(k, B, add(p.x, B), E));
    const auto C = gat(m2, 0), XB = gat(m2, 1), E2 = gat(m2, 2);
    const auto D = norm(dbl(sub(sub(XB, A), C)));  // 2 ((X + B)^2 - A - C)
    const auto X3 = sub(E2, dbl(D));
    const auto Y3 = sub(mulr(E, sub(D, X3)), dbl(norm(smul<4>(C))));  // E (D - X3) - 8 C
    return {reduce(X3), reduce(Y3), reduce(Z3)};
}

// qx, qy: a reduced affine point (AL) or a canonical table entry (F2<AN, BC>, as curve_lz.h jl_add_aff_c)
template <class QX, class QY>
DEV JL jl_add_aff_c(const JL& p, const QX& qx, const QY& qy) {
    if (jl_is_inf(p)) return {reduce(qx), reduce(qy), r_one()};
    const int k = pmember();
    const auto m1 = mulr(pick2(k, p.z, qy), p.z);  // Z1^2, y2 Z1
    const auto z1z1 = gat(m1, 0), t = gat(m1, 1);
    const auto m2 = mulr(pick2(k, qx, t), z1z1);  // u2, s2
    const F2R h = reduce(sub(gat(m2, 0), p.x));
    const F2R r0 = reduce(sub(gat(m2, 1), p.y));
    if (rz_is_zero(h)) return rz_is_zero(r0) ? wide::jl_dbl(p) : jl_inf();
    const auto rr = dbl(r0);
    const auto m3 = sqrr(pick2(k, h, rr, add(p.z, h)));  // h^2, rr^2, (Z1 + h)^2
    const auto hh = gat(m3, 0), rr2 = gat(m3, 1), zh = gat(m3, 2);
    const auto i = smul<4>(hh);
    const auto m4 = mulr(pick2(k, h, p.x), i);  // j = h i, v = X1 i
    const auto j = gat(m4, 0), v = gat(m4, 1);
    const auto X3 = sub(sub(rr2, j), dbl(v));
    const F2R X3r = reduce(X3);
    const auto m5 = mulr(pick2(k, rr, p.y), pick2(k, sub(v, X3r), j));  // rr (v - X3), Y1 j
    const auto Y3 = sub(gat(m5, 0), dbl(gat(m5, 1)));
    const auto Z3 = sub(sub(zh, z1z1), hh);
    return {X3r, reduce(Y3), reduce(Z3)};
}

DEV JL jl_add_aff(const JL& p, const AL& q) {
    if (jl_is_inf(p)) return jl_from_aff(q);
    return jl_add_aff_c(p, q.x, q.y);
}

DEV JL jl_add(const JL& p, const JL& q) {
    if (jl_is_inf(p)) return q;
    if (jl_is_inf(q)) return p;
    const int k = pmember();
    const auto m1 = mulr(pick2(k, p.z, q.z, p.y, q.y), pick2(k, p.z, q.z, q.z, p.z));
    const auto z1z1 = gat(m1, 0), z2z2 = gat(m1, 1);
    const auto m2 = mulr(pick2(k, p.x, q.x, gat(m1, 2), gat(m1, 3)), pick2(k, z2z2, z1z1, z2z2, z1z1));
    const auto u1 = gat(m2, 0), s1 = gat(m2, 2);
    const F2R h = reduce(sub(gat(m2, 1), u1));
    const F2R r0 = reduce(sub(gat(m2, 3), s1));
    if (rz_is_zero(h)) return rz_is_zero(r0) ? wide::jl_dbl(p) : jl_inf();
    const auto h2 = dbl(h), rr = dbl(r0);
    const auto m3 = mulr(pick2(k, h2, rr, p.z), pick2(k, h2, rr, q.z));  // (2h)^2, rr^2, Z1 Z2
    const auto i = gat(m3, 0), rr2 = gat(m3, 1);
    const auto m4 = mulr(pick2(k, h, u1, gat(m3, 2)), pick2(k, i, i, h2));  // j = h i, v = u1 i, Z3
    const auto j = gat(m4, 0), v = gat(m4, 1), Z3 = gat(m4, 2);
    const F2R X3 = reduce(sub(sub(rr2, j), dbl(v)));
    const auto m5 = mulr(pick2(k, rr, s1), pick2(k, sub(v, X3), j));  // rr (v - X3), s1 j
    const auto Y3 = sub(gat(m5, 0), dbl(gat(m5, 1)));
    return {X3, reduce(Y3), reduce(Z3)};
}

// curve_lz.h jg_to_aff_rp for a point every lane holds alike: the inversion in the quad divstep form
// (tower_q.h qinv: the iteration's four update chains one per lane of a quad)
DEV void jg_to_aff_rp(Fp& x, Fp& y, const JG& p) {
    const auto zi = qinv(p.z);
    const auto zi2 = sqrr1(zi);
    x = canon(mulr1(p.x, zi2));
    y = canon(mulr1(p.y, mulr1(zi2, zi)));
}

// curve.h jac_to_aff for a pair-lane G2 point every pair holds alike (storage form): the Fp2 inversion's
// norm inverted in the quad divstep form, as fexp_pl.hip f2_inv_q
DEV bool jac_to_aff(Aff<pl::Fp2>& r, const Jac<pl::Fp2>& p) {
    if (cc::jac_is_inf(p)) {
        pl::f2_zero(r.x);
        pl::f2_zero(r.y);
        return false;
    }
    pl::Fp2 zi, zi2, zi3;
    {
        const Fp zs = pl::swp(p.z.c);
        Fp nn = pl::fp_mul2_v(p.z.c, p.z.c, zs, zs), ni;  // |z|^2 on both lanes
        fp_inv_int_quad(ni, nn);                          // plain integer inverse of the Montgomery residue
        constexpr uint32_t R3[NL] = {CC_R3_LIMBS};
        Fp r3;
#pragma unroll
        for (int j = 0; j < NL; j++) r3.v[j] = R3[j];
        fp_mul(nn, ni, r3);  // |z|^-2 R (field.h fp_inv)
        pl::Fp2 t;
        fp_mul(t.c, p.z.c, nn);
        pl::f2_conj(zi, t);
    }
    pl::f2_sqr(zi2, zi);
    pl::f2_mul(zi3, zi2, zi);
    pl::f2_mul(r.x, p.x, zi2);
    pl::f2_mul(r.y, p.y, zi3);
    return true;
}

// ---------------------------------------------------------------- sums of the groups' points
// Every member of a group holds its group's point; a butterfly of spread additions (the lower group's
// point first, so every group ends with the same coordinates) leaves the sum of all groups' points on
// every lane.  G1: 16 groups a wave; G2: 8.
template <class P>
DEV P sel_pt(bool c, const P& a, const P& b) {
    P r;
    const int32_t* x = reinterpret_cast<const int32_t*>(&a);
    const int32_t* y = reinterpret_cast<const int32_t*>(&b);
    int32_t* o = reinterpret_cast<int32_t*>(&r);
#pragma unroll
    for (int w = 0; w < (int)(sizeof(P) / 4); w++) o[w] = c ? x[w] : y[w];
    return r;
}
template <class P>
DEV P shfl_xor_pt(const P& p, int m) {
    P r;
    const int32_t* x = reinterpret_cast<const int32_t*>(&p);
    int32_t* o = reinterpret_cast<int32_t*>(&r);
#pragma unroll
    for (int w = 0; w < (int)(sizeof(P) / 4); w++) o[w] = __shfl_xor(x[w], m);
    return r;
}
DEV JG jg_group_sum(JG a) {
#pragma unroll 1
    for (int m = G; m < 64; m <<= 1) {
        const JG o = shfl_xor_pt(a, m);
        const bool lo = (lane() & m) == 0;
        a = wide::jg_add(sel_pt(lo, a, o), sel_pt(lo, o, a));
    }
    return a;
}
DEV JL jl_group_sum(JL a) {
#pragma unroll 1
    for (int m = 2 * G; m < 64; m <<= 1) {
        const JL o = shfl_xor_pt(a, m);
        const bool lo = (lane() & m) == 0;
        a = wide::jl_add(sel_pt(lo, a, o), sel_pt(lo, o, a));
    }
    return a;
}

}  // namespace wide
}  // namespace lz
}  // namespace cc
