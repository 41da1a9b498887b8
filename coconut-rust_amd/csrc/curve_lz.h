// G2 Jacobian arithmetic on the lazy pair-lane field (lazy.h, tower_lz.h) — device code (the product
// path).  Same formulas as curve.h (dbl-2009-l, madd-2007-bl, add-2007-bl with their exceptional cases:
// AMCL's group law, reached by the reference through amcl_wrapper's multi-scalar multiplications,
// SURVEY.md §8a V4/V5/V8), one point per lane PAIR (each lane one half of every Fp2 coordinate), values
// in the lazy radix-2^28 form: no conversion per multiplication, additions carry-free.
//
// Points rest with REDUCED coordinates (lazy.h reduce(): normalised limbs, |V| < 0.5002 p).  A reduced
// value is zero iff all its limbs are (the only multiple of p below p / 2 in magnitude is 0, and
// normalised limbs represent 0 one way), so the identity (Z = 0) and the exceptional-case tests are an
// OR over 14 words, not a canonicalisation.
#pragma once
#include "tower_lz.h"

namespace cc {
namespace lz {

using F2R = F2<AN, 9>;  // reduced
struct JL {
    F2R x, y, z;
};
struct AL {
    F2R x, y;
};

// pair-uniform zero test of a reduced value
DEV bool rz_is_zero(const F2R& x) {
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < LN; k++) o |= (uint32_t)x.c.v[k];
    return pair_all(o == 0);
}
DEV F2R r_one() { return reduce(f2_one()); }
DEV JL jl_inf() { return {r_one(), r_one(), fit<AN, 9>(F2<AN, 0>{})}; }
DEV bool jl_is_inf(const JL& p) { return rz_is_zero(p.z); }
DEV JL jl_from_aff(const AL& a) { return {a.x, a.y, r_one()}; }

// dbl-2009-l (a = 0): 2M + 5S; the identity stays the identity (Z3 = 2 Y Z)
DEV JL jl_dbl(const JL& p) {
    const auto A = sqrr(p.x);
    const auto B = sqrr(p.y);
    const auto C = sqrr(B);
    const auto D = norm(dbl(sub(sub(sqrr(add(p.x, B)), A), C)));  // 2 ((X + B)^2 - A - C)
    const auto E = smul<3>(A);
    const auto X3 = sub(sqrr(E), dbl(D));
    const auto Y3 = sub(mulr(E, sub(D, X3)), dbl(norm(smul<4>(C))));  // E (D - X3) - 8 C
    const auto Z3 = dbl(mulr(p.y, p.z));
    return {reduce(X3), reduce(Y3), reduce(Z3)};
}

// madd-2007-bl: p (Jacobian) + q (affine, not the identity); 7M + 4S on the common path
DEV JL jl_add_aff(const JL& p, const AL& q) {
    if (jl_is_inf(p)) return jl_from_aff(q);
    const auto z1z1 = sqrr(p.z);
    const auto u2 = mulr(q.x, z1z1);
    const auto s2 = mulr(mulr(q.y, p.z), z1z1);
    const F2R h = reduce(sub(u2, p.x));
    const F2R r0 = reduce(sub(s2, p.y));
    if (rz_is_zero(h)) return rz_is_zero(r0) ? jl_dbl(p) : jl_inf();
    const auto rr = dbl(r0);
    const auto hh = sqrr(h);
    const auto i = smul<4>(hh);
    const auto j = mulr(h, i);
    const auto v = mulr(p.x, i);
    const auto X3 = sub(sub(sqrr(rr), j), dbl(v));
    const auto Y3 = sub(mulr(rr, sub(v, X3)), dbl(mulr(p.y, j)));
    const auto Z3 = sub(sub(sqrr(add(p.z, h)), z1z1), hh);
    return {reduce(X3), reduce(Y3), reduce(Z3)};
}

// madd-2007-bl with a canonical affine point (a table entry in the lazy Montgomery form, fixed.h)
DEV JL jl_add_aff_c(const JL& p, const F2<AN, BC>& qx, const F2<AN, BC>& qy) {
    if (jl_is_inf(p)) return {reduce(qx), reduce(qy), r_one()};
    const auto z1z1 = sqrr(p.z);
    const auto u2 = mulr(qx, z1z1);
    const auto s2 = mulr(mulr(qy, p.z), z1z1);
    const F2R h = reduce(sub(u2, p.x));
    const F2R r0 = reduce(sub(s2, p.y));
    if (rz_is_zero(h)) return rz_is_zero(r0) ? jl_dbl(p) : jl_inf();
    const auto rr = dbl(r0);
    const auto hh = sqrr(h);
    const auto i = smul<4>(hh);
    const auto j = mulr(h, i);
    const auto v = mulr(p.x, i);
    const auto X3 = sub(sub(sqrr(rr), j), dbl(v));
    const auto Y3 = sub(mulr(rr, sub(v, X3)), dbl(mulr(p.y, j)));
    const auto Z3 = sub(sub(sqrr(add(p.z, h)), z1z1), hh);
    return {reduce(X3), reduce(Y3), reduce(Z3)};
}

// add-2007-bl: general Jacobian addition with the exceptional cases
DEV JL jl_add(const JL& p, const JL& q) {
    if (jl_is_inf(p)) return q;
    if (jl_is_inf(q)) return p;
    const auto z1z1 = sqrr(p.z);
    const auto z2z2 = sqrr(q.z);
    const auto u1 = mulr(p.x, z2z2);
    const auto u2 = mulr(q.x, z1z1);
    const auto s1 = mulr(mulr(p.y, q.z), z2z2);
    const auto s2 = mulr(mulr(q.y, p.z), z1z1);
    const F2R h = reduce(sub(u2, u1));
    const F2R r0 = reduce(sub(s2, s1));
    if (rz_is_zero(h)) return rz_is_zero(r0) ? jl_dbl(p) : jl_inf();
    const auto rr = dbl(r0);
    const auto i = sqrr(dbl(h));
    const auto j = mulr(h, i);
    const auto v = mulr(u1, i);
    const auto X3 = sub(sub(sqrr(rr), j), dbl(v));
    const auto Y3 = sub(mulr(rr, sub(v, X3)), dbl(mulr(s1, j)));
    const auto Z3 = mulr(sub(sub(sqrr(add(p.z, q.z)), z1z1), z2z2), h);
    return {reduce(X3), reduce(Y3), reduce(Z3)};
}

DEV AL jl_neg_aff(const AL& a) { return {a.x, neg(a.y)}; }

// ================================================================ G1, one point per lane
// The same formulas over the lazy Fp on ONE lane (the G1 fixed-base MSMs of the verify / RLC / PoK
// preps and of Verkey::aggregate): additions carry-free, squarings on the upper triangle (lazy.h
// lz_sqr1, 105 product mads against 196), coordinates at rest reduced.
using FR = Fq<AN, 9>;
struct JG {
    FR x, y, z;
};
struct AG {
    Fq<AN, BC> x, y;  // canonical (a table entry)
};

template <int A1, int B1, int A2, int B2>
DEV auto mulr1(const Fq<A1, B1>& x, const Fq<A2, B2>& y) {
    if constexpr ((long long)A1 * A2 <= AMAX) return mul(x, y);
    else if constexpr (A1 >= A2 && (long long)AS * A2 <= AMAX) return mul(squeeze(x), y);
    else if constexpr (A2 > A1 && (long long)A1 * AS <= AMAX) return mul(x, squeeze(y));
    else return mul(squeeze(x), squeeze(y));
}
template <int A, int B>
DEV auto sqrr1(const Fq<A, B>& x) {
    if constexpr ((long long)A * A <= AMAX1S) return sqr(x);
    else return sqr(squeeze(x));
}
DEV bool r1_is_zero(const FR& x) {
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < LN; k++) o |= (uint32_t)x.v[k];
    return o == 0;
}
DEV FR r1_one() {
    constexpr int32_t O[LN] = {LZ_ONE_LIMBS};
    return reduce(fq_const(O));
}
DEV JG jg_inf() { return {r1_one(), r1_one(), fit<AN, 9>(Fq<AN, 0>{})}; }
DEV bool jg_is_inf(const JG& p) { return r1_is_zero(p.z); }

// dbl-2009-l (a = 0)
DEV JG jg_dbl(const JG& p) {
    const auto A = sqrr1(p.x);
    const auto B = sqrr1(p.y);
    const auto C = sqrr1(B);
    const auto t = sub(sub(sqrr1(add(p.x, B)), A), C);
    const auto D = squeeze(add(t, t));  // 2 ((X + B)^2 - A - C)
    const auto E = smul<3>(A);
    const auto X3 = sub(sqrr1(E), add(D, D));
    // E (D - X3) - 8 C  (8 C as 2 (4 C) squeezed: 8 normalised limbs would leave int32)
    const auto Y3 = sub(mulr1(E, sub(D, X3)), smul<2>(squeeze(smul<4>(C))));
    const auto Z3 = smul<2>(mulr1(p.y, p.z));
    return {reduce(X3), reduce(Y3), reduce(Z3)};
}

// madd-2007-bl: p (Jacobian) + q (affine, not the identity)
DEV JG jg_add_aff(const JG& p, const AG& q) {
    if (jg_is_inf(p)) return {reduce(q.x), reduce(q.y), r1_one()};
    const auto z1z1 = sqrr1(p.z);
    const auto u2 = mulr1(q.x, z1z1);
    const auto s2 = mulr1(mulr1(q.y, p.z), z1z1);
    const FR h = reduce(sub(u2, p.x));
    const FR r0 = reduce(sub(s2, p.y));
    if (r1_is_zero(h)) return r1_is_zero(r0) ? jg_dbl(p) : jg_inf();
    const auto rr = add(r0, r0);
    const auto hh = sqrr1(h);
    const auto i = smul<4>(hh);
    const auto j = mulr1(h, i);
    const auto v = mulr1(p.x, i);
    const FR X3 = reduce(sub(sub(sqrr1(rr), j), add(v, v)));
    // Y3 = rr (v - X3) - 2 y j = 2 (r0 (v - X3) - y j): both products under one reduction
    const auto Y3 = smul<2>(mul2(r0, sub(v, X3), neg(p.y), j));
    const auto Z3 = sub(sub(sqrr1(add(p.z, h)), z1z1), hh);
    return {X3, reduce(Y3), reduce(Z3)};
}

// add-2007-bl: general Jacobian addition with the exceptional cases
DEV JG jg_add(const JG& p, const JG& q) {
    if (jg_is_inf(p)) return q;
    if (jg_is_inf(q)) return p;
    const auto z1z1 = sqrr1(p.z);
    const auto z2z2 = sqrr1(q.z);
    const auto u1 = mulr1(p.x, z2z2);
    const auto u2 = mulr1(q.x, z1z1);
    const auto s1 = mulr1(mulr1(p.y, q.z), z2z2);
    const auto s2 = mulr1(mulr1(q.y, p.z), z1z1);
    const FR h = reduce(sub(u2, u1));
    const FR r0 = reduce(sub(s2, s1));
    if (r1_is_zero(h)) return r1_is_zero(r0) ? jg_dbl(p) : jg_inf();
    const auto rr = add(r0, r0);
    const auto i = sqrr1(add(h, h));
    const auto j = mulr1(h, i);
    const auto v = mulr1(u1, i);
    const FR X3 = reduce(sub(sub(sqrr1(rr), j), add(v, v)));
    const auto Y3 = smul<2>(mul2(r0, sub(v, X3), neg(s1), j));  // 2 (r0 (v - X3) - s1 j), one reduction
    const auto Z3 = mulr1(sub(sub(sqrr1(add(p.z, q.z)), z1z1), z2z2), h);
    return {X3, reduce(Y3), reduce(Z3)};
}

// p (not the identity) -> affine (x, y) in the R' form, canonical 12 x 32 words: the Miller loop's
// affine-R' operand (miller_lz.hip: its line's l0 needs no product, no Z to load).  One inversion
// (field.h divsteps) and four products.
DEV void jg_to_aff_rp(Fp& x, Fp& y, const JG& p) {
    const auto zi = inv(p.z);
    const auto zi2 = sqrr1(zi);
    x = canon(mulr1(p.x, zi2));
    y = canon(mulr1(p.y, mulr1(zi2, zi)));
}

// storage form (curve.h Jac<Fp>, canonical, R = 2^406) <-> lazy R' form
DEV JG jg_from(const Jac<Fp>& a) { return {reduce(in_r(a.x)), reduce(in_r(a.y)), reduce(in_r(a.z))}; }
DEV Jac<Fp> jg_to(const JG& a) { return {out_r(a.x), out_r(a.y), out_r(a.z)}; }

}  // namespace lz
}  // namespace cc
