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

}  // namespace lz
}  // namespace cc
