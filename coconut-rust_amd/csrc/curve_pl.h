// G2 point arithmetic on the pair-lane Fp2 (tower_pl.h) — device code (the product path).
//
// curve.h's Jacobian formulas are generic over a field-traits class; instantiated with
// FT<pl::Fp2> they run ONE G2 point per lane PAIR: each lane holds one half of every coordinate
// (3 Fp per lane for a Jacobian point against 6 on one lane), and every Fp2 multiplication costs
// 588 mads a lane instead of 1,176 (tower_pl.h header).  Used where the one-lane G2 code needs more
// than the 256 VGPRs of 2 waves/SIMD: the RLC batch mode's subgroup checks (rlc.hip).  As with
// every pair-lane code path, control flow is pair-uniform (the predicates below agree on both lanes).
#pragma once
#include "subgroup.h"
#include "tower_pl.h"

namespace cc {

template <>
struct FT<pl::Fp2> {
    using F2 = pl::Fp2;
    static DEV void add(F2& r, const F2& a, const F2& b) { pl::f2_add(r, a, b); }
    static DEV void sub(F2& r, const F2& a, const F2& b) { pl::f2_sub(r, a, b); }
    static DEV void dbl(F2& r, const F2& a) { pl::f2_dbl(r, a); }
    static DEV void neg(F2& r, const F2& a) { pl::f2_neg(r, a); }
    static DEV void mul(F2& r, const F2& a, const F2& b) { pl::f2_mul(r, a, b); }
    static DEV void sqr(F2& r, const F2& a) { pl::f2_sqr(r, a); }
    static DEV bool is_zero(const F2& a) { return pl::f2_is_zero(a); }
    static DEV bool eq(const F2& a, const F2& b) { return pl::f2_eq(a, b); }
    static DEV void zero(F2& r) { pl::f2_zero(r); }
    static DEV void one(F2& r) { pl::f2_one(r); }
    static DEV void inv(F2& r, const F2& a) { pl::f2_inv(r, a); }
    // twist constant 4 (1 + i): both halves are 4
    static DEV void curve_b(F2& r) { FT<Fp>::curve_b(r.c); }
};

namespace pl {

// psi(Q) == [x] Q (subgroup.h g2_in_subgroup, same constants) for Q held as a lane-pair value
DEV bool g2_in_subgroup(const Aff<Fp2>& q) {
    constexpr uint32_t CXB[NL] = {0x954030c4u, 0x1ed59d62u, 0x026053a5u, 0xc81fdd18u, 0xb49e2e0fu, 0xcb785f67u,
                                  0x6a65e5c3u, 0x689a6956u, 0x21724249u, 0x14cec802u, 0x7aaa6c42u, 0x00ba917au};
    constexpr uint32_t CYA[NL] = {0x699d9feeu, 0xfb9f5730u, 0x791f82c1u, 0x573fc3f8u, 0xc260bc18u, 0x774659b7u,
                                  0x65f57843u, 0x169c2180u, 0xf26ce7c9u, 0x477956cdu, 0x74beee42u, 0x191fce82u};
    constexpr uint32_t CYB[NL] = {0x96620abdu, 0xbe5fa8cfu, 0x38347d3du, 0xc76c3c06u, 0x34503a0bu, 0xefea78e9u,
                                  0x8d8f9a7bu, 0x4ddb2a04u, 0x50dec50eu, 0x03a250e8u, 0xc4c0f858u, 0x00e14367u};
    const bool im = half_id() != 0;
    Jac<Fp2> a, t;
    jac_from_aff(a, q);
    jac_mul_xabs(t, a);  // [|x|] Q = -[x] Q
    Aff<Fp2> ps;
    Fp2 c, u;
#pragma unroll
    for (int j = 0; j < NL; j++) c.c.v[j] = im ? CXB[j] : 0u;  // c_x = (0, CXB)
    f2_conj(u, q.x);
    f2_mul(ps.x, u, c);
#pragma unroll
    for (int j = 0; j < NL; j++) c.c.v[j] = im ? CYB[j] : CYA[j];
    f2_conj(u, q.y);
    f2_mul(ps.y, u, c);
    jac_add_aff(t, t, ps);  // [|x|] Q + psi(Q) == O  <=>  psi(Q) == [x] Q
    return jac_is_inf(t);
}

// the lane-pair form of a one-lane Fp2 value held by lane `src` of the pair (both lanes call it)
DEV Fp2 f2_from_lane(const cc::Fp2& v, int src) {
    const bool im = half_id() != 0;
    const Fp a = swp(v.a), b = swp(v.b);
    Fp2 r;
    if (src == 0) r.c = im ? b : v.a;  // lane 0 keeps its real half, lane 1 takes lane 0's imaginary
    else r.c = im ? v.b : a;           // lane 1 keeps its imaginary half, lane 0 takes lane 1's real
    return r;
}

}  // namespace pl
}  // namespace cc
