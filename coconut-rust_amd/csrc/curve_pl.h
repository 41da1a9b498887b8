// G2 point arithmetic on the pair-lane Fp2 (tower_pl.h) — device code (the product path).
//
// curve.h's Jacobian formulas are generic over a field-traits class; instantiated with
// FT<pl::Fp2> they run ONE G2 point per lane PAIR: each lane holds one half of every coordinate
// (3 Fp per lane for a Jacobian point against 6 on one lane), and every Fp2 multiplication costs
// 588 mads a lane instead of 1,176 (tower_pl.h header).  Used where the one-lane G2 code needs more
// than the 256 VGPRs of 2 waves/SIMD: the RLC batch mode's subgroup checks (rlc.hip).  As with
// every pair-lane code path, control flow is pair-uniform (the predicates below agree on both lanes).
#pragma once
#include "fixed.h"
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

// psi(Q) for Q held as a lane-pair value (subgroup.h g2_in_subgroup's constants)
DEV void g2_psi(Aff<Fp2>& r, const Aff<Fp2>& q) {
    constexpr uint32_t CXB[NL] = {0x954030c4u, 0x1ed59d62u, 0x026053a5u, 0xc81fdd18u, 0xb49e2e0fu, 0xcb785f67u,
                                  0x6a65e5c3u, 0x689a6956u, 0x21724249u, 0x14cec802u, 0x7aaa6c42u, 0x00ba917au};
    constexpr uint32_t CYA[NL] = {0x699d9feeu, 0xfb9f5730u, 0x791f82c1u, 0x573fc3f8u, 0xc260bc18u, 0x774659b7u,
                                  0x65f57843u, 0x169c2180u, 0xf26ce7c9u, 0x477956cdu, 0x74beee42u, 0x191fce82u};
    constexpr uint32_t CYB[NL] = {0x96620abdu, 0xbe5fa8cfu, 0x38347d3du, 0xc76c3c06u, 0x34503a0bu, 0xefea78e9u,
                                  0x8d8f9a7bu, 0x4ddb2a04u, 0x50dec50eu, 0x03a250e8u, 0xc4c0f858u, 0x00e14367u};
    const bool im = half_id() != 0;
    Fp2 c, u;
#pragma unroll
    for (int j = 0; j < NL; j++) c.c.v[j] = im ? CXB[j] : 0u;  // c_x = (0, CXB)
    f2_conj(u, q.x);
    f2_mul(r.x, u, c);
#pragma unroll
    for (int j = 0; j < NL; j++) c.c.v[j] = im ? CYB[j] : CYA[j];
    f2_conj(u, q.y);
    f2_mul(r.y, u, c);
}

// psi(Q) == [x] Q (subgroup.h g2_in_subgroup, same constants) for Q held as a lane-pair value
DEV bool g2_in_subgroup(const Aff<Fp2>& q) {
    Jac<Fp2> a, t;
    jac_from_aff(a, q);
    jac_mul_xabs(t, a);  // [|x|] Q = -[x] Q
    Aff<Fp2> ps;
    g2_psi(ps, q);
    jac_add_aff(t, t, ps);  // [|x|] Q + psi(Q) == O  <=>  psi(Q) == [x] Q
    return jac_is_inf(t);
}

// the same test on the lazy pair-lane field (curve_lz.h): [|x|] Q by double-and-add over |x|, plus psi(Q)
// (formed in the storage form, two Fp2 products), is the identity
DEV bool g2_in_subgroup_lz(const Aff<Fp2>& q) {
    const lz::AL a{lz::reduce(lz::in_r2(q.x)), lz::reduce(lz::in_r2(q.y))};
    lz::JL t = lz::jl_from_aff(a);
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        t = lz::jl_dbl(t);
        if ((X_ABS >> b) & 1ull) t = lz::jl_add_aff(t, a);
    }
    Aff<Fp2> ps;
    g2_psi(ps, q);
    t = lz::jl_add_aff(t, lz::AL{lz::reduce(lz::in_r2(ps.x)), lz::reduce(lz::in_r2(ps.y))});
    return lz::jl_is_inf(t);
}

// The Miller loop's twist point ends as T = [|x|] Q (homogeneous projective: x = X/Z, y = Y/Z; the
// loop walks |x|'s addition chain), so Q is in G2 iff psi(Q) == [x] Q = -T: X = psi_x Z, Y = -psi_y Z,
// Z != 0 (eprint 2021/1130 §4, the test of g2_in_subgroup at the cost of two Fp2 multiplications).
DEV bool miller_t_in_subgroup(const G2Proj& T, const Aff<Fp2>& q) {
    Aff<Fp2> ps;
    g2_psi(ps, q);
    Fp2 a, b;
    f2_mul(a, ps.x, T.z);
    f2_mul(b, ps.y, T.z);
    f2_neg(b, b);
    return !f2_is_zero(T.z) && f2_eq(a, T.x) && f2_eq(b, T.y);
}

// fixed.h ft_add on the pair-lane Fp2 over a G2 window table in the lazy Montgomery form (AoS entries
// x.a | x.b | y.a | y.b, 12 words each; the verkey and issuer tables, k_table_fill): each lane loads its
// own halves, the sum runs on the lazy pair-lane field (curve_lz.h)
DEV void ft_add_g2_lz(lz::JL& acc, const uint32_t k[8], const uint32_t* __restrict__ table, int wbits, int j,
                      int w0, int w1, bool negate = false) {  // negate: acc -= k B_j
    constexpr int EW = sizeof(cc::Aff<cc::Fp2>) / 4;
    const int h = (int)half_id();
    const size_t went = ft_went(wbits);
    const uint32_t* tj = table + (size_t)j * ft_base_words<cc::Fp2>(wbits);
#pragma unroll 1
    for (int w = w0; w < w1; w++) {
        const uint32_t d = ft_digit(k, w, wbits);  // pair-uniform: both lanes hold the same scalar
        if (!d) continue;
        const uint32_t* e = tj + ((size_t)w * went + d - 1) * EW;
        Fp x, y;
        uint32_t o = 0;
#pragma unroll
        for (int c = 0; c < NL; c++) {
            x.v[c] = e[NL * h + c];
            y.v[c] = e[2 * NL + NL * h + c];
            o |= x.v[c] | y.v[c];
        }
        if (pair_all(o == 0)) continue;  // (0, 0): an identity entry
        const lz::F2<lz::AN, lz::BC> ly{lz::from_fp(y)};
        acc = lz::jl_add_aff_c(acc, lz::F2<lz::AN, lz::BC>{lz::from_fp(x)}, negate ? lz::neg(ly) : ly);
    }
}
// storage-form (canonical, R = 2^406) pair-lane Jacobian points <-> the lazy field's (curve_lz.h)
DEV lz::JL jl_from_pl(const Jac<Fp2>& a) {
    return {lz::reduce(lz::in_r2(a.x)), lz::reduce(lz::in_r2(a.y)), lz::reduce(lz::in_r2(a.z))};
}
DEV Jac<Fp2> jl_to_pl(const lz::JL& a) { return {lz::out_r2(a.x), lz::out_r2(a.y), lz::out_r2(a.z)}; }
// curve.h lane_group_sum for lane-pair points: the sum over the L / 2 pairs of L consecutive lanes
// (L a power of two <= 64), butterfly at lane distances L/2 .. 2 so halves stay with halves; every
// pair ends with the same sum.
template <int L>
DEV void pair_group_sum(Jac<Fp2>& acc) {
    constexpr int JW = sizeof(Jac<Fp2>) / 4;
#pragma unroll 1
    for (int m = L >> 1; m >= 2; m >>= 1) {
        Jac<Fp2> o;
        const uint32_t* a = reinterpret_cast<const uint32_t*>(&acc);
        uint32_t* w = reinterpret_cast<uint32_t*>(&o);
        for (int c = 0; c < JW; c++) w[c] = (uint32_t)__shfl_xor((int)a[c], m);
        // same operand order on both partners so they hold the same representation
        if (threadIdx.x & m) {
            Jac<Fp2> t = acc;
            acc = o;
            o = t;
        }
        jac_add(acc, acc, o);
    }
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
