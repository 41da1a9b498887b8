// Pair-lane BLS12-381 tower for gfx950 — device code (the product path).
//
// Same field tower and pairing algorithms as field.h / pairing.h (AMCL's Fp2 -> Fp4 -> Fp12, which
// the reference reaches through amcl_wrapper 0.1.7), with ONE credential
// per PAIR of adjacent lanes: lane 2i holds the real half (a) of every Fp2 value, lane 2i+1 the
// imaginary half (b).  Why: one credential per lane needs ~600 live words in the Miller loop, so a
// 65,536-credential batch runs as 1,024 waves at one wave per SIMD with heavy scratch spills, and a
// lone wave issues VALU at half rate on gfx950 (profiles/r01_ubench_int.jsonl).  Splitting every
// Fp2 across a lane pair halves the per-lane state and doubles the wave count (2,048 waves, two per
// SIMD), while the multiplication count per credential stays the same:
//
//   Fp2 mul  (a + b i)(c + d i):  lane a computes a c + b (4p - d), lane b computes a d + b c — each
//            a SUM of two 381-bit products with ONE Montgomery reduction (fp_mul2): 3 x 196 mads
//            per lane vs 3 full multiplications (6 x 196) for Karatsuba on one lane.
//   Fp2 sqr: lane a (a + b)(a - b), lane b a (2b): one multiplication per lane.
//   Fp2 x Fp: one multiplication per lane.
//
// The partner's half is fetched with DPP quad_perm [1,0,3,2] (one v_mov_b32_dpp per word, no LDS).
// Every control-flow decision in code using this file must be uniform across a lane pair.
#pragma once
#include "pairing.h"
#include "soa.h"

namespace cc {
namespace pl {

// partner lane's word (lane ^ 1) via DPP quad_perm [1, 0, 3, 2]
DEV uint32_t swp(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true); }
DEV Fp swp(const Fp& x) {
    Fp r;
#pragma unroll
    for (int k = 0; k < NL; k++) r.v[k] = swp(x.v[k]);
    return r;
}
// 1 on the lane holding imaginary halves
DEV uint32_t half_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 1u; }
DEV Fp fp_sel(bool c, const Fp& x, const Fp& y) {
    Fp r;
#pragma unroll
    for (int k = 0; k < NL; k++) r.v[k] = c ? x.v[k] : y.v[k];
    return r;
}

// (a b + c d) * 2^-406 mod p, canonical, on radix-2^29 limbs: a, c < 2^29 per limb, b, d < 2^30 per
// limb, a b + c d < 3p^2.  Column sums: 14 products < 2^58 + 14 < 2^59 + 14 reduction products < 2^58
// + the carry < 56 * 2^58 < 2^64.  The second product runs in its own accumulator chain (ILP).
DEV Fp mul2_29(const uint32_t a[L29], const uint32_t b[L29], const uint32_t c[L29], const uint32_t d[L29]) {
    uint32_t m[L29], r[L29];
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * L29 - 1; k++) {
        uint64_t acc2 = 0;
#pragma unroll
        for (int i = 0; i < L29; i++) {
            const int j = k - i;
            if (j < 0 || j >= L29) continue;
            acc = mad64(a[i], b[j], acc);
            acc2 = mad64(c[i], d[j], acc2);
        }
        acc += acc2;
        redc_column(k, acc, m, r);
    }
    r[L29 - 1] = (uint32_t)acc;
    Fp o;
    from29(o, r);
    return o;
}

DEV Fp fp_mul2_v(const Fp& U1, const Fp& V1, const Fp& U2, const Fp& V2) {
    uint32_t a[L29], b[L29], c[L29], d[L29];
    to29(a, U1);
    to29(b, V1);
    to29(c, U2);
    to29(d, V2);
    return mul2_29(a, b, c, d);
}

// 4p in radix 2^29 with limbs 0..12 in [2^29 - 1, 2^30) and limb 13 = 51: 4p - y limb by limb needs
// no borrows for any y < 2p (y's limb 13 is then <= 26)
DEV uint32_t four_p29(int k) {
    constexpr uint32_t D[L29] = {0x3ffeaaacu, 0x3fdffffeu, 0x33ffffb8u, 0x3ffff589u, 0x3d8907a9u, 0x2541ed60u, 0x2bf6730cu,
                                 0x2279c288u, 0x3d91dd2du, 0x28697599u, 0x2b1ba7b5u, 0x2bff34d1u, 0x20447a8du, 0x00000033u};
    return D[k];
}

// own half of x * y (x, y: own halves of two Fp2 values, each < 2p: canonical or a lazy sum).  The
// operands are converted to radix 2^29 once and the partner's converted limbs fetched by DPP.
//   re: a c + b (4p - d) = x y + xs (4p - ys);   im: b c + a d = x ys + xs y
// a c + b (4p - d) < 12 p^2 < p R, so the Montgomery result is < 2p and one subtraction makes it canonical.
// 7 limbs of d <- 4p - d on the real-half lanes (limbs k0..k0+6 of four_p29), under an exec mask as
// lazy.h neg_re14: the imaginary-half lanes keep d
#define CC_4P_OPS7(k0)                                                                                        \
    asm volatile("s_mov_b64 %0, exec\n\t"                                                                     \
                 "s_and_b64 exec, exec, %8\n\t"                                                               \
                 "v_sub_u32 %1, %9, %1\n\tv_sub_u32 %2, %10, %2\n\tv_sub_u32 %3, %11, %3\n\t"                \
                 "v_sub_u32 %4, %12, %4\n\tv_sub_u32 %5, %13, %5\n\tv_sub_u32 %6, %14, %6\n\t"               \
                 "v_sub_u32 %7, %15, %7\n\t"                                                                  \
                 "s_mov_b64 exec, %0"                                                                         \
                 : "=&s"(save), "+v"(d[k0]), "+v"(d[k0 + 1]), "+v"(d[k0 + 2]), "+v"(d[k0 + 3]),               \
                   "+v"(d[k0 + 4]), "+v"(d[k0 + 5]), "+v"(d[k0 + 6])                                          \
                 : "s"(0x5555555555555555ull), "s"(four_p29(k0)), "s"(four_p29(k0 + 1)),                      \
                   "s"(four_p29(k0 + 2)), "s"(four_p29(k0 + 3)), "s"(four_p29(k0 + 4)), "s"(four_p29(k0 + 5)), \
                   "s"(four_p29(k0 + 6)))
DEV Fp f2_mul_half(const Fp& x, const Fp& y) {
    uint32_t a[L29], y29[L29], b[L29], c[L29], d[L29];
    to29(a, x);
    to29(y29, y);
#pragma unroll
    for (int k = 0; k < L29; k++) {
        c[k] = swp(a[k]);
        // the pair's real half of y on both lanes (b), its imaginary half (d), 4p - d on the real lane
        b[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)y29[k], 0xA0, 0xF, 0xF, true);
        d[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)y29[k], 0xF5, 0xF, 0xF, true);
    }
    uint64_t save;
    CC_4P_OPS7(0);
    CC_4P_OPS7(7);
    return mul2_29(a, b, c, d);
}
// 2p, 32-bit limbs
DEV uint32_t two_p_limb(int j) {
    constexpr uint32_t T[NL] = {0xffff5556u, 0x73fdffffu, 0x62a7ffffu, 0x3d57fffdu, 0xed61ec48u, 0xce61a541u,
                                0xe70a257eu, 0xc8ee9709u, 0x869759aeu, 0x96374f6cu, 0x72ffcd34u, 0x340223d4u};
    return T[j];
}
// own half of x^2 (x < 2p): re (a + b)(a - b) = (x + xs)(x + 2p - xs), im a (2b) = xs (x + x).  The
// factors are left unreduced (< 4p each): Montgomery takes them (16 p^2 < p R), the result is canonical.
DEV Fp f2_sqr_half(const Fp& x) {
    const bool im = half_id() != 0;
    const Fp xs = swp(x);
    Fp u, v;
    uint32_t c1 = 0, c2 = 0, b3 = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        u.v[j] = __builtin_addc(im ? 0u : x.v[j], xs.v[j], c1, &c1);           // im: xs, re: x + xs
        const uint32_t w = __builtin_subc(two_p_limb(j), xs.v[j], b3, &b3);   // 2p - xs > 0
        v.v[j] = __builtin_addc(x.v[j], im ? x.v[j] : w, c2, &c2);            // im: 2x, re: x + 2p - xs
    }
    return fp_mul_v(u, v);
}

#ifdef CC_FP_INLINE
DEV Fp f2_mul_call_(const Fp& x, const Fp& y) { return f2_mul_half(x, y); }
DEV Fp f2_sqr_call_(const Fp& x) { return f2_sqr_half(x); }
#else
static __device__ __noinline__ Fp f2_mul_call(CC_L12(a), CC_L12(b)) {
    const Fp A = {{CC_V12(a)}}, B = {{CC_V12(b)}};
    return f2_mul_half(A, B);
}
static __device__ __noinline__ Fp f2_sqr_call(CC_L12(a)) {
    const Fp A = {{CC_V12(a)}};
    return f2_sqr_half(A);
}
DEV Fp f2_mul_call_(const Fp& x, const Fp& y) { return f2_mul_call(CC_E12(x), CC_E12(y)); }
DEV Fp f2_sqr_call_(const Fp& x) { return f2_sqr_call(CC_E12(x)); }
#endif

// ============================== Fp2 (pair-lane) ==============================
struct Fp2 {
    Fp c;  // this lane's half: real part on even lanes, imaginary part on odd lanes
};

DEV void f2_zero(Fp2& r) { fp_zero(r.c); }
DEV void f2_one(Fp2& r) {
    Fp o, z;
    fp_one(o);
    fp_zero(z);
    r.c = fp_sel(half_id() != 0, z, o);
}
// pair-uniform predicates: both halves agree
DEV bool pair_all(bool own) { return (swp((uint32_t)own) & (uint32_t)own) != 0; }
DEV bool f2_is_zero(const Fp2& x) { return pair_all(fp_is_zero(x.c)); }
DEV bool f2_eq(const Fp2& x, const Fp2& y) { return pair_all(fp_eq(x.c, y.c)); }
DEV void f2_add(Fp2& r, const Fp2& x, const Fp2& y) { fp_add(r.c, x.c, y.c); }
// x + y without reduction (< 2p for canonical x, y): only for values consumed by f2_mul / f2_sqr
DEV void f2_add_lz(Fp2& r, const Fp2& x, const Fp2& y) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) r.c.v[j] = __builtin_addc(x.c.v[j], y.c.v[j], c, &c);
}
DEV void f2_sub(Fp2& r, const Fp2& x, const Fp2& y) { fp_sub(r.c, x.c, y.c); }
DEV void f2_dbl(Fp2& r, const Fp2& x) { fp_dbl(r.c, x.c); }
DEV void f2_neg(Fp2& r, const Fp2& x) { fp_neg(r.c, x.c); }
// conj: negate the imaginary half only
DEV void f2_conj(Fp2& r, const Fp2& x) {
    uint32_t t[NL], o = 0, br = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        t[j] = __builtin_subc(p_limb(j), x.c.v[j], br, &br);
        o |= x.c.v[j];
    }
    const bool neg = half_id() != 0 && o != 0;
#pragma unroll
    for (int j = 0; j < NL; j++) r.c.v[j] = neg ? t[j] : x.c.v[j];
}
DEV void f2_mul(Fp2& r, const Fp2& x, const Fp2& y) { r.c = f2_mul_call_(x.c, y.c); }
DEV void f2_sqr(Fp2& r, const Fp2& x) { r.c = f2_sqr_call_(x.c); }
DEV void f2_mul_fp(Fp2& r, const Fp2& x, const Fp& k) { fp_mul(r.c, x.c, k); }
// x * (1 + i) = (a - b) + (a + b) i: own + (im ? partner : p - partner), one reduced addition
DEV void f2_mul_xi(Fp2& r, const Fp2& x) {
    const Fp xs = swp(x.c);
    const bool im = half_id() != 0;
    Fp w;
    uint32_t br = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const uint32_t d = __builtin_subc(p_limb(j), xs.v[j], br, &br);  // p - xs in [1, p]
        w.v[j] = im ? xs.v[j] : d;
    }
    fp_add(r.c, x.c, w);  // x + w < 2p
}
// a must be equal on both lanes; both lanes run the same divsteps (field.h fp_inv), so the pair
// stays convergent and the result is returned on both.  The divstep inversion costs ~1/20 of the
// Fermat ladder it replaces, so splitting it across the pair no longer pays.
DEV void fp_inv_pair(Fp& r, const Fp& a) { fp_inv(r, a); }

// (a + b i)^-1 = (a - b i) / (a^2 + b^2); the norm is computed on both lanes, its inverse split
DEV void f2_inv(Fp2& r, const Fp2& x) {
    const Fp xs = swp(x.c);
    Fp n = fp_mul2_v(x.c, x.c, xs, xs);
    fp_inv_pair(n, n);
    Fp2 t;
    fp_mul(t.c, x.c, n);
    f2_conj(r, t);
}
DEV void f2_half(Fp2& r, const Fp2& a) { fp_half(r.c, a.c); }
DEV void load_f2c(Fp2& r, const F2c& c) {
    const bool im = half_id() != 0;
#pragma unroll
    for (int j = 0; j < NL; j++) r.c.v[j] = im ? c.b[j] : c.a[j];
}

#include "tower.inc"

DEV bool f12_is_one(const Fp12& x) {
    Fp one;
    fp_one(one);
    const bool im = half_id() != 0;
    // real halves: (1, 0, 0, 0, 0, 0); imaginary halves: all 0
    bool ok = im ? fp_is_zero(x.a.a.c) : fp_eq(x.a.a.c, one);
    ok = ok && fp_is_zero(x.a.b.c) && fp_is_zero(x.b.a.c) && fp_is_zero(x.b.b.c) && fp_is_zero(x.c.a.c) &&
         fp_is_zero(x.c.b.c);
    return pair_all(ok);
}

#include "pairing.inc"

// ---------------------------------------------------------------- SoA access (soa.h layout):
// an Fp2 occupies slots (slot, slot + 1) = (a, b); each lane moves its own half.
DEV void ld_f2(Fp2& x, const Soa& s, int slot, size_t i) { ld_fp(x.c, s, slot + (int)half_id(), i); }
DEV void st_f2(const Soa& s, int slot, size_t i, const Fp2& x) { st_fp(s, slot + (int)half_id(), i, x.c); }
DEV void ld_f12(Fp12& x, const Soa& s, size_t i) {
    Fp2* v = reinterpret_cast<Fp2*>(&x);
#pragma unroll
    for (int k = 0; k < 6; k++) ld_f2(v[k], s, 2 * k, i);
}
DEV void st_f12(const Soa& s, size_t i, const Fp12& x) {
    const Fp2* v = reinterpret_cast<const Fp2*>(&x);
#pragma unroll
    for (int k = 0; k < 6; k++) st_f2(s, 2 * k, i, v[k]);
}
// AoS Fp2 (a then b, 12 words each)
DEV void ld_f2_aos(Fp2& x, const uint32_t* p) {
    const uint32_t* q = p + NL * half_id();
#pragma unroll
    for (int k = 0; k < NL; k++) x.c.v[k] = q[k];
}

}  // namespace pl
}  // namespace cc
