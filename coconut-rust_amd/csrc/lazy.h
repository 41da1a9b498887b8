// Lazy-reduced pair-lane field layer for the pairing kernels (Miller loop, final exponentiation) on
// gfx950 — device code (the product path).  Same field, tower and lane-pair layout as tower_pl.h
// (AMCL's BLS12-381 tower, reached by the reference through amcl_wrapper 0.1.7; SURVEY.md §8a rows
// T3, V6); different number representation:
//
//   Fq   14 SIGNED 28-bit-radix limbs, V = sum v_k 2^(28k), Montgomery radix R' = 2^392.  Values are
//        neither reduced mod p nor limb-normalised: additions, subtractions and negations are 14
//        carry-free v_add/v_sub (no borrow chains, no conditional subtraction of p), and the
//        multiplication takes the limbs as they are (signed v_mad_i64_i32 product scanning, one
//        accumulator chain per column) and returns normalised limbs with V < 1.13 p.  Nothing is
//        converted per multiplication (tower_pl.h converts 12 x 32 <-> 14 x 29 at each one and
//        subtracts p).
//
// Correctness rests on two bounds carried in the TYPE of every value, checked at compile time:
//   A  limb magnitude, units of 2^20:   |v_k| < A 2^20 for every limb (normalised: A = 256)
//   B  value magnitude, units of p/16:  |V| < B p / 16          (canonical: 16; product: >= 18)
// * multiplication: every column of sum a_i b_j (+ c_i d_j) + m_i p_j + carry must fit a signed 64-bit
//   accumulator: 14 (sum A_a A_b) 2^40 + 14 2^56 + 2^36 < 2^63  <=>  sum A_a A_b <= 533,000.
//   Its result is (ab + cd + m p) / R' with 0 <= m < R', so |V| < (sum B_a B_b / 256) p^2 / R' + p,
//   i.e. B_out = 16 + ceil(sum B_a B_b / 40,304)  (p / R' < 1 / 2,520).
// * squeeze (parallel carry, 3 ops a limb): limbs back to A = 257, value unchanged; valid while the top
//   limb (V / 2^364) stays below 2^28, i.e. B <= 32,768.
// * limbs are int32: A <= 2,047.
// A formula that breaks a bound does not compile (static_assert), so overflow cannot happen at run
// time whatever the inputs; the squeezes in tower_lz.h are exactly the ones the bounds demand.
//
// Boundary: kernels keep their SoA inputs/outputs in the storage form of field.h (12 x 32 canonical,
// R = 2^406).  in_r() moves a value to R' form (x R * 2^378 / R' = x R'), out_r() back (x R' * R /
// R' = x R), each one Montgomery multiplication; canon() gives the canonical residue (rare: outputs,
// equality tests, inversion inputs).
#pragma once
#include "tower_pl.h"

namespace cc {
namespace lz {

constexpr int LN = 14;
constexpr int32_t LM = 0x0fffffff;
constexpr int AN = 256;  // normalised limbs (product output)
constexpr int AS = 257;  // squeezed limbs
constexpr int BC = 16;   // canonical value (< p)
constexpr long long AMAX = 533000;
constexpr int bprod(long long s) { return 16 + (int)((s + 40303) / 40304); }
constexpr int cmax(int a, int b) { return a > b ? a : b; }

#define LZ_P_LIMBS 0xfffaaab, 0xfefffff, 0x3ffffb9, 0xfffeb15, 0x6241eab, 0xa0f6b0f, 0xf6730d2, 0xf38512b, 0x4774b84, \
    0x4bacd76, 0xba7b643, 0xe69a4b1, 0x1ea397f, 0x001a011
constexpr uint32_t LZ_N0 = 0xffcfffdu;  // -p^-1 mod 2^28
// 2^406 mod p (= R mod p): R' form -> R form, and the line scaling of miller_lz.hip
#define LZ_C_OUT_LIMBS 0x3a9fb84, 0x7400d20, 0xc4a23c5, 0xacde629, 0x6cb6147, 0x0b7e6d2, 0x16b0f4b, 0xc2b7d6e, 0x1ecbde7, \
    0xdd80b89, 0xa23c34f, 0xd636d56, 0xc30f3a0, 0x0013317
// R'^3 mod p: inversion
#define LZ_R3_LIMBS 0x1f7b890, 0x294cc4d, 0x9f3af22, 0xb5ba56c, 0xcb5c0cc, 0xc0d975c, 0xc89a8c5, 0x6c968b4, 0x22672ea, \
    0x91de8c9, 0x35652a6, 0x84977c8, 0x424bbb9, 0x00141ab
// R' mod p (one)
#define LZ_ONE_LIMBS 0x347fcb8, 0xd800000, 0x002b119, 0x0cde6d2, 0xc7212e0, 0x83a2090, 0x037669f, 0xda0f73e, 0x9b09b42, \
    0x1297bb0, 0x515d98f, 0x012ca7c, 0x659fcfa, 0x000577a
constexpr double LZ_PH = 28591897852287.902;  // p / 2^336

DEV int32_t lz_p(int k) {
    constexpr int32_t P[LN] = {LZ_P_LIMBS};
    return P[k];
}

template <int A, int B>
struct Fq {
    static_assert(A <= 2047, "limbs must fit int32");
    static constexpr int AV = A, BV = B;
    int32_t v[LN];
};
struct W14 {
    int32_t v[LN];
};

template <int A2, int B2, int A, int B>
DEV Fq<A2, B2> fit(const Fq<A, B>& x) {
    static_assert(A <= A2 && B <= B2, "fit: bound exceeds the target type");
    Fq<A2, B2> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = x.v[k];
    return r;
}

// ---------------------------------------------------------------- Montgomery product scanning
// Column k: the caller's products are in acc; add m_i p_j, derive m_k (k < 14) or emit limb k - 14,
// shift.  All signed 64-bit (arithmetic shift): inputs may be negative, m and p are in [0, 2^28).
DEV void lz_redc_col(int k, int64_t& acc, int32_t m[LN], int32_t r[LN]) {
#pragma unroll
    for (int i = 0; i < LN; i++) {
        const int j = k - i;
        if (i >= k || j < 0 || j >= LN) continue;
        acc += (int64_t)m[i] * lz_p(j);
    }
    if (k < LN) {
        m[k] = (int32_t)(((uint32_t)acc * LZ_N0) & (uint32_t)LM);
        acc += (int64_t)m[k] * lz_p(0);
    } else {
        r[k - LN] = (int32_t)acc & LM;
    }
    acc >>= 28;
}

// (a b + c d) / R' mod p (NP = 2) or a b / R' (NP = 1); limbs 0..12 of the result in [0, 2^28)
template <int NP>
DEV W14 lz_mont(const int32_t a[LN], const int32_t b[LN], const int32_t c[LN], const int32_t d[LN]) {
    int32_t m[LN];
    W14 r;
    int64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * LN - 1; k++) {
        int64_t acc2 = 0;
#pragma unroll
        for (int i = 0; i < LN; i++) {
            const int j = k - i;
            if (j < 0 || j >= LN) continue;
            acc += (int64_t)a[i] * b[j];
            if (NP == 2) acc2 += (int64_t)c[i] * d[j];
        }
        if (NP == 2) acc += acc2;
        lz_redc_col(k, acc, m, r.v);
    }
    r.v[LN - 1] = (int32_t)acc;
    return r;
}


// a^2 / R' mod p for a one-lane value: product scanning over the upper triangle only (column k:
// sum over i < j of (2 a_i) a_j, plus a_{k/2}^2), 105 product mads instead of 196.  Column bound: at
// most 7 doubled cross terms and one square, 15 A^2 2^40 in all, so A^2 <= 498,000 (AMAX1S).
constexpr long long AMAX1S = 498000;
DEV W14 lz_sqr1(const int32_t a[LN]) {
    int32_t d[LN], m[LN];
#pragma unroll
    for (int i = 0; i < LN; i++) d[i] = a[i] + a[i];
    W14 r;
    int64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * LN - 1; k++) {
        int64_t acc2 = 0;
#pragma unroll
        for (int i = 0; i < LN; i++) {
            const int j = k - i;
            if (j <= i || j >= LN) continue;
            acc2 += (int64_t)d[i] * a[j];
        }
        if ((k & 1) == 0 && k / 2 < LN) acc2 += (int64_t)a[k / 2] * a[k / 2];
        acc += acc2;
        lz_redc_col(k, acc, m, r.v);
    }
    r.v[LN - 1] = (int32_t)acc;
    return r;
}

DEV int32_t swp(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true); }
// the pair's real / imaginary half on both lanes (DPP quad_perm [0,0,2,2] / [1,1,3,3])
DEV int32_t bc_re(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0xA0, 0xF, 0xF, true); }
DEV int32_t bc_im(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0xF5, 0xF, 0xF, true); }
using pl::half_id;

// Operand preparation under an exec mask: the two halves of a pair need different operations, and a
// per-limb select (v_cndmask) after computing both costs an instruction a limb more than running each
// half's operation on its own lanes.  The mask is restored inside the same asm statement, so the
// compiler never sees a partial exec; lanes that were inactive stay inactive.
constexpr uint64_t kEvenLanes = 0x5555555555555555ull;  // real halves
// d <- -d on the real-half lanes, all 14 limbs
DEV void neg_re14(int32_t d[LN]) {
    uint64_t save;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_and_b64 exec, exec, %15\n\t"
        "v_sub_u32 %1, 0, %1\n\tv_sub_u32 %2, 0, %2\n\tv_sub_u32 %3, 0, %3\n\tv_sub_u32 %4, 0, %4\n\t"
        "v_sub_u32 %5, 0, %5\n\tv_sub_u32 %6, 0, %6\n\tv_sub_u32 %7, 0, %7\n\tv_sub_u32 %8, 0, %8\n\t"
        "v_sub_u32 %9, 0, %9\n\tv_sub_u32 %10, 0, %10\n\tv_sub_u32 %11, 0, %11\n\tv_sub_u32 %12, 0, %12\n\t"
        "v_sub_u32 %13, 0, %13\n\tv_sub_u32 %14, 0, %14\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(save), "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]),
          "+v"(d[7]), "+v"(d[8]), "+v"(d[9]), "+v"(d[10]), "+v"(d[11]), "+v"(d[12]), "+v"(d[13])
        : "s"(kEvenLanes));
}
// squaring operands for 7 limbs: u holds xs on entry; re lanes u <- x + xs, w <- x - xs; im lanes w <- 2x
DEV void sqr_ops7(int32_t* u, int32_t* w, const int32_t* x) {
    uint64_t save;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_and_b64 exec, exec, %22\n\t"
        "v_sub_u32 %8, %15, %1\n\tv_add_u32 %1, %1, %15\n\t"
        "v_sub_u32 %9, %16, %2\n\tv_add_u32 %2, %2, %16\n\t"
        "v_sub_u32 %10, %17, %3\n\tv_add_u32 %3, %3, %17\n\t"
        "v_sub_u32 %11, %18, %4\n\tv_add_u32 %4, %4, %18\n\t"
        "v_sub_u32 %12, %19, %5\n\tv_add_u32 %5, %5, %19\n\t"
        "v_sub_u32 %13, %20, %6\n\tv_add_u32 %6, %6, %20\n\t"
        "v_sub_u32 %14, %21, %7\n\tv_add_u32 %7, %7, %21\n\t"
        "s_andn2_b64 exec, %0, %22\n\t"
        "v_add_u32 %8, %15, %15\n\tv_add_u32 %9, %16, %16\n\tv_add_u32 %10, %17, %17\n\tv_add_u32 %11, %18, %18\n\t"
        "v_add_u32 %12, %19, %19\n\tv_add_u32 %13, %20, %20\n\tv_add_u32 %14, %21, %21\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(save), "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(u[4]), "+v"(u[5]), "+v"(u[6]),
          "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(w[4]), "=&v"(w[5]), "=&v"(w[6])
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "s"(kEvenLanes));
}

// own half of x * y for pair-lane Fp2 values x = (a, b), y = (c, d):
//   re  x c + xs (-d) = a c - b d,  im  x c + xs d = b c + a d
// (c and d broadcast to both lanes of the pair, d negated on the real-half lane)
DEV W14 lz_f2_mul_v(const W14& x, const W14& y) {
    int32_t xs[LN], b[LN], d[LN];
#pragma unroll
    for (int k = 0; k < LN; k++) {
        xs[k] = swp(x.v[k]);
        b[k] = bc_re(y.v[k]);
        d[k] = bc_im(y.v[k]);
    }
    neg_re14(d);
    return lz_mont<2>(x.v, b, xs, d);
}
// own half of x^2: re (x + xs)(x - xs),  im xs (2 x)
DEV W14 lz_f2_sqr_v(const W14& x) {
    int32_t u[LN], w[LN];
#pragma unroll
    for (int k = 0; k < LN; k++) u[k] = swp(x.v[k]);
    sqr_ops7(u, w, x.v);
    sqr_ops7(u + 7, w + 7, x.v + 7);
    return lz_mont<1>(u, w, u, w);
}
DEV W14 lz_mul_v(const W14& x, const W14& y) { return lz_mont<1>(x.v, y.v, x.v, y.v); }

#define LZ_L14(x) int32_t x##0, int32_t x##1, int32_t x##2, int32_t x##3, int32_t x##4, int32_t x##5, int32_t x##6, \
    int32_t x##7, int32_t x##8, int32_t x##9, int32_t x##10, int32_t x##11, int32_t x##12, int32_t x##13
#define LZ_V14(x) x##0, x##1, x##2, x##3, x##4, x##5, x##6, x##7, x##8, x##9, x##10, x##11, x##12, x##13
#define LZ_E14(x) x.v[0], x.v[1], x.v[2], x.v[3], x.v[4], x.v[5], x.v[6], x.v[7], x.v[8], x.v[9], x.v[10], x.v[11], \
    x.v[12], x.v[13]
#ifdef CC_FP_INLINE
DEV void lz_opaque(W14& x) {
#pragma unroll
    for (int k = 0; k < LN; k++) asm volatile("" : "+v"(x.v[k]));
}
DEV W14 lz_f2_mul_c(W14 x, W14 y) {
    W14 r;
    do {
        lz_opaque(x);
        lz_opaque(y);
        r = lz_f2_mul_v(x, y);
    } while (cc_opaque_false());
    return r;
}
DEV W14 lz_f2_sqr_c(W14 x) {
    W14 r;
    do {
        lz_opaque(x);
        r = lz_f2_sqr_v(x);
    } while (cc_opaque_false());
    return r;
}
DEV W14 lz_mul_c(W14 x, W14 y) {
    W14 r;
    do {
        lz_opaque(x);
        lz_opaque(y);
        r = lz_mul_v(x, y);
    } while (cc_opaque_false());
    return r;
}
#else
static __device__ __noinline__ W14 lz_f2_mul_call(LZ_L14(a), LZ_L14(b)) {
    const W14 A = {{LZ_V14(a)}}, B = {{LZ_V14(b)}};
    return lz_f2_mul_v(A, B);
}
static __device__ __noinline__ W14 lz_f2_sqr_call(LZ_L14(a)) {
    const W14 A = {{LZ_V14(a)}};
    return lz_f2_sqr_v(A);
}
static __device__ __noinline__ W14 lz_mul_call(LZ_L14(a), LZ_L14(b)) {
    const W14 A = {{LZ_V14(a)}}, B = {{LZ_V14(b)}};
    return lz_mul_v(A, B);
}
DEV W14 lz_f2_mul_c(const W14& x, const W14& y) { return lz_f2_mul_call(LZ_E14(x), LZ_E14(y)); }
DEV W14 lz_f2_sqr_c(const W14& x) { return lz_f2_sqr_call(LZ_E14(x)); }
DEV W14 lz_mul_c(const W14& x, const W14& y) { return lz_mul_call(LZ_E14(x), LZ_E14(y)); }
#endif
// one-lane squaring (not in the pair-lane kernels' inlined build: only the G1 code uses it)
static __device__ __noinline__ W14 lz_sqr1_call(LZ_L14(a)) {
    const int32_t A[LN] = {LZ_V14(a)};
    return lz_sqr1(A);
}
DEV W14 lz_sqr1_c(const W14& x) { return lz_sqr1_call(LZ_E14(x)); }
// a wave-uniform false the compiler cannot see through (field.h cc_opaque_false)
DEV bool lz_opaque_false() {
    uint32_t x;
    asm volatile("s_mov_b32 %0, 0" : "=s"(x));
    return x != 0;
}
// a sum of two one-lane products under one reduction (the G1 point formulas' Y3), inlined: as a call
// the four 14-limb operands exceed the 32 argument registers and would pass through scratch (the
// pair-lane Fp2 form of the same sum, measured: more scratch in the G2 kernels, slower)
DEV W14 lz_mul2_c(W14 x, W14 y, W14 z, W14 w) {
    W14 r;
    do {
#pragma unroll
        for (int k = 0; k < LN; k++) asm volatile("" : "+v"(x.v[k]), "+v"(y.v[k]), "+v"(z.v[k]), "+v"(w.v[k]));
        r = lz_mont<2>(x.v, y.v, z.v, w.v);
    } while (lz_opaque_false());
    return r;
}

template <int A, int B>
DEV W14 w14(const Fq<A, B>& x) {
    W14 r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = x.v[k];
    return r;
}
template <int B>
DEV Fq<AN, B> fq(const W14& x) {
    Fq<AN, B> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = x.v[k];
    return r;
}

// ---------------------------------------------------------------- canonical residue (rare)
// the residue of x in [0, p) as 12 x 32-bit limbs (the integer V mod p; still R' form)
static __device__ __noinline__ Fp lz_canon_call(LZ_L14(a)) {
    int32_t u[LN] = {LZ_V14(a)};
    int32_t c = 0;
#pragma unroll
    for (int k = 0; k < LN - 1; k++) {
        const int32_t t = u[k] + c;
        u[k] = t & LM;
        c = t >> 28;
    }
    u[LN - 1] += c;
    // V = sum u_k 2^(28k), u_0..12 in [0, 2^28): subtract floor(V / p) p, estimated from the top
    // 56 bits (off by at most one), then fix up
    const int64_t h = ((int64_t)u[LN - 1] << 28) + u[LN - 2];
    const int32_t q = (int32_t)floor((double)h / LZ_PH);
    {
        int64_t cc = 0;
#pragma unroll
        for (int k = 0; k < LN; k++) {
            const int64_t t = (int64_t)u[k] - (int64_t)q * lz_p(k) + cc;
            if (k < LN - 1) {
                u[k] = (int32_t)(t & LM);
                cc = t >> 28;
            } else {
                u[k] = (int32_t)t;
            }
        }
    }
    for (int it = 0; it < 2; it++) {  // V < 0: add p
        if (u[LN - 1] >= 0) break;
        int32_t cc = 0;
#pragma unroll
        for (int k = 0; k < LN; k++) {
            const int32_t t = u[k] + lz_p(k) + cc;
            if (k < LN - 1) {
                u[k] = t & LM;
                cc = t >> 28;
            } else {
                u[k] = t;
            }
        }
    }
    for (int it = 0; it < 2; it++) {  // V >= p: subtract p
        int32_t w[LN], cc = 0;
#pragma unroll
        for (int k = 0; k < LN; k++) {
            const int32_t t = u[k] - lz_p(k) + cc;
            if (k < LN - 1) {
                w[k] = t & LM;
                cc = t >> 28;
            } else {
                w[k] = t;
            }
        }
        if (w[LN - 1] < 0) break;
#pragma unroll
        for (int k = 0; k < LN; k++) u[k] = w[k];
    }
    Fp r;
#pragma unroll
    for (int w = 0; w < NL; w++) {
        const int bit = 32 * w, k = bit / 28, s = bit % 28;
        uint32_t x = (uint32_t)u[k] >> s;
        if (k + 1 < LN) x |= (uint32_t)u[k + 1] << (28 - s);
        if (s > 24 && k + 2 < LN) x |= (uint32_t)u[k + 2] << (56 - s);
        r.v[w] = x;
    }
    return r;
}
template <int A, int B>
DEV Fp canon(const Fq<A, B>& x) {
    static_assert(B <= 32768, "canon: value bound");
    return lz_canon_call(LZ_E14(x));
}

// ---------------------------------------------------------------- storage-form conversions
// the integer of a 12 x 32 value (< 2^384) as normalised limbs; B is the caller's value bound
template <int B = BC>
DEV Fq<AN, B> from_fp(const Fp& x) {
    Fq<AN, B> r;
    r.v[0] = (int32_t)(x.v[0] & (uint32_t)LM);
#pragma unroll
    for (int k = 1; k < LN - 1; k++) {
        const int bit = 28 * k, w = bit >> 5, s = bit & 31;
        r.v[k] = (int32_t)((s ? __builtin_amdgcn_alignbit(x.v[w + 1], x.v[w], s) : x.v[w]) & (uint32_t)LM);
    }
    r.v[LN - 1] = (int32_t)(x.v[NL - 1] >> 12);
    return r;
}
DEV Fq<AN, BC> fq_const(const int32_t (&c)[LN]) {
    Fq<AN, BC> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = c[k];
    return r;
}

// ---------------------------------------------------------------- lane-local linear operations
template <int A1, int B1, int A2, int B2>
DEV Fq<A1 + A2, B1 + B2> add(const Fq<A1, B1>& x, const Fq<A2, B2>& y) {
    Fq<A1 + A2, B1 + B2> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = x.v[k] + y.v[k];
    return r;
}
template <int A1, int B1, int A2, int B2>
DEV Fq<A1 + A2, B1 + B2> sub(const Fq<A1, B1>& x, const Fq<A2, B2>& y) {
    Fq<A1 + A2, B1 + B2> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = x.v[k] - y.v[k];
    return r;
}
template <int A, int B>
DEV Fq<A, B> neg(const Fq<A, B>& x) {
    Fq<A, B> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = -x.v[k];
    return r;
}
template <int K, int A, int B>
DEV Fq<K * A, K * B> smul(const Fq<A, B>& x) {  // x * K for a small constant K
    Fq<K * A, K * B> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = x.v[k] * K;
    return r;
}
// limbs back to [-A/256 - 1, 2^28 + A/256]: one parallel carry step, value unchanged
template <int A, int B>
DEV Fq<AS, B> squeeze(const Fq<A, B>& x) {
    static_assert(B <= 32768, "squeeze: the top limb must stay below 2^28");
    Fq<AS, B> r;
    int32_t hi = 0;
#pragma unroll
    for (int k = 0; k < LN - 1; k++) {
        const int32_t h = x.v[k] >> 28;
        r.v[k] = (x.v[k] & LM) + hi;
        hi = h;
    }
    r.v[LN - 1] = x.v[LN - 1] + hi;
    return r;
}
// value reduction: x - q p with q = round(V / p) taken from the top limb (V / 2^364 / (p / 2^364); the
// lower limbs move V / p by < A 2^-24.7 and the float estimate by < 2^-11), carried limb by limb into
// normalised limbs: |result| < 0.5002 p (B = 9; tests/test_lazy_algebra.py).  For values that only grow through additions (the
// cyclotomic squarings' 3u +- 2v): ~70 simple ops against 392 mads for a product by one.
constexpr float LZ_INV_P13 = 1.0f / 106513.12f;  // 2^364 / p
template <int A, int B>
DEV Fq<AN, 9> reduce(const Fq<A, B>& x) {
    static_assert(B <= 32768, "reduce: |q| must stay small");
    const int32_t q = (int32_t)__builtin_rintf((float)x.v[LN - 1] * LZ_INV_P13);
    Fq<AN, 9> r;
    int64_t c = 0;
#pragma unroll
    for (int k = 0; k < LN - 1; k++) {
        // one v_mad_i64_i32 into the running carry: the opaque step keeps the compiler from hoisting
        // the 13 products as parallel 64-bit temporaries (they spilled in the squaring loop)
        c += x.v[k];
        asm volatile("" : "+v"(c));
        c += (int64_t)q * -lz_p(k);
        r.v[k] = (int32_t)c & LM;
        c >>= 28;
    }
    r.v[LN - 1] = x.v[LN - 1] - q * lz_p(LN - 1) + (int32_t)c;
    return r;
}

template <int A, int B>
DEV Fq<A, B> sel(bool c, const Fq<A, B>& x, const Fq<A, B>& y) {
    Fq<A, B> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.v[k] = c ? x.v[k] : y.v[k];
    return r;
}

// ---------------------------------------------------------------- packed LDS parking
// A lazy value parked in LDS column threadIdx.x of a [rows][MB] array: limbs carry-normalised to
// [0, 2^28) (value unchanged), limbs 0..12 packed into 12 words, the signed top limb in a 13th.
constexpr int PW = 13;  // packed words per Fq
template <int MB, int A, int B>
DEV void pack_fq(int32_t (*lds)[MB], int row, const Fq<A, B>& x) {
    int32_t u[LN], c = 0;
#pragma unroll
    for (int k = 0; k < LN - 1; k++) {
        const int32_t t = x.v[k] + c;
        u[k] = t & LM;
        c = t >> 28;
    }
    u[LN - 1] = x.v[LN - 1] + c;
#pragma unroll
    for (int w = 0; w < PW - 1; w++) {
        const int bit = 32 * w, k = bit / 28, s = bit % 28;
        uint32_t v = (uint32_t)u[k] >> s;
        if (k + 1 < LN - 1) v |= (uint32_t)u[k + 1] << (28 - s);
        if (s > 24 && k + 2 < LN - 1) v |= (uint32_t)u[k + 2] << (56 - s);
        lds[row + w][threadIdx.x] = (int32_t)v;
    }
    lds[row + PW - 1][threadIdx.x] = u[LN - 1];
}
template <int MB, int B>
DEV Fq<AN, B> unpack_fq(int32_t (*lds)[MB], int row) {
    uint32_t w[PW];
#pragma unroll
    for (int j = 0; j < PW; j++) w[j] = (uint32_t)lds[row + j][threadIdx.x];
    Fq<AN, B> r;
    r.v[0] = (int32_t)(w[0] & (uint32_t)LM);
#pragma unroll
    for (int k = 1; k < LN - 1; k++) {
        const int bit = 28 * k, j = bit >> 5, s = bit & 31;
        r.v[k] = (int32_t)((s ? __builtin_amdgcn_alignbit(w[j + 1], w[j], s) : w[j]) & (uint32_t)LM);
    }
    r.v[LN - 1] = (int32_t)w[PW - 1];
    return r;
}

// ---------------------------------------------------------------- pair-lane Fp2
template <int A, int B>
struct F2 {
    static constexpr int AV = A, BV = B;
    Fq<A, B> c;  // this lane's half: real part on even lanes, imaginary part on odd lanes
};
template <int A2, int B2, int A, int B>
DEV F2<A2, B2> fit(const F2<A, B>& x) { return {fit<A2, B2>(x.c)}; }

template <int A1, int B1, int A2, int B2>
DEV F2<A1 + A2, B1 + B2> add(const F2<A1, B1>& x, const F2<A2, B2>& y) { return {add(x.c, y.c)}; }
template <int A1, int B1, int A2, int B2>
DEV F2<A1 + A2, B1 + B2> sub(const F2<A1, B1>& x, const F2<A2, B2>& y) { return {sub(x.c, y.c)}; }
template <int A, int B>
DEV F2<A, B> neg(const F2<A, B>& x) { return {neg(x.c)}; }
template <int K, int A, int B>
DEV F2<K * A, K * B> smul(const F2<A, B>& x) { return {smul<K>(x.c)}; }
template <int A, int B>
DEV F2<2 * A, 2 * B> dbl(const F2<A, B>& x) { return {add(x.c, x.c)}; }
template <int A, int B>
DEV F2<AS, B> squeeze(const F2<A, B>& x) { return {squeeze(x.c)}; }
template <int A, int B>
DEV F2<AN, 9> reduce(const F2<A, B>& x) { return {reduce(x.c)}; }

// 7 limbs of s <- x - s on the real-half lanes, x + s on the imaginary-half lanes
DEV void xi_ops7(int32_t* s, const int32_t* x) {
    uint64_t save;
    asm volatile(
        "s_mov_b64 %0, exec\n\t"
        "s_and_b64 exec, exec, %15\n\t"
        "v_sub_u32 %1, %8, %1\n\tv_sub_u32 %2, %9, %2\n\tv_sub_u32 %3, %10, %3\n\tv_sub_u32 %4, %11, %4\n\t"
        "v_sub_u32 %5, %12, %5\n\tv_sub_u32 %6, %13, %6\n\tv_sub_u32 %7, %14, %7\n\t"
        "s_andn2_b64 exec, %0, %15\n\t"
        "v_add_u32 %1, %8, %1\n\tv_add_u32 %2, %9, %2\n\tv_add_u32 %3, %10, %3\n\tv_add_u32 %4, %11, %4\n\t"
        "v_add_u32 %5, %12, %5\n\tv_add_u32 %6, %13, %6\n\tv_add_u32 %7, %14, %7\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(save), "+v"(s[0]), "+v"(s[1]), "+v"(s[2]), "+v"(s[3]), "+v"(s[4]), "+v"(s[5]), "+v"(s[6])
        : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "s"(kEvenLanes));
}
// x (1 + i) = (a - b) + (a + b) i: own -+ partner (the partner's half, then one masked op a limb)
template <int A, int B>
DEV F2<2 * A, 2 * B> xi(const F2<A, B>& x) {
    F2<2 * A, 2 * B> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.c.v[k] = swp(x.c.v[k]);
    xi_ops7(r.c.v, x.c.v);
    xi_ops7(r.c.v + 7, x.c.v + 7);
    return r;
}
// conj: the imaginary half negated
template <int A, int B>
DEV F2<A, B> conj(const F2<A, B>& x) {
    const bool im = half_id() != 0;
    F2<A, B> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.c.v[k] = im ? -x.c.v[k] : x.c.v[k];
    return r;
}

template <int A1, int B1, int A2, int B2>
DEV F2<AN, bprod(2LL * B1 * B2)> mul(const F2<A1, B1>& x, const F2<A2, B2>& y) {
    static_assert(2LL * A1 * A2 <= AMAX, "f2 mul: limb bound");
    return {fq<bprod(2LL * B1 * B2)>(lz_f2_mul_c(w14(x.c), w14(y.c)))};
}
template <int A, int B>
DEV F2<AN, bprod(4LL * B * B)> sqr(const F2<A, B>& x) {
    static_assert(4LL * A * A <= AMAX, "f2 sqr: limb bound");
    return {fq<bprod(4LL * B * B)>(lz_f2_sqr_c(w14(x.c)))};
}
// x^2 with the multiplication inlined (its own basic block): for small hot loops whose whole body then
// runs without call boundaries (no values saved around calls)
template <int A, int B>
DEV F2<AN, bprod(4LL * B * B)> sqr_in(const F2<A, B>& x) {
    static_assert(4LL * A * A <= AMAX, "f2 sqr: limb bound");
    W14 r, a = w14(x.c);
    do {
#pragma unroll
        for (int k = 0; k < LN; k++) asm volatile("" : "+v"(a.v[k]));
        r = lz_f2_sqr_v(a);
    } while (lz_opaque_false());
    return {fq<bprod(4LL * B * B)>(r)};
}
// Fp2 x Fp (k held on both lanes)
template <int A1, int B1, int A2, int B2>
DEV F2<AN, bprod((long long)B1 * B2)> mul_fp(const F2<A1, B1>& x, const Fq<A2, B2>& k) {
    static_assert((long long)A1 * A2 <= AMAX, "mul_fp: limb bound");
    return {fq<bprod((long long)B1 * B2)>(lz_mul_c(w14(x.c), w14(k)))};
}
template <int A1, int B1, int A2, int B2>
DEV Fq<AN, bprod((long long)B1 * B2)> mul(const Fq<A1, B1>& x, const Fq<A2, B2>& y) {
    static_assert((long long)A1 * A2 <= AMAX, "fp mul: limb bound");
    return fq<bprod((long long)B1 * B2)>(lz_mul_c(w14(x), w14(y)));
}
// one-lane x y + z w, one reduction for both products
template <int A1, int B1, int A2, int B2, int A3, int B3, int A4, int B4>
DEV Fq<AN, bprod((long long)B1 * B2 + (long long)B3 * B4)> mul2(const Fq<A1, B1>& x, const Fq<A2, B2>& y,
                                                               const Fq<A3, B3>& z, const Fq<A4, B4>& w) {
    static_assert((long long)A1 * A2 + (long long)A3 * A4 <= AMAX, "fp mul2: limb bound");
    return fq<bprod((long long)B1 * B2 + (long long)B3 * B4)>(lz_mul2_c(w14(x), w14(y), w14(z), w14(w)));
}
// one-lane x^2 (upper-triangle product scanning)
template <int A, int B>
DEV Fq<AN, bprod((long long)B * B)> sqr(const Fq<A, B>& x) {
    static_assert((long long)A * A <= AMAX1S, "fp sqr: limb bound");
    return fq<bprod((long long)B * B)>(lz_sqr1_c(w14(x)));
}

// pair-uniform predicates (both halves agree)
DEV bool pair_all(bool own) { return pl::pair_all(own); }
template <int A, int B>
DEV bool is_zero(const F2<A, B>& x) { return pair_all(fp_is_zero(canon(x.c))); }
template <int A1, int B1, int A2, int B2>
DEV bool eq(const F2<A1, B1>& x, const F2<A2, B2>& y) { return pair_all(fp_eq(canon(x.c), canon(y.c))); }

// storage form (12 x 32 canonical, R = 2^406) <-> R' form
DEV auto in_r(const Fp& x) {
    constexpr int32_t C[LN] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x4000};  // 2^378
    return mul(from_fp(x), fq_const(C));
}
template <int A, int B>
DEV Fp out_r(const Fq<A, B>& x) {
    constexpr int32_t C[LN] = {LZ_C_OUT_LIMBS};
    return canon(mul(x, fq_const(C)));
}
DEV auto in_r2(const pl::Fp2& x) {
    const auto c = in_r(x.c);
    return F2<AN, decltype(c)::BV>{c};
}
template <int A, int B>
DEV pl::Fp2 out_r2(const F2<A, B>& x) { return {out_r(x.c)}; }

// x^-1 (x on both lanes of the pair)
template <int A, int B>
DEV auto inv(const Fq<A, B>& x) {
    constexpr int32_t C[LN] = {LZ_R3_LIMBS};
    Fp a = canon(x), ai;
    fp_inv_int(ai, a);  // (x R')^-1
    return mul(from_fp(ai), fq_const(C));
}
// (a + b i)^-1 = conj(x) / (a^2 + b^2)
template <int A, int B>
DEV auto inv(const F2<A, B>& x) {
    static_assert(2LL * A * A <= AMAX, "f2 inv: limb bound");
    int32_t xs[LN];
#pragma unroll
    for (int k = 0; k < LN; k++) xs[k] = swp(x.c.v[k]);
    const W14 n = lz_mont<2>(x.c.v, x.c.v, xs, xs);  // a^2 + b^2 on both lanes
    const auto ni = inv(fq<bprod(2LL * B * B)>(n));
    const auto r = mul(x.c, ni);
    return conj(F2<AN, decltype(r)::BV>{r});
}

DEV F2<AN, BC> f2_zero() {
    F2<AN, BC> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.c.v[k] = 0;
    return r;
}
DEV F2<AN, BC> f2_one() {
    constexpr int32_t O[LN] = {LZ_ONE_LIMBS};
    const bool im = half_id() != 0;
    F2<AN, BC> r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.c.v[k] = im ? 0 : O[k];
    return r;
}

}  // namespace lz
}  // namespace cc
