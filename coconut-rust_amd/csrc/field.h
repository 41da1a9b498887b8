// BLS12-381 field tower for gfx950 — device code (the product path).
//
// Replaces AMCL v3.2 FP/FP2/FP4/FP12 (reached by the reference through amcl_wrapper 0.1.7,
// reference Cargo.toml:16-19).  Same tower as AMCL so GT elements serialise
// in AMCL's byte order directly:
//     Fp2  = Fp[i]/(i^2 + 1)
//     Fp4  = Fp2[s]/(s^2 - xi),  xi = 1 + i
//     Fp12 = Fp4[w]/(w^3 - s)
//
// One field element per lane: 12 x 32-bit limbs in VGPRs (storage form, canonical, < p).
// Montgomery form with R = 2^406: multiplication converts its operands to radix 2^29 (14 limbs)
// and runs product scanning, so every column is ONE chain of v_mad_u64_u32 into a 64-bit
// accumulator (no carry words: 28 products of < 2^58 fit), then converts back and subtracts p once.
// Measured (tools/ubench_fpmul.hip, profiles/r01_ubench_fpmul.jsonl): 5.4e10 Fp mul/s chip-wide
// inlined at one wave per SIMD vs 2.4e10 for the 12x32 CIOS form it replaces.  Constants in
// Montgomery form come from tools/gen_constants.py.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

namespace cc {

constexpr int NL = 12;  // limbs per Fp

// p, little-endian 32-bit limbs
#define CC_P_LIMBS                                                                              \
    0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu, \
        0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau
// R mod p (Montgomery one), R = 2^406
#define CC_ONE_LIMBS                                                                            \
    0x03a9fb84u, 0xc57400d2u, 0x629c4a23u, 0x6147acdeu, 0x7e6d26cbu, 0x6b0f4b0bu, 0xc2b7d6e1u, \
        0x91ecbde7u, 0x4fdd80b8u, 0xd56a23c3u, 0xf3a0d636u, 0x13317c30u
// R^2 mod p
#define CC_R2_LIMBS                                                                             \
    0xd5bef7aeu, 0xa20639a1u, 0x918b764fu, 0xcd249131u, 0x9b54e6e2u, 0x3976e2d0u, 0x712d8c5cu, \
        0x36639944u, 0x8a6de8fbu, 0xb47e72f3u, 0xb13c5b3fu, 0x19ea66a2u
// p in radix 2^29 and -p^-1 mod 2^29
#define CC_P29_LIMBS                                                                                     \
    0x1fffaaabu, 0x0ff7ffffu, 0x14ffffeeu, 0x17fffd62u, 0x0f6241eau, 0x09507b58u, 0x0afd9cc3u, 0x109e70a2u, \
        0x1764774bu, 0x121a5d66u, 0x12c6e9edu, 0x12ffcd34u, 0x00111ea3u, 0x0000000du
constexpr uint32_t N0_29 = 0x1ffcfffdu;
constexpr int L29 = 14;
constexpr uint32_t M29 = 0x1fffffffu;

__constant__ static const uint32_t kP[NL] = {CC_P_LIMBS};

struct Fp {
    uint32_t v[NL];
};

DEV uint32_t p_limb(int j) {
    constexpr uint32_t P[NL] = {CC_P_LIMBS};
    return P[j];
}

DEV void fp_zero(Fp& r) {
#pragma unroll
    for (int j = 0; j < NL; j++) r.v[j] = 0;
}

DEV void fp_one(Fp& r) {
    constexpr uint32_t O[NL] = {CC_ONE_LIMBS};
#pragma unroll
    for (int j = 0; j < NL; j++) r.v[j] = O[j];
}

DEV bool fp_is_zero(const Fp& a) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) o |= a.v[j];
    return o == 0;
}

DEV bool fp_eq(const Fp& a, const Fp& b) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) o |= a.v[j] ^ b.v[j];
    return o == 0;
}

DEV bool fp_is_one(const Fp& a) {
    constexpr uint32_t O[NL] = {CC_ONE_LIMBS};
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) o |= a.v[j] ^ O[j];
    return o == 0;
}

// r = t >= p ? t - p : t   (t < 2p)
DEV void fp_reduce_once(Fp& r, const uint32_t t[NL]) {
    uint32_t s[NL];
    uint32_t br = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) s[j] = __builtin_subc(t[j], p_limb(j), br, &br);
#pragma unroll
    for (int j = 0; j < NL; j++) r.v[j] = br ? t[j] : s[j];
}

// Carry chains: gfx950 needs wait states between a VALU carry-out and the next carry-in of the same
// chain (the compiler pads them with s_nop), so each add/sub below runs two or three independent
// chains interleaved limb by limb.
DEV void fp_add(Fp& r, const Fp& a, const Fp& b) {
    uint32_t t[NL], s[NL];
    uint32_t c = 0, br = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        t[j] = __builtin_addc(a.v[j], b.v[j], c, &c);  // a + b < 2p < 2^384: no carry out
        s[j] = __builtin_subc(t[j], p_limb(j), br, &br);
    }
#pragma unroll
    for (int j = 0; j < NL; j++) r.v[j] = br ? t[j] : s[j];
}

DEV void fp_dbl(Fp& r, const Fp& a) { fp_add(r, a, a); }

// a - b, or a + (p - b) when a < b
DEV void fp_sub(Fp& r, const Fp& a, const Fp& b) {
    uint32_t t[NL], u[NL];
    uint32_t b1 = 0, b2 = 0, c3 = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        t[j] = __builtin_subc(a.v[j], b.v[j], b1, &b1);
        const uint32_t w = __builtin_subc(p_limb(j), b.v[j], b2, &b2);
        u[j] = __builtin_addc(a.v[j], w, c3, &c3);
    }
#pragma unroll
    for (int j = 0; j < NL; j++) r.v[j] = b1 ? u[j] : t[j];
}

// p - a for a != 0, 0 for a == 0 (one borrow chain and a mask)
DEV void fp_neg(Fp& r, const Fp& a) {
    uint32_t t[NL], o = 0, br = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        t[j] = __builtin_subc(p_limb(j), a.v[j], br, &br);
        o |= a.v[j];
    }
    const uint32_t mask = o ? ~0u : 0u;
#pragma unroll
    for (int j = 0; j < NL; j++) r.v[j] = t[j] & mask;
}

// ---------------------------------------------------------------- Montgomery multiplication
DEV uint32_t p29(int j) {
    constexpr uint32_t Q[L29] = {CC_P29_LIMBS};
    return Q[j];
}

// c + a*b: one v_mad_u64_u32.  Written in plain C, not inline asm: the hazard recognizer cannot see
// into an asm block and pads every asm mad with an s_nop (measured: ~1 nop per mad); the compiler's
// own v_mad_u64_u32 (dead SGPR carry-out) chains back to back.
DEV uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return c + (uint64_t)a * b; }
// same with a wave-uniform multiplier (a limb of p, an SGPR operand)
DEV uint64_t mad64s(uint32_t a, uint32_t b, uint64_t c) { return c + (uint64_t)a * b; }

// 12 x 32 -> 14 x 29 (value < 2^384)
DEV void to29(uint32_t o[L29], const Fp& x) {
    o[0] = x.v[0] & M29;
#pragma unroll
    for (int k = 1; k < L29 - 1; k++) {
        const int bit = 29 * k, w = bit >> 5, s = bit & 31;
        o[k] = (s ? __builtin_amdgcn_alignbit(x.v[w + 1], x.v[w], s) : x.v[w]) & M29;
    }
    o[L29 - 1] = x.v[NL - 1] >> 25;
}

// 14 x 29 (normalised limbs, value < 2p) -> canonical 12 x 32
DEV void from29(Fp& r, const uint32_t t[L29]) {
    uint32_t w32[NL];
#pragma unroll
    for (int w = 0; w < NL; w++) {
        const int bit = 32 * w, k = bit / 29, s = bit % 29;
        uint32_t x = t[k] >> s;
        if (k + 1 < L29) x |= t[k + 1] << (29 - s);
        if (s > 26 && k + 2 < L29) x |= t[k + 2] << (58 - s);
        w32[w] = x;
    }
    fp_reduce_once(r, w32);
}

// Montgomery reduction columns shared by mul and sqr: the caller has added column k's a*b terms
// to acc; this adds the m*p terms, derives m_k (k < 14) or emits limb k - 14, and shifts.
DEV void redc_column(int k, uint64_t& acc, uint32_t m[L29], uint32_t r[L29]) {
#pragma unroll
    for (int i = 0; i < L29; i++) {
        const int j = k - i;
        if (i >= k || j < 0 || j >= L29) continue;
        acc = mad64s(m[i], p29(j), acc);
    }
    if (k < L29) {
        m[k] = ((uint32_t)acc * N0_29) & M29;
        acc = mad64s(m[k], p29(0), acc);
    } else {
        r[k - L29] = (uint32_t)acc & M29;
    }
    acc >>= 29;
}

// a * b * 2^-406 mod p, canonical.  a, b < 2^384; column sums < 28 * 2^58 + 2^35 < 2^64.
DEV Fp fp_mul_v(const Fp& A, const Fp& B) {
    uint32_t a[L29], b[L29], m[L29], r[L29];
    to29(a, A);
    to29(b, B);
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * L29 - 1; k++) {
#pragma unroll
        for (int i = 0; i < L29; i++) {
            const int j = k - i;
            if (j < 0 || j >= L29) continue;
            acc = mad64(a[i], b[j], acc);
        }
        redc_column(k, acc, m, r);
    }
    r[L29 - 1] = (uint32_t)acc;
    Fp o;
    from29(o, r);
    return o;
}

// a^2 * 2^-406 mod p: off-diagonal products once against the doubled operand (105 + 196 mads)
DEV Fp fp_sqr_v(const Fp& A) {
    uint32_t a[L29], a2[L29], m[L29], r[L29];
    to29(a, A);
#pragma unroll
    for (int i = 0; i < L29; i++) a2[i] = a[i] << 1;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * L29 - 1; k++) {
#pragma unroll
        for (int i = 0; i < L29; i++) {
            const int j = k - i;
            if (j <= i || j >= L29) continue;
            acc = mad64(a2[i], a[j], acc);
        }
        if (!(k & 1) && k / 2 < L29) acc = mad64(a[k / 2], a[k / 2], acc);
        redc_column(k, acc, m, r);
    }
    r[L29 - 1] = (uint32_t)acc;
    Fp o;
    from29(o, r);
    return o;
}

// Translation units holding the hot loops (Miller loop, final exponentiation) define CC_FP_INLINE and
// get the multiplication inlined at every site; everywhere else it is one out-of-line copy called
// with its 24 limbs in argument VGPRs (compile time and code size stay small).
#ifdef CC_FP_INLINE
// Each inlined multiplication sits in its own basic block (a loop that runs once on an opaque,
// wave-uniform condition): instruction selection and scheduling work per block, and blocks of
// tens of thousands of instructions (a Miller step) make their compile time explode.
DEV bool cc_opaque_false() {
    uint32_t x;
    asm volatile("s_mov_b32 %0, 0" : "=s"(x));
    return x != 0;
}
// The operands pass through an empty volatile asm so their radix-2^29 conversions cannot be
// common-subexpression-eliminated across multiplication sites (that keeps 14-limb copies of every
// reused operand live and spills); the conversion is ~30 instructions against ~400 mads.
DEV void fp_opaque(Fp& x) {
#pragma unroll
    for (int k = 0; k < NL; k++) asm volatile("" : "+v"(x.v[k]));
}
DEV void fp_mul(Fp& r, const Fp& a, const Fp& b) {
    do {
        Fp x = a, y = b;
        fp_opaque(x);
        fp_opaque(y);
        r = fp_mul_v(x, y);
    } while (cc_opaque_false());
}
DEV void fp_sqr(Fp& r, const Fp& a) {
    do {
        Fp x = a;
        fp_opaque(x);
        r = fp_sqr_v(x);
    } while (cc_opaque_false());
}
#else
#define CC_L12(x) uint32_t x##0, uint32_t x##1, uint32_t x##2, uint32_t x##3, uint32_t x##4, uint32_t x##5, \
    uint32_t x##6, uint32_t x##7, uint32_t x##8, uint32_t x##9, uint32_t x##10, uint32_t x##11
#define CC_V12(x) x##0, x##1, x##2, x##3, x##4, x##5, x##6, x##7, x##8, x##9, x##10, x##11
#define CC_E12(x) x.v[0], x.v[1], x.v[2], x.v[3], x.v[4], x.v[5], x.v[6], x.v[7], x.v[8], x.v[9], x.v[10], x.v[11]
static __device__ __noinline__ Fp fp_mul_call(CC_L12(a), CC_L12(b)) {
    const Fp A = {{CC_V12(a)}}, B = {{CC_V12(b)}};
    return fp_mul_v(A, B);
}
static __device__ __noinline__ Fp fp_sqr_call(CC_L12(a)) {
    const Fp A = {{CC_V12(a)}};
    return fp_sqr_v(A);
}
DEV void fp_mul(Fp& r, const Fp& a, const Fp& b) { r = fp_mul_call(CC_E12(a), CC_E12(b)); }
DEV void fp_sqr(Fp& r, const Fp& a) { r = fp_sqr_call(CC_E12(a)); }
#endif

// a * small constant via additions (k <= 12)
DEV void fp_mul_small(Fp& r, const Fp& a, int k) {
    Fp acc = a;
    for (int i = 1; i < k; i++) fp_add(acc, acc, a);
    r = acc;
}

// convert canonical integer (< p) to Montgomery
DEV void fp_to_mont(Fp& r, const Fp& a) {
    constexpr uint32_t R2[NL] = {CC_R2_LIMBS};
    Fp r2;
#pragma unroll
    for (int j = 0; j < NL; j++) r2.v[j] = R2[j];
    fp_mul(r, a, r2);
}

DEV void fp_from_mont(Fp& r, const Fp& a) {
    Fp one;
    fp_zero(one);
    one.v[0] = 1;
    fp_mul(r, a, one);
}

// is the raw integer a (< 2^384) >= p ?
DEV bool fp_raw_geq_p(const Fp& a) {
    uint32_t br = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) (void)__builtin_subc(a.v[j], p_limb(j), br, &br);
    return br == 0;
}

// raw integer mod p (AMCL FP::new_big reduces); the loop runs only for non-canonical encodings
DEV void fp_raw_reduce(Fp& a) {
    while (fp_raw_geq_p(a)) {
        uint32_t br = 0;
#pragma unroll
        for (int j = 0; j < NL; j++) a.v[j] = __builtin_subc(a.v[j], p_limb(j), br, &br);
    }
}

// ---------------------------------------------------------------------------------------------
// Inversion: Bernstein-Yang divsteps ("safegcd", eprint 2019/266), variable-time variant with
// batches of 30 divsteps and the 2x2 transition matrix applied to signed radix-2^30 numbers
// (13 limbs, 390 bits).  Replaces Fermat's a^(p-2): ~25 batches of ~130 v_mad_i64_i32 plus
// ~300 scalar-width ops against ~580 full Montgomery multiplications.  Variable time is fine here:
// everything this engine inverts is public verification data.  Lanes diverge only inside the
// divstep inner loop (the wave runs the longest lane's count).
constexpr int S30N = 13;
constexpr int32_t M30 = 0x3fffffff;
struct S30 {
    int32_t v[S30N];
};
// p in signed radix 2^30, p^-1 mod 2^30, and R^3 mod p (R = 2^406) to return to Montgomery form
#define CC_P30_LIMBS                                                                                    \
    0x3fffaaab, 0x27fbffff, 0x153ffffb, 0x2affffac, 0x30f6241e, 0x034a83da, 0x112bf673, 0x12e13ce1, \
        0x2cd76477, 0x1ed90d2e, 0x29a4b1ba, 0x3a8e5ff9, 0x001a0111
constexpr uint32_t PINV30 = 0x30003u;
#define CC_R3_LIMBS                                                                             \
    0x49217d6au, 0x73ac2317u, 0x73c452c4u, 0x2c409357u, 0x79c0a55eu, 0xfe1f49acu, 0xaaa3c553u, \
        0x1bdc0da2u, 0xc3f31a9du, 0x75d3a486u, 0x84da1a2du, 0x15e5ecfbu
DEV int32_t p30_limb(int j) {
    constexpr int32_t P[S30N] = {CC_P30_LIMBS};
    return P[j];
}

// 30 divsteps on the low words of f, g (f odd); returns the new eta (= -delta) and the matrix t
// with 2^30 [f', g'] = t [f, g].  Zero runs of g are consumed at once; otherwise up to 8 low bits of
// g are cancelled by one multiple of f (-f^-1 mod 256 from two Newton steps).
DEV int32_t divsteps30(int32_t eta, uint32_t f, uint32_t g, int32_t t[4]) {
    uint32_t u = 1, v = 0, q = 0, r = 1;
    int i = 30;
    for (;;) {
        const int zeros = __builtin_ctz(g | (0xffffffffu << i));
        g >>= zeros;
        u <<= zeros;
        v <<= zeros;
        eta -= zeros;
        i -= zeros;
        if (i == 0) break;
        if (eta < 0) {
            eta = -eta;
            uint32_t tmp = f;
            f = g;
            g = 0u - tmp;
            tmp = u;
            u = q;
            q = 0u - tmp;
            tmp = v;
            v = r;
            r = 0u - tmp;
        }
        const int limit = (eta + 1) > i ? i : (eta + 1);
        const uint32_t m = (0xffffffffu >> (32 - limit)) & 255u;
        // -f^-1 mod 256 by Newton's iteration (f odd): (3f) ^ 2 is f^-1 to 5 bits, one step gives 10
        // (a table lookup here was a vector memory load with its full latency, every iteration)
        uint32_t fi = (3u * f) ^ 2u;
        fi *= 2u - f * fi;
        const uint32_t w = (g * (0u - fi)) & m;
        g += f * w;
        q += u * w;
        r += v * w;
    }
    t[0] = (int32_t)u;
    t[1] = (int32_t)v;
    t[2] = (int32_t)q;
    t[3] = (int32_t)r;
    return eta;
}

// c + a b for signed 32-bit a, b (one v_mad_i64_i32: left to itself the compiler multiplies these
// sign-extended, 64 x 64 bits, with two extra v_mul_lo_u32 and a v_add3)
DEV int64_t smad(int32_t a, int32_t b, int64_t c) {
    int64_t r;
    uint64_t cy;
    asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cy) : "v"(a), "v"(b), "v"(c));
    return r;
}
// [f, g] <- t [f, g] / 2^30 (exact)
DEV void s30_update_fg(S30& f, S30& g, const int32_t t[4]) {
    int64_t cf = smad(t[1], g.v[0], smad(t[0], f.v[0], 0));
    int64_t cg = smad(t[3], g.v[0], smad(t[2], f.v[0], 0));
    cf >>= 30;
    cg >>= 30;
#pragma unroll
    for (int i = 1; i < S30N; i++) {
        cf = smad(t[1], g.v[i], smad(t[0], f.v[i], cf));
        cg = smad(t[3], g.v[i], smad(t[2], f.v[i], cg));
        f.v[i - 1] = (int32_t)cf & M30;
        g.v[i - 1] = (int32_t)cg & M30;
        cf >>= 30;
        cg >>= 30;
    }
    f.v[S30N - 1] = (int32_t)cf;
    g.v[S30N - 1] = (int32_t)cg;
}

// [d, e] <- (t [d, e] + p [md, me]) / 2^30 with md, me making the division exact; d, e stay in
// (-2p, p) (Bernstein-Yang §5 / the libsecp256k1 modinv32 range argument, independent of width).
DEV void s30_update_de(S30& d, S30& e, const int32_t t[4]) {
    const int32_t sd = d.v[S30N - 1] >> 31, se = e.v[S30N - 1] >> 31;
    int32_t md = (t[0] & sd) + (t[1] & se);
    int32_t me = (t[2] & sd) + (t[3] & se);
    int64_t cd = smad(t[1], e.v[0], smad(t[0], d.v[0], 0));
    int64_t ce = smad(t[3], e.v[0], smad(t[2], d.v[0], 0));
    md -= (int32_t)((PINV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
    me -= (int32_t)((PINV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
    cd = smad(p30_limb(0), md, cd);
    ce = smad(p30_limb(0), me, ce);
    cd >>= 30;
    ce >>= 30;
#pragma unroll
    for (int i = 1; i < S30N; i++) {
        cd = smad(p30_limb(i), md, smad(t[1], e.v[i], smad(t[0], d.v[i], cd)));
        ce = smad(p30_limb(i), me, smad(t[3], e.v[i], smad(t[2], d.v[i], ce)));
        d.v[i - 1] = (int32_t)cd & M30;
        e.v[i - 1] = (int32_t)ce & M30;
        cd >>= 30;
        ce >>= 30;
    }
    d.v[S30N - 1] = (int32_t)cd;
    e.v[S30N - 1] = (int32_t)ce;
}

// limbs 0..11 into [0, 2^30), the signed remainder into the top limb
DEV void s30_carry(S30& a) {
#pragma unroll
    for (int i = 0; i < S30N - 1; i++) {
        a.v[i + 1] += a.v[i] >> 30;
        a.v[i] &= M30;
    }
}
// a += k p for k in {-1, 0, 1}
DEV void s30_add_kp(S30& a, int32_t k) {
#pragma unroll
    for (int i = 0; i < S30N; i++) a.v[i] += k * p30_limb(i);
    s30_carry(a);
}

DEV void s30_from_fp(S30& r, const Fp& a) {
#pragma unroll
    for (int i = 0; i < S30N; i++) {
        const int w = (30 * i) >> 5, sh = (30 * i) & 31;
        const uint64_t pair = (uint64_t)a.v[w] | ((w + 1 < NL ? (uint64_t)a.v[w + 1] : 0ull) << 32);
        r.v[i] = (int32_t)((uint32_t)(pair >> sh) & (uint32_t)M30);
    }
}
// a in [0, p), limbs normalised
DEV void fp_from_s30(Fp& r, const S30& a) {
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const int i = (32 * j) / 30, sh = (32 * j) % 30;
        uint64_t x = (uint64_t)(uint32_t)a.v[i] >> sh;
        if (i + 1 < S30N) x |= (uint64_t)(uint32_t)a.v[i + 1] << (30 - sh);
        if (i + 2 < S30N) x |= (uint64_t)(uint32_t)a.v[i + 2] << (60 - sh);
        r.v[j] = (uint32_t)x;
    }
}

// r = a^-1 mod p as a plain integer (a < p; 0 -> 0).  fp_inv below and the lazy layer (lazy.h) put
// it back into their own Montgomery forms.
DEV void fp_inv_int(Fp& r, const Fp& a) {
    S30 d, e, f, g;
#pragma unroll
    for (int i = 0; i < S30N; i++) {
        d.v[i] = 0;
        e.v[i] = 0;
        f.v[i] = p30_limb(i);
    }
    e.v[0] = 1;
    s30_from_fp(g, a);
    int32_t eta = -1;
    // Bernstein-Yang bound for 381-bit inputs: < 1110 divsteps = 37 batches
    for (int it = 0; it < 40; it++) {
        int32_t t[4];
        eta = divsteps30(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
        s30_update_de(d, e, t);
        s30_update_fg(f, g, t);
        int32_t o = 0;
#pragma unroll
        for (int i = 0; i < S30N; i++) o |= g.v[i];
        if (o == 0) break;
    }
    // f = +-1 (or p when a = 0, where d = 0): x = sign(f) d mod p, d in (-2p, p)
    if (f.v[S30N - 1] < 0) {
#pragma unroll
        for (int i = 0; i < S30N; i++) d.v[i] = -d.v[i];
        s30_carry(d);
    }
    s30_add_kp(d, d.v[S30N - 1] < 0 ? 1 : 0);
    s30_add_kp(d, d.v[S30N - 1] < 0 ? 1 : 0);
    S30 t = d;
    s30_add_kp(t, -1);
    if (t.v[S30N - 1] >= 0) d = t;
    fp_from_s30(r, d);
}

// r = a^-1 in Montgomery form (a in Montgomery form); 0 -> 0 like Fermat's a^(p-2).
DEV void fp_inv(Fp& r, const Fp& a) {
    Fp x, r3;
    fp_inv_int(x, a);
    constexpr uint32_t R3[NL] = {CC_R3_LIMBS};
#pragma unroll
    for (int j = 0; j < NL; j++) r3.v[j] = R3[j];
    fp_mul(r, x, r3);  // (aR)^-1 R^3 R^-1 = a^-1 R
}

// ============================== Fp2 ==============================
struct Fp2 {
    Fp a, b;  // a + b i
};

DEV void f2_zero(Fp2& r) { fp_zero(r.a); fp_zero(r.b); }
DEV void f2_one(Fp2& r) { fp_one(r.a); fp_zero(r.b); }
DEV bool f2_is_zero(const Fp2& x) { return fp_is_zero(x.a) && fp_is_zero(x.b); }
DEV bool f2_eq(const Fp2& x, const Fp2& y) { return fp_eq(x.a, y.a) && fp_eq(x.b, y.b); }
DEV void f2_add(Fp2& r, const Fp2& x, const Fp2& y) { fp_add(r.a, x.a, y.a); fp_add(r.b, x.b, y.b); }
DEV void f2_sub(Fp2& r, const Fp2& x, const Fp2& y) { fp_sub(r.a, x.a, y.a); fp_sub(r.b, x.b, y.b); }
// sum feeding only a multiplication (the pair-lane tower skips the reduction there; canonical here)
DEV void f2_add_lz(Fp2& r, const Fp2& x, const Fp2& y) { f2_add(r, x, y); }
DEV void f2_dbl(Fp2& r, const Fp2& x) { fp_dbl(r.a, x.a); fp_dbl(r.b, x.b); }
DEV void f2_neg(Fp2& r, const Fp2& x) { fp_neg(r.a, x.a); fp_neg(r.b, x.b); }
DEV void f2_conj(Fp2& r, const Fp2& x) { r.a = x.a; fp_neg(r.b, x.b); }

DEV void f2_mul(Fp2& r, const Fp2& x, const Fp2& y) {
    Fp t0, t1, s0, s1;
    fp_mul(t0, x.a, y.a);
    fp_mul(t1, x.b, y.b);
    fp_add(s0, x.a, x.b);
    fp_add(s1, y.a, y.b);
    fp_mul(s0, s0, s1);
    fp_sub(s0, s0, t0);
    fp_sub(r.b, s0, t1);
    fp_sub(r.a, t0, t1);
}

DEV void f2_sqr(Fp2& r, const Fp2& x) {
    Fp s, d, m;
    fp_add(s, x.a, x.b);
    fp_sub(d, x.a, x.b);
    fp_mul(m, x.a, x.b);
    fp_mul(r.a, s, d);
    fp_dbl(r.b, m);
}

DEV void f2_mul_fp(Fp2& r, const Fp2& x, const Fp& k) { fp_mul(r.a, x.a, k); fp_mul(r.b, x.b, k); }

// x * xi, xi = 1 + i
DEV void f2_mul_xi(Fp2& r, const Fp2& x) {
    Fp t;
    fp_sub(t, x.a, x.b);
    fp_add(r.b, x.a, x.b);
    r.a = t;
}

DEV void f2_inv(Fp2& r, const Fp2& x) {
    Fp n, t;
    fp_sqr(n, x.a);
    fp_sqr(t, x.b);
    fp_add(n, n, t);
    fp_inv(n, n);
    fp_mul(r.a, x.a, n);
    fp_mul(t, x.b, n);
    fp_neg(r.b, t);
}

#include "tower.inc"

DEV bool f12_is_one(const Fp12& x) {
    return fp_is_one(x.a.a.a) && fp_is_zero(x.a.a.b) && f2_is_zero(x.a.b) && f2_is_zero(x.b.a) &&
           f2_is_zero(x.b.b) && f2_is_zero(x.c.a) && f2_is_zero(x.c.b);
}


}  // namespace cc
