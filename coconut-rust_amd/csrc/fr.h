// Scalar-field (mod r) arithmetic and the RLC coefficient generator — device code.
//
//   Fm        : Fr in Montgomery form, 8 x 32-bit limbs, R = 2^256 (Lagrange coefficients of
//               secret_sharing `Polynomial::lagrange_basis_at_0` [EXT], reference
//               src/signature.rs:460,502; delta_i * m_ij products of the RLC batch mode)
//   chacha20  : RFC 8439 block function; the RLC batch mode draws its 128-bit coefficients
//               delta_i = ChaCha20(key = host seed, counter = global credential index)
#pragma once
#include "codec.h"

namespace cc {

constexpr int NR = 8;
#define CC_RR2 0xf3f29c6du, 0xc999e990u, 0x87925c23u, 0x2b6cedcbu, 0x7254398fu, 0x05d31496u, 0x9f59ff11u, 0x0748d9d9u
#define CC_RONE 0xfffffffeu, 0x00000001u, 0x00034802u, 0x5884b7fau, 0xecbc4ff5u, 0x998c4fefu, 0xacc5056fu, 0x1824b159u

struct Fm {
    uint32_t v[NR];
};

DEV uint32_t rl(int j) {
    constexpr uint32_t Rl[NR] = {CC_R_LIMBS};
    return Rl[j];
}

DEV void fm_reduce_once(Fm& r, const uint32_t t[NR]) {
    uint32_t s[NR], br = 0;
#pragma unroll
    for (int j = 0; j < NR; j++) s[j] = __builtin_subc(t[j], rl(j), br, &br);
#pragma unroll
    for (int j = 0; j < NR; j++) r.v[j] = br ? t[j] : s[j];
}

// CIOS Montgomery multiplication mod r (r < 2^255: no extra carry word)
static __device__ __noinline__ Fm fm_mul_v(Fm a, Fm b) {
    uint32_t t[NR];
#pragma unroll
    for (int i = 0; i < NR; i++) {
        const uint32_t bi = b.v[i];
        uint64_t A = (uint64_t)a.v[0] * bi + (i ? t[0] : 0u);
        const uint32_t t0 = (uint32_t)A;
        const uint32_t m = t0 * 0xffffffffu;  // -r^-1 mod 2^32
        uint64_t C = (uint64_t)m * rl(0) + t0;
#pragma unroll
        for (int j = 1; j < NR; j++) {
            A = (uint64_t)a.v[j] * bi + (uint64_t)(i ? t[j] : 0u) + (A >> 32);
            C = (uint64_t)m * rl(j) + (uint64_t)(uint32_t)A + (C >> 32);
            t[j - 1] = (uint32_t)C;
        }
        t[NR - 1] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
    }
    Fm r;
    fm_reduce_once(r, t);
    return r;
}

DEV void fm_sub(Fm& r, const Fm& a, const Fm& b) {
    uint32_t t[NR], br = 0;
#pragma unroll
    for (int j = 0; j < NR; j++) t[j] = __builtin_subc(a.v[j], b.v[j], br, &br);
    uint32_t mask = 0u - br, c = 0;
#pragma unroll
    for (int j = 0; j < NR; j++) r.v[j] = __builtin_addc(t[j], rl(j) & mask, c, &c);
}

DEV Fm fm_r2() {
    constexpr uint32_t R2[NR] = {CC_RR2};
    Fm r2;
#pragma unroll
    for (int j = 0; j < NR; j++) r2.v[j] = R2[j];
    return r2;
}

DEV Fm fm_from_u64(uint64_t x) {
    Fm a;
#pragma unroll
    for (int j = 0; j < NR; j++) a.v[j] = 0;
    a.v[0] = (uint32_t)x;
    a.v[1] = (uint32_t)(x >> 32);
    return fm_mul_v(a, fm_r2());  // x < 2^64 < r
}

DEV Fm fm_one() {
    constexpr uint32_t O[NR] = {CC_RONE};
    Fm a;
#pragma unroll
    for (int j = 0; j < NR; j++) a.v[j] = O[j];
    return a;
}

// ---------------------------------------------------------------- inversion mod r
// Bernstein-Yang divsteps as field.h fp_inv_int, for the 255-bit r: 9 signed radix-2^30 limbs, batches of
// 30 divsteps (field.h divsteps30) with the 2 x 2 matrix applied by signed 32 x 32 mads; r = 1 mod 2^30,
// so the exact-division multiple of r is the low 30 bits of -(c + m) directly.  ~25 batches against the
// ~384 Montgomery products of the Fermat ladder it replaces.
constexpr int R30N = 9;
struct R30 {
    int32_t v[R30N];
};
DEV int32_t r30_limb(int i) {
    constexpr int32_t L[R30N] = {0x1, 0x3ffffffc, 0x3fe5bfef, 0x2f6900bf, 0x21d80553,
                                 0x27602026, 0x17d48333, 0x29d4ca67, 0x73ed};
    return L[i];
}
DEV void r30_update_fg(R30& f, R30& g, const int32_t t[4]) {
    int64_t cf = smad(t[1], g.v[0], smad(t[0], f.v[0], 0));
    int64_t cg = smad(t[3], g.v[0], smad(t[2], f.v[0], 0));
    cf >>= 30;
    cg >>= 30;
#pragma unroll
    for (int i = 1; i < R30N; i++) {
        cf = smad(t[1], g.v[i], smad(t[0], f.v[i], cf));
        cg = smad(t[3], g.v[i], smad(t[2], f.v[i], cg));
        f.v[i - 1] = (int32_t)cf & M30;
        g.v[i - 1] = (int32_t)cg & M30;
        cf >>= 30;
        cg >>= 30;
    }
    f.v[R30N - 1] = (int32_t)cf;
    g.v[R30N - 1] = (int32_t)cg;
}
// [d, e] <- (t [d, e] + r [md, me]) / 2^30, d and e kept in (-2r, r)
DEV void r30_update_de(R30& d, R30& e, const int32_t t[4]) {
    const int32_t sd = d.v[R30N - 1] >> 31, se = e.v[R30N - 1] >> 31;
    int32_t md = (t[0] & sd) + (t[1] & se);
    int32_t me = (t[2] & sd) + (t[3] & se);
    int64_t cd = smad(t[1], e.v[0], smad(t[0], d.v[0], 0));
    int64_t ce = smad(t[3], e.v[0], smad(t[2], d.v[0], 0));
    md -= (int32_t)(((uint32_t)cd + (uint32_t)md) & (uint32_t)M30);  // r^-1 = 1 mod 2^30
    me -= (int32_t)(((uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
    cd = smad(r30_limb(0), md, cd);
    ce = smad(r30_limb(0), me, ce);
    cd >>= 30;
    ce >>= 30;
#pragma unroll
    for (int i = 1; i < R30N; i++) {
        cd = smad(r30_limb(i), md, smad(t[1], e.v[i], smad(t[0], d.v[i], cd)));
        ce = smad(r30_limb(i), me, smad(t[3], e.v[i], smad(t[2], d.v[i], ce)));
        d.v[i - 1] = (int32_t)cd & M30;
        e.v[i - 1] = (int32_t)ce & M30;
        cd >>= 30;
        ce >>= 30;
    }
    d.v[R30N - 1] = (int32_t)cd;
    e.v[R30N - 1] = (int32_t)ce;
}
DEV void r30_carry(R30& a) {
#pragma unroll
    for (int i = 0; i < R30N - 1; i++) {
        a.v[i + 1] += a.v[i] >> 30;
        a.v[i] &= M30;
    }
}
DEV void r30_add_kr(R30& a, int32_t k) {
#pragma unroll
    for (int i = 0; i < R30N; i++) a.v[i] += k * r30_limb(i);
    r30_carry(a);
}
// a^-1 mod r as a plain integer (a < r; 0 -> 0)
DEV void fr_inv_int(uint32_t out[NR], const uint32_t a[NR]) {
    R30 d, e, f, g;
#pragma unroll
    for (int i = 0; i < R30N; i++) {
        d.v[i] = 0;
        e.v[i] = 0;
        f.v[i] = r30_limb(i);
        const int w = (30 * i) >> 5, sh = (30 * i) & 31;
        const uint64_t pair = (uint64_t)a[w] | ((w + 1 < NR ? (uint64_t)a[w + 1] : 0ull) << 32);
        g.v[i] = (int32_t)((uint32_t)(pair >> sh) & (uint32_t)M30);
    }
    e.v[0] = 1;
    int32_t eta = -1;
    for (int it = 0; it < 30; it++) {  // Bernstein-Yang bound for 255-bit inputs: < 740 divsteps
        int32_t t[4];
        eta = divsteps30(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
        r30_update_de(d, e, t);
        r30_update_fg(f, g, t);
        int32_t o = 0;
#pragma unroll
        for (int i = 0; i < R30N; i++) o |= g.v[i];
        if (o == 0) break;
    }
    // f = +-1 (or r when a = 0, where d = 0): x = sign(f) d mod r, d in (-2r, r)
    if (f.v[R30N - 1] < 0) {
#pragma unroll
        for (int i = 0; i < R30N; i++) d.v[i] = -d.v[i];
        r30_carry(d);
    }
    r30_add_kr(d, d.v[R30N - 1] < 0 ? 1 : 0);
    r30_add_kr(d, d.v[R30N - 1] < 0 ? 1 : 0);
    R30 tt = d;
    r30_add_kr(tt, -1);
    if (tt.v[R30N - 1] >= 0) d = tt;
#pragma unroll
    for (int j = 0; j < NR; j++) {
        const int i = (32 * j) / 30, sh = (32 * j) % 30;
        uint64_t x = (uint64_t)(uint32_t)d.v[i] >> sh;
        if (i + 1 < R30N) x |= (uint64_t)(uint32_t)d.v[i + 1] << (30 - sh);
        if (i + 2 < R30N) x |= (uint64_t)(uint32_t)d.v[i + 2] << (60 - sh);
        out[j] = (uint32_t)x;
    }
}

// a^-1 in Montgomery form (a in Montgomery form): (a R)^-1 times R^3 R^-1 = a^-1 R; 0 -> 0
DEV Fm fm_inv(const Fm& a) {
    constexpr uint32_t R3[NR] = {0x439b73afu, 0xc62c1807u, 0x8cf06990u, 0x1b3e0d18u,
                                 0xc7b5f418u, 0x73d13c71u, 0xc8db33e9u, 0x6e2a5bb9u};  // R^3 mod r
    Fm x, r3;
    fr_inv_int(x.v, a.v);
#pragma unroll
    for (int j = 0; j < NR; j++) r3.v[j] = R3[j];
    return fm_mul_v(x, r3);
}

DEV Fm fm_to_canon(const Fm& a) {
    Fm one;
#pragma unroll
    for (int j = 0; j < NR; j++) one.v[j] = 0;
    one.v[0] = 1;
    return fm_mul_v(a, one);
}

// a * b mod r for canonical a, b (< r): (a b R^-1) R^2 R^-1
DEV void fr_mul_canon(uint32_t out[NR], const uint32_t a[NR], const uint32_t b[NR]) {
    Fm x, y;
#pragma unroll
    for (int j = 0; j < NR; j++) {
        x.v[j] = a[j];
        y.v[j] = b[j];
    }
    Fm z = fm_mul_v(fm_mul_v(x, y), fm_r2());
#pragma unroll
    for (int j = 0; j < NR; j++) out[j] = z.v[j];
}

// ---------------------------------------------------------------- ChaCha20 block (RFC 8439)
DEV uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

#define CC_QR(a, b, c, d)            \
    a += b, d ^= a, d = rotl32(d, 16); \
    c += d, b ^= c, b = rotl32(b, 12); \
    a += b, d ^= a, d = rotl32(d, 8);  \
    c += d, b ^= c, b = rotl32(b, 7)

DEV void chacha20_block(uint32_t out[16], const uint32_t key[8], uint32_t counter, uint32_t n0, uint32_t n1,
                        uint32_t n2) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4],      key[5],      key[6],      key[7],      counter, n0,     n1,     n2};
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = s[k];
#pragma unroll
    for (int r = 0; r < 10; r++) {
        CC_QR(x[0], x[4], x[8], x[12]);
        CC_QR(x[1], x[5], x[9], x[13]);
        CC_QR(x[2], x[6], x[10], x[14]);
        CC_QR(x[3], x[7], x[11], x[15]);
        CC_QR(x[0], x[5], x[10], x[15]);
        CC_QR(x[1], x[6], x[11], x[12]);
        CC_QR(x[2], x[7], x[8], x[13]);
        CC_QR(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) out[k] = x[k] + s[k];
}
#undef CC_QR

// delta for global credential index g: the first 128 bits of block (counter = low 32 bits of g,
// nonce = (high 32 bits of g, 0, 0)), low bit forced so delta != 0.  8 canonical limbs (< r).
DEV void rlc_delta(uint32_t d[NR], const uint32_t key[8], uint64_t g) {
    uint32_t blk[16];
    chacha20_block(blk, key, (uint32_t)g, (uint32_t)(g >> 32), 0u, 0u);
    d[0] = blk[0] | 1u;
    d[1] = blk[1];
    d[2] = blk[2];
    d[3] = blk[3];
    d[4] = d[5] = d[6] = d[7] = 0u;
}

// RLC coefficient as 16 signed base-256 digits: the 16 ChaCha20 bytes b_w read as int8 d_w in
// [-128, 127], delta = sum_w d_w 256^w (uniform over 2^128 consecutive integers around 0, so a
// forged batch still passes with probability <= 2^-127).  The g~-side fold (fold.hip) buckets by
// (w, |d_w|) with no carry digit.  d = delta mod r (canonical): with U = sum b_w 256^w and
// H = sum [b_w >= 128] 256^w, delta = U - 256 H.  dig: the 16 digit bytes (= the key-stream bytes).
DEV void rlc_delta_signed(uint32_t d[NR], uint32_t dig[4], const uint32_t key[8], uint64_t g) {
    uint32_t blk[16];
    chacha20_block(blk, key, (uint32_t)g, (uint32_t)(g >> 32), 0u, 0u);
    uint32_t h[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        dig[k] = blk[k];
        h[k] = (blk[k] >> 7) & 0x01010101u;
    }
    const uint32_t m[5] = {h[0] << 8, (h[1] << 8) | (h[0] >> 24), (h[2] << 8) | (h[1] >> 24),
                           (h[3] << 8) | (h[2] >> 24), h[3] >> 24};
    uint32_t br = 0;
#pragma unroll
    for (int k = 0; k < 5; k++) d[k] = __builtin_subc(k < 4 ? blk[k] : 0u, m[k], br, &br);
    const uint32_t ext = br ? 0xffffffffu : 0u;  // sign extension of U - 256 H
    d[5] = d[6] = d[7] = ext;
    if (br) {  // negative: + r
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < NR; k++) d[k] = __builtin_addc(d[k], rl(k), c, &c);
    }
}

// delta's magnitude and sign from its canonical residue d: |delta| < 2^136 (16 signed base-256 digits),
// so a residue with a nonzero word above bit 160 is r - |delta|.  delta X~ then runs over the
// magnitude's windows only (8-byte scalar: 7 of 12 windows at 22 bits) with the table entries negated.
DEV bool rlc_delta_abs(uint32_t a[NR], const uint32_t d[NR]) {
    const bool neg = (d[5] | d[6] | d[7]) != 0;
    uint32_t br = 0;
#pragma unroll
    for (int k = 0; k < NR; k++) {
        const uint32_t t = __builtin_subc(rl(k), d[k], br, &br);
        a[k] = neg ? t : d[k];
    }
    return neg;
}

}  // namespace cc
