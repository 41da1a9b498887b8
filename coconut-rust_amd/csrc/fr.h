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
__constant__ static const uint32_t kRm2[NR] = {0xffffffffu, 0xfffffffeu, 0xfffe5bfeu, 0x53bda402u,
                                               0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};

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

DEV Fm fm_inv(const Fm& a) {
    Fm acc = a;
    for (int bit = 254 - 1; bit >= 0; bit--) {  // r - 2 has its top bit at 254
        acc = fm_mul_v(acc, acc);
        if ((kRm2[bit >> 5] >> (bit & 31)) & 1u) acc = fm_mul_v(acc, a);
    }
    return acc;
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

}  // namespace cc
