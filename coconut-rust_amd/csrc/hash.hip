// Batched hash-to-curve for gfx950 — amcl_wrapper `from_msg_hash`: the
// generators of Params::new (reference src/signature.rs:22-32: label || " : g", " : g_tilde",
// " : y" || i) and SignatureRequest::compute_h (src/signature.rs:197-206).  One message per lane.
//
//   hash_msg  : SHAKE256(msg) squeezed to 48 bytes (Keccak-f[1600], rate 136, domain byte 0x1F)
//   G1 mapit  : x = hash mod p; try x, x+1, ...: y = (x^3 + 4)^((p+1)/4) when it is a root, negated
//               if its integer value is odd (AMCL ECP::new_bigint(x, 0)); P = [h1] P (cofactor),
//               retried if that is the identity
//   G2 mapit  : X = 1 + x i; try x, x+1, ...: y = AMCL FP2::sqrt(X^3 + 4(1+i)); then
//               [x^2 - x - 1] Q + psi([x - 1] Q) + psi^2(2 Q)  (Budroni-Pintore, AMCL ECP2::mapit)
// Restated from recalled AMCL v3.2 sources (not in this container): PARITY UNPINNED; the CPU mirror
// is oracle/hash_to_curve.py.
#include "codec.h"
#include "subgroup.h"

using namespace cc;

namespace {

// ---------------------------------------------------------------- SHAKE256
__constant__ static const uint64_t kRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

DEV uint64_t rotl64(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

DEV void keccak_f(uint64_t st[25]) {
    constexpr int ROTC[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
    constexpr int PILN[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
#pragma unroll 1
    for (int round = 0; round < 24; round++) {
        uint64_t bc[5];
#pragma unroll
        for (int i = 0; i < 5; i++) bc[i] = st[i] ^ st[i + 5] ^ st[i + 10] ^ st[i + 15] ^ st[i + 20];
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const uint64_t t = bc[(i + 4) % 5] ^ rotl64(bc[(i + 1) % 5], 1);
#pragma unroll
            for (int j = 0; j < 25; j += 5) st[j + i] ^= t;
        }
        uint64_t t = st[1];
#pragma unroll
        for (int i = 0; i < 24; i++) {
            const int j = PILN[i];
            const uint64_t b0 = st[j];
            st[j] = rotl64(t, ROTC[i]);
            t = b0;
        }
#pragma unroll
        for (int j = 0; j < 25; j += 5) {
#pragma unroll
            for (int i = 0; i < 5; i++) bc[i] = st[j + i];
#pragma unroll
            for (int i = 0; i < 5; i++) st[j + i] ^= (~bc[(i + 1) % 5]) & bc[(i + 2) % 5];
        }
        st[0] ^= kRC[round];
    }
}

// SHAKE256(msg[0..len)) -> 48 bytes
DEV void shake256_48(uint8_t out[48], const uint8_t* msg, size_t len) {
    constexpr int RATE = 136;
    uint64_t st[25];
#pragma unroll
    for (int i = 0; i < 25; i++) st[i] = 0;
    size_t off = 0;
#pragma unroll 1
    while (len - off >= RATE) {
        for (int i = 0; i < RATE / 8; i++) {
            uint64_t w = 0;
            for (int b = 0; b < 8; b++) w |= (uint64_t)msg[off + 8 * i + b] << (8 * b);
            st[i] ^= w;
        }
        keccak_f(st);
        off += RATE;
    }
    // last (partial) block with SHAKE padding: 0x1F ... 0x80
    const size_t rem = len - off;
    for (int i = 0; i < RATE / 8; i++) {
        uint64_t w = 0;
        for (int b = 0; b < 8; b++) {
            const size_t k = (size_t)(8 * i + b);
            uint8_t v = k < rem ? msg[off + k] : 0;
            if (k == rem) v ^= 0x1F;
            if (k == RATE - 1) v ^= 0x80;
            w |= (uint64_t)v << (8 * b);
        }
        st[i] ^= w;
    }
    keccak_f(st);
    for (int k = 0; k < 48; k++) out[k] = (uint8_t)(st[k >> 3] >> (8 * (k & 7)));
}

// ---------------------------------------------------------------- field helpers
// a^e for the fixed exponent e (12 LE limbs), square-and-multiply from the top set bit
DEV void fp_pow_fixed(Fp& r, const Fp& a, const uint32_t* e, int topbit) {
    Fp acc = a;
#pragma unroll 1
    for (int bit = topbit - 1; bit >= 0; bit--) {
        fp_sqr(acc, acc);
        if ((e[bit >> 5] >> (bit & 31)) & 1u) fp_mul(acc, acc, a);
    }
    r = acc;
}

// (p + 1) / 4, top bit 378
__constant__ static const uint32_t kSqrtE[NL] = {0xffffeaabu, 0xee7fbfffu, 0xac54ffffu, 0x07aaffffu, 0x3dac3d89u, 0xd9cc34a8u,
                                                 0x3ce144afu, 0xd91dd2e1u, 0x90d2eb35u, 0x92c6e9edu, 0x8e5ff9a6u, 0x0680447au};

// s = a^((p+1)/4); true iff s is a square root of a (a != 0)
DEV bool fp_sqrt_qr(Fp& s, const Fp& a) {
    fp_pow_fixed(s, a, kSqrtE, 378);
    Fp t;
    fp_sqr(t, s);
    return !fp_is_zero(a) && fp_eq(t, a);
}

// AMCL FP2::sqrt (see oracle/hash_to_curve.py f2_sqrt_amcl); false when x is not a square
DEV bool f2_sqrt_amcl(Fp2& r, const Fp2& x) {
    if (f2_is_zero(x)) {
        f2_zero(r);
        return true;
    }
    Fp w1, w2, t;
    fp_sqr(w1, x.b);
    fp_sqr(t, x.a);
    fp_add(w1, w1, t);
    if (!fp_sqrt_qr(t, w1)) return false;
    w1 = t;
    fp_add(w2, x.a, w1);
    fp_half(w2, w2);
    Fp s;
    if (!fp_sqrt_qr(s, w2)) {
        fp_sub(w2, x.a, w1);
        fp_half(w2, w2);
        if (!fp_sqrt_qr(s, w2)) return false;
    }
    r.a = s;
    fp_dbl(t, s);
    fp_inv(t, t);
    fp_mul(r.b, x.b, t);
    return true;
}

// 48 bytes big-endian -> Montgomery Fp (mod p)
DEV void fp_from_hash(Fp& r, const uint8_t h[48]) {
    Fp raw;
#pragma unroll
    for (int k = 0; k < NL; k++) {
        const uint8_t* q = h + 44 - 4 * k;
        raw.v[k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
    }
    fp_from_raw(r, raw);
}

// G1 cofactor h1 = (x - 1)^2 / 3 (126 bits)
constexpr uint64_t kH1Lo = 0x8C00AAAB0000AAABull, kH1Hi = 0x396C8C005555E156ull;

DEV bool g1_mapit(Aff<Fp>& out, const uint8_t h[48]) {
    Fp x, one, b;
    fp_from_hash(x, h);
    fp_one(one);
    FT<Fp>::curve_b(b);
#pragma unroll 1
    for (int tries = 0; tries < 4096; tries++) {
        Fp rhs, y;
        fp_sqr(rhs, x);
        fp_mul(rhs, rhs, x);
        fp_add(rhs, rhs, b);
        const Fp xc = x;
        fp_add(x, x, one);
        if (!fp_sqrt_qr(y, rhs)) continue;
        Fp yi;
        fp_from_mont(yi, y);
        if (yi.v[0] & 1u) fp_neg(y, y);  // ECP::new_bigint(x, 0): even y
        Aff<Fp> a{xc, y};
        Jac<Fp> acc;
        jac_from_aff(acc, a);
        for (int bit = 124; bit >= 0; bit--) {  // [h1] P, top bit 125 consumed by the start value
            jac_dbl(acc, acc);
            const uint64_t w = bit >= 64 ? kH1Hi : kH1Lo;
            if ((w >> (bit & 63)) & 1ull) jac_add_aff(acc, acc, a);
        }
        if (jac_to_aff(out, acc)) return true;
    }
    return false;
}

DEV void g2_psi(Jac<Fp2>& r, const Jac<Fp2>& p);

DEV bool g2_mapit(Aff<Fp2>& out, const uint8_t h[48]) {
    Fp x, one;
    fp_from_hash(x, h);
    fp_one(one);
    Fp2 b;
    FT<Fp2>::curve_b(b);
    Aff<Fp2> q;
    bool found = false;
#pragma unroll 1
    for (int tries = 0; tries < 4096 && !found; tries++) {
        Fp2 X, rhs, y;
        X.a = one;
        X.b = x;
        f2_sqr(rhs, X);
        f2_mul(rhs, rhs, X);
        f2_add(rhs, rhs, b);
        fp_add(x, x, one);
        if (f2_sqrt_amcl(y, rhs)) {
            q.x = X;
            q.y = y;
            found = true;
        }
    }
    if (!found) return false;
    // Budroni-Pintore: [x^2 - x - 1] Q + psi([x - 1] Q) + psi^2(2 Q), x < 0
    Jac<Fp2> Q, xQ, x2Q, t;
    jac_from_aff(Q, q);
    jac_mul_xabs(xQ, Q);   // [-x] Q
    jac_mul_xabs(x2Q, xQ); // [x^2] Q
    jac_neg(xQ, xQ);       // [x] Q
    Jac<Fp2> nQ;
    jac_neg(nQ, Q);
    jac_neg(t, xQ);        // [-x] Q
    jac_add(x2Q, x2Q, t);  // [x^2 - x] Q
    jac_add(x2Q, x2Q, nQ); // [x^2 - x - 1] Q
    jac_add(xQ, xQ, nQ);   // [x - 1] Q
    g2_psi(xQ, xQ);
    jac_dbl(Q, Q);
    g2_psi(Q, Q);
    g2_psi(Q, Q);
    jac_add(Q, Q, x2Q);
    jac_add(Q, Q, xQ);
    return jac_to_aff(out, Q);
}

// psi on Jacobian coordinates: (conj(X) c_x, conj(Y) c_y, conj(Z)) — the map is coordinate-wise
// Frobenius followed by constant scalings, so it commutes with the Jacobian scaling by Z
DEV void g2_psi(Jac<Fp2>& r, const Jac<Fp2>& p) {
    constexpr uint32_t CXB[NL] = {0x954030c4u, 0x1ed59d62u, 0x026053a5u, 0xc81fdd18u, 0xb49e2e0fu, 0xcb785f67u,
                                  0x6a65e5c3u, 0x689a6956u, 0x21724249u, 0x14cec802u, 0x7aaa6c42u, 0x00ba917au};
    constexpr uint32_t CYA[NL] = {0x699d9feeu, 0xfb9f5730u, 0x791f82c1u, 0x573fc3f8u, 0xc260bc18u, 0x774659b7u,
                                  0x65f57843u, 0x169c2180u, 0xf26ce7c9u, 0x477956cdu, 0x74beee42u, 0x191fce82u};
    constexpr uint32_t CYB[NL] = {0x96620abdu, 0xbe5fa8cfu, 0x38347d3du, 0xc76c3c06u, 0x34503a0bu, 0xefea78e9u,
                                  0x8d8f9a7bu, 0x4ddb2a04u, 0x50dec50eu, 0x03a250e8u, 0xc4c0f858u, 0x00e14367u};
    Fp2 c, u;
    fp_zero(c.a);
#pragma unroll
    for (int j = 0; j < NL; j++) c.b.v[j] = CXB[j];
    f2_conj(u, p.x);
    f2_mul(r.x, u, c);
#pragma unroll
    for (int j = 0; j < NL; j++) {
        c.a.v[j] = CYA[j];
        c.b.v[j] = CYB[j];
    }
    f2_conj(u, p.y);
    f2_mul(r.y, u, c);
    f2_conj(r.z, p.z);
}

template <int G>
__global__ __launch_bounds__(64) void k_hash_to_curve(size_t n, const uint8_t* __restrict__ data,
                                                      const uint64_t* __restrict__ offsets, uint8_t* __restrict__ out,
                                                      uint32_t* __restrict__ fail) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t h[48];
    shake256_48(h, data + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
    if (G == 1) {
        Aff<Fp> a;
        const bool ok = g1_mapit(a, h);
        g1_encode(out + i * 97, a, ok);
        if (!ok) atomicOr(fail, 1u);
    } else {
        Aff<Fp2> a;
        const bool ok = g2_mapit(a, h);
        g2_encode(out + i * 192, a, ok);
        if (!ok) atomicOr(fail, 1u);
    }
}

__global__ __launch_bounds__(64) void k_shake256(size_t n, const uint8_t* __restrict__ data,
                                                 const uint64_t* __restrict__ offsets, uint8_t* __restrict__ out) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t h[48];
    shake256_48(h, data + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
    for (int k = 0; k < 48; k++) out[i * 48 + k] = h[k];
}

}  // namespace

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

extern "C" {

int cck_hash_to_curve(int group, size_t n, const uint8_t* d_data, const uint64_t* d_offsets, uint8_t* d_out,
                      uint32_t* d_fail, hipStream_t st) {
    if (!n) return 0;
    if (group == 1)
        hipLaunchKernelGGL(k_hash_to_curve<1>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, d_data, d_offsets, d_out, d_fail);
    else
        hipLaunchKernelGGL(k_hash_to_curve<2>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, d_data, d_offsets, d_out, d_fail);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int cck_shake256_48(size_t n, const uint8_t* d_data, const uint64_t* d_offsets, uint8_t* d_out, hipStream_t st) {
    if (!n) return 0;
    hipLaunchKernelGGL(k_shake256, dim3(nblocks(n, 64)), dim3(64), 0, st, n, d_data, d_offsets, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
