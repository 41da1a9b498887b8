// Final-exponentiation kernel for gfx950 on the lazy field, ONE credential per QUAD of lanes (tower_q.h)
// — AMCL `pair::fexp` via amcl_wrapper `GT::ate_2_pairing` (reference src/lib.rs:13; SURVEY.md §8a
// V6/V7).  Same chain as fexp_pl.hip: easy part f^((p^6 - 1)(p^2 + 1)), hard part
// 3 + (x-1)^2 [p^3 + x p^2 + (x^2-1) p + x^3 - x] = 3 Phi_12(p) / r, each pow-by-x as 57 compressed
// cyclotomic squarings, one batched decompression (snapshots g^(2^16), g^(2^48), g^(2^57), one Fp2
// inversion) and 6 Granger-Scott squarings.
//
// The quad layout holds an Fp12 in 42 words a lane, so the whole chain stays in registers: no
// scratch round trips between steps (the pair layout's chain rested every Fp12 in an 84-slot HBM
// scratch and reloaded it for the next step).
#include "codec.h"
#include "tower_q.h"

namespace cc {
namespace lz {
// Build option CC_FEXP_PROF (tools/fexp_phases.py): per-wave shader-clock totals of the kernel's phases,
// written by lane 0 of each wave with plain vector stores to g_fq_prof[wave][slot].
#ifdef CC_FEXP_PROF
constexpr int kProfSlots = 8, kProfWaves = 8192;
__device__ unsigned long long g_fq_prof[kProfWaves][kProfSlots];
__device__ unsigned long long* fq_prof_acc() {
    static __shared__ unsigned long long acc[4][kProfSlots];  // per wave of the block
    return acc[threadIdx.x >> 6];
}
#define FXP_T(v) const unsigned long long v = clock64()
#define FXP_ADD(slot, t0)                                                          \
    do {                                                                           \
        const unsigned long long t1_ = clock64();                                  \
        if ((threadIdx.x & 63) == 0) fq_prof_acc()[slot] += t1_ - (t0);            \
    } while (0)
#else
#define FXP_T(v)
#define FXP_ADD(slot, t0)
#endif
namespace {

// ---------------------------------------------------------------- compressed cyclotomic squaring
// fexp_pl.hip cyc4_sqr (Karabina's compression restated for this tower) on b = b0 + b1 s, c = c0 + c1 s:
//     b0' = 3 (2 xi c0 c1) + 2 b0    b1' = 3 (c0^2 + xi c1^2) - 2 b1
//     c0' = 3 (b0^2 + xi b1^2) - 2 c0    c1' = 3 (2 b0 b1) + 2 c1
// Pair 0 holds V = c0, W = b0; pair 1 V = b1, W = c1.  Each lane squares S1 = V, S2 = W and S3 = W + V'
// (V' the other pair's V: b0 + b1 on pair 0, c1 + c0 on pair 1); with primes for the other pair's values
//     X = S3' - S2' - S1 = (S3 - S2)' - S1   (2 c0 c1 | 2 b0 b1; times xi on pair 0)
//     T = S1' + S2 + i B,  B = S1' (pair 0) | S2 (pair 1)   (b0^2 + xi b1^2 | c0^2 + xi c1^2)
//     V <- 3 T - 2 V,  W <- 3 X + 2 W
// — 3 Fp2 squarings a lane, three exchanges between the pairs, one select; the pair-0-only xi and the
// i B term run on their lanes under exec masks.
using F2R = F2<AN, 9>;
struct QZ {
    F2R V, W;
};
DEV QZ qz_from(const F2R& b, const F2R& c) {
    const bool j = qhi();
    return {qsel(j, b, c), qsel(j, c, b)};
}
DEV F2R qz_b(const QZ& x) { return qsel(qhi(), x.V, x.W); }
DEV F2R qz_c(const QZ& x) { return qsel(qhi(), x.W, x.V); }
DEV void qz_sqr(QZ& x) {
    const bool j = qhi();
    const auto S1 = sqrr_in(x.V);
    const auto S2 = sqrr_in(x.W);
    const auto S3 = sqrr_in(add(x.W, qx(x.V)));  // (b0 + b1)^2 | (c1 + c0)^2
    const auto pE = qx(sub(S3, S2));
    const auto pS1 = qx(S1);
    const auto Xs = norm(xi_pair0(sub(pE, S1)));          // xi 2 c0 c1 | 2 b0 b1
    const auto T = norm(add_i(add(pS1, S2), qsel(j, S2, pS1)));
    // 3T - 2V = T + 2 (T - V), 3X + 2W = X + 2 (X + W)
    x.V = reduce(add(T, dbl(sub(T, x.V))));
    x.W = reduce(add(Xs, dbl(add(Xs, x.W))));
}
// numerator of this lane's a_j and the common denominator D (fexp_pl.hip cyc4_num):
//     a0 = (b0 Nb + xi c1 Nc) / D,  a1 = (c0 Nc + b1 Nb) / D,
//     Nb = b0^2 - xi b1^2,  Nc = c0^2 - xi c1^2,  D = 2 (b0 c0 - xi b1 c1)
DEV void qz_num(F2R& nj, F2R& den, const QZ& z) {
    const bool j = qhi();
    const F2R B = qz_b(z), C = qz_c(z);
    const auto sB = sqrr(B), sC = sqrr(C);
    const auto pSB = qx(sB), pSC = qx(sC);
    const auto Nb = norm(qsel(j, sub(pSB, xi(sB)), sub(sB, xi(pSB))));  // the same on both pairs
    const auto Nc = norm(qsel(j, sub(pSC, xi(sC)), sub(sC, xi(pSC))));
    const auto P1 = mulr(B, Nb), P2 = mulr(C, Nc), P3 = mulr(B, C);
    const auto pP2 = qx(P2), pP3 = qx(P3);
    nj = reduce(qsel(j, add(pP2, P1), add(P1, xi(pP2))));
    den = reduce(dbl(qsel(j, sub(pP3, xi(P3)), sub(P3, xi(pP3)))));
}
template <class I>
DEV QR qz_expand(const QZ& x, const F2R& nj, const I& inv) {
    return {reduce(mulr(nj, inv)), qz_b(x), qz_c(x)};
}

// src^x by Granger-Scott square-and-multiply: the fallback of q_pow_x for a zero decompression
// denominator (never reached by honest inputs)
static __device__ __noinline__ QR q_pow_x_gs(QR src) {
    QR acc = src;
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        acc = rest(q12_cyc_sqr(acc));
        if ((X_ABS >> b) & 1ull) acc = rest(q12_mul(acc, src));
    }
    return q12_conj(acc);
}

// src^x, x = -|x| (bits 63, 62, 60, 57, 48, 16 of |x|)
DEV QR q_pow_x(const QR& src) {
    FXP_T(t_sq);
    QZ c = qz_from(src.b, src.c);
#pragma unroll 1
    for (int k = 0; k < 16; k++) qz_sqr(c);
    const QZ s16 = c;
#pragma unroll 1
    for (int k = 16; k < 48; k++) qz_sqr(c);
    const QZ s48 = c;
#pragma unroll 1
    for (int k = 48; k < 57; k++) qz_sqr(c);
    FXP_ADD(2, t_sq);
    FXP_T(t_dc);
    F2R n16, d16, n48, d48, n57, d57;
    qz_num(n16, d16, s16);
    qz_num(n48, d48, s48);
    qz_num(n57, d57, c);
    const auto p1 = mulr(d16, d48);
    const auto p2 = mulr(p1, d57);
    if (is_zero(p2)) return q_pow_x_gs(src);  // quad-uniform (D is the same on both pairs)
    const auto iv = qinv(p2);
    QR y = qz_expand(c, n57, mulr(iv, p1));    // g^(2^57)
    const auto iv2 = mulr(iv, d57);           // (d16 d48)^-1
    QR acc = rest(q12_mul(qz_expand(s16, n16, mulr(iv2, d48)), qz_expand(s48, n48, mulr(iv2, d16))));
    acc = rest(q12_mul(acc, y));
    FXP_ADD(3, t_dc);
    FXP_T(t_tl);
    // then y^2 three times, acc *= y (2^60), y^2 twice, acc *= y (2^62), y^2, acc *= y (2^63)
    constexpr uint32_t kSq = 0b010110111u;  // from bit 0: S S S M S S M S M  (1 = square)
#pragma unroll 1
    for (int st = 0; st < 9; st++) {
        if ((kSq >> st) & 1u) y = rest(q12_cyc_sqr(y));
        else acc = rest(q12_mul(acc, y));
    }
    FXP_ADD(4, t_tl);
    return q12_conj(acc);
}

// verdict and GT bytes of the result, through the storage form (12 x 32, R = 2^406)
DEV void qexp_out(size_t i, const QR& res, const uint32_t* flags, uint8_t* verdicts, uint8_t* gt_out) {
    const bool j = qhi();
    const int h = (int)half_id();
    const pl::Fp2 oa = out_r2(res.a), ob = out_r2(res.b), oc = out_r2(res.c);
    Fp one;
    fp_one(one);
    // one = (1, 0, 0, 0, 0, 0): only the real half of a's component 0 is non-zero
    bool own = (!j && !h ? fp_eq(oa.c, one) : fp_is_zero(oa.c)) && fp_is_zero(ob.c) && fp_is_zero(oc.c);
    const uint32_t fl = flags ? flags[i] : 0u;
    const bool ok = quad_all(own) && (fl & 11u) == 0;  // sigma_1/sigma_2 = O or PoK Schnorr failure
    if ((__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 3u) == 0) verdicts[i] = ok ? 1 : 0;
    if (gt_out) {  // Fp2 k of the AMCL FP12 order at 96 k, half h at + 48 h; component j of a, b, c is k = j, 2 + j, 4 + j
        uint8_t* o = gt_out + i * 576 + 48 * h + 96 * (int)j;
        Fp c;
        fp_from_mont(c, oa.c);
        store_be48_aligned(o, c);
        fp_from_mont(c, ob.c);
        store_be48_aligned(o + 192, c);
        fp_from_mont(c, oc.c);
        store_be48_aligned(o + 384, c);
    }
}

}  // namespace

// fbuf: Miller output f (12 x 32 SoA, 12 slots, R form); one credential per lane quad
__global__ __launch_bounds__(256, 2) void k_fexp_q(size_t n, const uint32_t* __restrict__ fbuf,
                                                const uint32_t* __restrict__ flags, uint8_t* __restrict__ verdicts,
                                                uint8_t* __restrict__ gt_out) {
    const size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 2;  // credential of this lane quad
    if (i >= n) return;                                                     // quad-uniform
#ifdef CC_FEXP_PROF
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < kProfSlots; k++) fq_prof_acc()[k] = 0;
#endif
    FXP_T(t_in);
    const int j = qhi() ? 1 : 0;
    const Soa S{const_cast<uint32_t*>(fbuf), n};
    const auto ld = [&](int k) {
        pl::Fp2 v;
        pl::ld_f2(v, S, 2 * k, i);
        return reduce(in_r2(v));
    };
    QR f{ld(j), ld(2 + j), ld(4 + j)};  // Fp2 k = a.a, a.b, b.a, b.b, c.a, c.b
    FXP_ADD(0, t_in);
    FXP_T(t_easy);
    // easy part: f^(p^6 - 1) = conj(f) f^-1, then ^(p^2 + 1)
#ifdef CC_FEXP_PROF
    FXP_T(t_qi);
    const QR fi = rest(q12_inv(f));
    FXP_ADD(7, t_qi);
    f = rest(q12_mul(q12_conj(f), fi));
#else
    f = rest(q12_mul(q12_conj(f), rest(q12_inv(f))));
#endif
    f = rest(q12_mul(rest(q12_frob2(f)), f));
    QR r = rest(q12_mul(rest(q12_cyc_sqr(f)), f));  // res = f^3
    FXP_ADD(1, t_easy);
    // hard part: five pow-by-x, each followed by its share of the chain (fexp_pl.hip fexp_chain)
    //   0: t = f^x, t *= conj(f)                       (f^(x-1))
    //   1: a = t^x, a *= conj(t), res *= (a^(p^2) conj(a))^p
    //   2: b = a^x, res *= b^(p^2) conj(b)
    //   3: c = b^x, res *= c^p
    //   4: d = c^x, res *= d
    QR cur = f;
#pragma unroll 1
    for (int it = 0; it < 5; it++) {
        QR y = q_pow_x(cur);
        FXP_T(t_ch);
        if (it <= 1) y = rest(q12_mul(y, q12_conj(cur)));
        QR z = y;
        if (it == 1 || it == 2) z = rest(q12_mul(rest(q12_frob2(y)), q12_conj(y)));
        if (it == 1 || it == 3) z = rest(q12_frob(z));
        if (it >= 1) r = rest(q12_mul(z, r));
        cur = y;
        FXP_ADD(5, t_ch);
    }
    FXP_T(t_out);
    qexp_out(i, r, flags, verdicts, gt_out);
    FXP_ADD(6, t_out);
#ifdef CC_FEXP_PROF
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0 && wave < (size_t)kProfWaves)
        for (int k = 0; k < kProfSlots; k++) g_fq_prof[wave][k] = fq_prof_acc()[k];
#endif
}

}  // namespace lz
}  // namespace cc

#ifdef CC_FEXP_PROF
extern "C" int cck_fexp_prof_read(unsigned long long* out, size_t nwaves) {
    if (nwaves > (size_t)cc::lz::kProfWaves) nwaves = cc::lz::kProfWaves;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(cc::lz::g_fq_prof), nwaves * cc::lz::kProfSlots * 8, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int cck_fexp_q(size_t n, const uint32_t* d_f, const uint32_t* d_flags, uint8_t* d_verdicts, uint8_t* d_gt,
                          hipStream_t st) {
    if (!n) return 0;
    hipLaunchKernelGGL(cc::lz::k_fexp_q, dim3((unsigned)((4 * n + 255) / 256)), dim3(256), 0, st, n, d_f, d_flags,
                       d_verdicts, d_gt);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
