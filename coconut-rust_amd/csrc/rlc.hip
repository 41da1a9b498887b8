// Random-linear-combination (RLC) batch verification for gfx950 (BASELINE config 3).
//
// Per credential i the reference checks e(sigma_1,i, pr_i) * e(-sigma_2,i, g~) == 1 (ps_sig
// Signature::verify [EXT], reference src/signature.rs:473-478).  RLC checks the whole batch at once:
//
//     prod_i e(sigma_1,i, delta_i pr_i) * e(-sigma_2,i, delta_i g~) == 1        (SigG2)
//     prod_i e(delta_i pr_i, sigma_1,i) * e(g~, -delta_i sigma_2,i) == 1        (SigG1)
//
// with independent delta_i (ChaCha20 keyed by a fresh host seed, 16 signed base-256 digits: fr.h
// rlc_delta_signed): the second pairs share g~ and are folded into 16 window pairs (fold.hip), so
// each credential keeps ONE pair (two credentials per shared-squaring Miller loop); then the product
// of all Miller values and ONE final exponentiation per batch (or, over several GPUs, one per
// gathered set of per-GPU partial products).  A forged credential passes with probability <= 2^-127.
// If the batch fails, or any sigma is the identity (which the per-credential semantics reject), the
// caller falls back to per-credential verification, so verdicts always equal the reference's.
//
//   k_rlc_check_* / k_rlc_msm_*        : decode, subgroup checks and the fold's inputs (-sigma_2,
//                                         delta's digits); the delta-scaled fixed-base MSM
//                                         (delta X + sum (delta m_j) Y_j) of pair 0 in the Miller
//                                         kernels' SoA layout (soa.h; G1 points affine in the R' form)
//   k_f12_reduce                        : one level of the pairwise product tree of Fp12 values (the
//                                         short levels: fexp_pl.hip k_f12_reduce_wide)
//   k_rlc_partial_out                   : the partial's product and flag words (rlc_part.h; the fold
//                                         writes its window section)
//   k_rlc_gather                        : the finish's inputs from the gathered partials: their products
//                                         and every shard's window pairs (S_w, P_w) for k_miller_wide
#include "codec.h"
#include "curve_pl.h"
#include "fixed.h"
#include "fr.h"
#include "pairing.h"
#include "rlc_part.h"
#include "soa.h"
#include "subgroup.h"

using namespace cc;

namespace {

// The RLC keeps one pair per credential and runs two credentials per Miller loop (miller_lz.hip
// kTwin): credential i's pair goes to SoA element i / 2 of the verify layout's pair-0 slots (even i)
// or pair-1 slots (odd i), so the loop loads both pairs exactly as a verify loop does (coalesced).
DEV int twin_slot(int s0, int s1, size_t i) { return (i & 1) ? s1 : s0; }

}  // namespace

// Tables: bases [Y~_0 .. Y~_{q-1}, g~, X~] (indices 0..q-1, q, q+1) of cc_set_verkey.
// flags: bit0 sigma_1 = O, bit1 sigma_2 = O, bit2 delta pr = O, bit5 sigma outside the subgroup.
// Per credential: its Miller pair (sigma_1 with delta pr, SoA slots of soa.h, twin_slot), the fold
// point X_i = -sigma_2,i (AoS affine, pts) and delta's 16 signed digits (dig[w * n + i]; all zero when
// sigma_2 is the identity, which fails the batch anyway).  delta X~ runs as +-|delta| X~ over the
// magnitude's windows (fr.h rlc_delta_abs); the products delta m_j use delta mod r.

template <class F>
DEV void st_aff_aos(uint32_t* p, const Aff<F>& a) {
    uint4* o = reinterpret_cast<uint4*>(p);
    const uint4* w = reinterpret_cast<const uint4*>(&a);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(Aff<F>) / 16); k++) o[k] = w[k];
}

// Two kernels per group mode (split so each keeps its registers within 2 waves/SIMD):
//   k_rlc_check_* : decode sigma_1 / sigma_2, subgroup checks, the fold's inputs (-sigma_2 and
//                   delta's digits), flags bits 0, 1, 5 and the batch's fall-back flag
//   k_rlc_msm_*   : delta X~ + sum (delta m_j) Y~_j (delta recomputed from the key stream) as pair 0's
//                   other argument, flag bit 2
// one credential per lane PAIR: lane h decodes sigma_{h+1} and writes its outputs (h = 0: sigma_1 as
// pair 0's Q; h = 1: the fold point -sigma_2); sigma_2's subgroup test runs on the pair-lane Fp2
// (curve_pl.h: 3 Fp a lane for a Jacobian G2 point) — sigma_1's comes free from the Miller loop's T;
// each lane writes 8 of delta's 16 digits.
__global__ __launch_bounds__(256, 2) void k_rlc_check_sigg2(size_t n, size_t ps, uint64_t base_index,
                                                            const uint32_t* __restrict__ key,
                                                            const uint8_t* __restrict__ s1b,
                                                            const uint8_t* __restrict__ s2b,
                                                            uint32_t* __restrict__ prep, uint32_t* __restrict__ flags,
                                                            uint32_t* __restrict__ any, uint32_t* __restrict__ pts,
                                                            int8_t* __restrict__ dig) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t i = g >> 1;
    const int h = (int)(g & 1);
    if (i >= n) return;  // pair-uniform
    const Soa S{prep, ps};
    uint32_t fl = 0;
    Aff<Fp2> a;
    if (!g2_decode(a, (h ? s2b : s1b) + i * 192)) fl |= h ? 2u : 1u;
    if (!h) {  // pair 0's Q in the twin layout (twin_slot)
        st_f2(S, twin_slot(S_Q1, S_Q2, i), i >> 1, a.x);
        st_f2(S, twin_slot(S_Q1, S_Q2, i) + 2, i >> 1, a.y);
    } else {
        Aff<Fp2> m = a;  // the fold point, in the lazy field's form (fold.hip sums it there)
        f2_neg(m.y, m.y);
        fp_to_lazy_form(m.x.a);
        fp_to_lazy_form(m.x.b);
        fp_to_lazy_form(m.y.a);
        fp_to_lazy_form(m.y.b);
        st_aff_aos<Fp2>(pts + i * (sizeof(Aff<Fp2>) / 4), m);
    }
    fl |= pl::swp(fl);  // both decode flags on both lanes
    // sigma_1's subgroup test runs in the Miller kernel, from its own T (miller_t_in_subgroup)
    Aff<pl::Fp2> p;
    p.x = pl::f2_from_lane(a.x, 1);
    p.y = pl::f2_from_lane(a.y, 1);
    if (!(fl & 2u) && !pl::g2_in_subgroup_lz(p)) fl |= 32u;
    uint32_t kk[NR], d[NR], w4[4];
    for (int k = 0; k < 8; k++) kk[k] = key[k];
    rlc_delta_signed(d, w4, kk, base_index + i);
    const bool on = (fl & 2u) == 0;
#pragma unroll
    for (int w = 8 * h; w < 8 * h + 8; w++)
        dig[(size_t)w * n + i] = on ? (int8_t)((w4[w >> 2] >> (8 * (w & 3))) & 0xffu) : 0;
    if (!h) {
        flags[i] = fl;
        if (fl & 35u) atomicOr(any, 1u);  // identity or non-subgroup sigma: the batch falls back
    }
}

__global__ __launch_bounds__(256, 2) void k_rlc_msm_sigg2(size_t n, size_t ps, int q, uint64_t base_index,
                                                          const uint32_t* __restrict__ key,
                                                          const uint8_t* __restrict__ msgs,
                                                          const uint32_t* __restrict__ table, int wbits,
                                                          const uint32_t* __restrict__ binf,
                                                          uint32_t* __restrict__ prep, uint32_t* __restrict__ flags) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Soa S{prep, ps};
    uint32_t kk[NR], d[NR], w4[4];
    for (int k = 0; k < 8; k++) kk[k] = key[k];
    rlc_delta_signed(d, w4, kk, base_index + i);
    lz::JG a = lz::jg_inf();  // the sum on the lazy field (fixed.h ft_add_lz)
    const int nwin = ft_nwin(wbits);
    if (!binf[q + 1]) {  // delta X~ as +-|delta| X~ (fr.h rlc_delta_abs)
        uint32_t da[NR];
        const bool neg = rlc_delta_abs(da, d);
        ft_add_lz(a, da, table, wbits, q + 1, 0, nwin, neg);
    }
    for (int j = 0; j < q; j++) {
        if (binf[j]) continue;
        Fr m;
        fr_from_be48(m, msgs + (i * (size_t)q + j) * 48);
        uint32_t dm[NR];
        fr_mul_canon(dm, d, m.v);
        ft_add_lz(a, dm, table, wbits, j, 0, nwin);
    }
    if (lz::jg_is_inf(a)) {
        flags[i] |= 4u;
    } else {  // affine in the R' form (the Miller loop's kAffRp operand)
        Fp x, y;
        lz::jg_to_aff_rp(x, y, a);
        st_fp(S, twin_slot(S_P1, S_P2, i), i >> 1, x);
        st_fp(S, twin_slot(S_P1, S_P2, i) + 1, i >> 1, y);
    }
}

// one credential per lane pair: lane h decodes and subgroup-checks sigma_{h+1} (one-lane G1)
__global__ __launch_bounds__(256, 2) void k_rlc_check_sigg1(size_t n, size_t ps, uint64_t base_index,
                                                            const uint32_t* __restrict__ key,
                                                            const uint8_t* __restrict__ s1b,
                                                            const uint8_t* __restrict__ s2b,
                                                            uint32_t* __restrict__ prep, uint32_t* __restrict__ flags,
                                                            uint32_t* __restrict__ any, uint32_t* __restrict__ pts,
                                                            int8_t* __restrict__ dig) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t i = g >> 1;
    const int h = (int)(g & 1);
    if (i >= n) return;  // pair-uniform
    const Soa S{prep, ps};
    uint32_t fl = 0;
    Aff<Fp> a;
    if (!g1_decode(a, (h ? s2b : s1b) + i * 97)) fl |= h ? 2u : 1u;
    else if (!g1_in_subgroup(a)) fl |= 32u;
    if (!h) {  // sigma_1 as the P side, affine in the R' form (the Miller loop's kAffRp operand)
        fp_to_lazy_form(a.x);
        fp_to_lazy_form(a.y);
        st_fp(S, twin_slot(S_P1, S_P2, i), i >> 1, a.x);
        st_fp(S, twin_slot(S_P1, S_P2, i) + 1, i >> 1, a.y);
    } else {
        fp_neg(a.y, a.y);
        fp_to_lazy_form(a.x);  // the fold point, in the lazy field's form (fold.hip sums it there)
        fp_to_lazy_form(a.y);
        st_aff_aos<Fp>(pts + i * (sizeof(Aff<Fp>) / 4), a);
    }
    fl |= pl::swp(fl);
    uint32_t kk[NR], d[NR], w4[4];
    for (int k = 0; k < 8; k++) kk[k] = key[k];
    rlc_delta_signed(d, w4, kk, base_index + i);
    const bool on = (fl & 2u) == 0;
#pragma unroll
    for (int w = 8 * h; w < 8 * h + 8; w++)
        dig[(size_t)w * n + i] = on ? (int8_t)((w4[w >> 2] >> (8 * (w & 3))) & 0xffu) : 0;
    if (!h) {
        flags[i] = fl;
        if (fl & 35u) atomicOr(any, 1u);  // identity or non-subgroup sigma: the batch falls back
    }
}

// one credential per lane PAIR: the G2 MSM on the pair-lane Fp2 (curve_pl.h ft_add_g2)
__global__ __launch_bounds__(256, 2) void k_rlc_msm_sigg1(size_t n, size_t ps, int q, uint64_t base_index,
                                                          const uint32_t* __restrict__ key,
                                                          const uint8_t* __restrict__ msgs,
                                                          const uint32_t* __restrict__ table, int wbits,
                                                          const uint32_t* __restrict__ binf,
                                                          uint32_t* __restrict__ prep, uint32_t* __restrict__ flags) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t i = g >> 1;
    if (i >= n) return;  // pair-uniform
    const Soa S{prep, ps};
    uint32_t kk[NR], d[NR], w4[4];
    for (int k = 0; k < 8; k++) kk[k] = key[k];
    rlc_delta_signed(d, w4, kk, base_index + i);
    lz::JL la = lz::jl_inf();  // the sum on the lazy pair-lane field (curve_pl.h ft_add_g2_lz)
    const int nwin = ft_nwin(wbits);
    if (!binf[q + 1]) {  // delta X~ as +-|delta| X~ (fr.h rlc_delta_abs)
        uint32_t da[NR];
        const bool neg = rlc_delta_abs(da, d);
        pl::ft_add_g2_lz(la, da, table, wbits, q + 1, 0, nwin, neg);
    }
    for (int j = 0; j < q; j++) {
        if (binf[j]) continue;
        Fr m;
        fr_from_be48(m, msgs + (i * (size_t)q + j) * 48);
        uint32_t dm[NR];
        fr_mul_canon(dm, d, m.v);
        pl::ft_add_g2_lz(la, dm, table, wbits, j, 0, nwin);
    }
    const Jac<pl::Fp2> acc = pl::jl_to_pl(la);
    Aff<pl::Fp2> a2;
    const bool fin = jac_to_aff(a2, acc);
    pl::st_f2(S, twin_slot(S_Q1, S_Q2, i), i >> 1, a2.x);
    pl::st_f2(S, twin_slot(S_Q1, S_Q2, i) + 2, i >> 1, a2.y);
    if (!fin && !pl::half_id()) flags[i] |= 4u;
}

// out[t] = in[2t] * in[2t+1] (in[2t] alone for an odd tail); SoA strides n_in / n_out.  One product
// per lane PAIR (tower_pl.h): the tree's short levels are latency-bound, and the pair-lane Fp12
// product has half the dependent multiplications of the one-lane one.
__global__ __launch_bounds__(256) void k_f12_reduce(size_t n_in, const uint32_t* __restrict__ in,
                                                    uint32_t* __restrict__ out) {
    const size_t t = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 1;
    const size_t n_out = (n_in + 1) / 2;
    if (t >= n_out) return;  // pair-uniform
    const Soa I{const_cast<uint32_t*>(in), n_in}, O{out, n_out};
    pl::Fp12 a;
    pl::ld_f12(a, I, 2 * t);
    if (2 * t + 1 < n_in) {
        pl::Fp12 b;
        pl::ld_f12(b, I, 2 * t + 1);
        pl::f12_mul(a, a, b);
    }
    pl::st_f12(O, t, a);
}

// the partial's product and flag words: the batch's Miller product (one element, Montgomery words in
// slot order) and the fall-back flag (any sigma = O or outside the subgroup, or a bad verkey)
__global__ void k_rlc_partial_out(const uint32_t* __restrict__ f1, const uint32_t* __restrict__ any,
                                  uint32_t* __restrict__ partial) {
    const int t = threadIdx.x;
    if (t < RLC_F12_WORDS) partial[t] = f1[t];
    if (t == RLC_FLAG) partial[t] = *any ? 1u : 0u;
}

// The finish's inputs from k gathered partials (stride RLC_PART_WORDS), one block per partial r:
//   fw element r (SoA stride fs)         : partial r's Miller product
//   window pair e = 16 r + w (prep SoA of stride 16 k, soa.h slots; k_miller_wide's operands): S_w of
//                                          partial r with P_w = (256^w) g~ (pw: SoA stride 16, finf: its
//                                          identity flags); flags2[e] bit 0 skips it (S_w = O or P_w = O)
//   flag (block 0)                       : OR of the partials' fall-back flags
// SigG2: S_w in G2 is the Q side, P_w (G1, evaluation form (x, y, 1)) the P side; SigG1 the reverse.
template <int MODE>
__global__ __launch_bounds__(256) void k_rlc_gather(size_t k, const uint32_t* __restrict__ parts,
                                                    const uint32_t* __restrict__ pw, const uint8_t* __restrict__ finf,
                                                    uint32_t* __restrict__ fw, size_t fs, uint32_t* __restrict__ prep,
                                                    uint32_t* __restrict__ flags2, uint32_t* __restrict__ flag) {
    const size_t r = blockIdx.x;
    const int t = threadIdx.x;
    const uint32_t* P = parts + r * RLC_PART_WORDS;
    if (t < RLC_F12_WORDS) fw[(size_t)t * fs + r] = P[t];
    if (t >= RLC_F12_WORDS && t < RLC_F12_WORDS + RLC_WINDOWS) {
        const int w = t - RLC_F12_WORDS;
        const size_t e = RLC_WINDOWS * r + w;
        const uint32_t* win = P + RLC_WIN_OFF + RLC_WIN_WORDS * w;
        const Soa S{prep, RLC_WINDOWS * k}, W{const_cast<uint32_t*>(pw), (size_t)RLC_WINDOWS};
        Fp v[4];
        for (int j = 0; j < 4; j++)
            for (int l = 0; l < NL; l++) v[j].v[l] = win[NL * j + l];
        if (MODE == 0) {  // S_w: affine G2 as Q; P_w: G1 in evaluation form as P
            for (int j = 0; j < 4; j++) st_fp(S, S_Q1 + j, e, v[j]);
            for (int j = 0; j < 3; j++) {
                Fp x;
                ld_fp(x, W, S_P1 + j, w);
                st_fp(S, S_P1 + j, e, x);
            }
        } else {  // S_w: G1 (x, y, 1) as P; P_w: affine G2 as Q
            Fp one;
            fp_one(one);
            st_fp(S, S_P1, e, v[0]);
            st_fp(S, S_P1 + 1, e, v[1]);
            st_fp(S, S_P1 + 2, e, one);
            for (int j = 0; j < 4; j++) {
                Fp x;
                ld_fp(x, W, S_Q1 + j, w);
                st_fp(S, S_Q1 + j, e, x);
            }
        }
        flags2[e] = (win[4 * NL] || finf[w]) ? 1u : 0u;
    }
    if (r == 0 && t == 255) {
        uint32_t fl = 0;
        for (size_t p = 0; p < k; p++) fl |= parts[p * RLC_PART_WORDS + RLC_FLAG];
        *flag = fl ? 1u : 0u;
    }
}

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

extern "C" int cck_f12_reduce_wide(size_t n, const uint32_t* d_in, uint32_t* d_out, hipStream_t st);

// levels with at most this many products run in the wide form (one wave a product): the packed form
// holds ~47 us a level (one product's latency on one lane pair) up to 16,384 products, the wide form
// ~17 us up to 256 products, 24 / 35 / 48 us at 512 / 1,024 / 2,048 (profiles/r04/rlc_wide_tree)
constexpr size_t kWideLevel = 1024;

extern "C" {

// d_pts: n fold points (AoS affine: 48 words SigG2, 24 SigG1); d_dig: 16 x n digit bytes; ps: the prep
// SoA's stride (>= (n + 1) / 2: credentials 2t and 2t + 1 share Miller loop t, twin_slot).
// part 0: decode + subgroup checks + the fold's inputs; part 1: the delta-scaled MSM
int cck_prep_rlc(int mode, int part, size_t n, size_t ps, int q, uint64_t base_index, const uint32_t* d_key,
                 const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_msgs, const uint32_t* d_table, int wbits,
                 const uint32_t* d_binf, uint32_t* d_prep, uint32_t* d_flags, uint32_t* d_any, uint32_t* d_pts,
                 int8_t* d_dig, hipStream_t st) {
    if (!n) return 0;
    const dim3 g2(nblocks(2 * n, 256)), g1(nblocks(n, 256)), b(256);
    if (part == 0) {
        if (mode == 0)
            hipLaunchKernelGGL(k_rlc_check_sigg2, g2, b, 0, st, n, ps, base_index, d_key, d_s1, d_s2, d_prep, d_flags,
                               d_any, d_pts, d_dig);
        else
            hipLaunchKernelGGL(k_rlc_check_sigg1, g2, b, 0, st, n, ps, base_index, d_key, d_s1, d_s2, d_prep, d_flags,
                               d_any, d_pts, d_dig);
    } else {
        if (mode == 0)
            hipLaunchKernelGGL(k_rlc_msm_sigg2, g1, b, 0, st, n, ps, q, base_index, d_key, d_msgs, d_table, wbits, d_binf,
                               d_prep, d_flags);
        else
            hipLaunchKernelGGL(k_rlc_msm_sigg1, g2, b, 0, st, n, ps, q, base_index, d_key, d_msgs, d_table, wbits, d_binf,
                               d_prep, d_flags);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// reduce n SoA Fp12 values in `a` to one, ping-ponging with `b` (`a` n, `b` (n + 1) / 2 elements of
// 144 words); writes the partial's product and flag words (rlc_part.h)
int cck_rlc_reduce(size_t n, uint32_t* d_a, uint32_t* d_b, const uint32_t* d_any, uint32_t* d_partial,
                   hipStream_t st) {
    if (!n) return -1;
    uint32_t *src = d_a, *dst = d_b;
    while (n > 1) {
        const size_t n_out = (n + 1) / 2;
        if (n_out <= kWideLevel) {
            if (cck_f12_reduce_wide(n, src, dst, st)) return -1;
        } else {
            hipLaunchKernelGGL(k_f12_reduce, dim3(nblocks(2 * n_out, 256)), dim3(256), 0, st, n, src, dst);
        }
        n = n_out;
        uint32_t* t = src;
        src = dst;
        dst = t;
    }
    hipLaunchKernelGGL(k_rlc_partial_out, dim3(1), dim3(192), 0, st, src, d_any, d_partial);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int cck_rlc_partial_words() { return RLC_PART_WORDS; }

// the finish's inputs (k_rlc_gather): d_fw >= 17 k Fp12 elements of stride fs (partial products at
// 0 .. k-1; k_miller_wide's window values go to k .. 17 k - 1), d_prep a 16 k-element prep SoA,
// d_flags2 16 k words, d_flag one word
int cck_rlc_gather(int mode, size_t k, const uint32_t* d_parts, const uint32_t* d_pw, const uint8_t* d_finf,
                   uint32_t* d_fw, size_t fs, uint32_t* d_prep, uint32_t* d_flags2, uint32_t* d_flag, hipStream_t st) {
    if (!k || fs < (RLC_WINDOWS + 1) * k) return -1;
    if (mode == 0)
        hipLaunchKernelGGL(k_rlc_gather<0>, dim3((unsigned)k), dim3(256), 0, st, k, d_parts, d_pw, d_finf, d_fw, fs,
                           d_prep, d_flags2, d_flag);
    else
        hipLaunchKernelGGL(k_rlc_gather<1>, dim3((unsigned)k), dim3(256), 0, st, k, d_parts, d_pw, d_finf, d_fw, fs,
                           d_prep, d_flags2, d_flag);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
