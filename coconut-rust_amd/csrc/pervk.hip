// Signature::verify with the CALLER's verkey per credential (the product path).
//
// Reference: src/signature.rs:473-478 -> ps_sig Signature::verify [EXT]: per call,
// pr = multi_scalar_mul_var_time([X~, Y~_1..Y~_q], [1, m_1..m_q]), then the
// 2-pairing check e(sigma_1, pr) e(-sigma_2, g~) == 1 that the shared-verkey path also ends in.
// With a verkey per credential the bases are not fixed, so no window tables exist: the MSM is a
// windowed Straus (straus.h) — signed radix-16 digits, per base the multiples 1..8 batch-normalised
// with one inversion per lane, 65 windows of 4 doublings + one mixed addition per base.  No per-lane
// branch on scalar bits (the round-1 bitwise double-and-add paid a mixed addition at nearly every bit
// in SIMT, some lane of the wave always having the bit set).
//
// Both group modes run one credential per lane PAIR, the layout the Miller loop and the shared-verkey
// preps use:
//   SigG2 (verkey in G1): lane h decodes sigma_{h+1} and runs the lazy one-lane G1 Straus over the
//     bases Y~_j with j = h mod 2 (lane 0 also adds X~); the two partial sums meet by DPP; pr is written
//     affine in the R' form.
//   SigG1 (verkey in G2): lane h decodes sigma_{h+1}; the pair runs the G2 Straus on the lazy pair-lane
//     field over every Y~_j (straus_g2lz_pair) and adds X~.
// The prep writes the SoA operands of kernels.hip's k_prep_*_pair, so k_miller / k_fexp finish.
#include "codec.h"
#include "curve_lz.h"
#include "curve_pl.h"
#include "curve_wide_lz.h"
#include "fixed.h"
#include "fr.h"
#include "pairing.h"
#include "soa.h"
#include "straus.h"

using namespace cc;

// messages (48-byte big-endian, any value) -> canonical 8-word little-endian scalars (mod r), the
// Straus digits' input
__global__ __launch_bounds__(256) void k_scalars_w8(size_t nm, const uint8_t* __restrict__ msgs,
                                                    uint32_t* __restrict__ out) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= nm) return;
    Fr m;
    fr_from_be48(m, msgs + i * 48);
    uint4* o = reinterpret_cast<uint4*>(out + i * 8);
    o[0] = make_uint4(m.v[0], m.v[1], m.v[2], m.v[3]);
    o[1] = make_uint4(m.v[4], m.v[5], m.v[6], m.v[7]);
}

// SigG2, per-credential verkey (G1 bases), ONE credential per LANE (round 6; round 4-5 ran one per
// lane pair, each lane over half the bases, both lanes running the whole 260-doubling chain): one chain
// of 65 windows over all q + 1 bases, so the doublings are paid once per credential (260 x 7 products
// instead of 2 x 260 x 7 a pair) and the two halves' Jacobian sum and storage-form round trip go away.
// 65,536 credentials are 1,024 waves, one a SIMD; a verifier keeps a second batch in flight
// (cc_set_concurrency), whose kernels fill the SIMD beside it (profiles/r06/pervk_lane).
__global__ __launch_bounds__(256, 2) void k_prep_sigg2_var(size_t n, int q, const uint8_t* __restrict__ s1b,
                                                           const uint8_t* __restrict__ s2b,
                                                           const uint8_t* __restrict__ vkX,
                                                           const uint8_t* __restrict__ vkY,
                                                           const uint32_t* __restrict__ scal,
                                                           uint32_t* __restrict__ scratch,
                                                           uint32_t* __restrict__ prep, uint32_t* __restrict__ flags) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Soa S{prep, n};
    uint32_t fl = 0;
#pragma unroll 1
    for (int h = 0; h < 2; h++) {  // sigma_1 -> Q1, -sigma_2 -> Q2
        Aff<Fp2> a;
        if (!g2_decode(a, (h ? s2b : s1b) + i * 192)) fl |= h ? 2u : 1u;
        if (h) f2_neg(a.y, a.y);
        const int slot = h ? S_Q2 : S_Q1;
        st_f2(S, slot, i, a.x);
        st_f2(S, slot + 2, i, a.y);
    }
    lz::JG a;
    straus_g1lz_lane(a, 1, 0, (size_t)q, vkY + i * (size_t)q * 97, scal + i * (size_t)q * 8,
                     scratch + i * straus_g1lz_words((size_t)q));
    {  // X~ with scalar 1
        Aff<Fp> X;
        if (g1_decode(X, vkX + i * 97)) a = lz::jg_add_aff(a, ag_of(lz::reduce(lz::in_r(X.x)), lz::reduce(lz::in_r(X.y))));
    }
    if (lz::jg_is_inf(a)) {
        fl |= 4u;
    } else {  // affine in the R' form (the Miller loop's kAffRp operand)
        Fp x, y;
        lz::jg_to_aff_rp(x, y, a);
        st_fp(S, S_P1, i, x);
        st_fp(S, S_P1 + 1, i, y);
    }
    flags[i] = fl;
}

// SigG1, per-credential verkey (G2 bases on the lazy pair-lane field), one credential per lane pair
__global__ __launch_bounds__(256, 2) void k_prep_sigg1_var(size_t n, int q, const uint8_t* __restrict__ s1b,
                                                           const uint8_t* __restrict__ s2b,
                                                           const uint8_t* __restrict__ vkX,
                                                           const uint8_t* __restrict__ vkY,
                                                           const uint32_t* __restrict__ scal,
                                                           uint32_t* __restrict__ scratch,
                                                           uint32_t* __restrict__ prep, uint32_t* __restrict__ flags) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t i = g >> 1;
    const int h = (int)(g & 1);
    if (i >= n) return;  // pair-uniform
    Soa S{prep, n};
    uint32_t fl = 0;
    {
        Aff<Fp> a;
        if (!g1_decode(a, (h ? s2b : s1b) + i * 97)) fl |= h ? 2u : 1u;
        if (h) fp_neg(a.y, a.y);  // -sigma_2
        const int slot = h ? S_P2 : S_P1;
        fp_to_lazy_form(a.x);  // the Miller loop's affine P in the lazy R' form (miller_lz.hip kAffRp)
        fp_to_lazy_form(a.y);
        st_fp(S, slot, i, a.x);
        st_fp(S, slot + 1, i, a.y);
    }
    fl |= pl::swp(fl);
    lz::JL la;
    straus_g2lz_pair(la, 1, 0, h, i, (size_t)q, vkY, (size_t)q * 192, 0, 192, scal, 1, scratch);
    {  // X~ with scalar 1 (both lanes decode it)
        Aff<Fp2> X;
        if (pl::pair_all(g2_decode(X, vkX + i * 192))) {
            pl::Fp2 hx, hy;
            hx.c = h ? X.x.b : X.x.a;
            hy.c = h ? X.y.b : X.y.a;
            la = lz::jl_add_aff(la, lz::AL{lz::reduce(lz::in_r2(hx)), lz::reduce(lz::in_r2(hy))});
        }
    }
    Jac<pl::Fp2> acc = pl::jl_to_pl(la);
    Aff<pl::Fp2> a;
    if (!jac_to_aff(a, acc)) fl |= 4u;
    pl::st_f2(S, S_Q1, i, a.x);
    pl::st_f2(S, S_Q1 + 2, i, a.y);
    if (!h) flags[i] = fl;
}

// Small batches (capi.cpp kFexpWideMax): ONE WAVE per credential.  A Straus chain's 260 doublings are
// the same for one base as for q, so the wave's lanes are split into GROUPS of 4 lanes (G1) or 4 lane
// pairs (G2), group g takes the bases k = g, g + NG, ..., and each group runs its chain with the
// products of every doubling and addition spread over its members (curve_wide_lz.h): 3 product times a
// doubling, 5 an addition.  The multiples 1P..8P stay Jacobian (a spread full addition costs what a
// spread mixed one does), so no batch inversion; the groups' sums meet in a butterfly of spread
// additions.  Same outputs as the pair kernels; the scratch holds the entries (x, y, flag; Z apart)
// and the digits at the pair kernels' offsets.
namespace {
using namespace cc::lz;
constexpr int WG = wide::G;

// group grp of NG: sum of scal_k P_k over its bases (pts: t G1 encodings of 97 bytes)
DEV void straus_g1lz_wide(JG& acc, int NG, int grp, size_t t, const uint8_t* __restrict__ pts,
                          const uint32_t* __restrict__ scal, uint32_t* __restrict__ ent) {
    uint32_t* zs = ent + t * 8 * SEW;
    int8_t* dig = reinterpret_cast<int8_t*>(zs + 2 * t * 8 * LN);
    acc = jg_inf();
#pragma unroll 1
    for (size_t k = grp; k < t; k += NG) {
        cc::Aff<cc::Fp> P1;
        const bool ok = g1_decode(P1, pts + k * 97);
        recode_w4(dig + k * 65, scal + k * 8);  // every member writes the same digits
        const FR px = reduce(in_r(P1.x)), py = reduce(in_r(P1.y));
        const AG P = ag_of(px, py);
        JG J = ok ? JG{px, py, r1_one()} : jg_inf();
#pragma unroll 1
        for (int d = 0; d < 8; d++) {
            if (d == 1) J = wide::jg_dbl(J);
            else if (d > 1 && ok) J = wide::jg_add_aff(J, P);
            const size_t e = k * 8 + d;
            uint32_t* w = ent + e * SEW;
            st_r1(w, J.x);
            st_r1(w + SEY, J.y);
            w[SEF] = jg_is_inf(J) ? 1u : 0u;
            st_r1(zs + e * LN, J.z);
        }
    }
#pragma unroll 1
    for (int win = 64; win >= 0; win--) {
        if (win != 64 && !jg_is_inf(acc))
#pragma unroll 1
            for (int z = 0; z < 4; z++) acc = wide::jg_dbl(acc);
#pragma unroll 1
        for (size_t k = grp; k < t; k += NG) {
            const int d = dig[k * 65 + win];
            if (!d) continue;
            const size_t e = k * 8 + (d < 0 ? -d : d) - 1;
            const uint32_t* w = ent + e * SEW;
            if (w[SEF]) continue;  // identity multiple
            JG E;
            ld16(E.x.v, w);
            ld16(E.y.v, w + SEY);
            E.z = ld_r1(zs + e * LN);
            if (d < 0) E.y = neg(E.y);
            acc = wide::jg_add(acc, E);
        }
    }
}

// G2 bases on lane-pair groups: pair group grp of NG, lane half h (straus_g2lz_pair's arguments)
DEV void straus_g2lz_wide(JL& acc, int NG, int grp, int h, size_t task, size_t t, const uint8_t* __restrict__ pts,
                          size_t pt_stride, const uint32_t* __restrict__ l, uint32_t* __restrict__ scratch) {
    const uint8_t* base = pts + task * pt_stride;
    const uint32_t* lk = l + task * t * 8;
    uint32_t* ent = scratch + task * straus_lz_words(t);
    uint32_t* zs = ent + t * 8 * 2 * SEW;
    int8_t* dig = reinterpret_cast<int8_t*>(zs + 2 * t * 8 * 2 * LN);
    acc = jl_inf();
#pragma unroll 1
    for (size_t k = grp; k < t; k += NG) {
        cc::Aff<cc::Fp2> P1;
        const bool ok = pl::pair_all(g2_decode(P1, base + k * 192));
        recode_w4(dig + k * 65, lk + k * 8);
        pl::Fp2 hx, hy;
        hx.c = h ? P1.x.b : P1.x.a;
        hy.c = h ? P1.y.b : P1.y.a;
        const AL P{reduce(in_r2(hx)), reduce(in_r2(hy))};
        JL J = ok ? jl_from_aff(P) : jl_inf();
#pragma unroll 1
        for (int d = 0; d < 8; d++) {
            if (d == 1) J = wide::jl_dbl(J);
            else if (d > 1 && ok) J = wide::jl_add_aff(J, P);
            const size_t e = k * 8 + d;
            uint32_t* w = ent + (e * 2 + h) * SEW;
            st_w(w, J.x);
            st_w(w + SEY, J.y);
            w[SEF] = jl_is_inf(J) ? 1u : 0u;
            st_w(zs + (e * 2 + h) * LN, J.z);
        }
    }
#pragma unroll 1
    for (int win = 64; win >= 0; win--) {
        if (win != 64 && !jl_is_inf(acc))
#pragma unroll 1
            for (int z = 0; z < 4; z++) acc = wide::jl_dbl(acc);
#pragma unroll 1
        for (size_t k = grp; k < t; k += NG) {
            const int d = dig[k * 65 + win];
            if (!d) continue;
            const size_t e = k * 8 + (d < 0 ? -d : d) - 1;
            const uint32_t* w = ent + (e * 2 + h) * SEW;
            if (w[SEF]) continue;  // identity multiple (both halves carry the flag)
            JL E;
            ld16(E.x.c.v, w);
            ld16(E.y.c.v, w + SEY);
            E.z = ld_w(zs + (e * 2 + h) * LN);
            if (d < 0) E.y = neg(E.y);
            acc = wide::jl_add(acc, E);
        }
    }
}
}  // namespace

__global__ __launch_bounds__(64) void k_prep_sigg2_var_wide(size_t n, int q, const uint8_t* __restrict__ s1b,
                                                            const uint8_t* __restrict__ s2b,
                                                            const uint8_t* __restrict__ vkX,
                                                            const uint8_t* __restrict__ vkY,
                                                            const uint32_t* __restrict__ scal,
                                                            uint32_t* __restrict__ scratch,
                                                            uint32_t* __restrict__ prep, uint32_t* __restrict__ flags) {
    const size_t i = blockIdx.x;
    if (i >= n) return;  // wave-uniform
    const int l = (int)threadIdx.x, h = l & 1;
    Soa S{prep, n};
    uint32_t fl = 0;
    {
        Aff<Fp2> a;
        if (!g2_decode(a, (h ? s2b : s1b) + i * 192)) fl |= h ? 2u : 1u;
        if (h) f2_neg(a.y, a.y);  // -sigma_2
        if (l < 2) {
            st_f2(S, h ? S_Q2 : S_Q1, i, a.x);
            st_f2(S, (h ? S_Q2 : S_Q1) + 2, i, a.y);
        }
    }
    fl = (uint32_t)__shfl((int)fl, 0) | (uint32_t)__shfl((int)fl, 1);
    constexpr int NG = 64 / WG;
    const int grp = l / WG;
    JG a;
    straus_g1lz_wide(a, NG, grp, (size_t)q, vkY + i * (size_t)q * 97, scal + i * (size_t)q * 8,
                     scratch + i * straus_g1lz_words((size_t)q));
    a = wide::jg_group_sum(a);  // the groups' sums
    {  // X~ with scalar 1
        Aff<Fp> X;
        if (g1_decode(X, vkX + i * 97)) a = wide::jg_add_aff(a, ag_of(reduce(in_r(X.x)), reduce(in_r(X.y))));
    }
    if (jg_is_inf(a)) {
        fl |= 4u;
    } else {
        Fp x, y;
        wide::jg_to_aff_rp(x, y, a);  // every lane the same point: the quad-form inversion
        if (l < 2) st_fp(S, S_P1 + h, i, h ? y : x);
    }
    if (l == 0) flags[i] = fl;
}

__global__ __launch_bounds__(64) void k_prep_sigg1_var_wide(size_t n, int q, const uint8_t* __restrict__ s1b,
                                                            const uint8_t* __restrict__ s2b,
                                                            const uint8_t* __restrict__ vkX,
                                                            const uint8_t* __restrict__ vkY,
                                                            const uint32_t* __restrict__ scal,
                                                            uint32_t* __restrict__ scratch,
                                                            uint32_t* __restrict__ prep, uint32_t* __restrict__ flags) {
    const size_t i = blockIdx.x;
    if (i >= n) return;  // wave-uniform
    const int l = (int)threadIdx.x, h = l & 1, p = l >> 1;
    Soa S{prep, n};
    uint32_t fl = 0;
    {
        Aff<Fp> a;
        if (!g1_decode(a, (h ? s2b : s1b) + i * 97)) fl |= h ? 2u : 1u;
        if (h) fp_neg(a.y, a.y);  // -sigma_2
        fp_to_lazy_form(a.x);     // the Miller loop's affine P in the lazy R' form (kAffRp)
        fp_to_lazy_form(a.y);
        if (l < 2) {
            st_fp(S, h ? S_P2 : S_P1, i, a.x);
            st_fp(S, (h ? S_P2 : S_P1) + 1, i, a.y);
        }
    }
    fl = (uint32_t)__shfl((int)fl, 0) | (uint32_t)__shfl((int)fl, 1);
    constexpr int NG = 32 / WG;
    const int grp = p / WG;
    JL la;
    straus_g2lz_wide(la, NG, grp, h, i, (size_t)q, vkY, (size_t)q * 192, scal, scratch);
    la = wide::jl_group_sum(la);  // the groups' sums
    {  // X~ with scalar 1
        Aff<Fp2> X;
        if (pl::pair_all(g2_decode(X, vkX + i * 192))) {
            pl::Fp2 hx, hy;
            hx.c = h ? X.x.b : X.x.a;
            hy.c = h ? X.y.b : X.y.a;
            la = wide::jl_add_aff(la, AL{reduce(in_r2(hx)), reduce(in_r2(hy))});
        }
    }
    Jac<pl::Fp2> acc = pl::jl_to_pl(la);
    Aff<pl::Fp2> a;
    if (!wide::jac_to_aff(a, acc)) fl |= 4u;  // every pair the same point: the quad-form inversion
    if (p == 0) {
        pl::st_f2(S, S_Q1, i, a.x);
        pl::st_f2(S, S_Q1 + 2, i, a.y);
    }
    if (l == 0) flags[i] = fl;
}

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

extern "C" {

// scratch words of cck_prep_var for n credentials of q messages
size_t cck_prep_var_words(int mode, size_t n, size_t q) {
    return straus_round32(n * q * 8) + n * (mode == 0 ? straus_g1lz_words(q) : straus_lz_words(q)) + 64;
}

// Per-credential-verkey prep: vkX n x OtherGroup, vkY n x q x OtherGroup, msgs n x q x 48 B;
// scratch: cck_prep_var_words words.  Writes the Miller-loop operands and flags like cck_prep.  wide:
// one wave per credential (the small-batch form above).
int cck_prep_var(int mode, size_t n, int q, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_vkX,
                 const uint8_t* d_vkY, const uint8_t* d_msgs, uint32_t* d_scratch, uint32_t* d_prep,
                 uint32_t* d_flags, int wide, hipStream_t st) {
    if (!n) return 0;
    uint32_t* scal = d_scratch;
    uint32_t* straus = d_scratch + straus_round32(n * (size_t)q * 8);  // 128-byte-aligned task regions
    if (q) hipLaunchKernelGGL(k_scalars_w8, dim3(nblocks(n * (size_t)q, 256)), dim3(256), 0, st, n * (size_t)q, d_msgs, scal);
    if (wide && mode == 0)
        hipLaunchKernelGGL(k_prep_sigg2_var_wide, dim3((unsigned)n), dim3(64), 0, st, n, q, d_s1, d_s2, d_vkX, d_vkY,
                           scal, straus, d_prep, d_flags);
    else if (wide)
        hipLaunchKernelGGL(k_prep_sigg1_var_wide, dim3((unsigned)n), dim3(64), 0, st, n, q, d_s1, d_s2, d_vkX, d_vkY,
                           scal, straus, d_prep, d_flags);
    else if (mode == 0)
        hipLaunchKernelGGL(k_prep_sigg2_var, dim3(nblocks(n, 256)), dim3(256), 0, st, n, q, d_s1, d_s2, d_vkX,
                           d_vkY, scal, straus, d_prep, d_flags);
    else
        hipLaunchKernelGGL(k_prep_sigg1_var, dim3(nblocks(2 * n, 256)), dim3(256), 0, st, n, q, d_s1, d_s2, d_vkX,
                           d_vkY, scal, straus, d_prep, d_flags);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"
