// Batch verification kernels for gfx950 (the product path).
//
// Hot path: Signature::verify = decode -> verkey MSM
// pr = X~ + sum_j Y~_j m_j -> 2-pair Miller loop -> final exponentiation -> is_one.
// Reference entry: src/signature.rs:473-478 (-> ps_sig Signature::verify [EXT]).
//
// One credential per lane; three launches per batch so each kernel's live state fits the
// 512-entry register file of one wave per SIMD:
//   k_prep_*   : decode sigma/messages, fixed-base (shared vk) MSM, write the Miller-loop operands
//                (SoA, limb-major: coalesced per limb); per-credential verkeys: pervk.hip
//   k_miller_* : shared-squaring 2-pair Miller loop -> f (Fp12, SoA)
//   k_fexp     : final exponentiation, is_one, identity check -> verdict (+ optional GT bytes)
// Group assignment is a template parameter: kSigG2 (reference default, sigma in G2, vk in G1)
// or SigG1 (sigma in G1, vk in G2).
#include "codec.h"
#include "fixed.h"
#include "pairing.h"
#include "soa.h"
#include "subgroup.h"
#include "curve_pl.h"  // pair-lane G2 (FT<pl::Fp2>), pl::swp
#include "curve_wide_lz.h"

using namespace cc;

namespace {

// AoS point loads (table entries, constants): F words contiguous
template <class F>
DEV void ld_aff_aos(Aff<F>& a, const uint32_t* p) {
    constexpr int W = sizeof(F) / 4;
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint32_t* dx = reinterpret_cast<uint32_t*>(&a.x);
    uint32_t* dy = reinterpret_cast<uint32_t*>(&a.y);
#pragma unroll
    for (int k = 0; k < W / 4; k++) {
        uint4 t = q[k];
        dx[4 * k] = t.x; dx[4 * k + 1] = t.y; dx[4 * k + 2] = t.z; dx[4 * k + 3] = t.w;
    }
#pragma unroll
    for (int k = 0; k < W / 4; k++) {
        uint4 t = q[W / 4 + k];
        dy[4 * k] = t.x; dy[4 * k + 1] = t.y; dy[4 * k + 2] = t.z; dy[4 * k + 3] = t.w;
    }
}


template <class F>
DEV void st_aff_aos(uint32_t* p, const Aff<F>& a) {
    constexpr int W = sizeof(F) / 4;
    const uint32_t* sx = reinterpret_cast<const uint32_t*>(&a.x);
    const uint32_t* sy = reinterpret_cast<const uint32_t*>(&a.y);
    for (int k = 0; k < W; k++) p[k] = sx[k];
    for (int k = 0; k < W; k++) p[W + k] = sy[k];
}

template <class F>
DEV void st_jac_aos(uint32_t* p, const Jac<F>& a) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(&a);
    for (int k = 0; k < (int)(sizeof(Jac<F>) / 4); k++) p[k] = s[k];
}
template <class F>
DEV void ld_jac_aos(Jac<F>& a, const uint32_t* p) {
    uint32_t* d = reinterpret_cast<uint32_t*>(&a);
    for (int k = 0; k < (int)(sizeof(Jac<F>) / 4); k++) d[k] = p[k];
}

template <class F>
DEV bool decode_point(Aff<F>& a, const uint8_t* p);
template <>
DEV bool decode_point<Fp>(Aff<Fp>& a, const uint8_t* p) { return g1_decode(a, p); }
template <>
DEV bool decode_point<Fp2>(Aff<Fp2>& a, const uint8_t* p) { return g2_decode(a, p); }

template <class F>
constexpr int enc_bytes() { return sizeof(F) == sizeof(Fp) ? 97 : 192; }

}  // namespace

// ================================================================ point decode (setup path)
// out: AoS affine (2*W words per point, Montgomery) + inf flags
template <class F>
__global__ __launch_bounds__(64) void k_decode_points(size_t n, const uint8_t* __restrict__ bytes, uint32_t* __restrict__ out,
                                uint32_t* __restrict__ inf) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<F> a;
    bool ok = decode_point<F>(a, bytes + i * enc_bytes<F>());
    st_aff_aos<F>(out + i * (sizeof(Aff<F>) / 4), a);
    inf[i] = ok ? 0u : 1u;
}

// ================================================================ subgroup membership (subgroup.h)
// status per point: 0 = identity (AMCL decodes a bad encoding / off-curve point to infinity),
// 1 = on the curve but outside the order-r subgroup, 2 = in G1 / G2
template <class F>
DEV bool in_subgroup(const Aff<F>& a);
template <>
DEV bool in_subgroup<Fp>(const Aff<Fp>& a) { return g1_in_subgroup(a); }
template <>
DEV bool in_subgroup<Fp2>(const Aff<Fp2>& a) { return g2_in_subgroup(a); }

template <class F>
__global__ __launch_bounds__(64) void k_subgroup(size_t n, const uint8_t* __restrict__ bytes,
                                                 uint8_t* __restrict__ status) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<F> a;
    if (!decode_point<F>(a, bytes + i * enc_bytes<F>())) {
        status[i] = 0;
        return;
    }
    status[i] = in_subgroup<F>(a) ? 2 : 1;
}

// ================================================================ fixed-base tables (fixed.h layout)
// T1: per (base j, window w): 2^(wbits w) * B_j (Jacobian, AoS)
template <class F>
__global__ __launch_bounds__(64) void k_table_pow2(int nbases, int wbits, const uint32_t* __restrict__ bases,
                                                   const uint32_t* __restrict__ inf, uint32_t* __restrict__ pw) {
    const int nwin = ft_nwin(wbits);
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nbases * nwin) return;
    int j = t / nwin, w = t % nwin;
    Jac<F> P;
    if (inf[j]) {
        jac_set_inf(P);
    } else {
        Aff<F> b;
        ld_aff_aos<F>(b, bases + (size_t)j * (sizeof(Aff<F>) / 4));
        jac_from_aff(P, b);
        for (int k = 0; k < wbits * w; k++) jac_dbl(P, P);
    }
    st_jac_aos<F>(pw + (size_t)t * (sizeof(Jac<F>) / 4), P);
}

// x R (storage form) -> x R' (the lazy field's Montgomery form, fixed.h): times 2^392 / R = 2^-14
DEV void g1_to_lazy_form(Fp& v) { fp_to_lazy_form(v); }
// table entries: G1 always in the lazy form; G2 when the table's consumers are the pair-lane lazy sums
// (verkey and issuer tables; cc_fixed_base_mul's one-lane tables stay in the storage form)
DEV void to_lazy_form(Fp& v, int) { g1_to_lazy_form(v); }
DEV void to_lazy_form(Fp2& v, int lazy_g2) {
    if (!lazy_g2) return;
    g1_to_lazy_form(v.a);
    g1_to_lazy_form(v.b);
}

// T2: entries d * 2^(wbits w) * B_j for a run of FILL_RUN consecutive digits per thread: the first by
// double-and-add, the rest by one mixed addition each, then ONE inversion for the whole run
// (Montgomery's trick) to write them affine (G1 entries in the lazy field's form, fixed.h).  Identity
// entries are written as (0, 0).
constexpr int FILL_RUN = 32;
template <class F>
__global__ __launch_bounds__(64) void k_table_fill(int nbases, int wbits, const uint32_t* __restrict__ pw,
                                                   uint32_t* __restrict__ table, int lazy_g2) {
    using T = FT<F>;
    constexpr int EW = sizeof(Aff<F>) / 4, PW = sizeof(F) / 4;
    const int nwin = ft_nwin(wbits);
    const size_t went = ft_went(wbits);
    const size_t runs = (went + FILL_RUN - 1) / FILL_RUN;
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (t >= (size_t)nbases * nwin * runs) return;
    const size_t jw = t / runs, r = t % runs;
    const size_t d0 = r * FILL_RUN + 1;
    const int cnt = (int)(went - d0 + 1 < (size_t)FILL_RUN ? went - d0 + 1 : FILL_RUN);
    uint32_t* out = table + (jw * went + d0 - 1) * EW;
    Jac<F> P;
    ld_jac_aos<F>(P, pw + jw * (sizeof(Jac<F>) / 4));
    Aff<F> Pa;
    if (!jac_to_aff(Pa, P)) {
        for (int i = 0; i < cnt * EW; i++) out[i] = 0u;
        return;
    }
    Jac<F> acc;
    jac_set_inf(acc);
    for (int b = wbits - 1; b >= 0; b--) {
        jac_dbl(acc, acc);
        if ((d0 >> b) & 1) jac_add_aff(acc, acc, Pa);
    }
    F z[FILL_RUN], pre[FILL_RUN];
    F run;
    T::one(run);
#pragma unroll 1
    for (int i = 0; i < cnt; i++) {
        if (i) jac_add_aff(acc, acc, Pa);
        uint32_t* o = out + (size_t)i * EW;
        const uint32_t* xw = reinterpret_cast<const uint32_t*>(&acc.x);
        const uint32_t* yw = reinterpret_cast<const uint32_t*>(&acc.y);
        for (int c = 0; c < PW; c++) {
            o[c] = xw[c];
            o[PW + c] = yw[c];
        }
        z[i] = acc.z;
        pre[i] = run;
        if (!jac_is_inf(acc)) T::mul(run, run, acc.z);
    }
    F inv;
    T::inv(inv, run);
#pragma unroll 1
    for (int i = cnt - 1; i >= 0; i--) {
        uint32_t* o = out + (size_t)i * EW;
        if (T::is_zero(z[i])) {
            for (int c = 0; c < EW; c++) o[c] = 0u;
            continue;
        }
        F zi, zi2, v;
        T::mul(zi, inv, pre[i]);
        T::mul(inv, inv, z[i]);
        T::sqr(zi2, zi);
        uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
        for (int c = 0; c < PW; c++) vw[c] = o[c];
        T::mul(v, v, zi2);
        to_lazy_form(v, lazy_g2);
        for (int c = 0; c < PW; c++) o[c] = vw[c];
        T::mul(zi2, zi2, zi);
        for (int c = 0; c < PW; c++) vw[c] = o[PW + c];
        T::mul(v, v, zi2);
        to_lazy_form(v, lazy_g2);
        for (int c = 0; c < PW; c++) o[PW + c] = vw[c];
    }
}

// ================================================================ MSM helpers
// acc += sum_j (m_j over windows [w0, w1)) Y~_j; G1 sums stay on the lazy field between the terms
template <class F>
DEV void msm_fixed_terms(Jac<F>& acc, const uint8_t* msgs, int q, const uint32_t* __restrict__ table, int wbits,
                         const uint32_t* __restrict__ binf, int w0, int w1) {
    if constexpr (std::is_same<F, Fp>::value) {
        lz::JG a = lz::jg_from(acc);
        for (int j = 0; j < q; j++) {
            if (binf[j]) continue;  // uniform across the batch (shared verkey)
            Fr m;
            fr_from_be48(m, msgs + (size_t)j * 48);
            ft_add_lz(a, m.v, table, wbits, j, w0, w1);
        }
        acc = lz::jg_to(a);
    } else {
        for (int j = 0; j < q; j++) {
            if (binf[j]) continue;
            Fr m;
            fr_from_be48(m, msgs + (size_t)j * 48);
            ft_add<F>(acc, m.v, table, wbits, j, w0, w1, true);  // the verkey table
        }
    }
}

// fixed-base: acc = X~ + sum_j m_j Y~_j using the window tables
template <class F>
DEV void msm_fixed(Jac<F>& acc, const uint8_t* msgs, int q, const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                   const uint32_t* __restrict__ table, int wbits, const uint32_t* __restrict__ binf) {
    if (Xinf) {
        jac_set_inf(acc);
    } else {
        Aff<F> x;
        ld_aff_aos<F>(x, Xaff);
        jac_from_aff(acc, x);
    }
    msm_fixed_terms<F>(acc, msgs, q, table, wbits, binf, 0, ft_nwin(wbits));
}

// fixed-base over windows [w0, w1) only, X~ included on request (the lane-pair split of msm_fixed)
template <class F>
DEV void msm_fixed_part(Jac<F>& acc, const uint8_t* msgs, int q, const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                        bool with_x, const uint32_t* __restrict__ table, int wbits,
                        const uint32_t* __restrict__ binf, int w0, int w1) {
    if (!with_x || Xinf) {
        jac_set_inf(acc);
    } else {
        Aff<F> x;
        ld_aff_aos<F>(x, Xaff);
        jac_from_aff(acc, x);
    }
    msm_fixed_terms<F>(acc, msgs, q, table, wbits, binf, w0, w1);
}


// ================================================================ prep kernels


// SigG2 + shared verkey, one credential per lane PAIR (the layout of the pairing kernels): the even
// lane decodes sigma_1, the odd lane sigma_2; each lane sums half of the fixed-base windows, the two
// partial sums are exchanged by DPP and added (same operand order on both lanes, so both hold the
// same Jacobian representation); the even lane writes (X Z, Y), the odd lane Z^3.
__global__ __launch_bounds__(256) void k_prep_sigg2_pair(size_t n, int q, const uint8_t* __restrict__ s1b,
                                                         const uint8_t* __restrict__ s2b,
                                                         const uint8_t* __restrict__ msgs,
                                                         const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                                                         const uint32_t* __restrict__ table, int wbits,
                                                         const uint32_t* __restrict__ binf_fixed,
                                                         uint32_t* __restrict__ prep, uint32_t* __restrict__ flags) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t i = g >> 1;
    const int h = (int)(g & 1);
    if (i >= n) return;  // pair-uniform
    Soa S{prep, n};
    uint32_t fl = 0;
    {
        Aff<Fp2> a;
        if (!g2_decode(a, (h ? s2b : s1b) + i * 192)) fl |= h ? 2u : 1u;
        if (h) f2_neg(a.y, a.y);  // -sigma_2
        const int slot = h ? S_Q2 : S_Q1;
        st_f2(S, slot, i, a.x);
        st_f2(S, slot + 2, i, a.y);
    }
    Jac<Fp> pr, o;
    const int nwin = ft_nwin(wbits);
    msm_fixed_part<Fp>(pr, msgs + i * (size_t)q * 48, q, Xaff, Xinf, h == 0, table, wbits, binf_fixed,
                       h ? nwin / 2 : 0, h ? nwin : nwin / 2);
    o.x = pl::swp(pr.x);
    o.y = pl::swp(pr.y);
    o.z = pl::swp(pr.z);
    fl |= pl::swp(fl);
    if (h) {
        Jac<Fp> t = pr;
        pr = o;
        o = t;
    }
    jac_add(pr, pr, o);  // (even half) + (odd half) on both lanes
    if (jac_is_inf(pr)) {
        fl |= 4u;
    } else {  // pr affine in the R' form (the Miller loop's kAffRp operand): x on the even lane, y on the odd
        Fp x, y;
        lz::jg_to_aff_rp(x, y, lz::jg_from(pr));
        st_fp(S, S_P1 + h, i, h ? y : x);
    }
    if (!h) flags[i] = fl;
}


// SigG1, shared verkey, one credential per lane PAIR: lane h decodes sigma_{h+1} (one-lane G1) and
// the G2 verkey MSM X~ + sum m_j Y~_j runs on the pair-lane Fp2 (curve_pl.h): both lanes hold halves
// of one Jacobian accumulator, each table entry is read as halves.  The one-lane form keeps a G2
// accumulator and entry in ~150 words a lane (1 wave/SIMD, spills); here they take half, and every
// Fp2 product costs half the mads a lane.
__global__ __launch_bounds__(256, 2) void k_prep_sigg1_pair(size_t n, int q, const uint8_t* __restrict__ s1b,
                                                            const uint8_t* __restrict__ s2b,
                                                            const uint8_t* __restrict__ msgs,
                                                            const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                                                            const uint32_t* __restrict__ table, int wbits,
                                                            const uint32_t* __restrict__ binf_fixed,
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
    Jac<pl::Fp2> acc;
    if (Xinf) {
        jac_set_inf(acc);
    } else {
        Aff<pl::Fp2> x;
        for (int c = 0; c < NL; c++) {
            x.x.c.v[c] = Xaff[NL * h + c];
            x.y.c.v[c] = Xaff[2 * NL + NL * h + c];
        }
        jac_from_aff(acc, x);
    }
    lz::JL la = pl::jl_from_pl(acc);  // the sum on the lazy pair-lane field
    for (int j = 0; j < q; j++) {
        if (binf_fixed[j]) continue;  // uniform across the batch (shared verkey)
        Fr m;
        fr_from_be48(m, msgs + (i * (size_t)q + j) * 48);
        pl::ft_add_g2_lz(la, m.v, table, wbits, j, 0, ft_nwin(wbits));
    }
    acc = pl::jl_to_pl(la);
    Aff<pl::Fp2> a;
    if (!jac_to_aff(a, acc)) fl |= 4u;
    pl::st_f2(S, S_Q1, i, a.x);
    pl::st_f2(S, S_Q1 + 2, i, a.y);
    if (!h) flags[i] = fl;
}

// Small batches (capi.cpp: n <= kWideMax): ONE WAVE per credential, its verkey MSM's window terms
// spread over the lanes.  The pair kernels above walk all q x nwin terms on one lane (pair) — the whole
// launch then lasts one such chain, however few credentials there are.  Here term t = (j, w) goes to
// lane (pair) t mod 64 (32), lane (pair) 0 also takes X~, and a butterfly sums the partial sums
// (curve.h lane_group_sum / curve_pl.h pair_group_sum).  Same outputs as the pair kernels: sigma_1 /
// -sigma_2 decoded by lanes 0 / 1, pr affine as the Miller loop's operand, flags.
__global__ __launch_bounds__(64) void k_prep_sigg2_wide(size_t n, int q, const uint8_t* __restrict__ s1b,
                                                        const uint8_t* __restrict__ s2b,
                                                        const uint8_t* __restrict__ msgs,
                                                        const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                                                        const uint32_t* __restrict__ table, int wbits,
                                                        const uint32_t* __restrict__ binf_fixed,
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
    // the window terms over 16 groups of 4 lanes (term t to group t mod 16), each group's sum by spread
    // mixed additions (curve_wide_lz.h: the products of a step on the group's members), then the
    // groups' butterfly of spread additions
    const int nwin = ft_nwin(wbits), nt = q * nwin;
    constexpr int NG = 64 / lz::wide::G, EW = sizeof(Aff<Fp>) / 4;
    const int grp = l / lz::wide::G;
    lz::JG a = lz::jg_inf();
    if (grp == 0 && !Xinf) {
        Aff<Fp> x;
        Jac<Fp> xj;
        ld_aff_aos<Fp>(x, Xaff);
        jac_from_aff(xj, x);
        a = lz::jg_from(xj);
    }
    const size_t went = ft_went(wbits);
#pragma unroll 1
    for (int t = grp; t < nt; t += NG) {  // group-uniform
        const int j = t / nwin, w = t - j * nwin;
        if (binf_fixed[j]) continue;
        Fr m;
        fr_from_be48(m, msgs + (i * (size_t)q + j) * 48);
        const uint32_t d = ft_digit(m.v, w, wbits);
        if (!d) continue;
        Aff<Fp> e;
        ft_load<Fp>(e, table + (size_t)j * ft_base_words<Fp>(wbits) + ((size_t)w * went + d - 1) * EW);
        if (ft_is_empty(e)) continue;
        a = lz::wide::jg_add_aff(a, lz::AG{lz::from_fp(e.x), lz::from_fp(e.y)});
    }
    a = lz::wide::jg_group_sum(a);  // every lane the same sum
    if (lz::jg_is_inf(a)) {
        fl |= 4u;
    } else {
        Fp x, y;
        lz::wide::jg_to_aff_rp(x, y, a);
        if (l < 2) st_fp(S, S_P1 + h, i, h ? y : x);
    }
    if (l == 0) flags[i] = fl;
}

__global__ __launch_bounds__(64) void k_prep_sigg1_wide(size_t n, int q, const uint8_t* __restrict__ s1b,
                                                        const uint8_t* __restrict__ s2b,
                                                        const uint8_t* __restrict__ msgs,
                                                        const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                                                        const uint32_t* __restrict__ table, int wbits,
                                                        const uint32_t* __restrict__ binf_fixed,
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
    // the window terms over 8 groups of 4 lane pairs (term t to group t mod 8), spread mixed additions
    // within a group, then the groups' butterfly (curve_wide_lz.h)
    constexpr int NG = 32 / lz::wide::G, EW = sizeof(Aff<Fp2>) / 4;
    const int grp = p / lz::wide::G;
    lz::JL la = lz::jl_inf();
    if (grp == 0 && !Xinf) {
        Aff<pl::Fp2> x;
        Jac<pl::Fp2> xj;
        for (int c = 0; c < NL; c++) {
            x.x.c.v[c] = Xaff[NL * h + c];
            x.y.c.v[c] = Xaff[2 * NL + NL * h + c];
        }
        jac_from_aff(xj, x);
        la = pl::jl_from_pl(xj);
    }
    {
        const int nwin = ft_nwin(wbits), nt = q * nwin;
        const size_t went = ft_went(wbits);
#pragma unroll 1
        for (int t = grp; t < nt; t += NG) {  // group-uniform
            const int j = t / nwin, w = t - j * nwin;
            if (binf_fixed[j]) continue;
            Fr m;
            fr_from_be48(m, msgs + (i * (size_t)q + j) * 48);
            const uint32_t d = ft_digit(m.v, w, wbits);
            if (!d) continue;
            const uint32_t* e = table + (size_t)j * ft_base_words<Fp2>(wbits) + ((size_t)w * went + d - 1) * EW;
            Fp ex, ey;
            uint32_t o = 0;
#pragma unroll
            for (int c = 0; c < NL; c++) {
                ex.v[c] = e[NL * h + c];
                ey.v[c] = e[2 * NL + NL * h + c];
                o |= ex.v[c] | ey.v[c];
            }
            if (pl::pair_all(o == 0)) continue;  // (0, 0): an identity entry
            la = lz::wide::jl_add_aff_c(la, lz::F2<lz::AN, lz::BC>{lz::from_fp(ex)}, lz::F2<lz::AN, lz::BC>{lz::from_fp(ey)});
        }
    }
    la = lz::wide::jl_group_sum(la);  // every pair the same sum
    Jac<pl::Fp2> acc = pl::jl_to_pl(la);
    Aff<pl::Fp2> a;
    if (!lz::wide::jac_to_aff(a, acc)) fl |= 4u;  // the quad-form inversion
    if (p == 0) {
        pl::st_f2(S, S_Q1, i, a.x);
        pl::st_f2(S, S_Q1 + 2, i, a.y);
    }
    if (l == 0) flags[i] = fl;
}

// Fixed-argument lines for the constant G2 point g~ (SigG1): per Miller step, (l0, l2c, l3c)
// — 63 doubling + 5 addition steps, stored in loop order.  One thread computes them at setup.
__global__ __launch_bounds__(64) void k_gtilde_lines(const uint32_t* __restrict__ gtilde, uint32_t* __restrict__ lines) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    Aff<Fp2> Q;
    ld_aff_aos<Fp2>(Q, gtilde);
    G2Proj T;
    T.x = Q.x;
    T.y = Q.y;
    f2_one(T.z);
    int k = 0;
    auto put = [&](const Fp2& l0, const Fp2& l2, const Fp2& l3) {
        uint32_t* p = lines + (size_t)k * 72;
        const uint32_t* a = reinterpret_cast<const uint32_t*>(&l0);
        const uint32_t* b = reinterpret_cast<const uint32_t*>(&l2);
        const uint32_t* c = reinterpret_cast<const uint32_t*>(&l3);
        for (int t = 0; t < 24; t++) {
            p[t] = a[t];
            p[24 + t] = b[t];
            p[48 + t] = c[t];
        }
        k++;
    };
    for (int b = 62; b >= 0; b--) {
        Fp2 l0, l2, l3;
        line_dbl(T, l0, l2, l3);
        put(l0, l2, l3);
        if ((X_ABS >> b) & 1ull) {
            line_add(T, Q, l0, l2, l3);
            put(l0, l2, l3);
        }
    }
}

// ================================================================ host-side launchers
#define CC_CHECK(x)                          \
    do {                                     \
        hipError_t e_ = (x);                 \
        if (e_ != hipSuccess) return (int)e_; \
    } while (0)

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

extern "C" {

int cck_decode_points(int group, size_t n, const uint8_t* d_bytes, uint32_t* d_out, uint32_t* d_inf,
                      hipStream_t st) {
    if (!n) return 0;
    if (group == 1)
        hipLaunchKernelGGL(k_decode_points<Fp>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, d_bytes, d_out, d_inf);
    else
        hipLaunchKernelGGL(k_decode_points<Fp2>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, d_bytes, d_out, d_inf);
    CC_CHECK(hipGetLastError());
    return 0;
}

// table: nbases * ft_base_words(wbits) words (fixed.h); pw scratch: nbases * ft_nwin(wbits) Jacobian points
int cck_build_table(int group, int nbases, int wbits, const uint32_t* d_bases, const uint32_t* d_inf, uint32_t* d_pw,
                    uint32_t* d_table, int lazy_g2, hipStream_t st) {
    if (!nbases) return 0;
    if (wbits < 8 || wbits > 22) return -1;
    size_t t1 = (size_t)nbases * ft_nwin(wbits), t2 = t1 * ((ft_went(wbits) + FILL_RUN - 1) / FILL_RUN);
    if (group == 1) {
        hipLaunchKernelGGL(k_table_pow2<Fp>, dim3(nblocks(t1, 64)), dim3(64), 0, st, nbases, wbits, d_bases, d_inf, d_pw);
        hipLaunchKernelGGL(k_table_fill<Fp>, dim3(nblocks(t2, 64)), dim3(64), 0, st, nbases, wbits, d_pw, d_table, 1);
    } else {
        hipLaunchKernelGGL(k_table_pow2<Fp2>, dim3(nblocks(t1, 64)), dim3(64), 0, st, nbases, wbits, d_bases, d_inf, d_pw);
        hipLaunchKernelGGL(k_table_fill<Fp2>, dim3(nblocks(t2, 64)), dim3(64), 0, st, nbases, wbits, d_pw, d_table,
                           lazy_g2);
    }
    CC_CHECK(hipGetLastError());
    return 0;
}

int cck_subgroup(int group, size_t n, const uint8_t* d_bytes, uint8_t* d_status, hipStream_t st) {
    if (!n) return 0;
    if (group == 1)
        hipLaunchKernelGGL(k_subgroup<Fp>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, d_bytes, d_status);
    else
        hipLaunchKernelGGL(k_subgroup<Fp2>, dim3(nblocks(n, 64)), dim3(64), 0, st, n, d_bytes, d_status);
    CC_CHECK(hipGetLastError());
    return 0;
}

// n values of the storage form (x R, canonical 12 x 32) -> the lazy field's R' form (x R' mod p, canonical)
__global__ __launch_bounds__(64) void k_lazy_form(size_t n, const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fp v;
    for (int k = 0; k < NL; k++) v.v[k] = in[i * NL + k];
    fp_to_lazy_form(v);
    for (int k = 0; k < NL; k++) out[i * NL + k] = v.v[k];
}

int cck_lazy_form(size_t n, const uint32_t* d_in, uint32_t* d_out, hipStream_t st) {
    if (!n) return 0;
    hipLaunchKernelGGL(k_lazy_form, dim3(nblocks(n, 64)), dim3(64), 0, st, n, d_in, d_out);
    CC_CHECK(hipGetLastError());
    return 0;
}

int cck_gtilde_lines(const uint32_t* d_gtilde_aff, uint32_t* d_lines, hipStream_t st) {
    hipLaunchKernelGGL(k_gtilde_lines, dim3(1), dim3(64), 0, st, d_gtilde_aff, d_lines);
    CC_CHECK(hipGetLastError());
    return 0;
}


// shared-verkey prep (the fixed-base tables); per-credential verkeys: pervk.hip cck_prep_var
int cck_prep(int mode, size_t n, int q, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_msgs,
             const uint32_t* d_Xaff, uint32_t Xinf, const uint32_t* d_table, int wbits, const uint32_t* d_binf_fixed,
             uint32_t* d_prep, uint32_t* d_flags, hipStream_t st) {
    if (!n) return 0;
    if (mode == 0)
        hipLaunchKernelGGL(k_prep_sigg2_pair, dim3(nblocks(2 * n, 256)), dim3(256), 0, st, n, q, d_s1, d_s2, d_msgs,
                           d_Xaff, Xinf, d_table, wbits, d_binf_fixed, d_prep, d_flags);
    else
        hipLaunchKernelGGL(k_prep_sigg1_pair, dim3(nblocks(2 * n, 256)), dim3(256), 0, st, n, q, d_s1, d_s2, d_msgs,
                           d_Xaff, Xinf, d_table, wbits, d_binf_fixed, d_prep, d_flags);
    CC_CHECK(hipGetLastError());
    return 0;
}

// the small-batch form (one wave per credential, k_prep_*_wide): same arguments and outputs as cck_prep
int cck_prep_wide(int mode, size_t n, int q, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_msgs,
                  const uint32_t* d_Xaff, uint32_t Xinf, const uint32_t* d_table, int wbits,
                  const uint32_t* d_binf_fixed, uint32_t* d_prep, uint32_t* d_flags, hipStream_t st) {
    if (!n) return 0;
    if (mode == 0)
        hipLaunchKernelGGL(k_prep_sigg2_wide, dim3((unsigned)n), dim3(64), 0, st, n, q, d_s1, d_s2, d_msgs, d_Xaff, Xinf,
                           d_table, wbits, d_binf_fixed, d_prep, d_flags);
    else
        hipLaunchKernelGGL(k_prep_sigg1_wide, dim3((unsigned)n), dim3(64), 0, st, n, q, d_s1, d_s2, d_msgs, d_Xaff, Xinf,
                           d_table, wbits, d_binf_fixed, d_prep, d_flags);
    CC_CHECK(hipGetLastError());
    return 0;
}

}  // extern "C"
