// Threshold aggregation and PoK-of-signature verification kernels for gfx950 (the product path).
//
//   k_lagrange     : secret_sharing `Polynomial::lagrange_basis_at_0` [EXT] over the de-duplicated
//                    id set of the first t entries (reference src/signature.rs:454-463, 496-509)
//   k_msm_straus   : one Lagrange-weighted MSM per 16-lane group, windowed Straus over variable
//                    bases — Signature::aggregate (signature.rs:465, SignatureGroup) and the q+1 MSMs
//                    of Verkey::aggregate (signature.rs:512-524, OtherGroup) given per-entry verkeys;
//                    output encoded as amcl_wrapper `to_bytes`
//   k_vk_agg_fixed : Verkey::aggregate from the resident issuer table (fixed-base windows)
//   k_prep_pok     : ps_sig PoKOfSignatureProof::verify [EXT] (reference pok_sig.rs:103-105):
//                    Schnorr check MSM(g~, Y~_hidden.., J; responses.., chal) == T, then
//                    J' = X~ + J + sum_revealed Y~_i m_i, written in the verify kernels' Miller-loop
//                    operand layout so k_miller_* / k_fexp finish the 2-pairing check.
#include <cmath>
#include <cstdlib>

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

namespace {

template <class F>
DEV bool decode_pt(Aff<F>& a, const uint8_t* p);
template <>
DEV bool decode_pt<Fp>(Aff<Fp>& a, const uint8_t* p) { return g1_decode(a, p); }
template <>
DEV bool decode_pt<Fp2>(Aff<Fp2>& a, const uint8_t* p) { return g2_decode(a, p); }

template <class F>
DEV void encode_pt(uint8_t* p, const Aff<F>& a, bool finite);
template <>
DEV void encode_pt<Fp>(uint8_t* p, const Aff<Fp>& a, bool finite) { g1_encode(p, a, finite); }
template <>
DEV void encode_pt<Fp2>(uint8_t* p, const Aff<Fp2>& a, bool finite) { g2_encode(p, a, finite); }

template <class F>
constexpr int ebytes() { return sizeof(F) == sizeof(Fp) ? 97 : 192; }

template <class F>
DEV void ld_aff_aos(Aff<F>& a, const uint32_t* p) {
    uint32_t* d = reinterpret_cast<uint32_t*>(&a);
    for (int k = 0; k < (int)(sizeof(Aff<F>) / 4); k++) d[k] = p[k];
}

}  // namespace

// ================================================================ Lagrange coefficients
// l[(cred * t + i) * 8 ..]: canonical l_i(0) for the i-th of the first t ids of credential `cred`.
// LT tasks (credential, i) per lane.
// - The factors enter as raw integers, not Montgomery images: num and den take the same number of
//   factors, so the R^-1 each product picks up cancels in num / den (no conversion multiply).
// - The numerator is shared: with P = the product of the credential's distinct ids, l_i =
//   P / (x_i den_i), so a task multiplies only its t - 1 differences (P is formed once per
//   credential a lane touches; a credential holding the id 0 takes the per-task numerator instead).
// - The tasks' denominators share ONE Fermat inversion (Montgomery's trick: with
//   P_q = den_0 ... den_{q-1}, l_q = (num_q P_q) / P_{q+1}, walking q down from 1 / P_cnt and
//   multiplying den_q back in).
// - The O(t^2) duplicate scan (HashSet semantics) runs once per credential a lane touches; a
//   credential without repeated ids takes the plain product loop.
// - kLds: the block's credentials' first t ids are staged in LDS first (the out-of-line products
//   begin with s_waitcnt vmcnt(0), so a global id load per factor waited its full latency).
template <int LT, bool kLds>
__global__ __launch_bounds__(64) void k_lagrange(size_t n, size_t len, size_t t, const uint64_t* __restrict__ ids,
                                                 uint32_t* __restrict__ l) {
    extern __shared__ uint64_t sid[];
    const size_t first = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) * LT;
    size_t c0 = 0;
    if (kLds) {
        const size_t b0 = blockIdx.x * (size_t)blockDim.x * LT;
        const size_t b1 = b0 + (size_t)blockDim.x * LT < n * t ? b0 + (size_t)blockDim.x * LT : n * t;
        c0 = b0 / t;
        const size_t nc = (b1 - 1) / t - c0 + 1;
        for (size_t e = threadIdx.x; e < nc * t; e += blockDim.x) sid[e] = ids[(c0 + e / t) * len + e % t];
        __syncthreads();
    }
    if (first >= n * t) return;
    const int cnt = (int)((n * t - first) < (size_t)LT ? (n * t - first) : (size_t)LT);
    Fm nump[LT], den[LT];
    Fm pre = fm_one();  // P_q (a Montgomery 1: the raw factors' R^-k cancel between num and den)
    Fm prod = fm_one();  // the current credential's product of distinct ids
    size_t have = ~(size_t)0;
    bool dups = false, zero = false;
#pragma unroll
    for (int q = 0; q < LT; q++) {
        if (q >= cnt) break;
        const size_t task = first + q, cred = task / t, i = task % t;
        const uint64_t* id = kLds ? sid + (cred - c0) * t : ids + cred * len;
        if (cred != have) {
            have = cred;
            dups = false;
            zero = false;
            for (size_t j = 1; j < t && !dups; j++)
                for (size_t k = 0; k < j; k++)
                    if (id[k] == id[j]) { dups = true; break; }
            prod = fm_one();
            for (size_t j = 0; j < t; j++) {
                const uint64_t xj = id[j];
                zero |= xj == 0;
                if (dups) {
                    bool seen = false;
                    for (size_t k = 0; k < j; k++)
                        if (id[k] == xj) { seen = true; break; }
                    if (seen) continue;
                }
                Fm fxj;
#pragma unroll
                for (int k = 0; k < NR; k++) fxj.v[k] = 0;
                fxj.v[0] = (uint32_t)xj;
                fxj.v[1] = (uint32_t)(xj >> 32);
                prod = fm_mul_v(prod, fxj);
            }
        }
        const uint64_t xi = id[i];
        Fm nm = fm_one(), fxi;
#pragma unroll
        for (int k = 0; k < NR; k++) fxi.v[k] = 0;
        fxi.v[0] = (uint32_t)xi;
        fxi.v[1] = (uint32_t)(xi >> 32);
        Fm dn = zero ? fm_one() : fxi;  // x_i den_i, or den_i with its own numerator
        for (size_t j = 0; j < t; j++) {
            const uint64_t xj = id[j];
            if (xj == xi) continue;
            if (dups) {
                bool seen = false;
                for (size_t k = 0; k < j; k++)
                    if (id[k] == xj) { seen = true; break; }
                if (seen) continue;
            }
            Fm fxj, d;
#pragma unroll
            for (int k = 0; k < NR; k++) fxj.v[k] = 0;
            fxj.v[0] = (uint32_t)xj;
            fxj.v[1] = (uint32_t)(xj >> 32);
            if (zero) nm = fm_mul_v(nm, fxj);
            fm_sub(d, fxj, fxi);
            dn = fm_mul_v(dn, d);
        }
        nump[q] = fm_mul_v(zero ? nm : prod, pre);
        den[q] = dn;
        pre = fm_mul_v(pre, dn);
    }
    Fm inv = fm_inv(pre);  // 1 / P_cnt
#pragma unroll
    for (int q = LT - 1; q >= 0; q--) {
        if (q >= cnt) continue;
        const Fm li = fm_to_canon(fm_mul_v(nump[q], inv));  // num_q P_q / P_{q+1}
        uint32_t* o = l + (first + q) * 8;
        for (int k = 0; k < 8; k++) o[k] = li.v[k];
        inv = fm_mul_v(inv, den[q]);  // 1 / P_q
    }
}

// ================================================================ windowed Straus MSM (variable bases)
// One Lagrange-weighted MSM per lane with signed 4-bit windows: per base the multiples 1P..8P are
// built in Jacobian form, batch-normalised to affine with ONE inversion per task (Montgomery's
// trick over all 8t entries), then 65 windows x (4 doublings + t mixed additions).  For t = 67 in G2
// that is ~147k Fp multiplications per task against ~253k for the bitwise double-and-add it
// replaces.  Identity bases (AMCL decodes an off-curve point to infinity) and identity multiples of
// small-order points are flagged and skipped, so every input gives the reference's group element.
// Scratch per task (AoS, contiguous): 8t Jacobian entries (3*FS*12 words, affine x,y written back in
// place, word 2*FS*12 = infinity flag), 8t prefix products (FS*12 words), 65t digit bytes.
template <class F>
__host__ __device__ inline size_t straus_words(size_t t) {
    constexpr int FS = sizeof(F) / sizeof(Fp);
    return t * 8 * (3 * FS * NL) + t * 8 * (FS * NL) + (t * 65 + 3) / 4;
}



// L lanes per task: lane l takes the bases k = l, l + L, ... (t = 67, L = 16: 4-5 bases per lane),
// builds and normalises their multiples, runs the 65 windows over them, and the L partial sums are
// added across the lane group.  One lane per task would leave 10,000 tasks as 157 waves — a
// latency-bound GPU (each lane doing ~146k serial Fp multiplications).
template <class F, int L>
__global__ __launch_bounds__(256, 2) void k_msm_straus(size_t ntask, size_t t, const uint8_t* __restrict__ pts,
                                                    size_t pt_stride, size_t pt_jstride, size_t pt_step,
                                                    const uint32_t* __restrict__ l, size_t l_div,
                                                    uint32_t* __restrict__ scratch, uint8_t* __restrict__ out) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t task = g / L;
    const int lane = (int)(g % L);
    if (task >= ntask) return;  // uniform over the lane group (L divides the block)
    using T = FT<F>;
    constexpr int FS = sizeof(F) / sizeof(Fp);
    constexpr int JW = 3 * FS * NL, PW = FS * NL;
    const size_t cred = task / l_div;
    const uint8_t* base = pts + cred * pt_stride + (task % l_div) * pt_jstride;
    const uint32_t* lk = l + cred * t * 8;
    uint32_t* ent = scratch + task * straus_words<F>(t);
    uint32_t* pre = ent + t * 8 * JW;
    int8_t* dig = reinterpret_cast<int8_t*>(pre + t * 8 * PW);
    // multiples 1P..8P (Jacobian) of this lane's bases and the running product of their Z
    F acc_z;
    T::one(acc_z);
#pragma unroll 1
    for (size_t k = lane; k < t; k += L) {
        Aff<F> P;
        const bool ok = decode_pt<F>(P, base + k * pt_step);
        recode_w4(dig + k * 65, lk + k * 8);
        Jac<F> J;
        if (ok) {
            jac_from_aff(J, P);
        } else {
            jac_set_inf(J);
        }
#pragma unroll 1
        for (int d = 0; d < 8; d++) {
            if (d == 1) {
                jac_dbl(J, J);
            } else if (d > 1) {
                if (ok) jac_add_aff(J, J, P);
            }
            const size_t e = k * 8 + d;
            uint32_t* w = ent + e * JW;
            const uint32_t* jw = reinterpret_cast<const uint32_t*>(&J);
            for (int c = 0; c < JW; c++) w[c] = jw[c];
            const uint32_t* zw = reinterpret_cast<const uint32_t*>(&acc_z);
            for (int c = 0; c < PW; c++) pre[e * PW + c] = zw[c];
            if (!jac_is_inf(J)) T::mul(acc_z, acc_z, J.z);
        }
    }
    // one inversion per lane, then walk back: z_e^-1 = inv * prefix_e; inv *= z_e
    F inv;
    T::inv(inv, acc_z);
    if (t > (size_t)lane) {
        const long long kmax = (long long)(((t - 1 - lane) / L) * L + lane);
#pragma unroll 1
        for (long long kk = kmax; kk >= lane; kk -= L) {
            for (int d = 7; d >= 0; d--) {
                const size_t e = (size_t)kk * 8 + d;
                Jac<F> J;
                uint32_t* w = ent + e * JW;
                uint32_t* jw = reinterpret_cast<uint32_t*>(&J);
                for (int c = 0; c < JW; c++) jw[c] = w[c];
                const bool inf = jac_is_inf(J);
                if (!inf) {
                    F pz, zi, zi2;
                    uint32_t* pw = reinterpret_cast<uint32_t*>(&pz);
                    for (int c = 0; c < PW; c++) pw[c] = pre[e * PW + c];
                    T::mul(zi, inv, pz);
                    T::mul(inv, inv, J.z);
                    T::sqr(zi2, zi);
                    T::mul(J.x, J.x, zi2);
                    T::mul(zi2, zi2, zi);
                    T::mul(J.y, J.y, zi2);
                }
                for (int c = 0; c < 2 * PW; c++) w[c] = jw[c];  // affine x, y
                w[2 * PW] = inf ? 1u : 0u;
            }
        }
    }
    // 65 signed windows over this lane's bases, most significant first
    Jac<F> acc;
    jac_set_inf(acc);
#pragma unroll 1
    for (int win = 64; win >= 0; win--) {
        if (win != 64 && !jac_is_inf(acc))
            for (int z = 0; z < 4; z++) jac_dbl(acc, acc);
#pragma unroll 1
        for (size_t k = lane; k < t; k += L) {
            const int d = dig[k * 65 + win];
            if (!d) continue;
            const uint32_t* w = ent + (k * 8 + (d < 0 ? -d : d) - 1) * JW;
            if (w[2 * PW]) continue;  // identity multiple
            Aff<F> e;
            uint32_t* ew = reinterpret_cast<uint32_t*>(&e);
            for (int c = 0; c < 2 * PW; c++) ew[c] = w[c];
            if (d < 0) T::neg(e.y, e.y);
            jac_add_aff(acc, acc, e);
        }
    }
    lane_group_sum<F, L>(acc);
    if (lane == 0) {
        Aff<F> r;
        bool fin = jac_to_aff(r, acc);
        encode_pt<F>(out + task * ebytes<F>(), r, fin);
    }
}

// straus_lz_words, straus_g2lz_pair: straus.h

// affine encoding (amcl_wrapper to_bytes) of a lane-pair point; lane h = 0 writes
DEV void straus_g2lz_out(const lz::JL& acc, int h, uint8_t* out) {
    using namespace lz;
    cc::Aff<cc::Fp2> o;
    const bool fin = !jl_is_inf(acc);
    pl::Fp2 x, y;
    if (fin) {
        const auto zi = inv(acc.z);
        const auto zi2 = sqrr(zi);
        x = out_r2(mulr(acc.x, zi2));
        y = out_r2(mulr(acc.y, mulr(zi2, zi)));
    } else {
        fp_zero(x.c);
        fp_zero(y.c);
    }
    const Fp xs = pl::swp(x.c), ys = pl::swp(y.c);
    o.x.a = h ? xs : x.c;
    o.x.b = h ? x.c : xs;
    o.y.a = h ? ys : y.c;
    o.y.b = h ? y.c : ys;
    if (!h) g2_encode(out, o, fin);
}

// G lane pairs per task for any G (not only powers of two): blockDim = 2G floor(256 / 2G), the
// pairs' partial sums meet in LDS and pair 0 adds them.  G is chosen so the launch's waves
// fill whole rounds of the 2 waves/SIMD the registers allow (cck_msm_straus): 10,000 tasks at 8 pairs
// are 2,500 waves, 1.22 rounds of an MI355X's 2,048 slots, the last one a fifth full.
__global__ __launch_bounds__(256, 2) void k_msm_straus_g2lz_g(int G, size_t ntask, size_t t,
                                                             const uint8_t* __restrict__ pts, size_t pt_stride,
                                                             size_t pt_jstride, size_t pt_step,
                                                             const uint32_t* __restrict__ l, size_t l_div,
                                                             uint32_t* __restrict__ scratch,
                                                             uint8_t* __restrict__ out) {
    constexpr int JW = 3 * lz::LN;
    __shared__ int32_t red[256 * JW];
    const int L = 2 * G, TB = (int)blockDim.x / L;
    const int tib = (int)threadIdx.x / L, lit = (int)threadIdx.x % L;
    const size_t task = (size_t)blockIdx.x * TB + tib;
    const int pair = lit >> 1, h = lit & 1;
    const bool active = task < ntask;  // pair-uniform; every lane reaches the barrier
    lz::JL acc;
    if (active)
        straus_g2lz_pair(acc, G, pair, h, task, t, pts, pt_stride, pt_jstride, pt_step, l, l_div, scratch);
    else
        acc = lz::jl_inf();
    {
        int32_t* my = red + threadIdx.x * JW;
        for (int c = 0; c < lz::LN; c++) {
            my[c] = acc.x.c.v[c];
            my[lz::LN + c] = acc.y.c.v[c];
            my[2 * lz::LN + c] = acc.z.c.v[c];
        }
    }
    __syncthreads();
    if (active && pair == 0) {
#pragma unroll 1
        for (int p = 1; p < G; p++) {
            lz::JL o;
            const int32_t* src = red + (tib * L + 2 * p + h) * JW;
            for (int c = 0; c < lz::LN; c++) {
                o.x.c.v[c] = src[c];
                o.y.c.v[c] = src[lz::LN + c];
                o.z.c.v[c] = src[2 * lz::LN + c];
            }
            acc = lz::jl_add(acc, o);
        }
        straus_g2lz_out(acc, h, out + task * 192);
    }
}

// SigG2 PoK prep split by WAVE: a block of 256 lanes serves 128 proofs; its waves 0-1 (role A) decode
// sigma', add g~ resp_0 and the first `split` hidden responses' table terms and run chal J, waves
// 2-3 (role B) the other hidden responses, -T and J'.  The partial Schnorr sums meet in LDS and role A
// checks their sum.  Roles are wave-uniform (no divergence); the launch is 2 waves per proof group,
// so the 65,536-proof batch fills the 2 waves/SIMD the registers allow instead of 1.
constexpr int PK_PB = 128;  // proofs per block
__global__ __launch_bounds__(256, 2) void k_prep_pok_split(size_t n, int q, int r, int split,
                                                          const uint8_t* __restrict__ s1b,
                                                          const uint8_t* __restrict__ s2b,
                                                          const uint8_t* __restrict__ Jb,
                                                          const uint8_t* __restrict__ Tb,
                                                          const uint8_t* __restrict__ resp,
                                                          const uint8_t* __restrict__ chal,
                                                          const uint8_t* __restrict__ rev_msgs,
                                                          const uint32_t* __restrict__ rev_idx,
                                                          const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                                                          const uint32_t* __restrict__ table, int wbits,
                                                          const uint32_t* __restrict__ binf,
                                                          uint32_t* __restrict__ prep, uint32_t* __restrict__ flags,
                                                          uint32_t* __restrict__ jtab) {
    using FS_ = Fp2;
    using FO = Fp;
    constexpr int JW = sizeof(Jac<FO>) / 4;
    __shared__ uint32_t part[PK_PB][JW + 1];  // role B's partial Schnorr sum and flags
    const bool roleB = threadIdx.x >= PK_PB;   // wave-uniform
    const int slot_in_block = (int)(threadIdx.x & (PK_PB - 1));
    const size_t i = blockIdx.x * (size_t)PK_PB + slot_in_block;
    const bool active = i < n;
    constexpr int SB = ebytes<FS_>(), OB = ebytes<FO>();
    Soa S{prep, n};
    uint32_t fl = 0;
    Jac<FO> acc;
    jac_set_inf(acc);
    if (active) {
        Aff<FO> Ja;
        const bool Jok = decode_pt<FO>(Ja, Jb + i * OB);
        const uint8_t* rp = resp + i * (size_t)(q - r + 1) * 48;
        const int nwin = ft_nwin(wbits);
        Fr k;
        lz::JG la = lz::jg_inf();  // the table terms on the lazy field (fixed.h ft_add_lz)
        if (!roleB) {
            {
                Aff<FS_> a;
                if (!decode_pt<FS_>(a, s1b + i * SB)) fl |= 1u;
                const Fp* pa = reinterpret_cast<const Fp*>(&a);
                for (int c = 0; c < 4; c++) st_fp(S, S_Q1 + c, i, pa[c]);
                if (!decode_pt<FS_>(a, s2b + i * SB)) fl |= 2u;
                FT<FS_>::neg(a.y, a.y);
                for (int c = 0; c < 4; c++) st_fp(S, S_Q2 + c, i, pa[c]);
            }
            fr_from_be48(k, rp);
            if (!binf[q]) ft_add_lz(la, k.v, table, wbits, q, 0, nwin);  // table base q = g~
        }
        // hidden responses: role A the first `split`, role B the rest
        int slot = 1, hid = 0;
        for (int h = 0; h < q; h++) {
            bool revealed = false;
            for (int z = 0; z < r; z++) revealed |= rev_idx[z] == (uint32_t)h;
            if (revealed) continue;
            const bool mine = roleB ? hid >= split : hid < split;
            hid++;
            if (mine) {
                fr_from_be48(k, rp + (size_t)slot * 48);
                if (!binf[h]) ft_add_lz(la, k.v, table, wbits, h, 0, nwin);
            }
            slot++;
        }
        acc = lz::jg_to(la);
        if (!roleB) {
            // J * chal in fixed 4-bit windows (k_prep_pok)
            fr_from_be48(k, chal + i * 48);
            if (Jok) {
                // on the lazy field (curve_lz.h); the table of d J, d = 1..15, in the scratch as lazy points
                constexpr int LW = sizeof(lz::JG) / 4;
                auto tab = [&](int d, int w) -> uint32_t& { return jtab[((size_t)(d - 1) * LW + w) * n + i]; };
                const lz::AG Jl{lz::fit<lz::AN, lz::BC>(lz::reduce(lz::in_r(Ja.x))), lz::fit<lz::AN, lz::BC>(lz::reduce(lz::in_r(Ja.y)))};
                lz::JG t = lz::jg_add_aff(lz::jg_inf(), Jl);
#pragma unroll 1
                for (int d = 1; d <= 15; d++) {
                    if (d > 1) t = lz::jg_add_aff(t, Jl);
                    const uint32_t* tw = reinterpret_cast<const uint32_t*>(&t);
                    for (int w = 0; w < LW; w++) tab(d, w) = tw[w];
                }
                lz::JG sacc = lz::jg_inf();
#pragma unroll 1
                for (int win = 63; win >= 0; win--) {
                    for (int b = 0; b < 4; b++) sacc = lz::jg_dbl(sacc);
                    const uint32_t d = (k.v[win >> 3] >> ((win & 7) * 4)) & 15u;
                    if (d) {
                        uint32_t* tw = reinterpret_cast<uint32_t*>(&t);
                        for (int w = 0; w < LW; w++) tw[w] = tab((int)d, w);
                        sacc = lz::jg_add(sacc, t);
                    }
                }
                jac_add(acc, acc, lz::jg_to(sacc));
            }
        } else {
            Aff<FO> Ta;
            if (decode_pt<FO>(Ta, Tb + i * OB)) {
                FT<FO>::neg(Ta.y, Ta.y);
                jac_add_aff(acc, acc, Ta);
            }
            // J' = X~ + J + sum_revealed Y~_i m_i; P1 = J' affine in the R' form (the Miller loop's kAffRp)
            Jac<FO> jp;
            if (Xinf) {
                jac_set_inf(jp);
            } else {
                Aff<FO> x;
                ld_aff_aos<FO>(x, Xaff);
                jac_from_aff(jp, x);
            }
            if (Jok) jac_add_aff(jp, jp, Ja);
            lz::JG lj = lz::jg_from(jp);
            for (int z = 0; z < r; z++) {
                Fr m;
                fr_from_be48(m, rev_msgs + ((size_t)i * r + z) * 48);
                const int h = (int)rev_idx[z];
                if (!binf[h]) ft_add_lz(lj, m.v, table, wbits, h, 0, nwin);
            }
            if (lz::jg_is_inf(lj)) {
                fl |= 4u;
            } else {
                Fp x, y;
                lz::jg_to_aff_rp(x, y, lj);
                st_fp(S, S_P1, i, x);
                st_fp(S, S_P1 + 1, i, y);
            }
        }
    }
    if (roleB) {
        const uint32_t* aw = reinterpret_cast<const uint32_t*>(&acc);
        for (int c = 0; c < JW; c++) part[slot_in_block][c] = aw[c];
        part[slot_in_block][JW] = fl;
    }
    __syncthreads();
    if (roleB || !active) return;
    Jac<FO> o;
    uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
    for (int c = 0; c < JW; c++) ow[c] = part[slot_in_block][c];
    fl |= part[slot_in_block][JW];
    jac_add(acc, acc, o);
    if (!jac_is_inf(acc)) fl |= 8u;
    flags[i] = fl;
}

// ================================================================ issuer-table Verkey::aggregate
// Verkey::aggregate (signature.rs:483-526) over a resident issuer table: the bases X~_k, Y~_k,j of
// the n_iss issuers are FIXED, so cc_set_issuers gives each one an 8-bit window table (32 x 255
// affine multiples, the layout of the shared-verkey tables) and every Lagrange-weighted MSM is a
// fixed-base sum: t x 32 mixed additions, no doublings.  Task = (credential, j): j = 0 -> X~,
// j = 1..q -> Y~_{j-1}.  Issuer ids are sorted; each entry's id is found by binary search.  An id
// that is not in the table (the host entry point rejects those before launching; the device entry
// point cannot) makes the task write the identity and raise bit CC_DEVERR_UNKNOWN_ID in *err.  Table
// entries that are the identity (possible only for small-order bases) are stored as (0, 0), which is
// on neither curve, and skipped.
template <class F, int L>
__global__ __launch_bounds__(256) void k_vk_agg_fixed(size_t n, size_t len, size_t t, int q,
                                                      const uint64_t* __restrict__ ids,
                                                      const uint32_t* __restrict__ l,
                                                      const uint64_t* __restrict__ iss_ids, int n_iss,
                                                      const uint32_t* __restrict__ table, int wbits,
                                                      const uint32_t* __restrict__ binf,
                                                      uint8_t* __restrict__ outX, uint8_t* __restrict__ outY,
                                                      uint32_t* __restrict__ err) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t task = g / L;
    const int lane = (int)(g % L);
    if (task >= n * (size_t)(q + 1)) return;  // uniform over the lane group
    const size_t cred = task / (q + 1);
    const int j = (int)(task % (q + 1));
    int bad = 0;
    // this lane's share of the t terms into accum (a lazy G1 accumulator, or a storage-form one)
    auto lane_terms = [&](auto& accum, auto&& add_term) {
#pragma unroll 1
        for (size_t k = lane; k < t; k += L) {
            const uint64_t id = ids[cred * len + k];
            int lo = 0, hi = n_iss;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (iss_ids[mid] < id) lo = mid + 1; else hi = mid;
            }
            if (lo >= n_iss || iss_ids[lo] != id) {  // no issuer verkey for this id
                bad = 1;
                continue;
            }
            const int b = lo * (q + 1) + j;
            if (binf[b]) continue;
            add_term(accum, l + (cred * t + k) * 8, b);
        }
    };
    Jac<F> acc;
    if constexpr (std::is_same<F, Fp>::value) {  // G1: the whole lane sum on the lazy field
        lz::JG a = lz::jg_inf();
        lane_terms(a, [&](lz::JG& x, const uint32_t* kk, int b) { ft_add_lz(x, kk, table, wbits, b, 0, ft_nwin(wbits)); });
        acc = lz::jg_to(a);
    } else {
        jac_set_inf(acc);
        lane_terms(acc, [&](Jac<F>& x, const uint32_t* kk, int b) { ft_add<F>(x, kk, table, wbits, b, 0, ft_nwin(wbits), true); });
    }
    lane_group_sum<F, L>(acc);
#pragma unroll
    for (int o = 1; o < L; o <<= 1) bad |= __shfl_xor(bad, o, L);
    if (lane) return;
    if (bad) {
        atomicOr(err, 1u);  // CC_DEVERR_UNKNOWN_ID
        jac_set_inf(acc);
    }
    Aff<F> r;
    const bool fin = jac_to_aff(r, acc);
    uint8_t* o = j == 0 ? outX + cred * ebytes<F>() : outY + (cred * q + (j - 1)) * ebytes<F>();
    encode_pt<F>(o, r, fin);
}

// SigG1 (G2 issuer keys): the same task on lane PAIRS (curve_pl.h: one point per pair, each lane one
// half of every Fp2 coordinate, the storage-form table add pl::ft_add_g2), L lanes = L / 2 pairs a task.
// The one-lane G2 form needed all 512 VGPRs (one wave per SIMD); the pair form fits two.
template <int L>
__global__ __launch_bounds__(256, 2) void k_vk_agg_fixed_g2pl(size_t n, size_t len, size_t t, int q,
                                                            const uint64_t* __restrict__ ids,
                                                            const uint32_t* __restrict__ l,
                                                            const uint64_t* __restrict__ iss_ids, int n_iss,
                                                            const uint32_t* __restrict__ table, int wbits,
                                                            const uint32_t* __restrict__ binf,
                                                            uint8_t* __restrict__ outX, uint8_t* __restrict__ outY,
                                                            uint32_t* __restrict__ err) {
    constexpr int NPR = L / 2;
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t task = g / L;
    const int lane = (int)(g % L), pair = lane >> 1, h = lane & 1;
    if (task >= n * (size_t)(q + 1)) return;  // uniform over the lane group
    const size_t cred = task / (q + 1);
    const int j = (int)(task % (q + 1));
    lz::JL la = lz::jl_inf();  // the pair's share on the lazy pair-lane field
    int bad = 0;
#pragma unroll 1
    for (size_t k = pair; k < t; k += NPR) {  // pair-uniform
        const uint64_t id = ids[cred * len + k];
        int lo = 0, hi = n_iss;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (iss_ids[mid] < id) lo = mid + 1; else hi = mid;
        }
        if (lo >= n_iss || iss_ids[lo] != id) {  // no issuer verkey for this id
            bad = 1;
            continue;
        }
        const int b = lo * (q + 1) + j;
        if (binf[b]) continue;
        pl::ft_add_g2_lz(la, l + (cred * t + k) * 8, table, wbits, b, 0, ft_nwin(wbits));
    }
    Jac<pl::Fp2> acc = pl::jl_to_pl(la);
    pl::pair_group_sum<L>(acc);
#pragma unroll
    for (int o = 1; o < L; o <<= 1) bad |= __shfl_xor(bad, o, L);
    if (pair) return;  // pair 0 writes
    if (bad) {
        if (!h) atomicOr(err, 1u);  // CC_DEVERR_UNKNOWN_ID
        jac_set_inf(acc);
    }
    Aff<pl::Fp2> r;
    const bool fin = jac_to_aff(r, acc);
    Aff<Fp2> o;  // both halves on lane h = 0 for the encoding
    const Fp xs = pl::swp(r.x.c), ys = pl::swp(r.y.c);
    o.x.a = h ? xs : r.x.c;
    o.x.b = h ? r.x.c : xs;
    o.y.a = h ? ys : r.y.c;
    o.y.b = h ? r.y.c : ys;
    uint8_t* out = j == 0 ? outX + cred * 192 : outY + (cred * q + (j - 1)) * 192;
    if (!h) g2_encode(out, o, fin);
}

// ================================================================ PoK verify prep
// Prep layout (soa.h: Q1 0..3 | Q2 4..7 | P1 8..10 | P2 11..12) and flag bits as kernels.hip,
// plus flag bit3 = Schnorr check failed.

// SigG1 PoK prep (sigma' in G1, the Schnorr MSM and J' in G2), one proof per lane PAIR (curve_pl.h): lane h
// decodes sigma'_{h+1} (G1), the G2 sums run on the pair-lane Fp2 (pl::ft_add_g2 over the verkey tables,
// chal J in fixed 4-bit windows from a per-lane table of d J, d = 1..15, in jtab), the pair writes J' as
// pair 0's Q.  The one-lane form needed all 512 VGPRs and spilled (one wave per SIMD).
__global__ __launch_bounds__(256, 2) void k_prep_pok_g1pl(size_t n, int q, int r, const uint8_t* __restrict__ s1b,
                                                        const uint8_t* __restrict__ s2b,
                                                        const uint8_t* __restrict__ Jb,
                                                        const uint8_t* __restrict__ Tb,
                                                        const uint8_t* __restrict__ resp,
                                                        const uint8_t* __restrict__ chal,
                                                        const uint8_t* __restrict__ rev_msgs,
                                                        const uint32_t* __restrict__ rev_idx,
                                                        const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                                                        const uint32_t* __restrict__ table, int wbits,
                                                        const uint32_t* __restrict__ binf,
                                                        uint32_t* __restrict__ prep, uint32_t* __restrict__ flags,
                                                        uint32_t* __restrict__ jtab) {
    using G2 = pl::Fp2;
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t i = g >> 1;
    const int h = (int)(g & 1);
    if (i >= n) return;  // pair-uniform
    Soa S{prep, n};
    uint32_t fl = 0;
    {  // sigma'_1 on lane 0 (P1), -sigma'_2 on lane 1 (P2)
        Aff<Fp> a;
        if (!g1_decode(a, (h ? s2b : s1b) + i * 97)) fl |= h ? 2u : 1u;
        if (h) fp_neg(a.y, a.y);
        const int slot = h ? S_P2 : S_P1;
        fp_to_lazy_form(a.x);  // the Miller loop's affine P in the lazy R' form (miller_lz.hip kAffRp)
        fp_to_lazy_form(a.y);
        st_fp(S, slot, i, a.x);
        st_fp(S, slot + 1, i, a.y);
    }
    fl |= pl::swp(fl);
    // a G2 point as this lane's halves (both lanes decode it)
    auto own = [&](Aff<G2>& o, const Aff<Fp2>& a) {
        o.x.c = h ? a.x.b : a.x.a;
        o.y.c = h ? a.y.b : a.y.a;
    };
    Aff<Fp2> Jf;
    const bool Jok = pl::pair_all(g2_decode(Jf, Jb + i * 192));
    Aff<G2> Ja;
    own(Ja, Jf);
    // Schnorr: acc = g~ resp[0] + sum_hidden Y~_h resp[k] + J chal - T == O ?
    Jac<G2> acc;
    jac_set_inf(acc);
    {
        Fr k;
        const uint8_t* rp = resp + i * (size_t)(q - r + 1) * 48;
        fr_from_be48(k, rp);
        const int nwin = ft_nwin(wbits);
        lz::JL la = lz::jl_inf();  // the table terms on the lazy pair-lane field
        if (!binf[q]) pl::ft_add_g2_lz(la, k.v, table, wbits, q, 0, nwin);  // table base q = g~
        int slot = 1;
        for (int hh = 0; hh < q; hh++) {
            bool revealed = false;
            for (int z = 0; z < r; z++) revealed |= rev_idx[z] == (uint32_t)hh;
            if (revealed) continue;
            fr_from_be48(k, rp + (size_t)slot * 48);
            slot++;
            if (!binf[hh]) pl::ft_add_g2_lz(la, k.v, table, wbits, hh, 0, nwin);
        }
        fr_from_be48(k, chal + i * 48);
        if (Jok) {
            // chal J in fixed 4-bit windows on the lazy pair-lane field (curve_lz.h), the table of d J,
            // d = 1..15, in the scratch as lazy points (this lane's halves: 42 words an entry)
            constexpr int LW = sizeof(lz::JL) / 4;
            auto tab = [&](int d, int w) -> uint32_t& { return jtab[((size_t)(d - 1) * LW + w) * 2 * n + g]; };
            const lz::AL Jl{lz::reduce(lz::in_r2(Ja.x)), lz::reduce(lz::in_r2(Ja.y))};
            lz::JL t = lz::jl_from_aff(Jl);
#pragma unroll 1
            for (int d = 1; d <= 15; d++) {
                if (d > 1) t = lz::jl_add_aff(t, Jl);
                const uint32_t* tw = reinterpret_cast<const uint32_t*>(&t);
                for (int w = 0; w < LW; w++) tab(d, w) = tw[w];
            }
            lz::JL sacc = lz::jl_inf();
#pragma unroll 1
            for (int win = 63; win >= 0; win--) {
                for (int b = 0; b < 4; b++) sacc = lz::jl_dbl(sacc);
                const uint32_t d = (k.v[win >> 3] >> ((win & 7) * 4)) & 15u;
                if (d) {
                    uint32_t* tw = reinterpret_cast<uint32_t*>(&t);
                    for (int w = 0; w < LW; w++) tw[w] = tab((int)d, w);
                    sacc = lz::jl_add(sacc, t);
                }
            }
            la = lz::jl_add(la, sacc);
        }
        acc = pl::jl_to_pl(la);
        Aff<Fp2> Tf;
        if (pl::pair_all(g2_decode(Tf, Tb + i * 192))) {
            Aff<G2> Ta;
            own(Ta, Tf);
            FT<G2>::neg(Ta.y, Ta.y);
            jac_add_aff(acc, acc, Ta);
        }
        if (!jac_is_inf(acc)) fl |= 8u;
    }
    // J' = X~ + J + sum_revealed Y~_i m_i
    Jac<G2> jp;
    if (Xinf) {
        jac_set_inf(jp);
    } else {
        Aff<G2> x;
        for (int c = 0; c < NL; c++) {
            x.x.c.v[c] = Xaff[NL * h + c];
            x.y.c.v[c] = Xaff[2 * NL + NL * h + c];
        }
        jac_from_aff(jp, x);
    }
    if (Jok) jac_add_aff(jp, jp, Ja);
    lz::JL lj = pl::jl_from_pl(jp);
    for (int z = 0; z < r; z++) {
        Fr m;
        fr_from_be48(m, rev_msgs + ((size_t)i * r + z) * 48);
        const int hh = (int)rev_idx[z];
        if (!binf[hh]) pl::ft_add_g2_lz(lj, m.v, table, wbits, hh, 0, ft_nwin(wbits));
    }
    jp = pl::jl_to_pl(lj);
    Aff<G2> a;
    if (!jac_to_aff(a, jp)) fl |= 4u;
    pl::st_f2(S, S_Q1, i, a.x);
    pl::st_f2(S, S_Q1 + 2, i, a.y);
    if (!h) flags[i] = fl;
}

// ---------------------------------------------------------------- small batches: one block per proof
// The two PoK preps above walk a proof's whole Schnorr MSM (g~ and every hidden Y~ times its response,
// nwin table windows each), chal J and J' on one lane (pair) or two waves' lanes: for a small batch the
// launch then lasts that chain (~9 ms at n = 1).  Here one BLOCK of two waves takes one proof: wave 0
// decodes sigma' (sigma'_1 and sigma'_2 on its two halves) and runs chal J — a 256-doubling chain no
// lane split shortens, so each doubling's and addition's products are spread over lane groups instead
// (curve_wide_lz.h: 3 product times a doubling, 5 an addition), the multiples dJ in LDS (the jtab
// argument is unused here) — while wave 1 spreads the table terms over its lanes (G1) or lane pairs
// (G2) — term t = (response or revealed message, window) to lane t mod L — adds -T and X~ + J on two of
// them, and butterfly-sums the Schnorr part and J'.  The Schnorr parts meet in LDS.  Same outputs as
// the kernels above.
DEV bool pok_revealed(int hh, int r, const uint32_t* rev_idx) {
    bool rv = false;
    for (int z = 0; z < r; z++) rv |= rev_idx[z] == (uint32_t)hh;
    return rv;
}
DEV int rot_start(int lane, int t0, int L) { return ((lane - t0) % L + L) % L; }

__global__ __launch_bounds__(128) void k_prep_pok_wide_sigg2(size_t n, int q, int r, const uint8_t* __restrict__ s1b,
                                                            const uint8_t* __restrict__ s2b,
                                                            const uint8_t* __restrict__ Jb,
                                                            const uint8_t* __restrict__ Tb,
                                                            const uint8_t* __restrict__ resp,
                                                            const uint8_t* __restrict__ chal,
                                                            const uint8_t* __restrict__ rev_msgs,
                                                            const uint32_t* __restrict__ rev_idx,
                                                            const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                                                            const uint32_t* __restrict__ table, int wbits,
                                                            const uint32_t* __restrict__ binf,
                                                            uint32_t* __restrict__ prep, uint32_t* __restrict__ flags,
                                                            uint32_t* __restrict__ jtab) {
    using FS_ = Fp2;
    using FO = Fp;
    constexpr int JW = sizeof(Jac<FO>) / 4;
    constexpr int SB = ebytes<FS_>(), OB = ebytes<FO>();
    __shared__ uint32_t part[JW + 1];  // wave 1's Schnorr part and flag bits
    const size_t i = blockIdx.x;
    if (i >= n) return;  // block-uniform
    const int l = (int)(threadIdx.x & 63);
    const bool w1 = threadIdx.x >= 64;  // wave-uniform
    Soa S{prep, n};
    Aff<FO> Ja;
    const bool Jok = decode_pt<FO>(Ja, Jb + i * OB);
    if (!w1) {
        uint32_t fl = 0;
        {  // sigma'_1 on lanes 0-31, -sigma'_2 on lanes 32-63
            const bool second = l >= 32;
            Aff<FS_> a;
            const Fp* pa = reinterpret_cast<const Fp*>(&a);
            if (!decode_pt<FS_>(a, (second ? s2b : s1b) + i * SB)) fl |= second ? 2u : 1u;
            if (second) FT<FS_>::neg(a.y, a.y);
            if ((l & 31) == 0)
                for (int c = 0; c < 4; c++) st_fp(S, (second ? S_Q2 : S_Q1) + c, i, pa[c]);
            fl = (uint32_t)__shfl((int)fl, 0) | (uint32_t)__shfl((int)fl, 32);
        }
        Jac<FO> acc;
        jac_set_inf(acc);
        if (Jok) {  // chal J in fixed 4-bit windows (k_prep_pok_split): one chain, its products spread over lanes
            Fr k;
            fr_from_be48(k, chal + i * 48);
            constexpr int LW = sizeof(lz::JG) / 4;
            __shared__ uint32_t tabl[15][LW];  // d J, d = 1..15 (every lane holds the same point)
            const lz::AG Jl{lz::fit<lz::AN, lz::BC>(lz::reduce(lz::in_r(Ja.x))), lz::fit<lz::AN, lz::BC>(lz::reduce(lz::in_r(Ja.y)))};
            lz::JG t = lz::wide::jg_add_aff(lz::jg_inf(), Jl);
            const int grp = l / lz::wide::G, mem = l & (lz::wide::G - 1);
            auto ld_tab = [&](int d) {
                lz::JG v;
                uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
                for (int w = 0; w < LW; w++) vw[w] = tabl[d - 1][w];
                return v;
            };
            if (l == 0) {
                const uint32_t* tw = reinterpret_cast<const uint32_t*>(&t);
                for (int w = 0; w < LW; w++) tabl[0][w] = tw[w];
            }
            __builtin_amdgcn_wave_barrier();
            // d J, d = 2..15, as a tree: level s forms d = s + 1 .. 2s as (s J) + ((d - s) J), one multiple
            // a lane group (2s J through the addition's P = Q branch): 4 levels instead of 14 additions
#pragma unroll 1
            for (int s = 1; s <= 8; s <<= 1) {
                const int d = s + 1 + grp;
                const bool mine = grp < s && d <= 15;
                const lz::JG r = lz::wide::jg_add(ld_tab(s), ld_tab(mine ? d - s : 1));
                if (mine && mem == 0) {
                    const uint32_t* rw = reinterpret_cast<const uint32_t*>(&r);
                    for (int w = 0; w < LW; w++) tabl[d - 1][w] = rw[w];
                }
                __builtin_amdgcn_wave_barrier();
            }
            lz::JG sacc = lz::jg_inf();
#pragma unroll 1
            for (int win = 63; win >= 0; win--) {
                for (int b = 0; b < 4; b++) sacc = lz::wide::jg_dbl(sacc);
                const uint32_t d = (k.v[win >> 3] >> ((win & 7) * 4)) & 15u;
                if (d) {
                    uint32_t* tw = reinterpret_cast<uint32_t*>(&t);
                    for (int w = 0; w < LW; w++) tw[w] = tabl[d - 1][w];
                    sacc = lz::wide::jg_add(sacc, t);
                }
            }
            acc = lz::jg_to(sacc);
        }
        __syncthreads();
        Jac<FO> o;
        uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
        for (int c = 0; c < JW; c++) ow[c] = part[c];
        fl |= part[JW];
        jac_add(acc, acc, o);
        if (!jac_is_inf(acc)) fl |= 8u;
        if (l == 0) flags[i] = fl;
        return;
    }
    const uint8_t* rp = resp + i * (size_t)(q - r + 1) * 48;
    const int nwin = ft_nwin(wbits), nresp = q - r + 1;
    lz::JG la = lz::jg_inf(), lj = lz::jg_inf();
    int hh = -1;
#pragma unroll 1
    for (int s = 0; s < nresp; s++) {  // response s: g~ (s = 0, table base q) or the s-th hidden Y~
        int base = q;
        if (s) {
            do hh++;
            while (pok_revealed(hh, r, rev_idx));
            base = hh;
        }
        if (binf[base]) continue;
        Fr k;
        fr_from_be48(k, rp + (size_t)s * 48);
#pragma unroll 1
        for (int w = rot_start(l, s * nwin, 64); w < nwin; w += 64) ft_add_lz(la, k.v, table, wbits, base, w, w + 1);
    }
#pragma unroll 1
    for (int z = 0; z < r; z++) {  // J' terms: revealed messages, the lane rotation continued
        const int base = (int)rev_idx[z];
        if (binf[base]) continue;
        Fr m;
        fr_from_be48(m, rev_msgs + ((size_t)i * r + z) * 48);
#pragma unroll 1
        for (int w = rot_start(l, (nresp + z) * nwin, 64); w < nwin; w += 64) ft_add_lz(lj, m.v, table, wbits, base, w, w + 1);
    }
    Jac<FO> acc = lz::jg_to(la), jp = lz::jg_to(lj);
    if (l == 63) {  // -T
        Aff<FO> Ta;
        if (decode_pt<FO>(Ta, Tb + i * OB)) {
            FT<FO>::neg(Ta.y, Ta.y);
            jac_add_aff(acc, acc, Ta);
        }
    }
    if (l == 62) {  // X~ + J
        if (!Xinf) {
            Aff<FO> x;
            ld_aff_aos<FO>(x, Xaff);
            jac_add_aff(jp, jp, x);
        }
        if (Jok) jac_add_aff(jp, jp, Ja);
    }
    lane_group_sum<FO, 64>(acc);
    lane_group_sum<FO, 64>(jp);
    uint32_t fl = 0;
    if (jac_is_inf(jp)) {
        fl |= 4u;
    } else {
        Fp x, y;
        lz::wide::jg_to_aff_rp(x, y, lz::jg_from(jp));  // every lane the same point (lane_group_sum)
        if (l == 0) {
            st_fp(S, S_P1, i, x);
            st_fp(S, S_P1 + 1, i, y);
        }
    }
    if (l == 0) {
        const uint32_t* aw = reinterpret_cast<const uint32_t*>(&acc);
        for (int c = 0; c < JW; c++) part[c] = aw[c];
        part[JW] = fl;
    }
    __syncthreads();
}

__global__ __launch_bounds__(128) void k_prep_pok_wide_sigg1(size_t n, int q, int r, const uint8_t* __restrict__ s1b,
                                                            const uint8_t* __restrict__ s2b,
                                                            const uint8_t* __restrict__ Jb,
                                                            const uint8_t* __restrict__ Tb,
                                                            const uint8_t* __restrict__ resp,
                                                            const uint8_t* __restrict__ chal,
                                                            const uint8_t* __restrict__ rev_msgs,
                                                            const uint32_t* __restrict__ rev_idx,
                                                            const uint32_t* __restrict__ Xaff, uint32_t Xinf,
                                                            const uint32_t* __restrict__ table, int wbits,
                                                            const uint32_t* __restrict__ binf,
                                                            uint32_t* __restrict__ prep, uint32_t* __restrict__ flags,
                                                            uint32_t* __restrict__ jtab) {
    using G2 = pl::Fp2;
    constexpr int JW = sizeof(Jac<G2>) / 4;  // one lane's halves
    __shared__ uint32_t part[2][JW + 1];     // wave 1 pair 0's Schnorr part (each half) and flag bits
    const size_t i = blockIdx.x;
    if (i >= n) return;  // block-uniform
    const int l = (int)(threadIdx.x & 63), h = l & 1, p = l >> 1;
    const bool w1 = threadIdx.x >= 64;  // wave-uniform
    Soa S{prep, n};
    auto own = [&](Aff<G2>& o, const Aff<Fp2>& a) {
        o.x.c = h ? a.x.b : a.x.a;
        o.y.c = h ? a.y.b : a.y.a;
    };
    Aff<Fp2> Jf;
    const bool Jok = pl::pair_all(g2_decode(Jf, Jb + i * 192));
    Aff<G2> Ja;
    own(Ja, Jf);
    if (!w1) {
        uint32_t fl = 0;
        {  // sigma'_1 on lane 0 (P1), -sigma'_2 on lane 1 (P2)
            Aff<Fp> a;
            if (!g1_decode(a, (h ? s2b : s1b) + i * 97)) fl |= h ? 2u : 1u;
            if (h) fp_neg(a.y, a.y);
            fp_to_lazy_form(a.x);  // the Miller loop's affine P in the lazy R' form (kAffRp)
            fp_to_lazy_form(a.y);
            if (l < 2) {
                st_fp(S, h ? S_P2 : S_P1, i, a.x);
                st_fp(S, (h ? S_P2 : S_P1) + 1, i, a.y);
            }
        }
        fl = (uint32_t)__shfl((int)fl, 0) | (uint32_t)__shfl((int)fl, 1);
        lz::JL sacc = lz::jl_inf();
        if (Jok) {  // chal J in fixed 4-bit windows (k_prep_pok_g1pl): one chain, its products spread over pairs
            Fr k;
            fr_from_be48(k, chal + i * 48);
            constexpr int LW = sizeof(lz::JL) / 4;
            __shared__ uint32_t tabl[15][2][LW];  // d J, d = 1..15, by half (every pair holds the same point)
            const lz::AL Jl{lz::reduce(lz::in_r2(Ja.x)), lz::reduce(lz::in_r2(Ja.y))};
            lz::JL t = lz::jl_from_aff(Jl);
            const int grp = p / lz::wide::G, mem = p & (lz::wide::G - 1);
            auto ld_tab = [&](int d) {
                lz::JL v;
                uint32_t* vw = reinterpret_cast<uint32_t*>(&v);
                for (int w = 0; w < LW; w++) vw[w] = tabl[d - 1][h][w];
                return v;
            };
            if (l < 2) {
                const uint32_t* tw = reinterpret_cast<const uint32_t*>(&t);
                for (int w = 0; w < LW; w++) tabl[0][h][w] = tw[w];
            }
            __builtin_amdgcn_wave_barrier();
            // d J, d = 2..15, as a tree (8 lane-pair groups), as in k_prep_pok_wide_sigg2
#pragma unroll 1
            for (int s = 1; s <= 8; s <<= 1) {
                const int d = s + 1 + grp;
                const bool mine = grp < s && d <= 15;
                const lz::JL r = lz::wide::jl_add(ld_tab(s), ld_tab(mine ? d - s : 1));
                if (mine && mem == 0) {
                    const uint32_t* rw = reinterpret_cast<const uint32_t*>(&r);
                    for (int w = 0; w < LW; w++) tabl[d - 1][h][w] = rw[w];
                }
                __builtin_amdgcn_wave_barrier();
            }
#pragma unroll 1
            for (int win = 63; win >= 0; win--) {
                for (int b = 0; b < 4; b++) sacc = lz::wide::jl_dbl(sacc);
                const uint32_t d = (k.v[win >> 3] >> ((win & 7) * 4)) & 15u;
                if (d) {
                    uint32_t* tw = reinterpret_cast<uint32_t*>(&t);
                    for (int w = 0; w < LW; w++) tw[w] = tabl[d - 1][h][w];
                    sacc = lz::wide::jl_add(sacc, t);
                }
            }
        }
        Jac<G2> acc = pl::jl_to_pl(sacc);
        __syncthreads();
        Jac<G2> o;
        uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
        for (int c = 0; c < JW; c++) ow[c] = part[h][c];
        fl |= part[0][JW];
        jac_add(acc, acc, o);
        if (!pl::pair_all(jac_is_inf(acc))) fl |= 8u;
        if (l == 0) flags[i] = fl;
        return;
    }
    const uint8_t* rp = resp + i * (size_t)(q - r + 1) * 48;
    const int nwin = ft_nwin(wbits), nresp = q - r + 1;
    lz::JL la = lz::jl_inf(), lj = lz::jl_inf();
    int hh = -1;
#pragma unroll 1
    for (int s = 0; s < nresp; s++) {  // response s: g~ (s = 0, table base q) or the s-th hidden Y~
        int base = q;
        if (s) {
            do hh++;
            while (pok_revealed(hh, r, rev_idx));
            base = hh;
        }
        if (binf[base]) continue;
        Fr k;
        fr_from_be48(k, rp + (size_t)s * 48);
#pragma unroll 1
        for (int w = rot_start(p, s * nwin, 32); w < nwin; w += 32) pl::ft_add_g2_lz(la, k.v, table, wbits, base, w, w + 1);
    }
#pragma unroll 1
    for (int z = 0; z < r; z++) {  // J' terms: revealed messages, the pair rotation continued
        const int base = (int)rev_idx[z];
        if (binf[base]) continue;
        Fr m;
        fr_from_be48(m, rev_msgs + ((size_t)i * r + z) * 48);
#pragma unroll 1
        for (int w = rot_start(p, (nresp + z) * nwin, 32); w < nwin; w += 32)
            pl::ft_add_g2_lz(lj, m.v, table, wbits, base, w, w + 1);
    }
    Jac<G2> acc = pl::jl_to_pl(la), jp = pl::jl_to_pl(lj);
    if (p == 31) {  // -T (both lanes of the pair)
        Aff<Fp2> Tf;
        if (pl::pair_all(g2_decode(Tf, Tb + i * 192))) {
            Aff<G2> Ta;
            own(Ta, Tf);
            FT<G2>::neg(Ta.y, Ta.y);
            jac_add_aff(acc, acc, Ta);
        }
    }
    if (p == 30) {  // X~ + J
        if (!Xinf) {
            Aff<G2> x;
            for (int c = 0; c < NL; c++) {
                x.x.c.v[c] = Xaff[NL * h + c];
                x.y.c.v[c] = Xaff[2 * NL + NL * h + c];
            }
            jac_add_aff(jp, jp, x);
        }
        if (Jok) jac_add_aff(jp, jp, Ja);
    }
    pl::pair_group_sum<64>(acc);
    pl::pair_group_sum<64>(jp);
    Aff<G2> a;
    const uint32_t fl = lz::wide::jac_to_aff(a, jp) ? 0u : 4u;  // every pair the same J': quad-form inversion
    if (p == 0) {
        pl::st_f2(S, S_Q1, i, a.x);
        pl::st_f2(S, S_Q1 + 2, i, a.y);
        const uint32_t* aw = reinterpret_cast<const uint32_t*>(&acc);
        for (int c = 0; c < JW; c++) part[h][c] = aw[c];
        part[h][JW] = fl;
    }
    __syncthreads();
}

// ================================================================ fixed-base scalar multiplication
// out_i = k_i * B for one base B with a prebuilt 8-bit window table (keygen-style derivations:
// reference keygen.rs:27-32 g~ * x_i, and issuer-side h * e).  Scalars are 48-byte BE Fr.
template <class F>
__global__ __launch_bounds__(256) void k_fixed_mul(size_t n, const uint8_t* __restrict__ ks,
                                                   const uint32_t* __restrict__ table, uint32_t base_inf,
                                                   uint8_t* __restrict__ out) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Jac<F> acc;
    jac_set_inf(acc);
    if (!base_inf) {
        Fr k;
        fr_from_be48(k, ks + i * 48);
        ft_add<F>(acc, k.v, table, 8, 0, 0, ft_nwin(8));
    }
    Aff<F> r;
    bool fin = jac_to_aff(r, acc);
    encode_pt<F>(out + i * ebytes<F>(), r, fin);
}

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

// sigma_1 = sigs[0].sigma_1 (signature.rs:452): row i of n (sb bytes) from src + i * pitch, one byte a
// thread (hipMemcpy2DAsync's rectangle-copy kernel took 8.4 ms for 10,000 rows of 192 B, 20 ms for 97-B rows)
__global__ __launch_bounds__(256) void k_copy_rows(size_t n, size_t sb, const uint8_t* __restrict__ src,
                                                   size_t pitch, uint8_t* __restrict__ dst) {
    const size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n * sb) return;
    const size_t i = g / sb, b = g % sb;
    dst[g] = src[i * pitch + b];
}

extern "C" {

int cck_copy_rows(size_t n, size_t sb, const uint8_t* d_src, size_t pitch, uint8_t* d_dst, hipStream_t st) {
    if (!n || !sb) return 0;
    const size_t tot = n * sb;
    hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, n, sb, d_src, pitch, d_dst);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int cck_lagrange(size_t n, size_t len, size_t t, const uint64_t* d_ids, uint32_t* d_l, hipStream_t st) {
    if (!n || !t) return 0;
    constexpr int lt = 2;  // tasks per lane: with the divstep inversion 1.82 / 2.01 ms for 2 / 4 at config 4
                           // (the Fermat ladder measured 3.96 / 3.62 / 4.10 for 2 / 4 / 8)
    // ids of the credentials one block's 64 x lt tasks touch: at most 64 lt / t + 2 rows of t; past
    // 64 KiB (t > 3,968) the ids are read from global memory
    const size_t lds = (64 * (size_t)lt + 2 * t) * 8;
    const unsigned nb = nblocks((n * t + lt - 1) / lt, 64);
    if (lds <= 64 * 1024)
        hipLaunchKernelGGL((k_lagrange<lt, true>), dim3(nb), dim3(64), lds, st, n, len, t, d_ids, d_l);
    else
        hipLaunchKernelGGL((k_lagrange<lt, false>), dim3(nb), dim3(64), 0, st, n, len, t, d_ids, d_l);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t cck_straus_words(int group, size_t t) { return group == 1 ? straus_words<Fp>(t) : straus_lz_words(t); }

int cck_msm_straus(int group, size_t ntask, size_t t, const uint8_t* d_pts, size_t pt_stride, size_t pt_jstride,
                   size_t pt_step, const uint32_t* d_l, size_t l_div, uint32_t* d_scratch, uint8_t* d_out,
                   hipStream_t st) {
    if (!ntask) return 0;
    if (group == 1) {
        constexpr int L = 16;
        hipLaunchKernelGGL((k_msm_straus<Fp, L>), dim3(nblocks(ntask * L, 256)), dim3(256), 0, st, ntask, t, d_pts,
                           pt_stride, pt_jstride, pt_step, d_l, l_div, d_scratch, d_out);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    // G2: lane pairs per task G chosen for the fewest rounds of wave slots (2 waves/SIMD), then the least
    // work a wave (a pair's work modelled as ceil(t / G) 73 + 143 additions)
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const double slots = (double)cus * 4 * 2;
    int G = 0;
    double best = 0;
    for (int c = 4; c <= 16; c++) {
        const double per = (double)((t + c - 1) / c) * 73.0 + 143.0;
        const int tb = 256 / (2 * c);
        const double waves = (double)((ntask + tb - 1) / tb) * ((2 * c * tb + 63) / 64);
        const double est = per * std::ceil(waves / slots);
        if (!G || est < best) {
            G = c;
            best = est;
        }
    }
    const int L = 2 * G, tb = 256 / L;
    hipLaunchKernelGGL(k_msm_straus_g2lz_g, dim3((unsigned)((ntask + tb - 1) / tb)), dim3(tb * L), 0, st, G, ntask, t,
                       d_pts, pt_stride, pt_jstride, pt_step, d_l, l_div, d_scratch, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int cck_vk_agg_fixed(int group, size_t n, size_t len, size_t t, int q, const uint64_t* d_ids, const uint32_t* d_l,
                     const uint64_t* d_iss_ids, int n_iss, const uint32_t* d_table, int wbits, const uint32_t* d_binf,
                     uint8_t* d_outX, uint8_t* d_outY, uint32_t* d_err, hipStream_t st) {
    if (!n) return 0;
    constexpr int L = 8;  // 8 lanes per (credential, key) task: 34.1 ms vs 35.8 (4) and 43.3 (2) at config 4
    const size_t ntask = n * (size_t)(q + 1);
    dim3 g(nblocks(ntask * L, 256)), b(256);
    if (group == 1)
        hipLaunchKernelGGL((k_vk_agg_fixed<Fp, L>), g, b, 0, st, n, len, t, q, d_ids, d_l, d_iss_ids, n_iss, d_table,
                           wbits, d_binf, d_outX, d_outY, d_err);
    else
        hipLaunchKernelGGL((k_vk_agg_fixed_g2pl<L>), g, b, 0, st, n, len, t, q, d_ids, d_l, d_iss_ids, n_iss,
                           d_table, wbits, d_binf, d_outX, d_outY, d_err);  // G2 keys: 4 lane pairs a task
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int cck_prep_pok(int mode, size_t n, int q, int r, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_J,
                 const uint8_t* d_T, const uint8_t* d_resp, const uint8_t* d_chal, const uint8_t* d_rev_msgs,
                 const uint32_t* d_rev_idx, const uint32_t* d_Xaff, uint32_t Xinf, const uint32_t* d_table, int wbits,
                 const uint32_t* d_binf, uint32_t* d_prep, uint32_t* d_flags, uint32_t* d_jtab, hipStream_t st) {
    if (!n) return 0;
    dim3 g(nblocks(n, 256)), b(256);
    // d_jtab: 15 Jacobian points of the other group per element (<= 15 x 84 words a proof: SigG1's lazy
    // pair-lane G2 points, 42 words a lane)
    if (mode == 0) {
        // hidden responses for role A: balance nwin (1 + split) + ~233 (chal J) against
        // nwin (hidden - split) + nwin r + ~10 (mixed-addition units)
        const int hidden = q - r, nwin = ft_nwin(wbits);
        int split = (nwin * (hidden + r - 1) - 223) / (2 * nwin);
        split = split < 0 ? 0 : (split > hidden ? hidden : split);
        hipLaunchKernelGGL(k_prep_pok_split, dim3(nblocks(n, PK_PB)), dim3(2 * PK_PB), 0, st, n, q, r, split, d_s1,
                           d_s2, d_J, d_T, d_resp, d_chal, d_rev_msgs, d_rev_idx, d_Xaff, Xinf, d_table, wbits, d_binf,
                           d_prep, d_flags, d_jtab);
    } else
        hipLaunchKernelGGL(k_prep_pok_g1pl, dim3(nblocks(2 * n, 256)), b, 0, st, n, q, r, d_s1, d_s2, d_J, d_T, d_resp,
                           d_chal, d_rev_msgs, d_rev_idx, d_Xaff, Xinf, d_table, wbits, d_binf, d_prep, d_flags, d_jtab);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the small-batch form (one block of two waves per proof, k_prep_pok_wide_*): same arguments and outputs
int cck_prep_pok_wide(int mode, size_t n, int q, int r, const uint8_t* d_s1, const uint8_t* d_s2, const uint8_t* d_J,
                      const uint8_t* d_T, const uint8_t* d_resp, const uint8_t* d_chal, const uint8_t* d_rev_msgs,
                      const uint32_t* d_rev_idx, const uint32_t* d_Xaff, uint32_t Xinf, const uint32_t* d_table,
                      int wbits, const uint32_t* d_binf, uint32_t* d_prep, uint32_t* d_flags, uint32_t* d_jtab,
                      hipStream_t st) {
    if (!n) return 0;
    if (mode == 0)
        hipLaunchKernelGGL(k_prep_pok_wide_sigg2, dim3((unsigned)n), dim3(128), 0, st, n, q, r, d_s1, d_s2, d_J, d_T,
                           d_resp, d_chal, d_rev_msgs, d_rev_idx, d_Xaff, Xinf, d_table, wbits, d_binf, d_prep, d_flags,
                           d_jtab);
    else
        hipLaunchKernelGGL(k_prep_pok_wide_sigg1, dim3((unsigned)n), dim3(128), 0, st, n, q, r, d_s1, d_s2, d_J, d_T,
                           d_resp, d_chal, d_rev_msgs, d_rev_idx, d_Xaff, Xinf, d_table, wbits, d_binf, d_prep, d_flags,
                           d_jtab);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int cck_fixed_mul(int group, size_t n, const uint8_t* d_ks, const uint32_t* d_table, uint32_t base_inf,
                  uint8_t* d_out, hipStream_t st) {
    if (!n) return 0;
    dim3 g(nblocks(n, 256)), b(256);
    if (group == 1)
        hipLaunchKernelGGL(k_fixed_mul<Fp>, g, b, 0, st, n, d_ks, d_table, base_inf, d_out);
    else
        hipLaunchKernelGGL(k_fixed_mul<Fp2>, g, b, 0, st, n, d_ks, d_table, base_inf, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
