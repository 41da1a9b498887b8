// Miller-loop kernels for gfx950 — the shared-squaring 2-pair loop of ate_2_pairing
// (ps_sig `ate_2_pairing` -> AMCL `pair::ate2`, reference src/lib.rs:13).
//
// Pair-lane form (tower_pl.h): one credential per PAIR of adjacent lanes, each lane holding one
// half of every Fp2 value, so a block of 256 lanes serves 128 credentials.
//
// Compiled once per group assignment (-DCC_MILLER_SIG=2: sigma in G2, the reference default;
// -DCC_MILLER_SIG=1: sigma in G1) so the two heavy kernels build in parallel.  CC_FP_INLINE puts
// every Fp multiplication inline in the loop body.
//
// One credential per lane.  Per Miller step the two pairs are processed by ONE copy of the
// line/evaluate/multiply code (a rolled loop over the pair index): the pair that is not being
// processed parks its twist point T in LDS (72 words per lane), and the G1 evaluation point is
// re-read from the prep SoA (L2-resident) at each use, so the registers hold f, one T, the line and
// the multiplication temporaries.  The 5 addition steps run out of line (rare; keeps code size down).
//
//   SigG2: pair 0 = (sigma_1, pr) with pr in Jacobian-evaluation form (XZ, Y, Z^3);
//          pair 1 = (-sigma_2, g~): g~ affine constant, or per lane (lane2: the RLC fold's
//          pseudo-credentials, two (bucket, fixed point) pairs each, fold.hip).
//   SigG1: pair 0 = (pr [affine G2], sigma_1); pair 1 = (g~ [precomputed lines], -sigma_2).
//   RLC mode runs pair 0 alone (NP = 1): its second pairs are folded (fold.hip).
#ifndef CC_MILLER_SIG
#define CC_MILLER_SIG 2
#endif
#ifdef CC_HOT_INLINE  // build option (Makefile HOT_INLINE=1): inline every Fp multiplication
#define CC_FP_INLINE 1
#endif
#include <cstdlib>
#include <cstring>
#include "codec.h"
#include "curve_pl.h"

namespace cc {
namespace pl {
namespace {

constexpr int MB = 256;        // lanes per block
constexpr int TW = 3 * NL;     // words of a parked G2Proj (this lane's halves)

// where a pair's G1 evaluation point lives: word (slot * NL + limb) * n + i * is
struct PSrc {
    const uint32_t* p;
    size_t n, is;
    bool jac;  // (XZ, Y, Z^3) form; affine (x, y) [z = 1] otherwise
};

DEV void ld_P(G1Eval& P, const PSrc& s, size_t i) {
#pragma unroll
    for (int k = 0; k < NL; k++) {
        P.px.v[k] = s.p[(size_t)k * s.n + i * s.is];
        P.py.v[k] = s.p[(size_t)(NL + k) * s.n + i * s.is];
    }
    if (s.jac) {
#pragma unroll
        for (int k = 0; k < NL; k++) P.pz.v[k] = s.p[(size_t)(2 * NL + k) * s.n + i * s.is];
    } else {
        fp_one(P.pz);
    }
}

// f *= line(P); a skipped pair (identity argument) contributes the constant 1.  P's coordinates are
// loaded one at a time, right before their multiplication (fewer live registers across the calls).
DEV void ld_Pc(Fp& x, const PSrc& s, int slot, size_t i) {
#pragma unroll
    for (int k = 0; k < NL; k++) x.v[k] = s.p[(size_t)(slot * NL + k) * s.n + i * s.is];
}
DEV void eval_mul(Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3, const PSrc& ps, size_t i, bool skip) {
    if (skip) return;  // e(O, Q) = e(P, O) = 1
    Fp2 a0, a2, a3;
    Fp c;
    if (ps.jac) {
        ld_Pc(c, ps, 2, i);
        f2_mul_fp(a0, l0, c);
    } else {
        a0 = l0;
    }
    ld_Pc(c, ps, 0, i);
    f2_mul_fp(a2, l2, c);
    ld_Pc(c, ps, 1, i);
    f2_mul_fp(a3, l3, c);
    f12_mul_line(f, a0, a2, a3);
}

DEV void park(uint32_t (*lds)[MB], const G2Proj& T) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&T);
#pragma unroll
    for (int k = 0; k < TW; k++) lds[k][threadIdx.x] = w[k];
}
DEV void unpark(G2Proj& T, uint32_t (*lds)[MB]) {
    uint32_t* w = reinterpret_cast<uint32_t*>(&T);
#pragma unroll
    for (int k = 0; k < TW; k++) w[k] = lds[k][threadIdx.x];
}

DEV void ld_line(Fp2& l0, Fp2& l2, Fp2& l3, const uint32_t* L) {
    ld_f2_aos(l0, L);
    ld_f2_aos(l2, L + 24);
    ld_f2_aos(l3, L + 48);
}

struct StepState {
    Fp12 f;
    G2Proj T;
};

// addition step of one pair: T <- T + Q, f *= line; or (line != nullptr) f *= precomputed line
static __device__ __noinline__ void miller_add(StepState* st, const uint32_t* qsrc, size_t n, size_t i,
                                               const uint32_t* line, PSrc ps, bool skip) {
    Fp12 f = st->f;
    Fp2 l0, l2, l3;
    if (line) {
        ld_line(l0, l2, l3, line);
    } else {
        G2Proj T = st->T;
        Aff<Fp2> Q;
        const Soa S{const_cast<uint32_t*>(qsrc), n};
        ld_f2(Q.x, S, 0, i);
        ld_f2(Q.y, S, 2, i);
        line_add(T, Q, l0, l2, l3);
        st->T = T;
    }
    eval_mul(f, l0, l2, l3, ps, i, skip);
    st->f = f;
}

}  // namespace

// prep: SoA slots of soa.h; flags: bit0 sigma_1 = O, bit1 sigma_2 = O, bit2 pr = O, bit4 pair-1 P = O
// cst: SigG2 -> g~ affine (24 words, used when !kLane2); SigG1 -> g~ lines (68 x 72 words)
// SIG is a template parameter (not only the macro) so the two objects' instantiations have distinct
// symbol names: the same name in both would be merged by the linker as one weak definition.
// NP = 1: pair 0 only (RLC mode, whose second pairs are folded into per-bucket pairs, fold.hip).
// The Miller value of credential i goes to fout as SoA element foff + i of stride fstride.
// qcheck (NP = 1, SigG2): pair 0's Q (sigma_1) gets the G2 subgroup test from the loop's own T
// (curve_pl.h miller_t_in_subgroup); a failure sets *qcheck (the RLC batch then falls back).
template <int SIG, bool kLane2, int NP>
__global__ __launch_bounds__(MB, 2) void k_miller(size_t n, const uint32_t* __restrict__ prep,
                                               const uint32_t* __restrict__ flags, const uint32_t* __restrict__ cst,
                                               uint32_t* __restrict__ fout, size_t fstride, size_t foff,
                                               uint32_t* __restrict__ qcheck) {
    __shared__ uint32_t lds[NP == 2 ? TW : 1][MB];
    const size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 1;  // credential of this lane pair
    if (i >= n) return;  // pair-uniform
    constexpr bool kSigG2 = SIG == 2;
    const uint32_t fl = flags[i];
    // pair 0 is degenerate if sigma_1 = O or pr = O; pair 1 if sigma_2 = O (or its P = O in RLC mode)
    const bool skip0 = (fl & 5u) != 0, skip1 = (fl & 18u) != 0;
    PSrc ps0, ps1;
    if (kSigG2) {
        ps0 = PSrc{prep + (size_t)S_P1 * NL * n, n, 1, true};
        ps1 = kLane2 ? PSrc{prep + (size_t)S_P2 * NL * n, n, 1, true} : PSrc{cst, 1, 0, false};
    } else {
        ps0 = PSrc{prep + (size_t)S_P1 * NL * n, n, 1, false};
        ps1 = PSrc{prep + (size_t)S_P2 * NL * n, n, 1, kLane2};
    }
    const uint32_t* q0 = prep + (size_t)S_Q1 * NL * n;
    const uint32_t* q1 = prep + (size_t)S_Q2 * NL * n;
    const Soa S{const_cast<uint32_t*>(prep), n};
    G2Proj T;
    if (kSigG2 && NP == 2) {  // park pair 1's T = -sigma_2
        ld_f2(T.x, S, S_Q2, i);
        ld_f2(T.y, S, S_Q2 + 2, i);
        f2_one(T.z);
        park(lds, T);
    }
    ld_f2(T.x, S, S_Q1, i);
    ld_f2(T.y, S, S_Q1 + 2, i);
    f2_one(T.z);
    Fp12 f;
    f12_one(f);
    const uint32_t* gl = cst;  // SigG1: next precomputed g~ line
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        if (b != 62) f12_sqr(f, f);
#pragma unroll 1
        for (int k = 0; k < NP; k++) {
            Fp2 l0, l2, l3;
            if (!kSigG2 && k == 1) {
                ld_line(l0, l2, l3, gl);
                gl += 72;
            } else {
                line_dbl(T, l0, l2, l3);
            }
            eval_mul(f, l0, l2, l3, k ? ps1 : ps0, i, k ? skip1 : skip0);
            if (kSigG2 && NP == 2) {  // swap T with the parked one
                G2Proj U;
                unpark(U, lds);
                park(lds, T);
                T = U;
            }
        }
        if ((X_ABS >> b) & 1ull) {
#pragma unroll 1
            for (int k = 0; k < NP; k++) {
                StepState st;
                st.f = f;
                st.T = T;
                const bool const_line = !kSigG2 && k == 1;
                miller_add(&st, k ? q1 : q0, n, i, const_line ? gl : nullptr, k ? ps1 : ps0, k ? skip1 : skip0);
                if (const_line) gl += 72;
                f = st.f;
                T = st.T;
                if (kSigG2 && NP == 2) {
                    G2Proj U;
                    unpark(U, lds);
                    park(lds, T);
                    T = U;
                }
            }
        }
    }
    if (NP == 1 && kSigG2 && qcheck && !skip0) {
        Aff<Fp2> q;
        ld_f2(q.x, S, S_Q1, i);
        ld_f2(q.y, S, S_Q1 + 2, i);
        if (!miller_t_in_subgroup(T, q) && !half_id()) atomicOr(qcheck, 1u);
    }
    f12_conj(f, f);
    st_f12(Soa{fout, fstride}, foff + i, f);
}

}  // namespace pl
}  // namespace cc

#if CC_MILLER_SIG == 2
#define CC_MILLER_LAUNCH cck_miller_pl_g2
#define CC_MILLER_LZ cck_miller_lz_g2
#else
#define CC_MILLER_LAUNCH cck_miller_pl_g1
#define CC_MILLER_LZ cck_miller_lz_g1
#endif
// the lazy-field kernels (miller_lz.hip), same arguments
extern "C" int CC_MILLER_LZ(int lane2, int np, size_t n, const uint32_t* d_prep, const uint32_t* d_flags,
                            const uint32_t* d_const, uint32_t* d_f, size_t fstride, size_t foff, uint32_t* d_qcheck,
                            hipStream_t st);

// lane2: per-lane second-pair P; np: pairs per credential (1 or 2); the Miller values go to SoA
// elements [foff, foff + n) of stride fstride (>= foff + n); d_qcheck (np = 1, SigG2, or null): the
// sigma_1 subgroup test from the loop's T
extern "C" int CC_MILLER_LAUNCH(int lane2, int np, size_t n, const uint32_t* d_prep, const uint32_t* d_flags,
                                const uint32_t* d_const, uint32_t* d_f, size_t fstride, size_t foff,
                                uint32_t* d_qcheck, hipStream_t st) {
    if (!n) return 0;
    if (fstride < foff + n || (np != 1 && np != 2)) return -1;
    // The lazy-field loop (miller_lz.hip) runs by default: 11 % fewer VALU instructions, same wait
    // fraction (profiles/r02/lz: config 2 Miller 16.1 -> 14.3 ms, config 3 21.7 -> 20.1 ms, same box).
    // CC_MILLER = pl | lz1 (this loop for 2 | for 1 and 2 pairs) keeps this file's loop for A/B runs.
    static const int sel = [] {
        const char* e = getenv("CC_MILLER");
        return !e ? 3 : !strcmp(e, "pl") ? 0 : !strcmp(e, "lz1") ? 1 : 3;
    }();
    if (sel & np)
        return CC_MILLER_LZ(lane2, np, n, d_prep, d_flags, d_const, d_f, fstride, foff, d_qcheck, st);
    constexpr int MB = cc::pl::MB;
    dim3 g((unsigned)((2 * n + MB - 1) / MB)), b(MB);
    if (np == 1)
        hipLaunchKernelGGL((cc::pl::k_miller<CC_MILLER_SIG, false, 1>), g, b, 0, st, n, d_prep, d_flags, d_const, d_f,
                           fstride, foff, d_qcheck);
    else if (lane2)
        hipLaunchKernelGGL((cc::pl::k_miller<CC_MILLER_SIG, true, 2>), g, b, 0, st, n, d_prep, d_flags, d_const, d_f,
                           fstride, foff, d_qcheck);
    else
        hipLaunchKernelGGL((cc::pl::k_miller<CC_MILLER_SIG, false, 2>), g, b, 0, st, n, d_prep, d_flags, d_const, d_f,
                           fstride, foff, d_qcheck);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
