// Miller-loop kernels for gfx950 on the lazy radix-2^28 field (lazy.h, tower_lz.h) — the
// shared-squaring 2-pair loop of ate_2_pairing (ps_sig `ate_2_pairing` -> AMCL `pair::ate2`,
// reference src/lib.rs:13).  Replaces miller_pl.hip (same launchers, same SoA
// inputs and outputs); one credential per PAIR of adjacent lanes as there.
//
//   SigG2: pair 0 = (sigma_1, pr) with pr in Jacobian-evaluation form (XZ, Y, Z^3);
//          pair 1 = (-sigma_2, g~): g~ affine constant.
//   SigG1: pair 0 = (pr [affine G2], sigma_1); pair 1 = (g~ [precomputed lines], -sigma_2); sigma_1,
//          -sigma_2 arrive in the lazy R' form (kAffRp: no product for l0).
//   RLC mode keeps pair 0 of every credential (its second pairs are folded, fold.hip) and runs FOUR
//   credentials through one loop (k_miller4, built as its own object with CC_MILLER_QUAD; kTwin, two
//   credentials through the 2-pair loop, is the round-3 form): the RLC only needs the product of the
//   credentials' Miller values, and the shared squaring divides the Fp12 work per credential (5,002 Fp
//   multiplications against 5,548 for two a loop, 6,664 for a loop of its own).  The fold's 16 window
//   pairs run in the finish in the wide one-wave form (fexp_pl.hip k_miller_wide).
//
// Representation boundary: the prep SoA holds canonical 12 x 32 values in R = 2^406 form.  The twist
// points are moved to R' form once (in_r: T's start and the addition steps' Q).  The G1 evaluation
// coordinates are NOT converted: multiplied in R form straight into the R'-form line, every
// coefficient of a line comes out scaled by the same 2^14 (R / R'), and affine points use the constant
// R mod p as their Z; a line scaled by an Fp constant leaves the pairing unchanged (the final
// exponentiation's easy part kills Fp^*), as does the doubling step's 4x scale of T (lines are
// homogeneous of degree 2 in T).  The Miller value leaves in R form, canonical (out_r), for k_fexp.
#ifndef CC_MILLER_SIG
#define CC_MILLER_SIG 2
#endif
#ifdef CC_HOT_INLINE  // build option (Makefile HOT_INLINE=1): inline every Fp multiplication
#define CC_FP_INLINE 1
#endif
#include "codec.h"
#include "curve_pl.h"
#include "tower_lz.h"

namespace cc {
namespace lz {
namespace {

constexpr int MB = 256;  // lanes per block
// loop-carried value bounds (units of p/16; lazy.h): the step functions fit their results into
// these, so a bound that does not hold is a compile error
// f: after a line multiplication (BF), after the squaring (BS)
constexpr int BX = 128, BY = 1024, BZ = 128, BF = 512, BS = 2048, BL = 2048;
using Tw = G2P<BX, BY, BZ>;
using F12S = F12<AS, BF>;
using F2L = F2<AS, BL>;
using LineS = Line<F2L, F2L, F2L>;

template <class L>
DEV LineS fit_line(const L& l) { return {fit<AS, BL>(l.l0), fit<AS, BL>(l.l2), fit<AS, BL>(l.l3)}; }

// where a pair's G1 evaluation point lives: word (slot * NL + limb) * n + i * is.  form:
//   kJac    (XZ, Y, Z^3), R form: every line coefficient scaled by 2^14 (header)
//   kAffR   affine (x, y), R form: l0 times R mod p (the affine Z), scale 2^14
//   kAffRp  affine (x, y) in the lazy field's R' form (x R' mod p, canonical): l2 x, l3 y come out
//           unscaled and l0 needs no product (SigG2's constant g~: one Fp product less per step)
enum { kJac = 0, kAffR = 1, kAffRp = 2 };
struct PSrc {
    const uint32_t* p;
    size_t n, is;
    int form;
};

DEV Fq<AN, BC> ld_Pc(const PSrc& s, int slot, size_t i) {
    Fp x;
#pragma unroll
    for (int k = 0; k < NL; k++) x.v[k] = s.p[(size_t)(slot * NL + k) * s.n + i * s.is];
    return from_fp(x);
}

// f * line(P), the line scaled by 2^14 (header).  A skipped pair (identity argument: e(O, Q) =
// e(P, O) = 1) multiplies by the unit line (1, 0, 0) instead of returning early: the product's type
// bound then holds on every path (f's value bound only shrinks through a multiplication), and the
// lanes of a mixed wave would wait for the others anyway.
template <int B>
DEV F12S eval_mul(const F12<AS, B>& f, const LineS& ln, const PSrc& ps, size_t i, bool skip) {
    constexpr int32_t ONE_R[LN] = {LZ_C_OUT_LIMBS};
    using A0 = decltype(mul_fpr(ln.l0, fq_const(ONE_R)));
    A0 a0;
    if (ps.form == kAffRp) a0 = fit<AN, A0::BV>(reduce(ln.l0));  // pair-uniform branch
    else a0 = mul_fpr(ln.l0, ps.form == kJac ? ld_Pc(ps, 2, i) : fq_const(ONE_R));
    const auto a2 = mul_fpr(ln.l2, ld_Pc(ps, 0, i));
    const auto a3 = mul_fpr(ln.l3, ld_Pc(ps, 1, i));
    using L = decltype(a0);
    const L one = fit<AN, L::BV>(f2_one()), zero = fit<AN, L::BV>(f2_zero());
    return fit<AS, BF>(f12_mul_line(f, L{sel(skip, one.c, a0.c)}, L{sel(skip, zero.c, fit<AN, L::BV>(a2).c)},
                                    L{sel(skip, zero.c, fit<AN, L::BV>(a3).c)}));
}

// Two-pair loop: both twist points are parked in LDS while f is multiplied by their lines (the values
// live across the out-of-line multiplications must fit the callee-saved registers; f, a line and a T
// (84 + 42 + 42 words a lane) do not).  A T is packed for it: limbs carry-normalised to [0, 2^28),
// 13 limbs in 12 words + the signed top limb = 39 words, so both T's of the 512 lanes a CU holds fit
// its 160 KiB (78 x 4 B x 512).
constexpr int TP = 3 * PW;  // packed words per T
DEV void park(int32_t (*lds)[MB], int k, const Tw& T) {
    pack_fq<MB>(lds, TP * k, T.x.c);
    pack_fq<MB>(lds, TP * k + PW, T.y.c);
    pack_fq<MB>(lds, TP * k + 2 * PW, T.z.c);
}
DEV Tw unpark(int32_t (*lds)[MB], int k) {
    return {fit<AS, BX>(F2<AN, BX>{unpack_fq<MB, BX>(lds, TP * k)}), fit<AS, BY>(F2<AN, BY>{unpack_fq<MB, BY>(lds, TP * k + PW)}),
            fit<AS, BZ>(F2<AN, BZ>{unpack_fq<MB, BZ>(lds, TP * k + 2 * PW)})};
}

// a precomputed g~ line (SigG1): AoS l0 | l2 | l3, (a, b) halves of 12 words, R form
DEV LineS ld_line(const uint32_t* L) {
    const int h = (int)half_id();
    Fp c[3];
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int k = 0; k < NL; k++) c[j].v[k] = L[24 * j + NL * h + k];
    return {fit<AS, BL>(F2<AN, BC>{from_fp(c[0])}), fit<AS, BL>(F2<AN, BC>{from_fp(c[1])}),
            fit<AS, BL>(F2<AN, BC>{from_fp(c[2])})};
}

// an affine twist point from the prep SoA, in R' form
DEV void ld_q(F2<AN, 17>& x, F2<AN, 17>& y, const Soa& S, int slot, size_t i) {
    pl::Fp2 a, b;
    pl::ld_f2(a, S, slot, i);
    pl::ld_f2(b, S, slot + 2, i);
    x = in_r2(a);
    y = in_r2(b);
}
DEV Tw t_from(const F2<AN, 17>& x, const F2<AN, 17>& y) {
    return {fit<AS, BX>(x), fit<AS, BY>(y), fit<AS, BZ>(f2_one())};
}

// g's value came from eval_mul (F12S), stored in a wider variable: back to F12S
template <int B2, int B>
DEV F12<AS, B2> narrow_to(const F12<AS, B>& g) {
    static_assert(B2 == BF, "narrow_to: only for eval_mul results");
    F12<AS, B2> r;
    static_assert(sizeof(r) == sizeof(g), "same layout");
    __builtin_memcpy(&r, &g, sizeof(r));
    return r;
}

struct StepState {
    F12S f;
    Tw T;
};

// addition step of one pair: T <- T + Q, f *= line; or (line != nullptr) f *= precomputed line
static __device__ __noinline__ void miller_add(StepState* st, const uint32_t* prep, size_t n, int qslot, size_t i,
                                               const uint32_t* line, PSrc ps, bool skip) {
    F12S f = st->f;
    LineS ln;
    if (line) {
        ln = ld_line(line);
    } else {
        Tw T = st->T;
        F2<AN, 17> qx, qy;
        ld_q(qx, qy, Soa{const_cast<uint32_t*>(prep), n}, qslot, i);
        ln = fit_line(line_add(T, qx, qy));
        st->T = T;
    }
    st->f = eval_mul(f, ln, ps, i, skip);
}

// sigma_1's G2 subgroup test from the loop's final T (curve_pl.h miller_t_in_subgroup): out of line,
// so its registers do not add to the loop's
static __device__ __noinline__ void t_check(const Tw* T, const uint32_t* prep, size_t n, int qslot, size_t i,
                                            uint32_t* qcheck) {
    pl::G2Proj Tp;
    Tp.x = out_r2(T->x);
    Tp.y = out_r2(T->y);
    Tp.z = out_r2(T->z);
    const Soa S{const_cast<uint32_t*>(prep), n};
    Aff<pl::Fp2> q;
    pl::ld_f2(q.x, S, qslot, i);
    pl::ld_f2(q.y, S, qslot + 2, i);
    if (!pl::miller_t_in_subgroup(Tp, q) && !half_id()) atomicOr(qcheck, 1u);
}

}  // namespace

#ifndef CC_MILLER_QUAD
// prep: SoA slots of soa.h, stride ps (>= the elements read); flags: bit0 sigma_1 = O, bit1 sigma_2 = O,
// bit2 pr = O, bit4 pair-1 P = O
// cst: SigG2 -> g~ affine in the lazy R' form (24 words, cck_lazy_form); SigG1 -> g~ lines (68 x 72
// words); unused by kTwin.
// The Miller value of credential i goes to fout as SoA element foff + i of stride fstride.  kTwin (RLC
// credentials): the one pair of credentials 2j and 2j + 1, laid out as pairs 0 and 1 of element j
// (rlc.hip twin_slot; the second skipped when n is odd); their product goes to element foff + j.
// qcheck (kTwin, SigG2): each credential's Q (sigma_1) gets the G2 subgroup test from the loop's own T
// (curve_pl.h miller_t_in_subgroup); a failure sets *qcheck.
template <int SIG, bool kTwin>
__global__ __launch_bounds__(MB, 2) void k_miller(size_t n, size_t ps, const uint32_t* __restrict__ prep,
                                               const uint32_t* __restrict__ flags, const uint32_t* __restrict__ cst,
                                               uint32_t* __restrict__ fout, size_t fstride, size_t foff,
                                               uint32_t* __restrict__ qcheck, int pform) {
    constexpr int NP = 2;  // pairs per loop
    __shared__ int32_t lds[2 * TP][MB];
    const size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 1;  // lane pair: credential (twin: pair)
    if (i >= (kTwin ? (n + 1) / 2 : n)) return;  // pair-uniform
    constexpr bool kSigG2 = SIG == 2;
    // twin: credentials 2 i and 2 i + 1 have their pairs at element i of the pair-0 and pair-1 slots
    // (rlc.hip twin_slot); with n odd the last pair 1 is skipped (its element was never written)
    const uint32_t fl = flags[kTwin ? 2 * i : i];
    const bool skip0 = (fl & 5u) != 0;
    const bool skip1 = kTwin ? (2 * i + 1 >= n || (flags[2 * i + 1] & 5u) != 0) : (fl & 18u) != 0;
    // pform: the form of the preps' P (kAffRp), a kernel argument so that both eval_mul paths stay
    // compiled as one runtime branch: with the branch folded away the loop's registers allocate
    // differently and spill more (measured: +80 static scratch instructions, Miller +4 %)
    PSrc ps0, ps1;
    if (kTwin) {
        ps0 = PSrc{prep + (size_t)S_P1 * NL * ps, ps, 1, pform};
        ps1 = PSrc{prep + (size_t)S_P2 * NL * ps, ps, 1, pform};
    } else if (kSigG2) {
        ps0 = PSrc{prep + (size_t)S_P1 * NL * ps, ps, 1, pform};
        ps1 = PSrc{cst, 1, 0, kAffRp};
    } else {
        ps0 = PSrc{prep + (size_t)S_P1 * NL * ps, ps, 1, pform};
        ps1 = PSrc{prep + (size_t)S_P2 * NL * ps, ps, 1, pform};
    }
    const Soa S{const_cast<uint32_t*>(prep), ps};
    // both T's parked in LDS between their uses
    Tw T;
    {
        F2<AN, 17> qx, qy;
        if (kSigG2 || kTwin) {  // pair 1's T: -sigma_2 (twin: the second credential's Q)
            ld_q(qx, qy, S, S_Q2, i);
            park(lds, 1, t_from(qx, qy));
        }
        ld_q(qx, qy, S, S_Q1, i);
        T = t_from(qx, qy);
        park(lds, 0, T);
    }
    F12S f = fit<AS, BF>(f12_one());
    const uint32_t* gl = cst;  // SigG1: next precomputed g~ line
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        // g: the squared f, then f times each pair's line; one eval_mul instantiation serves both pairs
        F12<AS, BS> g = b != 62 ? fit<AS, BS>(f12_sqr(f)) : fit<AS, BS>(f);
#pragma unroll 1
        for (int k = 0; k < NP; k++) {
            LineS ln;
            if (!kSigG2 && !kTwin && k == 1) {
                ln = ld_line(gl);
                gl += 72;
            } else {
                T = unpark(lds, k);
                ln = fit_line(line_dbl(T));
                park(lds, k, T);
            }
            g = fit<AS, BS>(eval_mul(g, ln, k ? ps1 : ps0, i, k ? skip1 : skip0));
        }
        // both passes ran, so g holds an eval_mul result, whose type bound is BF
        f = narrow_to<BF>(g);
        if ((X_ABS >> b) & 1ull) {
#pragma unroll 1
            for (int k = 0; k < NP; k++) {
                const bool const_line = !kSigG2 && !kTwin && k == 1;
                StepState st;
                st.f = f;
                if (!const_line) st.T = unpark(lds, k);
                miller_add(&st, prep, ps, k ? S_Q2 : S_Q1, i, const_line ? gl : nullptr, k ? ps1 : ps0,
                           k ? skip1 : skip0);
                if (const_line) gl += 72;
                else park(lds, k, st.T);
                f = st.f;
            }
        }
    }
    if (kTwin && kSigG2 && qcheck) {
#pragma unroll 1
        for (int k = 0; k < NP; k++) {
            if (k ? skip1 : skip0) continue;  // pair-uniform
            const Tw Tk = unpark(lds, k);
            t_check(&Tk, prep, ps, k ? S_Q2 : S_Q1, i, qcheck);
        }
    }
    f = f12_conj(f);
    const Soa O{fout, fstride};
    const F2<AS, BF>* v = reinterpret_cast<const F2<AS, BF>*>(&f);
#pragma unroll
    for (int k = 0; k < 6; k++) st_fp(O, 2 * k + (int)half_id(), foff + i, out_r(v[k].c));
}

#else  // CC_MILLER_QUAD: its own object (Makefile miller4_*), so the 1-wave kernel's register budget does
       // not reach the out-of-line helpers of the 2-wave kernels above
// RLC, FOUR credentials' pairs per shared-squaring loop (twice kTwin's): the Fp12 squaring is shared by
// four pairs instead of two (per credential 26 Fp2 products a step against 29).  Reads the twin layout
// (credentials 4 j .. 4 j + 3 = pairs 0 / 1 of elements 2 j and 2 j + 1); the four T's are parked packed
// in LDS (4 x 39 words a lane: the whole 160 KiB of a CU at 1 wave/SIMD, 256 lanes), the loop body is
// the two-pair loop's with one pair at a time; the product of the four Miller values goes to element
// foff + j.
template <int SIG>
__global__ __launch_bounds__(MB, 1) void k_miller4(size_t n, size_t ps, const uint32_t* __restrict__ prep,
                                                const uint32_t* __restrict__ flags, uint32_t* __restrict__ fout,
                                                size_t fstride, size_t foff, uint32_t* __restrict__ qcheck,
                                                int pform) {
    constexpr int NP = 4;
    __shared__ int32_t lds[NP * TP][MB];
    const size_t j = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 1;
    if (j >= (n + 3) / 4) return;  // pair-uniform
    const Soa S{const_cast<uint32_t*>(prep), ps};
    uint32_t skipm = 0;  // bit k: pair k skipped (credential absent, or an identity argument)
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const size_t c = 4 * j + k;
        const bool in = c < n;
        if (!in || (flags[in ? c : 0] & 5u) != 0) skipm |= 1u << k;
        F2<AN, 17> qx, qy;
        ld_q(qx, qy, S, (k & 1) ? S_Q2 : S_Q1, in ? c >> 1 : 0);
        park(lds, k, t_from(qx, qy));
    }
    // pair k: credential 4 j + k at twin element 2 j + k / 2, slots pair (k & 1)
    auto elem = [&](int k) -> size_t { return 4 * j + k < n ? 2 * j + (k >> 1) : 0; };
    auto psrc = [&](int k) { return PSrc{prep + (size_t)((k & 1) ? S_P2 : S_P1) * NL * ps, ps, 1, pform}; };
    F12S f = fit<AS, BF>(f12_one());
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        F12<AS, BS> g = b != 62 ? fit<AS, BS>(f12_sqr(f)) : fit<AS, BS>(f);
#pragma unroll 1
        for (int k = 0; k < NP; k++) {
            Tw T = unpark(lds, k);
            const LineS ln = fit_line(line_dbl(T));
            park(lds, k, T);
            g = fit<AS, BS>(eval_mul(g, ln, psrc(k), elem(k), (skipm >> k) & 1u));
        }
        f = narrow_to<BF>(g);
        if ((X_ABS >> b) & 1ull) {
#pragma unroll 1
            for (int k = 0; k < NP; k++) {
                StepState st;
                st.f = f;
                st.T = unpark(lds, k);
                miller_add(&st, prep, ps, (k & 1) ? S_Q2 : S_Q1, elem(k), nullptr, psrc(k), (skipm >> k) & 1u);
                park(lds, k, st.T);
                f = st.f;
            }
        }
    }
    if (SIG == 2 && qcheck) {
#pragma unroll 1
        for (int k = 0; k < NP; k++) {
            if ((skipm >> k) & 1u) continue;  // pair-uniform
            const Tw Tk = unpark(lds, k);
            t_check(&Tk, prep, ps, (k & 1) ? S_Q2 : S_Q1, elem(k), qcheck);
        }
    }
    f = f12_conj(f);
    const Soa O{fout, fstride};
    const F2<AS, BF>* v = reinterpret_cast<const F2<AS, BF>*>(&f);
#pragma unroll
    for (int k = 0; k < 6; k++) st_fp(O, 2 * k + (int)half_id(), foff + j, out_r(v[k].c));
}

#endif  // CC_MILLER_QUAD

}  // namespace lz
}  // namespace cc

#ifdef CC_MILLER_QUAD
#if CC_MILLER_SIG == 2
#define CC_MILLER4_LAUNCH cck_miller4_lz_g2
#else
#define CC_MILLER4_LAUNCH cck_miller4_lz_g1
#endif
// four credentials per lane pair (k_miller4) over the twin layout (pstride >= ceil(n / 2)): ceil(n / 4)
// Miller values to SoA elements [foff, foff + m) of stride fstride; d_qcheck as the twin launch's
extern "C" int CC_MILLER4_LAUNCH(size_t n, size_t pstride, const uint32_t* d_prep, const uint32_t* d_flags,
                                 uint32_t* d_f, size_t fstride, size_t foff, uint32_t* d_qcheck, hipStream_t st) {
    if (!n) return 0;
    const size_t m = (n + 3) / 4;
    if (fstride < foff + m || pstride < (n + 1) / 2) return -1;
    constexpr int MB = cc::lz::MB;
    hipLaunchKernelGGL((cc::lz::k_miller4<CC_MILLER_SIG>), dim3((unsigned)((2 * m + MB - 1) / MB)), dim3(MB), 0, st, n,
                       pstride, d_prep, d_flags, d_f, fstride, foff, d_qcheck, (int)cc::lz::kAffRp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#else
#if CC_MILLER_SIG == 2
#define CC_MILLER_LAUNCH cck_miller_lz_g2
#else
#define CC_MILLER_LAUNCH cck_miller_lz_g1
#endif

// twin: two credentials per lane pair (their one pair each), one Miller value (their product) per
// two credentials; otherwise two pairs per credential.  pstride: the prep SoA's stride.  The m Miller values (m = n, twin:
// ceil(n / 2)) go to SoA elements [foff, foff + m) of stride fstride (>= foff + m); d_qcheck (twin,
// SigG2, or null): the sigma_1 subgroup tests from the loop's T
extern "C" int CC_MILLER_LAUNCH(int twin, size_t n, size_t pstride, const uint32_t* d_prep, const uint32_t* d_flags,
                                const uint32_t* d_const, uint32_t* d_f, size_t fstride, size_t foff,
                                uint32_t* d_qcheck, hipStream_t st) {
    if (!n) return 0;
    const size_t m = twin ? (n + 1) / 2 : n;
    if (fstride < foff + m || pstride < m) return -1;
    constexpr int MB = cc::lz::MB;
    dim3 g((unsigned)((2 * m + MB - 1) / MB)), b(MB);
    if (twin)
        hipLaunchKernelGGL((cc::lz::k_miller<CC_MILLER_SIG, true>), g, b, 0, st, n, pstride, d_prep, d_flags, d_const, d_f,
                           fstride, foff, d_qcheck, (int)cc::lz::kAffRp);
    else
        hipLaunchKernelGGL((cc::lz::k_miller<CC_MILLER_SIG, false>), g, b, 0, st, n, pstride, d_prep, d_flags, d_const, d_f,
                           fstride, foff, d_qcheck, (int)cc::lz::kAffRp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif  // CC_MILLER_QUAD
