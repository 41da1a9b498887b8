// The g~-side fold of the RLC batch mode (BASELINE config 3) for gfx950.
//
// RLC checks prod_i e(sigma_1,i, delta_i pr_i) e(-sigma_2,i, delta_i g~) == 1 (SigG2; SigG1 swaps the
// pairing arguments, rlc.hip).  The second factors share g~, so
//     prod_i e(-sigma_2,i, delta_i g~) = e(sum_i delta_i (-sigma_2,i), g~).
// delta_i is drawn as 16 signed base-256 digits d_w,i in [-128, 127] (fr.h rlc_delta_signed), so
//     sum_i delta_i X_i = sum_w sum_{d=1..128} (256^w d) B_w,d,   B_w,d = sum_{i: |d_w,i| = d} sign X_i
// and instead of ONE sequential Horner combination over all 16 windows (~2k dependent Fp
// multiplications on one lane, milliseconds of latency) each window is combined on its own wave and
// the window weights 256^w move to the OTHER pairing argument, whose points P_w = (256^w) g~ are fixed
// per verkey:
//     prod = prod_w e(S_w, P_w),   S_w = sum_{d=1..128} d B_w,d      (16 one-pair pseudo-credentials)
// S_w is a bucket-method sum spread over the wave's lanes (k_fold_window): lane t takes the CK
// digits d = CK t + k + 1 and forms U_t = sum_k (k + 1) B and T_t = sum_k B by running sums, then
// U_t + [CK t] T_t; a butterfly adds the lanes.  The per-credential Miller loop keeps pair 0 only and
// runs two credentials per shared-squaring loop (miller_lz.hip kTwin); the fold costs ~16 mixed
// additions per credential (one per window) and ~30 point operations per window lane.
//
//   k_fold_count / k_fold_scan / k_fold_scatter : counting sort of the (w, i) digits into 2,048
//                                                 bucket lists, each padded to FS-entry chunks
//   k_fold_sum_g1                               : one lane per chunk: mixed additions of its points
//                                                 (lazy field: the fold points come in its form)
//   k_fold_reduce<F>                            : one wave per bucket: chunk partials, butterfly
//   k_fold_window                               : one wave per window: S_w (lazy field), affine
//   k_fold_sum_g2pl / k_fold_reduce_g2pl /      : the same for G2 buckets (SigG2) on the pair-lane
//   k_fold_window_g2pl                            Fp2 (curve_pl.h): one LANE PAIR per chunk / 32 pairs
//                                                 per bucket or window, 2 waves/SIMD where the one-lane
//                                                 G2 forms need 448-512 registers (1 wave/SIMD)
//   k_fold_fixed<F>                             : the fixed points P_w (once per verkey, cck_fold_fixed)
// X_i = -sigma_2,i (AoS affine in the lazy field's form, fixed.h fp_to_lazy_form; written by the RLC
// prep); S_w lands in the shard's partial (rlc_part.h: affine words + identity flag per window), and
// the finish pairs every shard's S_w with P_w (rlc.hip k_rlc_gather, then k_miller_wide): SigG2 S in
// G2 (the Q side), SigG1 S in G1 (the P side), P_w on the other side.
#include "codec.h"
#include "curve_pl.h"
#include "fixed.h"
#include "rlc_part.h"
#include "soa.h"

using namespace cc;

namespace {

constexpr int FW = RLC_WINDOWS;  // windows: signed base-256 digits of delta
constexpr int FD = 128;       // |digit| values per window
constexpr int FB = FW * FD;   // buckets
constexpr int FS = 16;        // list entries per chunk (one lane)
constexpr uint32_t PAD = 0xffffffffu;

template <class F>
DEV void ld_aff_aos(Aff<F>& a, const uint32_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4* d = reinterpret_cast<uint4*>(&a);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(Aff<F>) / 16); k++) d[k] = q[k];
}
template <class F>
DEV void st_jac_aos(uint32_t* p, const Jac<F>& a) {
    uint4* q = reinterpret_cast<uint4*>(p);
    const uint4* s = reinterpret_cast<const uint4*>(&a);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(Jac<F>) / 16); k++) q[k] = s[k];
}
template <class F>
DEV void ld_jac_aos(Jac<F>& a, const uint32_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4* d = reinterpret_cast<uint4*>(&a);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(Jac<F>) / 16); k++) d[k] = q[k];
}

// a point as the pair argument of a pseudo-credential: Q (affine G2, slots Q1) or P (G1, evaluation
// form (x, y, 1), slots P1)
DEV void st_as_q(const Soa& S, size_t j, const Aff<Fp2>& a) {
    st_f2(S, S_Q1, j, a.x);
    st_f2(S, S_Q1 + 2, j, a.y);
}
DEV void st_as_p(const Soa& S, size_t j, const Aff<Fp>& a) {
    const int s = S_P1;
    Fp one;
    fp_one(one);
    st_fp(S, s, j, a.x);
    st_fp(S, s + 1, j, a.y);
    st_fp(S, s + 2, j, one);
}

}  // namespace

// per-window histograms of |digit| (LDS, then one global add per bucket and block)
__global__ __launch_bounds__(256) void k_fold_count(size_t n, const int8_t* __restrict__ dig,
                                                    uint32_t* __restrict__ cnt) {
    __shared__ uint32_t h[FD];
    const int w = blockIdx.y;
    for (int t = threadIdx.x; t < FD; t += blockDim.x) h[t] = 0;
    __syncthreads();
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int d = dig[(size_t)w * n + i];
        if (d) atomicAdd(&h[(d < 0 ? -d : d) - 1], 1u);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < FD; t += blockDim.x)
        if (h[t]) atomicAdd(&cnt[w * FD + t], h[t]);
}

// padded bucket offsets (off[FB] = total) and scatter cursors; one block
__global__ __launch_bounds__(256) void k_fold_scan(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ off,
                                                   uint32_t* __restrict__ cur) {
    constexpr int PT = FB / 256;
    __shared__ uint32_t s[256];
    const int t = threadIdx.x;
    uint32_t loc[PT], pc[PT], sum = 0;
#pragma unroll
    for (int k = 0; k < PT; k++) {
        pc[k] = (cnt[t * PT + k] + FS - 1) / FS * FS;
        loc[k] = sum;
        sum += pc[k];
    }
    s[t] = sum;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const uint32_t v = t >= o ? s[t - o] : 0u;
        __syncthreads();
        s[t] += v;
        __syncthreads();
    }
    const uint32_t base = t ? s[t - 1] : 0u;
#pragma unroll
    for (int k = 0; k < PT; k++) {
        const int b = t * PT + k;
        const uint32_t o = base + loc[k];
        off[b] = o;
        cur[b] = o;
    }
    if (t == 255) off[FB] = s[255];
}

// list[pos] = i | sign << 31 for every nonzero digit (order inside a bucket is irrelevant: sums)
__global__ __launch_bounds__(256) void k_fold_scatter(size_t n, const int8_t* __restrict__ dig,
                                                      uint32_t* __restrict__ cur, uint32_t* __restrict__ list) {
    const int w = blockIdx.y;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int d = dig[(size_t)w * n + i];
        if (!d) continue;
        const uint32_t pos = atomicAdd(&cur[w * FD + (d < 0 ? -d : d) - 1], 1u);
        list[pos] = (uint32_t)i | (d < 0 ? 0x80000000u : 0u);
    }
}

// one lane per FS-entry chunk (all of one bucket): Jacobian partial sum of its signed G1 points (the
// fold points are in the lazy field's form: mixed additions on the lazy field, curve_lz.h), written in
// the storage form
__global__ __launch_bounds__(256) void k_fold_sum_g1(size_t maxchunks, const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ pts, uint32_t* __restrict__ part) {
    constexpr int AW = sizeof(Aff<Fp>) / 4, JW = sizeof(Jac<Fp>) / 4;
    const size_t c = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (c >= maxchunks || c * FS >= off[FB]) return;
    lz::JG acc = lz::jg_inf();
#pragma unroll 1
    for (int e = 0; e < FS; e++) {
        const uint32_t v = list[c * FS + e];
        if (v == PAD) continue;
        Aff<Fp> a;
        ld_aff_aos<Fp>(a, pts + (size_t)(v & 0x7fffffffu) * AW);
        const auto y = lz::from_fp(a.y);
        acc = lz::jg_add_aff(acc, lz::AG{lz::from_fp(a.x), lz::sel((v >> 31) != 0, lz::neg(y), y)});
    }
    st_jac_aos<Fp>(part + c * JW, lz::jg_to(acc));
}

// one wave per bucket: lane-strided sum of the bucket's chunk partials, butterfly across the wave;
// the Jacobian sum B_b goes to bkt (AoS, JW words a bucket)
template <class F>
__global__ __launch_bounds__(64) void k_fold_reduce(const uint32_t* __restrict__ off, const uint32_t* __restrict__ part,
                                                    uint32_t* __restrict__ bkt) {
    constexpr int JW = sizeof(Jac<F>) / 4;
    const int b = blockIdx.x;
    const uint32_t c0 = off[b] / FS, c1 = off[b + 1] / FS;
    Jac<F> acc;
    jac_set_inf(acc);
#pragma unroll 1
    for (uint32_t c = c0 + threadIdx.x; c < c1; c += 64) {
        Jac<F> p;
        ld_jac_aos<F>(p, part + (size_t)c * JW);
        jac_add(acc, acc, p);
    }
    lane_group_sum<F, 64>(acc);
    if (threadIdx.x == 0) st_jac_aos<F>(bkt + (size_t)b * JW, acc);
}

// one wave per window (one lane per CK = 2 digits): lane t's share of S_w = sum_d d B_d over the
// digits d = CK t + k + 1 (k < CK) is U + [CK t] T with U = sum_k (k + 1) B and T = sum_k B (running
// sums from the top digit down), on the lazy field; a butterfly adds the lanes.  S_w (SigG1: in G1),
// affine, and its identity flag go to the partial's window w (rlc_part.h)
__global__ __launch_bounds__(64) void k_fold_window(const uint32_t* __restrict__ bkt, uint32_t* __restrict__ part) {
    constexpr int JW = sizeof(Jac<Fp>) / 4, CK = FD / 64;
    const int w = blockIdx.x, t = threadIdx.x;
    lz::JG run = lz::jg_inf(), u = lz::jg_inf(), v = lz::jg_inf();
#pragma unroll 1
    for (int k = CK - 1; k >= 0; k--) {
        Jac<Fp> b;
        ld_jac_aos<Fp>(b, bkt + (size_t)(w * FD + CK * t + k) * JW);
        run = lz::jg_add(run, lz::jg_from(b));
        u = lz::jg_add(u, run);
    }
#pragma unroll 1
    for (int s = 5; s >= 0; s--) {  // [t] run (t < 64), then [CK] of it
        v = lz::jg_dbl(v);
        if ((t >> s) & 1) v = lz::jg_add(v, run);
    }
#pragma unroll 1
    for (int c = 1; c < CK; c <<= 1) v = lz::jg_dbl(v);
    Jac<Fp> acc = lz::jg_to(lz::jg_add(u, v));
    lane_group_sum<Fp, 64>(acc);
    if (threadIdx.x != 0) return;
    Aff<Fp> a;
    const bool fin = jac_to_aff(a, acc);
    uint32_t* o = part + RLC_WIN_OFF + RLC_WIN_WORDS * w;
#pragma unroll
    for (int k = 0; k < NL; k++) {
        o[k] = fin ? a.x.v[k] : 0u;
        o[NL + k] = fin ? a.y.v[k] : 0u;
        o[2 * NL + k] = 0u;
        o[3 * NL + k] = 0u;
    }
    o[4 * NL] = fin ? 0u : 1u;  // e(O, .) = 1: the finish skips the pair
}

// k_fold_sum for G2 points on the pair-lane Fp2: one lane pair per chunk, each lane adds its halves.
// part: chunk c's partial at c * 72 words, lane h's half (X, Y, Z halves: 36 words) at + 36 h.
__global__ __launch_bounds__(256, 2) void k_fold_sum_g2pl(size_t maxchunks, const uint32_t* __restrict__ off,
                                                          const uint32_t* __restrict__ list,
                                                          const uint32_t* __restrict__ pts,
                                                          uint32_t* __restrict__ part) {
    constexpr int AW = sizeof(Aff<Fp2>) / 4, JW = sizeof(Jac<Fp2>) / 4, HW = sizeof(Jac<pl::Fp2>) / 4;
    const size_t c = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 1;  // pair-uniform
    const int h = (int)pl::half_id();
    if (c >= maxchunks || c * FS >= off[FB]) return;
    lz::JL acc = lz::jl_inf();  // the lazy pair-lane field (curve_lz.h); the points are in its form
#pragma unroll 1
    for (int e = 0; e < FS; e++) {
        const uint32_t v = list[c * FS + e];  // pair-uniform
        if (v == PAD) continue;
        const uint32_t* p = pts + (size_t)(v & 0x7fffffffu) * AW;
        Fp x, y;
#pragma unroll
        for (int k = 0; k < NL; k++) {
            x.v[k] = p[NL * h + k];
            y.v[k] = p[2 * NL + NL * h + k];
        }
        const lz::F2<lz::AN, lz::BC> ly{lz::from_fp(y)};
        const lz::F2<lz::AN, lz::BC> qy{lz::sel((v >> 31) != 0, lz::neg(ly).c, ly.c)};
        acc = lz::jl_add_aff_c(acc, lz::F2<lz::AN, lz::BC>{lz::from_fp(x)}, qy);
    }
    st_jac_aos<pl::Fp2>(part + c * JW + h * HW, pl::jl_to_pl(acc));
}

// k_fold_reduce<Fp2> on the pair-lane Fp2: one wave (32 lane pairs) per bucket; bkt as part
__global__ __launch_bounds__(64, 2) void k_fold_reduce_g2pl(const uint32_t* __restrict__ off,
                                                           const uint32_t* __restrict__ part,
                                                           uint32_t* __restrict__ bkt) {
    constexpr int JW = sizeof(Jac<Fp2>) / 4, HW = sizeof(Jac<pl::Fp2>) / 4;
    const int b = blockIdx.x;
    const int h = (int)pl::half_id();
    const uint32_t c0 = off[b] / FS, c1 = off[b + 1] / FS;
    Jac<pl::Fp2> acc;
    jac_set_inf(acc);
#pragma unroll 1
    for (uint32_t c = c0 + (threadIdx.x >> 1); c < c1; c += 32) {
        Jac<pl::Fp2> p;
        ld_jac_aos<pl::Fp2>(p, part + (size_t)c * JW + h * HW);
        jac_add(acc, acc, p);
    }
    pl::pair_group_sum<64>(acc);
    if (threadIdx.x < 2) st_jac_aos<pl::Fp2>(bkt + (size_t)b * JW + h * HW, acc);
}

// k_fold_window for G2 buckets on the pair-lane Fp2 (one lane pair per CK = 4 digits), S_w in G2
// (SigG2).  The lane pair's share runs on the lazy pair-lane field (curve_lz.h): latency-bound (16
// waves), and beside the delta MSM's waves every dependent step counts.  Lane h of pair 0 writes the
// h-halves (x.a / x.b, y.a / y.b) of the partial's window w.
__global__ __launch_bounds__(64, 2) void k_fold_window_g2pl(const uint32_t* __restrict__ bkt, uint32_t* __restrict__ part) {
    constexpr int JW = sizeof(Jac<Fp2>) / 4, HW = sizeof(Jac<pl::Fp2>) / 4, CK = FD / 32;
    const int w = blockIdx.x, t = threadIdx.x >> 1;  // pair-uniform
    const int h = (int)pl::half_id();
    lz::JL run = lz::jl_inf(), u = lz::jl_inf(), v = lz::jl_inf();
#pragma unroll 1
    for (int k = CK - 1; k >= 0; k--) {  // running sums: run = sum B, u = sum (k + 1) B
        Jac<pl::Fp2> b;
        ld_jac_aos<pl::Fp2>(b, bkt + (size_t)(w * FD + CK * t + k) * JW + h * HW);
        run = lz::jl_add(run, pl::jl_from_pl(b));
        u = lz::jl_add(u, run);
    }
#pragma unroll 1
    for (int s = 4; s >= 0; s--) {  // [t] run (t < 32), then [CK] of it
        v = lz::jl_dbl(v);
        if ((t >> s) & 1) v = lz::jl_add(v, run);
    }
#pragma unroll 1
    for (int c = 1; c < CK; c <<= 1) v = lz::jl_dbl(v);
    Jac<pl::Fp2> acc = pl::jl_to_pl(lz::jl_add(u, v));
    pl::pair_group_sum<64>(acc);
    if (threadIdx.x >= 2) return;
    Aff<pl::Fp2> a;
    const bool fin = jac_to_aff(a, acc);  // pair-uniform
    uint32_t* o = part + RLC_WIN_OFF + RLC_WIN_WORDS * w;
#pragma unroll
    for (int k = 0; k < NL; k++) {
        o[NL * h + k] = fin ? a.x.c.v[k] : 0u;
        o[2 * NL + NL * h + k] = fin ? a.y.c.v[k] : 0u;
    }
    if (!h) o[4 * NL] = fin ? 0u : 1u;  // e(O, .) = 1: the finish skips the pair
}

// P_w = (256^w) g~ from g~'s fixed-base table (base index q of the verkey tables); G is g~'s field
template <class G>
__global__ __launch_bounds__(64) void k_fold_fixed(int q, const uint32_t* __restrict__ table, int wbits,
                                                   const uint32_t* __restrict__ binf, uint32_t* __restrict__ pw,
                                                   uint8_t* __restrict__ fixed_inf) {
    const int w = threadIdx.x;
    if (w >= FW) return;
    uint32_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    s[w >> 2] = 1u << (8 * (w & 3));
    Jac<G> acc;
    jac_set_inf(acc);
    if (!binf[q]) ft_add<G>(acc, s, table, wbits, q, 0, ft_nwin(wbits), true);  // the verkey table: lazy form
    Aff<G> a;
    const bool fin = jac_to_aff(a, acc);
    fixed_inf[w] = fin ? 0 : 1;
    const Soa S{pw, FW};
    if constexpr (sizeof(G) == sizeof(Fp)) st_as_p(S, w, a);  // SigG2: g~ in G1
    else st_as_q(S, w, a);                                     // SigG1: g~ in G2
}

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

// work-buffer layout (32-bit words): cnt FB | off FB+1 | cur FB (+3) | list maxchunks*FS |
// part maxchunks*JW (16-byte aligned) | bkt FB*JW
static size_t fold_maxchunks(size_t n) { return (FW * n + (size_t)FB * (FS - 1)) / FS + 1; }
struct FoldWork {
    uint32_t *cnt, *off, *cur, *list, *part, *bkt;
};
static FoldWork fold_work(int mode, size_t n, uint32_t* d_work) {
    const size_t mc = fold_maxchunks(n);
    FoldWork w;
    w.cnt = d_work;
    w.off = w.cnt + FB;
    w.cur = w.off + FB + 1;
    w.list = w.cur + FB + 3;
    w.part = reinterpret_cast<uint32_t*>(((uintptr_t)(w.list + mc * FS) + 15) & ~(uintptr_t)15);
    w.bkt = w.part + mc * (mode == 0 ? sizeof(Jac<Fp2>) / 4 : sizeof(Jac<Fp>) / 4);
    return w;
}

extern "C" {

size_t cck_fold_words(int mode, size_t n) {
    const size_t jw = mode == 0 ? sizeof(Jac<Fp2>) / 4 : sizeof(Jac<Fp>) / 4;
    const size_t mc = fold_maxchunks(n);
    return 3 * (size_t)FB + 1 + 3 + mc * FS + mc * jw + 4 + (size_t)FB * jw;
}

int cck_fold_pseudo() { return FW; }

// P_w = (256^w) g~, w < 16, from the verkey tables (g~ = base q): d_pw (PREP_SLOTS x FW SoA, soa.h:
// SigG2 the P side in evaluation form (x, y, 1), SigG1 the Q side) and their identity flags d_finf
// (FW bytes); once per verkey (cc_set_verkey), read by every finish
int cck_fold_fixed(int mode, int q, const uint32_t* d_table, int wbits, const uint32_t* d_binf, uint32_t* d_pw,
                   uint8_t* d_finf, hipStream_t st) {
    if (mode == 0)
        hipLaunchKernelGGL(k_fold_fixed<Fp>, dim3(1), dim3(64), 0, st, q, d_table, wbits, d_binf, d_pw, d_finf);
    else
        hipLaunchKernelGGL(k_fold_fixed<Fp2>, dim3(1), dim3(64), 0, st, q, d_table, wbits, d_binf, d_pw, d_finf);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// mode 0 (SigG2): X_i in G2 (AoS affine, 48 words); mode 1: X_i in G1 (24 words).
// d_dig: [FW][n] int8 digits (0 for credentials to leave out).  The bucket sums; cck_fold_window, which
// the host launches after this, forms the window sums.
int cck_fold(int mode, size_t n, const int8_t* d_dig, const uint32_t* d_pts, uint32_t* d_work, hipStream_t st) {
    if (!n) return -1;
    const size_t mc = fold_maxchunks(n);
    const FoldWork fw = fold_work(mode, n, d_work);
    uint32_t *cnt = fw.cnt, *off = fw.off, *cur = fw.cur, *list = fw.list, *part = fw.part, *bkt = fw.bkt;
    if (hipMemsetAsync(cnt, 0, FB * 4, st) != hipSuccess || hipMemsetAsync(list, 0xff, mc * FS * 4, st) != hipSuccess)
        return -1;
    const dim3 gw(nblocks(n, 256) < 64 ? nblocks(n, 256) : 64, FW);
    hipLaunchKernelGGL(k_fold_count, gw, dim3(256), 0, st, n, d_dig, cnt);
    hipLaunchKernelGGL(k_fold_scan, dim3(1), dim3(256), 0, st, cnt, off, cur);
    hipLaunchKernelGGL(k_fold_scatter, gw, dim3(256), 0, st, n, d_dig, cur, list);
    if (mode == 0) {
        hipLaunchKernelGGL(k_fold_sum_g2pl, dim3(nblocks(2 * mc, 256)), dim3(256), 0, st, mc, off, list, d_pts, part);
        hipLaunchKernelGGL(k_fold_reduce_g2pl, dim3(FB), dim3(64), 0, st, off, part, bkt);
    } else {
        hipLaunchKernelGGL(k_fold_sum_g1, dim3(nblocks(mc, 256)), dim3(256), 0, st, mc, off, list, d_pts, part);
        hipLaunchKernelGGL(k_fold_reduce<Fp>, dim3(FB), dim3(64), 0, st, off, part, bkt);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the fold's last step, after cck_fold (16 waves, latency-bound: the host runs it beside other
// work): the window sums S_w into the partial's window section (rlc_part.h)
int cck_fold_window(int mode, size_t n, uint32_t* d_work, uint32_t* d_partial, hipStream_t st) {
    if (!n) return -1;
    uint32_t* bkt = fold_work(mode, n, d_work).bkt;
    if (mode == 0)
        hipLaunchKernelGGL(k_fold_window_g2pl, dim3(FW), dim3(64), 0, st, bkt, d_partial);
    else
        hipLaunchKernelGGL(k_fold_window, dim3(FW), dim3(64), 0, st, bkt, d_partial);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
