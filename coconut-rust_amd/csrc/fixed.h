// Fixed-base window tables — device code shared by the prep, RLC, PoK and aggregation kernels.
//
// The verifier's MSMs (multi_scalar_mul_var_time over X~, Y~_j, g~) have FIXED
// bases per verkey, so cc_set_verkey precomputes, per base B, nwin = ceil(256 / wbits) windows of the
// 2^wbits - 1 affine multiples d * 2^(wbits w) * B (AoS, Montgomery).  A scalar multiplication is then
// nwin mixed additions and no doublings.  The shared-verkey tables use the widest of wbits = 22 / 20 /
// 16 that fits the HBM budget (capi.cpp rebuild_tables; 22 bits: 12 windows, 4.8 GB per G1 base — the
// tables live in HBM and every lookup is one random 96/192-byte read, which the ~8 TB/s HBM serves far
// faster than the VALU-bound additions consume them); the issuer tables (hundreds of bases) take the widest window
// in {16, 13, 12, 10, 8} whose tables fit a memory budget (cc_set_issuers), the one-off
// cc_fixed_base_mul wbits = 8.
// An entry equal to the identity (only possible for a small-order base) is stored as (0, 0), which
// lies on neither curve, and skipped.
#pragma once
#include <type_traits>
#include "curve.h"
#include "curve_lz.h"

namespace cc {

__host__ __device__ constexpr int ft_nwin(int wbits) { return (256 + wbits - 1) / wbits; }
__host__ __device__ constexpr size_t ft_went(int wbits) { return ((size_t)1 << wbits) - 1; }
// words of one base's table
template <class F>
__host__ __device__ constexpr size_t ft_base_words(int wbits) {
    return (size_t)ft_nwin(wbits) * ft_went(wbits) * (sizeof(Aff<F>) / 4);
}

// window w of a canonical scalar given as 8 little-endian 32-bit limbs (wbits in [8, 22])
DEV uint32_t ft_digit(const uint32_t k[8], int w, int wbits) {
    if (wbits == 16) return (k[w >> 1] >> (16 * (w & 1))) & 0xffffu;
    if (wbits == 8) return (k[w >> 2] >> (8 * (w & 3))) & 0xffu;
    const int o = w * wbits, i = o >> 5, sh = o & 31;
    uint32_t v = k[i] >> sh;
    if (sh && i + 1 < 8) v |= k[i + 1] << (32 - sh);
    return v & ((1u << wbits) - 1u);
}

template <class F>
DEV void ft_load(Aff<F>& a, const uint32_t* p) {
    constexpr int W = sizeof(Aff<F>) / 16;
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4* d = reinterpret_cast<uint4*>(&a);
#pragma unroll
    for (int k = 0; k < W; k++) d[k] = q[k];
}

template <class F>
DEV bool ft_is_empty(const Aff<F>& a) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&a);
    uint32_t o = 0;
#pragma unroll
    for (int c = 0; c < (int)(sizeof(Aff<F>) / 4); c++) o |= w[c];
    return o == 0;
}

// G1 tables hold their entries in the lazy field's Montgomery form (x R' mod p, R' = 2^392, canonical
// 12 x 32 words; k_table_fill rescales them), so the lazy G1 mixed addition (curve_lz.h) loads an
// entry with shifts only.  acc += (k over windows [w0, w1)) * B_j on a lazy accumulator:
DEV void ft_add_lz(lz::JG& acc, const uint32_t k[8], const uint32_t* __restrict__ table, int wbits, int j, int w0,
                   int w1, bool negate = false) {  // negate: acc -= k B_j
    constexpr int EW = sizeof(Aff<Fp>) / 4;
    const size_t went = ft_went(wbits);
    const uint32_t* tj = table + (size_t)j * ft_base_words<Fp>(wbits);
#pragma unroll 1
    for (int w = w0; w < w1; w++) {
        const uint32_t d = ft_digit(k, w, wbits);
        if (!d) continue;
        Aff<Fp> e;
        ft_load<Fp>(e, tj + ((size_t)w * went + d - 1) * EW);
        if (ft_is_empty(e)) continue;
        const auto y = lz::from_fp(e.y);
        acc = lz::jg_add_aff(acc, lz::AG{lz::from_fp(e.x), negate ? lz::neg(y) : y});
    }
}

// storage form (x R, R = 2^406, canonical) -> the lazy field's form as a canonical 12 x 32 value
// (x R', R' = 2^392): fp_mul by 2^392 mod p.  Table entries and the RLC fold's points are stored so,
// and the lazy sums read them with from_fp alone.
DEV void fp_to_lazy_form(Fp& v) {
    constexpr uint32_t C[NL] = {0x0347fcb8u, 0x19d80000u, 0x6d2002b1u, 0x12e00cdeu, 0xa2090c72u, 0x37669f83u,
                                0xda0f73e0u, 0x09b09b42u, 0x8f1297bbu, 0xa7c515d9u, 0xfcfa012cu, 0x0577a659u};  // 2^392 mod p
    Fp c;
#pragma unroll
    for (int j = 0; j < NL; j++) c.v[j] = C[j];
    fp_mul(v, v, c);
}

// a G2 entry of a lazy-form table back to the storage form (one-lane consumers of the verkey tables:
// the RLC fold's fixed points in SigG1 mode): x R' -> x R, times 2^14 = R^2 / R' (fp_mul by 2^420 mod p)
DEV void g2_entry_from_lazy_form(Aff<Fp2>& e) {
    constexpr uint32_t C[NL] = {0x8e9f9aecu, 0x977080eau, 0x16d8fe47u, 0x26e7d667u, 0xfb088639u, 0xaca5f496u,
                                0x7416d1f5u, 0xbca6d4cfu, 0xb5b6168du, 0xdaab0ee4u, 0x403d5566u, 0x14820974u};
    Fp c;
#pragma unroll
    for (int i = 0; i < NL; i++) c.v[i] = C[i];
    fp_mul(e.x.a, e.x.a, c);
    fp_mul(e.x.b, e.x.b, c);
    fp_mul(e.y.a, e.y.a, c);
    fp_mul(e.y.b, e.y.b, c);
}

// acc += (k restricted to windows [w0, w1)) * B_j; lazy_g2: a G2 table in the lazy form (the verkey and
// issuer tables; cc_fixed_base_mul's tables are in the storage form)
template <class F>
DEV void ft_add(Jac<F>& acc, const uint32_t k[8], const uint32_t* __restrict__ table, int wbits, int j, int w0,
                int w1, bool lazy_g2 = false) {
    if constexpr (std::is_same<F, Fp>::value) {  // G1: on the lazy field, storage form at the boundary
        lz::JG a = lz::jg_from(acc);
        ft_add_lz(a, k, table, wbits, j, w0, w1);
        acc = lz::jg_to(a);
    } else {
        constexpr int EW = sizeof(Aff<F>) / 4;
        const size_t went = ft_went(wbits);
        const uint32_t* tj = table + (size_t)j * ft_base_words<F>(wbits);
#pragma unroll 1
        for (int w = w0; w < w1; w++) {
            const uint32_t d = ft_digit(k, w, wbits);
            if (!d) continue;
            Aff<F> e;
            ft_load<F>(e, tj + ((size_t)w * went + d - 1) * EW);
            if (ft_is_empty(e)) continue;
            if constexpr (std::is_same<F, Fp2>::value)
                if (lazy_g2) g2_entry_from_lazy_form(e);
            jac_add_aff(acc, acc, e);
        }
    }
}

}  // namespace cc
