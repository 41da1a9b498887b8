// Windowed Straus MSM over variable bases — device code shared by Signature::aggregate (aggregate.hip)
// and Signature::verify with per-credential verkeys (pervk.hip).  Signed radix-16 digits (65 windows),
// per base the multiples 1P..8P built in Jacobian form and batch-normalised to affine with ONE inversion
// per lane (Montgomery's trick), then 65 windows x (4 doublings + one mixed addition per base).
// Identity bases (AMCL decodes an off-curve point to infinity) and identity multiples of small-order
// points are flagged and skipped, so every input gives the reference's group element.
#pragma once
#include "codec.h"
#include "curve_lz.h"
#include "curve_pl.h"

namespace cc {

// signed radix-16 digits of a canonical 255-bit scalar: 65 digits in [-8, 8], least significant first.
// The scalar's 8 words are loaded once, up front (two 16-byte loads; k is 16-byte aligned): read
// inside the loop, every digit waited on a global load, since the digit stores may alias them.
DEV void recode_w4(int8_t* d, const uint32_t k[8]) {
    const uint4 a = reinterpret_cast<const uint4*>(k)[0], b = reinterpret_cast<const uint4*>(k)[1];
    const uint32_t kk[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    int carry = 0;
#pragma unroll
    for (int w = 0; w < 64; w++) {
        const int v = (int)((kk[w >> 3] >> (4 * (w & 7))) & 0xfu) + carry;
        carry = v > 8;
        d[w] = (int8_t)(v - 16 * carry);
    }
    d[64] = (int8_t)carry;
}

// G2 bases on the lazy pair-lane field (curve_lz.h): the same algorithm with ONE task lane per lane
// PAIR (lane 2i + h holds half h of every Fp2 coordinate) and lazy radix-2^28 arithmetic (no conversion
// per multiplication, carry-free additions, identity and exceptional cases tested on reduced values).
// The pair form keeps a Jacobian G2 point in 3 Fp a lane (2 waves/SIMD) and halves each lane's share of
// every Fp2 product; the one-lane G2 form needed 512 VGPRs.  NG pairs per task take the bases
// k = pair, pair + NG, ...  Scratch per task (lazy words, each entry's two halves side by side), laid
// out so the window loop's reads are whole cache lines: 8t entries [entry][half][32] (x at 0, y at 16,
// infinity flag at 30: one 128-byte line a half, Jacobian x, y first, affine x, y written back in
// place), then 8t Z's [entry][half][LN], 8t prefix products [entry][half][LN], 65t digit bytes; the
// task's share rounded up to 32 words (the scratch base is 256-byte aligned).
constexpr int SEW = 32, SEY = 16, SEF = 30;  // entry words, y offset, flag offset
__host__ __device__ inline size_t straus_round32(size_t w) { return (w + 31) / 32 * 32; }
__host__ __device__ inline size_t straus_lz_words(size_t t) {
    return straus_round32(t * 8 * 2 * (SEW + 2 * lz::LN) + (t * 65 + 3) / 4);
}
// 14 words from a 16-byte-aligned address as four 16-byte loads
DEV void ld16(int32_t (&v)[lz::LN], const uint32_t* w) {
    const uint4* q = reinterpret_cast<const uint4*>(w);
    uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    const uint32_t t[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
#pragma unroll
    for (int k = 0; k < lz::LN; k++) v[k] = (int32_t)t[k];
}
DEV void st_w(uint32_t* w, const lz::F2R& x) {
#pragma unroll
    for (int c = 0; c < lz::LN; c++) w[c] = (uint32_t)x.c.v[c];
}
DEV lz::F2R ld_w(const uint32_t* w) {
    lz::F2R x;
#pragma unroll
    for (int c = 0; c < lz::LN; c++) x.c.v[c] = (int32_t)w[c];
    return x;
}
// One task's share on one lane pair: multiples of its bases built and batch-normalised, then the 65
// windows over them into acc
DEV void straus_g2lz_pair(lz::JL& acc, int NG, int pair, int h, size_t task, size_t t,
                          const uint8_t* __restrict__ pts, size_t pt_stride, size_t pt_jstride, size_t pt_step,
                          const uint32_t* __restrict__ l, size_t l_div, uint32_t* __restrict__ scratch) {
    using namespace lz;
    const size_t cred = task / l_div;
    const uint8_t* base = pts + cred * pt_stride + (task % l_div) * pt_jstride;
    const uint32_t* lk = l + cred * t * 8;
    uint32_t* ent = scratch + task * straus_lz_words(t);
    uint32_t* zs = ent + t * 8 * 2 * SEW;
    uint32_t* pre = zs + t * 8 * 2 * LN;
    int8_t* dig = reinterpret_cast<int8_t*>(pre + t * 8 * 2 * LN);
    acc = jl_inf();
    F2R acc_z = r_one();
#pragma unroll 1
    for (size_t k = pair; k < t; k += NG) {
        cc::Aff<cc::Fp2> P1;
        const bool ok = pl::pair_all(g2_decode(P1, base + k * pt_step));  // both lanes decode the point
        recode_w4(dig + k * 65, lk + k * 8);                            // both write the same digits
        pl::Fp2 hx, hy;
        hx.c = h ? P1.x.b : P1.x.a;
        hy.c = h ? P1.y.b : P1.y.a;
        const AL P{reduce(in_r2(hx)), reduce(in_r2(hy))};
        JL J = ok ? jl_from_aff(P) : jl_inf();
#pragma unroll 1
        for (int d = 0; d < 8; d++) {
            if (d == 1) J = jl_dbl(J);
            else if (d > 1 && ok) J = jl_add_aff(J, P);
            const size_t e = k * 8 + d;
            uint32_t* w = ent + (e * 2 + h) * SEW;
            const bool inf = jl_is_inf(J);
            st_w(w, J.x);
            st_w(w + SEY, J.y);
            w[SEF] = inf ? 1u : 0u;
            st_w(zs + (e * 2 + h) * LN, J.z);
            st_w(pre + (e * 2 + h) * LN, acc_z);
            if (!inf) acc_z = reduce(mulr(acc_z, J.z));
        }
    }
    F2R zinv = reduce(inv(acc_z));
    if (t > (size_t)pair) {
        const long long kmax = (long long)(((t - 1 - pair) / NG) * NG + pair);
#pragma unroll 1
        for (long long kk = kmax; kk >= pair; kk -= NG) {
#pragma unroll 1
            for (int d = 7; d >= 0; d--) {
                const size_t e = (size_t)kk * 8 + d;
                uint32_t* w = ent + (e * 2 + h) * SEW;
                if (w[SEF]) continue;  // identity multiple (pair-uniform: both halves carry the flag)
                const F2R z = ld_w(zs + (e * 2 + h) * LN);
                const auto zi = mulr(zinv, ld_w(pre + (e * 2 + h) * LN));
                zinv = reduce(mulr(zinv, z));
                const auto zi2 = sqrr(zi);
                st_w(w, reduce(mulr(ld_w(w), zi2)));
                st_w(w + SEY, reduce(mulr(ld_w(w + SEY), mulr(zi2, zi))));
            }
        }
    }
#pragma unroll 1
    for (int win = 64; win >= 0; win--) {
        if (win != 64 && !jl_is_inf(acc))
#pragma unroll 1
            for (int z = 0; z < 4; z++) acc = jl_dbl(acc);
#pragma unroll 1
        for (size_t k = pair; k < t; k += NG) {
            const int d = dig[k * 65 + win];
            if (!d) continue;
            const uint32_t* w = ent + ((k * 8 + (d < 0 ? -d : d) - 1) * 2 + h) * SEW;
            if (w[SEF]) continue;  // identity multiple
            AL e;
            ld16(e.x.c.v, w);
            ld16(e.y.c.v, w + SEY);
            if (d < 0) e = jl_neg_aff(e);
            acc = jl_add_aff(acc, e);
        }
    }
}

// G1 bases on the lazy field, one task share per LANE (curve_lz.h JG: squarings on the upper triangle,
// carry-free additions, coordinates at rest reduced).  NG lanes per task take the bases k = part,
// part + NG, ...  Scratch per task (lazy words): 8t Jacobian entries [entry][3 LN + 1] (x, y, z,
// infinity flag; affine x, y written back in place), 8t prefix products [entry][LN], 65t digit bytes —
// entries as in straus_g2lz_pair: [entry][32] (x at 0, y at 16, flag at 30), Z's apart.
// Bases: t encodings of 97 bytes at pts; scalars: t canonical 8-word little-endian values at scal.
__host__ __device__ inline size_t straus_g1lz_words(size_t t) {
    return straus_round32(t * 8 * (SEW + 2 * lz::LN) + (t * 65 + 3) / 4);
}
DEV void st_r1(uint32_t* w, const lz::FR& x) {
#pragma unroll
    for (int c = 0; c < lz::LN; c++) w[c] = (uint32_t)x.v[c];
}
DEV lz::FR ld_r1(const uint32_t* w) {
    lz::FR x;
#pragma unroll
    for (int c = 0; c < lz::LN; c++) x.v[c] = (int32_t)w[c];
    return x;
}
// an affine point with reduced coordinates as the mixed addition's operand
DEV lz::AG ag_of(const lz::FR& x, const lz::FR& y) { return {lz::fit<lz::AN, lz::BC>(x), lz::fit<lz::AN, lz::BC>(y)}; }

DEV void straus_g1lz_lane(lz::JG& acc, int NG, int part, size_t t, const uint8_t* __restrict__ pts,
                          const uint32_t* __restrict__ scal, uint32_t* __restrict__ ent) {
    using namespace lz;
    uint32_t* zs = ent + t * 8 * SEW;
    uint32_t* pre = zs + t * 8 * LN;
    int8_t* dig = reinterpret_cast<int8_t*>(pre + t * 8 * LN);
    acc = jg_inf();
    FR acc_z = r1_one();
#pragma unroll 1
    for (size_t k = part; k < t; k += NG) {
        cc::Aff<cc::Fp> P1;
        const bool ok = g1_decode(P1, pts + k * 97);
        recode_w4(dig + k * 65, scal + k * 8);
        const FR px = reduce(in_r(P1.x)), py = reduce(in_r(P1.y));
        const AG P = ag_of(px, py);
        JG J = ok ? JG{px, py, r1_one()} : jg_inf();
#pragma unroll 1
        for (int d = 0; d < 8; d++) {
            if (d == 1) J = jg_dbl(J);
            else if (d > 1 && ok) J = jg_add_aff(J, P);
            const size_t e = k * 8 + d;
            uint32_t* w = ent + e * SEW;
            const bool inf = jg_is_inf(J);
            st_r1(w, J.x);
            st_r1(w + SEY, J.y);
            w[SEF] = inf ? 1u : 0u;
            st_r1(zs + e * LN, J.z);
            st_r1(pre + e * LN, acc_z);
            if (!inf) acc_z = reduce(mulr1(acc_z, J.z));
        }
    }
    // one inversion (the storage form's divsteps), then walk back: z_e^-1 = inv * prefix_e; inv *= z_e
    cc::Fp zinv_s;
    fp_inv(zinv_s, out_r(acc_z));
    FR zinv = reduce(in_r(zinv_s));
    if (t > (size_t)part) {
        const long long kmax = (long long)(((t - 1 - part) / NG) * NG + part);
#pragma unroll 1
        for (long long kk = kmax; kk >= part; kk -= NG) {
#pragma unroll 1
            for (int d = 7; d >= 0; d--) {
                const size_t e = (size_t)kk * 8 + d;
                uint32_t* w = ent + e * SEW;
                if (w[SEF]) continue;  // identity multiple
                const FR z = ld_r1(zs + e * LN);
                const FR zi = reduce(mulr1(zinv, ld_r1(pre + e * LN)));
                zinv = reduce(mulr1(zinv, z));
                const FR zi2 = reduce(sqrr1(zi));
                st_r1(w, reduce(mulr1(ld_r1(w), zi2)));
                st_r1(w + SEY, reduce(mulr1(ld_r1(w + SEY), mulr1(zi2, zi))));
            }
        }
    }
#pragma unroll 1
    for (int win = 64; win >= 0; win--) {
        if (win != 64 && !jg_is_inf(acc))
#pragma unroll 1
            for (int z = 0; z < 4; z++) acc = jg_dbl(acc);
#pragma unroll 1
        for (size_t k = part; k < t; k += NG) {
            const int d = dig[k * 65 + win];
            if (!d) continue;
            const uint32_t* w = ent + (k * 8 + (d < 0 ? -d : d) - 1) * SEW;
            if (w[SEF]) continue;  // identity multiple
            FR ex, ey;
            ld16(ex.v, w);
            ld16(ey.v, w + SEY);
            acc = jg_add_aff(acc, ag_of(ex, d < 0 ? neg(ey) : ey));
        }
    }
}

}  // namespace cc
