// Structure-of-arrays operand layout shared by the verify kernels: slot-major,
// limb-major u32 words, `n` lanes per limb, so each limb access of a wave is 256 contiguous bytes.
#pragma once
#include "field.h"

namespace cc {

struct Soa {
    uint32_t* p;
    size_t n;  // stride between limbs (= batch capacity)
};

DEV void st_fp(const Soa& s, int slot, size_t i, const Fp& x) {
#pragma unroll
    for (int k = 0; k < NL; k++) s.p[((size_t)slot * NL + k) * s.n + i] = x.v[k];
}
DEV void ld_fp(Fp& x, const Soa& s, int slot, size_t i) {
#pragma unroll
    for (int k = 0; k < NL; k++) x.v[k] = s.p[((size_t)slot * NL + k) * s.n + i];
}
DEV void st_f2(const Soa& s, int slot, size_t i, const Fp2& x) { st_fp(s, slot, i, x.a); st_fp(s, slot + 1, i, x.b); }
DEV void ld_f2(Fp2& x, const Soa& s, int slot, size_t i) { ld_fp(x.a, s, slot, i); ld_fp(x.b, s, slot + 1, i); }

DEV void st_f12(const Soa& s, size_t i, const Fp12& x) {
    const Fp* v = reinterpret_cast<const Fp*>(&x);
#pragma unroll
    for (int k = 0; k < 12; k++) st_fp(s, k, i, v[k]);
}
DEV void ld_f12(Fp12& x, const Soa& s, size_t i) {
    Fp* v = reinterpret_cast<Fp*>(&x);
#pragma unroll
    for (int k = 0; k < 12; k++) ld_fp(v[k], s, k, i);
}

DEV void ld_f2_aos(Fp2& a, const uint32_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint32_t* d = reinterpret_cast<uint32_t*>(&a);
#pragma unroll
    for (int k = 0; k < 6; k++) {
        uint4 t = q[k];
        d[4 * k] = t.x; d[4 * k + 1] = t.y; d[4 * k + 2] = t.z; d[4 * k + 3] = t.w;
    }
}

// Prep SoA slots written by k_prep_* / k_prep_pok and read by the Miller kernels:
//   Q1 0..3 | Q2 4..7 | P1 8..10 (px, py, pz) | P2 11..13 (pz only in RLC mode) ; flags word per lane:
//   bit0 sigma_1 = O, bit1 sigma_2 = O, bit2 pair-0 degenerate (pr = O), bit3 PoK Schnorr failed,
//   bit4 pair-1 degenerate (RLC: delta * point = O), bit5 sigma outside G1/G2 (RLC: forces fallback)
enum { S_Q1 = 0, S_Q2 = 4, S_P1 = 8, S_P2 = 11, PREP_SLOTS = 14 };
constexpr int NLINES = 68;  // Miller steps: 63 doublings + 5 additions

}  // namespace cc
