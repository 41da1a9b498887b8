// amcl_wrapper / AMCL byte codec on the device.
//   Fr  : 48 B big-endian, reduced mod r
//   G1  : 97 B = 0x04 || x || y (48 B BE each); any other prefix, or an off-curve point,
//         decodes to the identity (AMCL ECP::frombytes / ECP::new_bigs)
//   G2  : 192 B = x.a || x.b || y.a || y.b; off-curve -> identity (AMCL ECP2::new_fp2s)
//   GT  : 576 B, AMCL FP12 order a.a.a, a.a.b, ..., c.b.b (= the Fp12 struct order here)
//   identity encodes as AMCL's projective infinity (x = 0, y = 1).
#pragma once
#include "curve.h"

namespace cc {

// r (255-bit), little-endian 32-bit limbs
#define CC_R_LIMBS 0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u, 0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u

struct Fr {
    uint32_t v[8];  // canonical, < r
};

DEV void be48_aligned(Fp& r, const uint8_t* p) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int k = 0; k < NL; k++) r.v[k] = __builtin_bswap32(w[NL - 1 - k]);
}

DEV void be48_bytes(Fp& r, const uint8_t* p) {
#pragma unroll
    for (int k = 0; k < NL; k++) {
        const uint8_t* q = p + 44 - 4 * k;
        r.v[k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
    }
}

DEV void store_be48_aligned(uint8_t* p, const Fp& canon) {
    uint32_t* w = reinterpret_cast<uint32_t*>(p);
#pragma unroll
    for (int k = 0; k < NL; k++) w[NL - 1 - k] = __builtin_bswap32(canon.v[k]);
}

DEV void store_be48_bytes(uint8_t* p, const Fp& canon) {
#pragma unroll
    for (int k = 0; k < NL; k++) {
        uint8_t* q = p + 44 - 4 * k;
        uint32_t v = canon.v[k];
        q[0] = (uint8_t)(v >> 24);
        q[1] = (uint8_t)(v >> 16);
        q[2] = (uint8_t)(v >> 8);
        q[3] = (uint8_t)v;
    }
}

// raw 48-byte integer -> Montgomery Fp (mod p first)
DEV void fp_from_raw(Fp& r, Fp raw) {
    fp_raw_reduce(raw);
    fp_to_mont(r, raw);
}

DEV uint32_t r_limb(int j) {
    constexpr uint32_t Rl[8] = {CC_R_LIMBS};
    return Rl[j];
}

// v (12 limbs, < 2^384) mod r by shift-and-subtract.  Slow path: only non-canonical scalars.
__device__ __noinline__ void fr_reduce_slow(uint32_t v[NL]) {
    for (int s = 384 - 255; s >= 0; s--) {
        // m = r << s (12 limbs)
        uint32_t m[NL];
        const int ws = s >> 5, bs = s & 31;
        for (int j = 0; j < NL; j++) {
            uint32_t lo = 0, hi = 0;
            int k = j - ws;
            if (k >= 0 && k < 8) lo = r_limb(k) << bs;
            if (bs && k - 1 >= 0 && k - 1 < 8) hi = r_limb(k - 1) >> (32 - bs);
            m[j] = lo | hi;
        }
        uint32_t t[NL], br = 0;
        for (int j = 0; j < NL; j++) t[j] = __builtin_subc(v[j], m[j], br, &br);
        if (!br)
            for (int j = 0; j < NL; j++) v[j] = t[j];
    }
}

DEV void fr_from_be48(Fr& out, const uint8_t* p) {
    Fp raw;
    be48_aligned(raw, p);
    uint32_t hi = raw.v[8] | raw.v[9] | raw.v[10] | raw.v[11];
    // canonical iff hi == 0 and low 256 bits < r
    uint32_t br = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) (void)__builtin_subc(raw.v[j], r_limb(j), br, &br);
    if (hi != 0 || br == 0) fr_reduce_slow(raw.v);
#pragma unroll
    for (int j = 0; j < 8; j++) out.v[j] = raw.v[j];
}

// G1 from 97 bytes (byte-addressed: the 0x04 prefix misaligns the coordinates)
DEV bool g1_decode(Aff<Fp>& a, const uint8_t* p) {
    bool ok = p[0] == 0x04;
    Fp raw;
    be48_bytes(raw, p + 1);
    fp_from_raw(a.x, raw);
    be48_bytes(raw, p + 49);
    fp_from_raw(a.y, raw);
    ok = ok && aff_on_curve(a);
    if (!ok) {
        fp_zero(a.x);
        fp_zero(a.y);
    }
    return ok;  // false => identity
}

DEV bool g2_decode(Aff<Fp2>& a, const uint8_t* p) {
    Fp raw;
    be48_aligned(raw, p);
    fp_from_raw(a.x.a, raw);
    be48_aligned(raw, p + 48);
    fp_from_raw(a.x.b, raw);
    be48_aligned(raw, p + 96);
    fp_from_raw(a.y.a, raw);
    be48_aligned(raw, p + 144);
    fp_from_raw(a.y.b, raw);
    bool ok = aff_on_curve(a);
    if (!ok) {
        f2_zero(a.x);
        f2_zero(a.y);
    }
    return ok;
}

DEV void g1_encode(uint8_t* p, const Aff<Fp>& a, bool finite) {
    p[0] = 0x04;
    Fp c;
    if (finite) {
        fp_from_mont(c, a.x);
        store_be48_bytes(p + 1, c);
        fp_from_mont(c, a.y);
        store_be48_bytes(p + 49, c);
    } else {
        fp_zero(c);
        store_be48_bytes(p + 1, c);
        c.v[0] = 1;
        store_be48_bytes(p + 49, c);
    }
}

DEV void g2_encode(uint8_t* p, const Aff<Fp2>& a, bool finite) {
    Fp c;
    if (finite) {
        fp_from_mont(c, a.x.a);
        store_be48_aligned(p, c);
        fp_from_mont(c, a.x.b);
        store_be48_aligned(p + 48, c);
        fp_from_mont(c, a.y.a);
        store_be48_aligned(p + 96, c);
        fp_from_mont(c, a.y.b);
        store_be48_aligned(p + 144, c);
    } else {
        fp_zero(c);
        store_be48_aligned(p, c);
        store_be48_aligned(p + 48, c);
        store_be48_aligned(p + 144, c);
        c.v[0] = 1;
        store_be48_aligned(p + 96, c);
    }
}

}  // namespace cc
