// Optimal-ate pairing pieces for gfx950 — device code (the product path).
//
// Replaces AMCL `pair::ate2` + `pair::fexp` reached through amcl_wrapper
// `GT::ate_2_pairing` (ps_sig `ate_2_pairing`, reference src/lib.rs:13).
//
// Miller loop: homogeneous projective T on the M-type twist, lines through psi(T) evaluated at
// P in G1 and kept sparse: l = l0 + l2 W^2 + l3 W^3, i.e. in the AMCL tower a = (l0, l3),
// b = 0, c = (l2, 0).  Lines may be scaled by any element of Fp2 * W^k (and the Jacobian
// P's Z^3): the easy part of the final exponentiation kills those factors, so GT values equal
// AMCL's.  Final exponentiation: easy part (p^6-1)(p^2+1), hard part 3*Phi_12(p)/r (AMCL's
// exponent), computed as 3 + (x-1)^2 [p^3 + x p^2 + (x^2-1) p + x^3 - x] with a low-liveness
// chain (5 exponentiations by x, cyclotomic squarings).
#pragma once
#include "curve.h"

namespace cc {

constexpr uint64_t X_ABS = 0xd201000000010000ull;  // |x|, x < 0

// ---------------------------------------------------------------- constants (Montgomery)
struct F2c {
    uint32_t a[NL], b[NL];
};
// gamma_k = xi^(k(p-1)/6) for W^k, k = 0..5
__constant__ static const F2c kGamma1[6] = {
    {{0x0002fffdu, 0x76090000u, 0xc40c0002u, 0xebf4000bu, 0x53c758bau, 0x5f489857u, 0x70525745u, 0x77ce5853u,
      0xa256ec6du, 0x5c071a97u, 0xfa80e493u, 0x15f65ec3u},
     {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}},
    {{0xb319d465u, 0x07089552u, 0xb50a8313u, 0xc6695f92u, 0xd117228fu, 0x97e83cccu, 0xb2dc29eeu, 0xa35baecau,
      0x5daace4du, 0x1ce393eau, 0xb0fb66ebu, 0x08f2220fu},
     {0x4ce5d646u, 0xb2f66aadu, 0xfc497cecu, 0x5842a06bu, 0x2599d394u, 0xcf4895d4u, 0x40a8e8d0u, 0xc11b9cbau,
      0xe5a0de89u, 0x2e3813cbu, 0x88847fafu, 0x110eefdau}},
    {{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
     {0x8671f071u, 0xcd03c9e4u, 0x1fcda5d2u, 0x5dab2246u, 0xd3851b95u, 0x587042afu, 0x01bacb9eu, 0x8eb60ebeu,
      0x83d050d2u, 0x03f97d6eu, 0x54638741u, 0x18f02065u}},
    {{0x5aa30fdau, 0x7bcfa7a2u, 0x2a927e7cu, 0xdc17dec1u, 0x6b4ebef1u, 0x2f088dd8u, 0xda74d4a7u, 0xd1ca2087u,
      0x96cebc1du, 0x2da25966u, 0xbbfd87d2u, 0x0e2b7eedu},
     {0x5aa30fdau, 0x7bcfa7a2u, 0x2a927e7cu, 0xdc17dec1u, 0x6b4ebef1u, 0x2f088dd8u, 0xda74d4a7u, 0xd1ca2087u,
      0x96cebc1du, 0x2da25966u, 0xbbfd87d2u, 0x0e2b7eedu}},
    {{0x867545c3u, 0x890dc9e4u, 0x3285a5d5u, 0x2af32253u, 0x309b7e2cu, 0x50880866u, 0x7e881024u, 0xa20d1b8cu,
      0xe2db9068u, 0x14e4f04fu, 0x1564853au, 0x14e56d3fu},
     {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}},
    {{0x0dbce43fu, 0x82d83cf5u, 0xdf9d018fu, 0xa2813e53u, 0x3c65e181u, 0xc6f0caa5u, 0x8d50fe95u, 0x7525cf52u,
      0xf4798a6bu, 0x4a85ed50u, 0x6cf8eebdu, 0x171da0fdu},
     {0xf242c66cu, 0x3726c30au, 0xd1b6fe70u, 0x7c2ac1aau, 0xba4b14a2u, 0xa04007fbu, 0x66341429u, 0xef517c32u,
      0x4ed2226bu, 0x0095ba65u, 0xcc86f7ddu, 0x02e370ecu}},
};
// gamma2_k = xi^(k(p^2-1)/6) (in Fp)
__constant__ static const uint32_t kGamma2[6][NL] = {
    {0x0002fffdu, 0x76090000u, 0xc40c0002u, 0xebf4000bu, 0x53c758bau, 0x5f489857u, 0x70525745u, 0x77ce5853u,
     0xa256ec6du, 0x5c071a97u, 0xfa80e493u, 0x15f65ec3u},
    {0x798dba3au, 0xecfb361bu, 0x91865a2cu, 0xc100ddb8u, 0x232bda8eu, 0x0ec08ff1u, 0xf1ca4721u, 0xd5c13cc6u,
     0xbf7b5c04u, 0x47222a47u, 0xe51c5f59u, 0x0110f184u},
    {0x798a64e8u, 0x30f1361bu, 0x7ece5a2au, 0xf3b8ddabu, 0xc61577f7u, 0x16a8ca3au, 0x74fd029bu, 0xc26a2ff8u,
     0x60701c6eu, 0x3636b766u, 0x241b6160u, 0x051ba4abu},
    {0xfffcaaaeu, 0x43f5ffffu, 0xed47fffdu, 0x32b7fff2u, 0xa2e99d69u, 0x07e83a49u, 0x8332bb7au, 0xeca8f331u,
     0xa0f4c069u, 0xef148d1eu, 0x3eff0206u, 0x040ab326u},
    {0x8671f071u, 0xcd03c9e4u, 0x1fcda5d2u, 0x5dab2246u, 0xd3851b95u, 0x587042afu, 0x01bacb9eu, 0x8eb60ebeu,
     0x83d050d2u, 0x03f97d6eu, 0x54638741u, 0x18f02065u},
    {0x867545c3u, 0x890dc9e4u, 0x3285a5d5u, 0x2af32253u, 0x309b7e2cu, 0x50880866u, 0x7e881024u, 0xa20d1b8cu,
     0xe2db9068u, 0x14e4f04fu, 0x1564853au, 0x14e56d3fu},
};

DEV void load_f2c(Fp2& r, const F2c& c) {
#pragma unroll
    for (int j = 0; j < NL; j++) {
        r.a.v[j] = c.a[j];
        r.b.v[j] = c.b[j];
    }
}

// x^p coefficient-wise: conj(c) * gamma_k for the coefficient of W^k.
// AMCL slots -> W power: a.a 0, a.b 3, b.a 1, b.b 4, c.a 2, c.b 5.
DEV void frob_coef(Fp2& c, int k) {
    Fp2 g, t;
    load_f2c(g, kGamma1[k]);
    f2_conj(t, c);
    f2_mul(c, t, g);
}

DEV void f12_frob(Fp12& r, const Fp12& x) {
    r = x;
    // a.a (k=0): gamma_0 = 1 -> conj only
    f2_conj(r.a.a, r.a.a);
    frob_coef(r.a.b, 3);
    frob_coef(r.b.a, 1);
    frob_coef(r.b.b, 4);
    frob_coef(r.c.a, 2);
    frob_coef(r.c.b, 5);
}

DEV void frob2_coef(Fp2& c, int k) {
    Fp g;
#pragma unroll
    for (int j = 0; j < NL; j++) g.v[j] = kGamma2[k][j];
    f2_mul_fp(c, c, g);
}

DEV void f12_frob2(Fp12& r, const Fp12& x) {
    r = x;
    frob2_coef(r.a.b, 3);
    frob2_coef(r.b.a, 1);
    frob2_coef(r.b.b, 4);
    frob2_coef(r.c.a, 2);
    frob2_coef(r.c.b, 5);
}

// ---------------------------------------------------------------- sparse line multiply
// f *= (A + C w^2) with A = (l0, l3) in Fp4 and C = (l2, 0): 13 Fp2 multiplications.
DEV void f12_mul_line(Fp12& f, const Fp2& l0, const Fp2& l2, const Fp2& l3) {
    Fp4 A;
    A.a = l0;
    A.b = l3;
    Fp4 t0, t2, s, u;
    f4_mul(t0, f.a, A);       // a A
    f4_mul_f2(t2, f.c, l2);   // c C
    // r.c = (a + c)(A + C) - t0 - t2 = c A + a C
    Fp4 AC = A;
    f2_add(AC.a, AC.a, l2);
    f4_add(s, f.a, f.c);
    f4_mul(s, s, AC);
    f4_sub(s, s, t0);
    Fp4 rc;
    f4_sub(rc, s, t2);
    // r.a = a A + s (b C)
    f4_mul_f2(u, f.b, l2);
    f4_mul_s(u, u);
    Fp4 ra;
    f4_add(ra, t0, u);
    // r.b = b A + s (c C)
    f4_mul(u, f.b, A);
    f4_mul_s(t2, t2);
    f4_add(f.b, u, t2);
    f.a = ra;
    f.c = rc;
}

// ---------------------------------------------------------------- line functions
struct G2Proj {
    Fp2 x, y, z;  // homogeneous projective on the twist
};

DEV void fp_half(Fp& r, const Fp& a) {
    // (a + (a odd ? p : 0)) / 2 ; a < p so a + p < 2^382
    uint32_t mask = 0u - (a.v[0] & 1u);
    uint32_t t[NL];
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) t[j] = __builtin_addc(a.v[j], p_limb(j) & mask, c, &c);
#pragma unroll
    for (int j = 0; j < NL - 1; j++) r.v[j] = (t[j] >> 1) | (t[j + 1] << 31);
    r.v[NL - 1] = t[NL - 1] >> 1;
}

DEV void f2_half(Fp2& r, const Fp2& a) { fp_half(r.a, a.a); fp_half(r.b, a.b); }

// x * 12
DEV void f2_mul12(Fp2& r, const Fp2& x) {
    Fp2 t4;
    f2_dbl(t4, x);
    f2_dbl(t4, t4);
    Fp2 t8;
    f2_dbl(t8, t4);
    f2_add(r, t8, t4);
}

// Doubling step: T <- 2T; line coefficients before evaluation at P:
//   l0 = 3b'Z^2 - Y^2, l2c = 3X^2 (times x_P), l3c = -2YZ (times y_P).   b' = 4(1+i).
DEV void line_dbl(G2Proj& T, Fp2& l0, Fp2& l2c, Fp2& l3c) {
    Fp2 a, b, c, e, f, g, h, t;
    f2_mul(a, T.x, T.y);
    f2_half(a, a);
    f2_sqr(b, T.y);
    f2_sqr(c, T.z);
    // e = 3 b' c = 12 (1 + i) c
    f2_mul_xi(e, c);
    f2_mul12(e, e);
    f2_dbl(f, e);
    f2_add(f, f, e);
    f2_add(g, b, f);
    f2_half(g, g);
    f2_add(h, T.y, T.z);
    f2_sqr(h, h);
    f2_sub(h, h, b);
    f2_sub(h, h, c);
    f2_sub(l0, e, b);
    f2_sqr(t, T.x);
    f2_dbl(l2c, t);
    f2_add(l2c, l2c, t);
    f2_neg(l3c, h);
    // T
    f2_sub(t, b, f);
    f2_mul(T.x, a, t);
    f2_sqr(t, e);
    f2_sqr(T.y, g);
    f2_sub(T.y, T.y, t);
    f2_sub(T.y, T.y, t);
    f2_sub(T.y, T.y, t);
    f2_mul(T.z, b, h);
}

// Addition step with affine Q: T <- T + Q;
//   l0 = theta x_Q - lambda y_Q, l2c = -theta (times x_P), l3c = lambda (times y_P).
DEV void line_add(G2Proj& T, const Aff<Fp2>& Q, Fp2& l0, Fp2& l2c, Fp2& l3c) {
    Fp2 theta, lambda, c, d, e, f, g, h, t;
    f2_mul(t, Q.y, T.z);
    f2_sub(theta, T.y, t);
    f2_mul(t, Q.x, T.z);
    f2_sub(lambda, T.x, t);
    f2_sqr(c, theta);
    f2_sqr(d, lambda);
    f2_mul(e, lambda, d);
    f2_mul(f, T.z, c);
    f2_mul(g, T.x, d);
    f2_add(h, e, f);
    f2_sub(h, h, g);
    f2_sub(h, h, g);
    f2_mul(l0, theta, Q.x);
    f2_mul(t, lambda, Q.y);
    f2_sub(l0, l0, t);
    f2_neg(l2c, theta);
    l3c = lambda;
    f2_mul(T.x, lambda, h);
    f2_sub(t, g, h);
    f2_mul(t, theta, t);
    f2_mul(c, e, T.y);
    f2_sub(T.y, t, c);
    f2_mul(T.z, T.z, e);
}

// P in G1 prepared for line evaluation: line = l0*pz + l2c*px W^2 + l3c*py W^3.
// Affine P: (x, y, 1).  Jacobian (X, Y, Z): (X Z, Y, Z^3) — the line times Z^3 (an Fp factor).
struct G1Eval {
    Fp px, py, pz;
};

template <bool kAffine>
DEV void eval_line(Fp12& f, const Fp2& l0, const Fp2& l2c, const Fp2& l3c, const G1Eval& P) {
    Fp2 a0, a2, a3;
    if (kAffine) {
        a0 = l0;
    } else {
        f2_mul_fp(a0, l0, P.pz);
    }
    f2_mul_fp(a2, l2c, P.px);
    f2_mul_fp(a3, l3c, P.py);
    f12_mul_line(f, a0, a2, a3);
}

// ---------------------------------------------------------------- final exponentiation
// y^|x| for cyclotomic y (square-and-multiply over the 64-bit constant), then conj: y^x.
DEV void cyc_pow_x(Fp12& r, const Fp12& y) {
    Fp12 acc = y;
    for (int i = 62; i >= 0; i--) {
        f12_cyc_sqr(acc, acc);
        if ((X_ABS >> i) & 1ull) f12_mul(acc, acc, y);
    }
    f12_conj(r, acc);
}

}  // namespace cc
