// G1 / G2 point arithmetic for gfx950 — device code (the product path).
//
// Replaces AMCL ECP / ECP2 (via amcl_wrapper `G1`, `G2`).
// G1: y^2 = x^3 + 4 over Fp.   G2: the M-type twist y^2 = x^3 + 4(1+i) over Fp2.
// Jacobian coordinates (x = X/Z^2, y = Y/Z^3), Z = 0 is the point at infinity.  Exceptional
// additions (P == Q, P == -Q, O) are handled exactly so every input — including the
// deliberately corrupted fixtures — gives the group element the reference would.
#pragma once
#include "field.h"

namespace cc {

// Field traits so one template serves both groups.
template <class F>
struct FT;

template <>
struct FT<Fp> {
    static DEV void add(Fp& r, const Fp& a, const Fp& b) { fp_add(r, a, b); }
    static DEV void sub(Fp& r, const Fp& a, const Fp& b) { fp_sub(r, a, b); }
    static DEV void dbl(Fp& r, const Fp& a) { fp_dbl(r, a); }
    static DEV void neg(Fp& r, const Fp& a) { fp_neg(r, a); }
    static DEV void mul(Fp& r, const Fp& a, const Fp& b) { fp_mul(r, a, b); }
    static DEV void sqr(Fp& r, const Fp& a) { fp_sqr(r, a); }
    static DEV bool is_zero(const Fp& a) { return fp_is_zero(a); }
    static DEV bool eq(const Fp& a, const Fp& b) { return fp_eq(a, b); }
    static DEV void zero(Fp& r) { fp_zero(r); }
    static DEV void one(Fp& r) { fp_one(r); }
    static DEV void inv(Fp& r, const Fp& a) { fp_inv(r, a); }
    // curve constant b = 4 (Montgomery, R = 2^406; tools/gen_constants.py)
    static DEV void curve_b(Fp& r) {
        constexpr uint32_t B[NL] = {0x0ea898bau, 0xa1d20348u, 0x27c9288fu, 0x47c6b37cu, 0x0c52aee5u, 0xdddb86ecu,
                                    0x23d53606u, 0x7ec46095u, 0xb8dea933u, 0xbf713fa0u, 0x5b838ba6u, 0x18c3ccefu};
#pragma unroll
        for (int j = 0; j < NL; j++) r.v[j] = B[j];
    }
};

template <>
struct FT<Fp2> {
    static DEV void add(Fp2& r, const Fp2& a, const Fp2& b) { f2_add(r, a, b); }
    static DEV void sub(Fp2& r, const Fp2& a, const Fp2& b) { f2_sub(r, a, b); }
    static DEV void dbl(Fp2& r, const Fp2& a) { f2_dbl(r, a); }
    static DEV void neg(Fp2& r, const Fp2& a) { f2_neg(r, a); }
    static DEV void mul(Fp2& r, const Fp2& a, const Fp2& b) { f2_mul(r, a, b); }
    static DEV void sqr(Fp2& r, const Fp2& a) { f2_sqr(r, a); }
    static DEV bool is_zero(const Fp2& a) { return f2_is_zero(a); }
    static DEV bool eq(const Fp2& a, const Fp2& b) { return f2_eq(a, b); }
    static DEV void zero(Fp2& r) { f2_zero(r); }
    static DEV void one(Fp2& r) { f2_one(r); }
    static DEV void inv(Fp2& r, const Fp2& a) { f2_inv(r, a); }
    // twist constant 4 (1 + i)
    static DEV void curve_b(Fp2& r) {
        FT<Fp>::curve_b(r.a);
        FT<Fp>::curve_b(r.b);
    }
};

template <class F>
struct Jac {
    F x, y, z;
};

template <class F>
struct Aff {
    F x, y;
};

template <class F>
DEV bool jac_is_inf(const Jac<F>& p) {
    return FT<F>::is_zero(p.z);
}

template <class F>
DEV void jac_set_inf(Jac<F>& p) {
    FT<F>::one(p.x);
    FT<F>::one(p.y);
    FT<F>::zero(p.z);
}

template <class F>
DEV void jac_from_aff(Jac<F>& r, const Aff<F>& a) {
    r.x = a.x;
    r.y = a.y;
    FT<F>::one(r.z);
}

// dbl-2009-l (a = 0): 2M + 5S.  Infinity maps to infinity (Z3 = 2YZ = 0).
template <class F>
DEV void jac_dbl(Jac<F>& r, const Jac<F>& p) {
    using T = FT<F>;
    F A, B, C, D, E, G, t;
    T::sqr(A, p.x);
    T::sqr(B, p.y);
    T::sqr(C, B);
    T::add(t, p.x, B);
    T::sqr(t, t);
    T::sub(t, t, A);
    T::sub(t, t, C);
    T::dbl(D, t);
    T::dbl(E, A);
    T::add(E, E, A);
    T::sqr(G, E);
    F z3;
    T::mul(z3, p.y, p.z);
    T::dbl(z3, z3);
    F x3;
    T::sub(x3, G, D);
    T::sub(x3, x3, D);
    T::sub(t, D, x3);
    T::mul(r.y, E, t);
    T::dbl(C, C);
    T::dbl(C, C);
    T::dbl(C, C);
    T::sub(r.y, r.y, C);
    r.x = x3;
    r.z = z3;
}

// madd-2007-bl: p (Jacobian) + q (affine, not infinity). 7M + 4S on the common path.
template <class F>
DEV void jac_add_aff(Jac<F>& r, const Jac<F>& p, const Aff<F>& q) {
    using T = FT<F>;
    if (jac_is_inf(p)) {
        jac_from_aff(r, q);
        return;
    }
    F z1z1, u2, s2, h, rr, t;
    T::sqr(z1z1, p.z);
    T::mul(u2, q.x, z1z1);
    T::mul(s2, q.y, p.z);
    T::mul(s2, s2, z1z1);
    T::sub(h, u2, p.x);
    T::sub(rr, s2, p.y);
    if (T::is_zero(h)) {
        if (T::is_zero(rr)) {
            jac_dbl(r, p);
        } else {
            jac_set_inf(r);
        }
        return;
    }
    T::dbl(rr, rr);
    F hh, i, j, v;
    T::sqr(hh, h);
    T::dbl(i, hh);
    T::dbl(i, i);
    T::mul(j, h, i);
    T::mul(v, p.x, i);
    F x3, y3, z3;
    T::sqr(x3, rr);
    T::sub(x3, x3, j);
    T::sub(x3, x3, v);
    T::sub(x3, x3, v);
    T::sub(t, v, x3);
    T::mul(y3, rr, t);
    T::mul(t, p.y, j);
    T::dbl(t, t);
    T::sub(y3, y3, t);
    T::add(z3, p.z, h);
    T::sqr(z3, z3);
    T::sub(z3, z3, z1z1);
    T::sub(z3, z3, hh);
    r.x = x3;
    r.y = y3;
    r.z = z3;
}

// add-2007-bl: general Jacobian addition with exceptional cases.
template <class F>
DEV void jac_add(Jac<F>& r, const Jac<F>& p, const Jac<F>& q) {
    using T = FT<F>;
    if (jac_is_inf(p)) {
        r = q;
        return;
    }
    if (jac_is_inf(q)) {
        r = p;
        return;
    }
    F z1z1, z2z2, u1, u2, s1, s2, h, rr, t;
    T::sqr(z1z1, p.z);
    T::sqr(z2z2, q.z);
    T::mul(u1, p.x, z2z2);
    T::mul(u2, q.x, z1z1);
    T::mul(s1, p.y, q.z);
    T::mul(s1, s1, z2z2);
    T::mul(s2, q.y, p.z);
    T::mul(s2, s2, z1z1);
    T::sub(h, u2, u1);
    T::sub(rr, s2, s1);
    if (T::is_zero(h)) {
        if (T::is_zero(rr)) {
            jac_dbl(r, p);
        } else {
            jac_set_inf(r);
        }
        return;
    }
    T::dbl(rr, rr);
    F i, j, v;
    T::dbl(i, h);
    T::sqr(i, i);
    T::mul(j, h, i);
    T::mul(v, u1, i);
    F x3, y3, z3;
    T::sqr(x3, rr);
    T::sub(x3, x3, j);
    T::sub(x3, x3, v);
    T::sub(x3, x3, v);
    T::sub(t, v, x3);
    T::mul(y3, rr, t);
    T::mul(t, s1, j);
    T::dbl(t, t);
    T::sub(y3, y3, t);
    T::add(z3, p.z, q.z);
    T::sqr(z3, z3);
    T::sub(z3, z3, z1z1);
    T::sub(z3, z3, z2z2);
    T::mul(z3, z3, h);
    r.x = x3;
    r.y = y3;
    r.z = z3;
}

template <class F>
DEV void jac_neg(Jac<F>& r, const Jac<F>& p) {
    r.x = p.x;
    FT<F>::neg(r.y, p.y);
    r.z = p.z;
}

template <class F>
DEV bool aff_on_curve(const Aff<F>& a) {
    using T = FT<F>;
    F l, rr, b;
    T::sqr(l, a.y);
    T::sqr(rr, a.x);
    T::mul(rr, rr, a.x);
    T::curve_b(b);
    T::add(rr, rr, b);
    return T::eq(l, rr);
}

// Jacobian -> affine (one inversion); returns false for infinity.
template <class F>
DEV bool jac_to_aff(Aff<F>& r, const Jac<F>& p) {
    using T = FT<F>;
    if (jac_is_inf(p)) {
        T::zero(r.x);
        T::zero(r.y);
        return false;
    }
    F zi, zi2, zi3;
    T::inv(zi, p.z);
    T::sqr(zi2, zi);
    T::mul(zi3, zi2, zi);
    T::mul(r.x, p.x, zi2);
    T::mul(r.y, p.y, zi3);
    return true;
}

// Sum of Jacobian points across the L consecutive lanes of a task (L a power of two <= 64):
// butterfly over __shfl_xor, every lane ends with the same sum.
template <class F, int L>
DEV void lane_group_sum(Jac<F>& acc) {
    constexpr int JW = sizeof(Jac<F>) / 4;
#pragma unroll 1
    for (int m = L >> 1; m > 0; m >>= 1) {
        Jac<F> o;
        const uint32_t* a = reinterpret_cast<const uint32_t*>(&acc);
        uint32_t* w = reinterpret_cast<uint32_t*>(&o);
        for (int c = 0; c < JW; c++) w[c] = (uint32_t)__shfl_xor((int)a[c], m);
        // same operand order on both partners so they hold the same representation
        if (threadIdx.x & m) {
            Jac<F> t = acc;
            acc = o;
            o = t;
        }
        jac_add(acc, acc, o);
    }
}

}  // namespace cc
