/* bls_oracle.c — C restatement of the reference hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Used only by tests/ (as a fast independent checker), __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg (timed as the "port" CPU baseline).  Never linked into the product library.
 *
 * Restates:
 *   V1/V3  Signature::verify  (reference src/signature.rs:473-478 -> ps_sig verify [EXT]):
 *          len check, identity check, pr = MSM_var([X~, Y~..], [1, m..]),
 *          ate_2_pairing(sigma1, pr, -sigma2, g~).is_one()
 *   V4     multi_scalar_mul_var_time [EXT] as interleaved width-5 wNAF (Straus)
 *   V6     AMCL ate2 (shared-squaring 2-pair Miller loop over |x|, conj for x<0) + fexp
 *          (easy part, then the Ghammam-Fouotsa BLS12 hard-part chain = 3*Phi_12(p)/r)
 *   V8/V9  Signature::aggregate / Verkey::aggregate (signature.rs:448-526)
 *   P1     PoKOfSignatureProof::verify [EXT] (exercised at reference pok_sig.rs:103-105)
 *
 * Representation is deliberately independent of the device code: 6 x 64-bit Montgomery limbs
 * (R = 2^384) and the Fp2 -> Fp6 = Fp2[v]/(v^3 - xi) -> Fp12 = Fp6[w]/(w^2 - v) tower; the GT
 * serialiser permutes into AMCL's FP4-tower byte order.  Pinned against tests/golden/ (made by
 * the Python restatement oracle/bls12_381.py, a third representation).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

typedef unsigned __int128 u128;

/* ============================== Fp ============================== */
typedef struct { uint64_t l[6]; } fp;

static const uint64_t PM[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                               0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static const uint64_t N0 = 0x89f3fffcfffcfffdULL;
static const uint64_t RM[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                               0x73eda753299d7d48ULL};
static fp FP_ONE, FP_R2, FP_INV2;

static int geq6(const uint64_t* a, const uint64_t* b) {
    for (int i = 5; i >= 0; i--) {
        if (a[i] != b[i]) return a[i] > b[i];
    }
    return 1;
}

static void sub6(uint64_t* r, const uint64_t* a, const uint64_t* b) {
    uint64_t br = 0;
    for (int i = 0; i < 6; i++) {
        u128 t = (u128)a[i] - b[i] - br;
        r[i] = (uint64_t)t;
        br = (uint64_t)(t >> 64) & 1;
    }
}

static void fp_add(fp* r, const fp* a, const fp* b) {
    uint64_t c = 0, t[6];
    for (int i = 0; i < 6; i++) {
        u128 s = (u128)a->l[i] + b->l[i] + c;
        t[i] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
    }
    if (geq6(t, PM)) sub6(t, t, PM);
    memcpy(r->l, t, sizeof t);
}

static void fp_sub(fp* r, const fp* a, const fp* b) {
    uint64_t t[6], br = 0;
    for (int i = 0; i < 6; i++) {
        u128 d = (u128)a->l[i] - b->l[i] - br;
        t[i] = (uint64_t)d;
        br = (uint64_t)(d >> 64) & 1;
    }
    if (br) {
        uint64_t c = 0;
        for (int i = 0; i < 6; i++) {
            u128 s = (u128)t[i] + PM[i] + c;
            t[i] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
    }
    memcpy(r->l, t, sizeof t);
}

static int fp_is_zero(const fp* a) {
    uint64_t o = 0;
    for (int i = 0; i < 6; i++) o |= a->l[i];
    return o == 0;
}

static int fp_eq(const fp* a, const fp* b) { return memcmp(a->l, b->l, sizeof a->l) == 0; }

static void fp_neg(fp* r, const fp* a) {
    if (fp_is_zero(a)) { *r = *a; return; }
    sub6(r->l, PM, a->l);
}

/* CIOS Montgomery multiplication, 6 x 64-bit limbs */
static void fp_mul(fp* r, const fp* a, const fp* b) {
    uint64_t t[8] = {0};
    for (int i = 0; i < 6; i++) {
        u128 c = 0;
        for (int j = 0; j < 6; j++) {
            c += (u128)a->l[j] * b->l[i] + t[j];
            t[j] = (uint64_t)c;
            c >>= 64;
        }
        c += t[6];
        t[6] = (uint64_t)c;
        t[7] = (uint64_t)(c >> 64);
        uint64_t m = t[0] * N0;
        c = ((u128)m * PM[0] + t[0]) >> 64;
        for (int j = 1; j < 6; j++) {
            c += (u128)m * PM[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[6];
        t[5] = (uint64_t)c;
        t[6] = t[7] + (uint64_t)(c >> 64);
    }
    if (t[6] || geq6(t, PM)) sub6(t, t, PM);
    memcpy(r->l, t, 6 * sizeof(uint64_t));
}

static void fp_sqr(fp* r, const fp* a) { fp_mul(r, a, a); }
static void fp_set_one(fp* r) { *r = FP_ONE; }
static void fp_set_zero(fp* r) { memset(r, 0, sizeof *r); }

/* a^e, e little-endian u64[n] */
static void fp_pow(fp* r, const fp* a, const uint64_t* e, int n) {
    fp acc = FP_ONE, b = *a;
    for (int i = 0; i < n * 64; i++) {
        if ((e[i / 64] >> (i % 64)) & 1) fp_mul(&acc, &acc, &b);
        fp_sqr(&b, &b);
    }
    *r = acc;
}

static void fp_inv(fp* r, const fp* a) {
    uint64_t e[6];
    memcpy(e, PM, sizeof e);
    e[0] -= 2;
    fp_pow(r, a, e, 6);
}

/* 48-byte big-endian -> Montgomery, reducing mod p (AMCL FP::new_big reduces) */
static void fp_from_be(fp* r, const uint8_t* b) {
    uint64_t v[6];
    for (int i = 0; i < 6; i++) {
        uint64_t w = 0;
        for (int k = 0; k < 8; k++) w = (w << 8) | b[(5 - i) * 8 + k];
        v[i] = w;
    }
    while (geq6(v, PM)) sub6(v, v, PM);
    fp t;
    memcpy(t.l, v, sizeof v);
    fp_mul(r, &t, &FP_R2);
}

static void fp_to_be(uint8_t* b, const fp* a) {
    fp one_raw, t;
    memset(&one_raw, 0, sizeof one_raw);
    one_raw.l[0] = 1;
    fp_mul(&t, a, &one_raw);
    for (int i = 0; i < 6; i++)
        for (int k = 0; k < 8; k++) b[(5 - i) * 8 + k] = (uint8_t)(t.l[i] >> (56 - 8 * k));
}

static void fp_from_hex(fp* r, const char* h) {
    uint8_t b[48];
    memset(b, 0, sizeof b);
    size_t n = strlen(h);
    for (size_t i = 0; i < n; i++) {
        char c = h[n - 1 - i];
        int v = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : c - 'A' + 10;
        b[47 - i / 2] |= (uint8_t)(v << (4 * (i % 2)));
    }
    fp_from_be(r, b);
}

/* ============================== Fp2 ============================== */
typedef struct { fp a, b; } fp2;

static void fp2_add(fp2* r, const fp2* x, const fp2* y) { fp_add(&r->a, &x->a, &y->a); fp_add(&r->b, &x->b, &y->b); }
static void fp2_sub(fp2* r, const fp2* x, const fp2* y) { fp_sub(&r->a, &x->a, &y->a); fp_sub(&r->b, &x->b, &y->b); }
static void fp2_neg(fp2* r, const fp2* x) { fp_neg(&r->a, &x->a); fp_neg(&r->b, &x->b); }
static void fp2_conj(fp2* r, const fp2* x) { r->a = x->a; fp_neg(&r->b, &x->b); }
static int fp2_is_zero(const fp2* x) { return fp_is_zero(&x->a) && fp_is_zero(&x->b); }
static int fp2_eq(const fp2* x, const fp2* y) { return fp_eq(&x->a, &y->a) && fp_eq(&x->b, &y->b); }
static void fp2_set_one(fp2* r) { r->a = FP_ONE; fp_set_zero(&r->b); }
static void fp2_set_zero(fp2* r) { memset(r, 0, sizeof *r); }

static void fp2_mul(fp2* r, const fp2* x, const fp2* y) {
    fp t0, t1, s0, s1;
    fp_mul(&t0, &x->a, &y->a);
    fp_mul(&t1, &x->b, &y->b);
    fp_add(&s0, &x->a, &x->b);
    fp_add(&s1, &y->a, &y->b);
    fp_mul(&s0, &s0, &s1);
    fp_sub(&s0, &s0, &t0);
    fp_sub(&r->b, &s0, &t1);
    fp_sub(&r->a, &t0, &t1);
}

static void fp2_sqr(fp2* r, const fp2* x) {
    fp s, d, m;
    fp_add(&s, &x->a, &x->b);
    fp_sub(&d, &x->a, &x->b);
    fp_mul(&m, &x->a, &x->b);
    fp_mul(&r->a, &s, &d);
    fp_add(&r->b, &m, &m);
}

static void fp2_mul_fp(fp2* r, const fp2* x, const fp* k) { fp_mul(&r->a, &x->a, k); fp_mul(&r->b, &x->b, k); }

static void fp2_mul_xi(fp2* r, const fp2* x) {
    fp t;
    fp_sub(&t, &x->a, &x->b);
    fp_add(&r->b, &x->a, &x->b);
    r->a = t;
}

static void fp2_inv(fp2* r, const fp2* x) {
    fp n, t;
    fp_sqr(&n, &x->a);
    fp_sqr(&t, &x->b);
    fp_add(&n, &n, &t);
    fp_inv(&n, &n);
    fp_mul(&r->a, &x->a, &n);
    fp_mul(&t, &x->b, &n);
    fp_neg(&r->b, &t);
}

/* ============================== Fp6 / Fp12 (standard tower) ============================== */
typedef struct { fp2 c0, c1, c2; } fp6;
typedef struct { fp6 c0, c1; } fp12;

static void fp6_add(fp6* r, const fp6* a, const fp6* b) { fp2_add(&r->c0, &a->c0, &b->c0); fp2_add(&r->c1, &a->c1, &b->c1); fp2_add(&r->c2, &a->c2, &b->c2); }
static void fp6_sub(fp6* r, const fp6* a, const fp6* b) { fp2_sub(&r->c0, &a->c0, &b->c0); fp2_sub(&r->c1, &a->c1, &b->c1); fp2_sub(&r->c2, &a->c2, &b->c2); }
static void fp6_neg(fp6* r, const fp6* a) { fp2_neg(&r->c0, &a->c0); fp2_neg(&r->c1, &a->c1); fp2_neg(&r->c2, &a->c2); }

static void fp6_mul(fp6* r, const fp6* a, const fp6* b) {
    fp2 t0, t1, t2, s, u, c0, c1, c2;
    fp2_mul(&t0, &a->c0, &b->c0);
    fp2_mul(&t1, &a->c1, &b->c1);
    fp2_mul(&t2, &a->c2, &b->c2);
    fp2_add(&s, &a->c1, &a->c2); fp2_add(&u, &b->c1, &b->c2); fp2_mul(&s, &s, &u);
    fp2_sub(&s, &s, &t1); fp2_sub(&s, &s, &t2); fp2_mul_xi(&s, &s); fp2_add(&c0, &s, &t0);
    fp2_add(&s, &a->c0, &a->c1); fp2_add(&u, &b->c0, &b->c1); fp2_mul(&s, &s, &u);
    fp2_sub(&s, &s, &t0); fp2_sub(&s, &s, &t1); fp2_mul_xi(&u, &t2); fp2_add(&c1, &s, &u);
    fp2_add(&s, &a->c0, &a->c2); fp2_add(&u, &b->c0, &b->c2); fp2_mul(&s, &s, &u);
    fp2_sub(&s, &s, &t0); fp2_sub(&s, &s, &t2); fp2_add(&c2, &s, &t1);
    r->c0 = c0; r->c1 = c1; r->c2 = c2;
}

/* a * (b0 + b1 v) */
static void fp6_mul_by_01(fp6* r, const fp6* a, const fp2* b0, const fp2* b1) {
    fp2 t0, t1, s, u, c0, c1, c2;
    fp2_mul(&t0, &a->c0, b0);
    fp2_mul(&t1, &a->c1, b1);
    fp2_mul(&s, &a->c2, b1); fp2_mul_xi(&s, &s); fp2_add(&c0, &s, &t0);
    fp2_add(&s, &a->c0, &a->c1); fp2_add(&u, b0, b1); fp2_mul(&s, &s, &u);
    fp2_sub(&s, &s, &t0); fp2_sub(&c1, &s, &t1);
    fp2_mul(&s, &a->c2, b0); fp2_add(&c2, &s, &t1);
    r->c0 = c0; r->c1 = c1; r->c2 = c2;
}

/* a * (b1 v) */
static void fp6_mul_by_1(fp6* r, const fp6* a, const fp2* b1) {
    fp2 c0, c1, c2;
    fp2_mul(&c0, &a->c2, b1); fp2_mul_xi(&c0, &c0);
    fp2_mul(&c1, &a->c0, b1);
    fp2_mul(&c2, &a->c1, b1);
    r->c0 = c0; r->c1 = c1; r->c2 = c2;
}

static void fp6_mul_by_v(fp6* r, const fp6* a) {
    fp2 t;
    fp2_mul_xi(&t, &a->c2);
    r->c2 = a->c1; r->c1 = a->c0; r->c0 = t;
}

static void fp6_inv(fp6* r, const fp6* a) {
    fp2 A, Bv, C, F, t;
    fp2_sqr(&A, &a->c0); fp2_mul(&t, &a->c1, &a->c2); fp2_mul_xi(&t, &t); fp2_sub(&A, &A, &t);
    fp2_sqr(&Bv, &a->c2); fp2_mul_xi(&Bv, &Bv); fp2_mul(&t, &a->c0, &a->c1); fp2_sub(&Bv, &Bv, &t);
    fp2_sqr(&C, &a->c1); fp2_mul(&t, &a->c0, &a->c2); fp2_sub(&C, &C, &t);
    fp2_mul(&F, &a->c2, &Bv); fp2_mul(&t, &a->c1, &C); fp2_add(&F, &F, &t); fp2_mul_xi(&F, &F);
    fp2_mul(&t, &a->c0, &A); fp2_add(&F, &F, &t);
    fp2_inv(&F, &F);
    fp2_mul(&r->c0, &A, &F); fp2_mul(&r->c1, &Bv, &F); fp2_mul(&r->c2, &C, &F);
}

static void fp12_set_one(fp12* r) {
    memset(r, 0, sizeof *r);
    r->c0.c0.a = FP_ONE;
}

static int fp12_is_one(const fp12* a) {
    fp12 one;
    fp12_set_one(&one);
    return memcmp(a, &one, sizeof one) == 0;
}

static void fp12_mul(fp12* r, const fp12* a, const fp12* b) {
    fp6 t0, t1, s, u;
    fp6_mul(&t0, &a->c0, &b->c0);
    fp6_mul(&t1, &a->c1, &b->c1);
    fp6_add(&s, &a->c0, &a->c1); fp6_add(&u, &b->c0, &b->c1); fp6_mul(&s, &s, &u);
    fp6_sub(&s, &s, &t0); fp6_sub(&r->c1, &s, &t1);
    fp6_mul_by_v(&t1, &t1); fp6_add(&r->c0, &t0, &t1);
}

static void fp12_sqr(fp12* r, const fp12* a) {
    fp6 t, s, u;
    fp6_mul(&t, &a->c0, &a->c1);
    fp6_add(&s, &a->c0, &a->c1);
    fp6_mul_by_v(&u, &a->c1); fp6_add(&u, &u, &a->c0);
    fp6_mul(&s, &s, &u);
    fp6_sub(&s, &s, &t);
    fp6_mul_by_v(&u, &t); fp6_sub(&r->c0, &s, &u);
    fp6_add(&r->c1, &t, &t);
}

static void fp12_conj(fp12* r, const fp12* a) { r->c0 = a->c0; fp6_neg(&r->c1, &a->c1); }

static void fp12_inv(fp12* r, const fp12* a) {
    fp6 t0, t1;
    fp6_mul(&t0, &a->c0, &a->c0);
    fp6_mul(&t1, &a->c1, &a->c1);
    fp6_mul_by_v(&t1, &t1);
    fp6_sub(&t0, &t0, &t1);
    fp6_inv(&t0, &t0);
    fp6_mul(&r->c0, &a->c0, &t0);
    fp6_mul(&t1, &a->c1, &t0);
    fp6_neg(&r->c1, &t1);
}

/* f * (l0 + l2 W^2 + l3 W^3) = f * ((l0, l2, 0) + (0, l3, 0) w) */
static void fp12_mul_line(fp12* r, const fp12* f, const fp2* l0, const fp2* l2, const fp2* l3) {
    fp6 t0, t1, s;
    fp2 u;
    fp6_mul_by_01(&t0, &f->c0, l0, l2);
    fp6_mul_by_1(&t1, &f->c1, l3);
    fp6_add(&s, &f->c0, &f->c1);
    fp2_add(&u, l2, l3);
    fp6_mul_by_01(&s, &s, l0, &u);
    fp6_sub(&s, &s, &t0);
    fp6_sub(&r->c1, &s, &t1);
    fp6_mul_by_v(&t1, &t1);
    fp6_add(&r->c0, &t0, &t1);
}

/* Frobenius: (c W^k)^p = conj(c) gamma_k W^k, c0.j <-> W^(2j), c1.j <-> W^(2j+1) */
static fp2 FROB_G[6];

static void fp12_frob(fp12* r, const fp12* a) {
    fp2* src[6] = {(fp2*)&a->c0.c0, (fp2*)&a->c1.c0, (fp2*)&a->c0.c1,
                   (fp2*)&a->c1.c1, (fp2*)&a->c0.c2, (fp2*)&a->c1.c2};
    fp12 t;
    fp2* dst[6] = {&t.c0.c0, &t.c1.c0, &t.c0.c1, &t.c1.c1, &t.c0.c2, &t.c1.c2};
    for (int k = 0; k < 6; k++) {
        fp2 c;
        fp2_conj(&c, src[k]);
        fp2_mul(dst[k], &c, &FROB_G[k]);
    }
    *r = t;
}

/* Granger-Scott cyclotomic squaring (standard tower) */
static void fp12_cyc_sqr(fp12* r, const fp12* a) {
    fp2 z0 = a->c0.c0, z4 = a->c0.c1, z3 = a->c0.c2, z2 = a->c1.c0, z1 = a->c1.c1, z5 = a->c1.c2;
    fp2 tmp, t0, t1, t2, t3, t4, t5, u, v;
#define SQ4(x, y, ta, tb)                                                   \
    fp2_mul(&tmp, &x, &y);                                                  \
    fp2_add(&u, &x, &y); fp2_mul_xi(&v, &y); fp2_add(&v, &v, &x);           \
    fp2_mul(&ta, &u, &v); fp2_sub(&ta, &ta, &tmp); fp2_mul_xi(&u, &tmp);    \
    fp2_sub(&ta, &ta, &u); fp2_add(&tb, &tmp, &tmp);
    SQ4(z0, z1, t0, t1)
    SQ4(z2, z3, t2, t3)
    SQ4(z4, z5, t4, t5)
#undef SQ4
    /* z0 = 3 t0 - 2 z0 */
    fp2_sub(&z0, &t0, &z0); fp2_add(&z0, &z0, &z0); fp2_add(&z0, &z0, &t0);
    fp2_add(&z1, &t1, &z1); fp2_add(&z1, &z1, &z1); fp2_add(&z1, &z1, &t1);
    fp2_mul_xi(&tmp, &t5);
    fp2_add(&z2, &tmp, &z2); fp2_add(&z2, &z2, &z2); fp2_add(&z2, &z2, &tmp);
    fp2_sub(&z3, &t4, &z3); fp2_add(&z3, &z3, &z3); fp2_add(&z3, &z3, &t4);
    fp2_sub(&z4, &t2, &z4); fp2_add(&z4, &z4, &z4); fp2_add(&z4, &z4, &t2);
    fp2_add(&z5, &t3, &z5); fp2_add(&z5, &z5, &z5); fp2_add(&z5, &z5, &t3);
    r->c0.c0 = z0; r->c0.c1 = z4; r->c0.c2 = z3;
    r->c1.c0 = z2; r->c1.c1 = z1; r->c1.c2 = z5;
}

static const uint64_t X_ABS = 0xd201000000010000ULL;

/* y^e for cyclotomic y; e > 0 64-bit; AMCL FP12::pow with usqr */
static void fp12_cyc_pow(fp12* r, const fp12* a, uint64_t e) {
    fp12 acc = *a;
    int nb = 64 - __builtin_clzll(e);
    for (int i = nb - 2; i >= 0; i--) {
        fp12_cyc_sqr(&acc, &acc);
        if ((e >> i) & 1) fp12_mul(&acc, &acc, a);
    }
    *r = acc;
}

/* pow by x (negative): conj(y^|x|) */
static void pow_x(fp12* r, const fp12* a) { fp12_cyc_pow(r, a, X_ABS); fp12_conj(r, r); }
static void pow_x2(fp12* r, const fp12* a) { fp12_cyc_pow(r, a, X_ABS >> 1); fp12_conj(r, r); }

/* AMCL fexp for BLS12 (easy part + Ghammam-Fouotsa hard part) */
static void final_exp(fp12* out, const fp12* f) {
    fp12 r, t, y0, y1, y2, y3;
    fp12_conj(&t, f);
    fp12_inv(&r, f);
    fp12_mul(&r, &t, &r);       /* f^(p^6-1) */
    fp12_frob(&t, &r);
    fp12_frob(&t, &t);
    fp12_mul(&r, &t, &r);       /* ^(p^2+1) */
    fp12_cyc_sqr(&y0, &r);
    pow_x(&y1, &y0);
    pow_x2(&y2, &y1);
    fp12_conj(&y3, &r);
    fp12_mul(&y1, &y1, &y3);
    fp12_conj(&y1, &y1);
    fp12_mul(&y1, &y1, &y2);
    pow_x(&y2, &y1);
    pow_x(&y3, &y2);
    fp12_conj(&y1, &y1);
    fp12_mul(&y3, &y3, &y1);
    fp12_conj(&y1, &y1);
    fp12_frob(&y1, &y1); fp12_frob(&y1, &y1); fp12_frob(&y1, &y1);
    fp12_frob(&y2, &y2); fp12_frob(&y2, &y2);
    fp12_mul(&y1, &y1, &y2);
    pow_x(&y2, &y3);
    fp12_mul(&y2, &y2, &y0);
    fp12_mul(&y2, &y2, &r);
    fp12_mul(&y1, &y1, &y2);
    fp12_frob(&y2, &y3);
    fp12_mul(out, &y1, &y2);
}

/* ============================== curves ============================== */
static fp g1_B;   /* 4 */
static fp2 g2_B;  /* 4 (1 + i) */
static fp2 g2_B3; /* 3 * 4 (1 + i) */

#define F fp
#define G g1
#include "ec_tmpl.h"
#undef F
#undef G
#define F fp2
#define G g2
#include "ec_tmpl.h"
#undef F
#undef G

static g1_aff G1_GEN_A;
static g2_aff G2_GEN_A;

/* ============================== Miller loop ============================== */
typedef struct { fp2 x, y, z; } g2_proj; /* homogeneous projective on the twist */

static void line_dbl(g2_proj* T, fp2* l0, fp2* l2, fp2* l3, const fp* xp, const fp* yp) {
    fp2 a, b, c, e, f, g, h, j, t;
    const fp inv2 = FP_INV2;
    fp2_mul(&a, &T->x, &T->y); fp2_mul_fp(&a, &a, &inv2);
    fp2_sqr(&b, &T->y);
    fp2_sqr(&c, &T->z);
    fp2_mul(&e, &c, &g2_B3);
    fp2_add(&f, &e, &e); fp2_add(&f, &f, &e);
    fp2_add(&g, &b, &f); fp2_mul_fp(&g, &g, &inv2);
    fp2_add(&h, &T->y, &T->z); fp2_sqr(&h, &h); fp2_sub(&h, &h, &b); fp2_sub(&h, &h, &c);
    fp2_sqr(&j, &T->x);
    fp2_sub(l0, &e, &b);                                   /* 3b'Z^2 - Y^2 */
    fp2_add(&t, &j, &j); fp2_add(&t, &t, &j); fp2_mul_fp(l2, &t, xp);  /* 3X^2 x_P */
    fp2_neg(&t, &h); fp2_mul_fp(l3, &t, yp);               /* -2YZ y_P */
    fp2 x3, y3, z3, e2;
    fp2_sub(&t, &b, &f); fp2_mul(&x3, &a, &t);
    fp2_sqr(&y3, &g); fp2_sqr(&e2, &e); fp2_sub(&y3, &y3, &e2); fp2_sub(&y3, &y3, &e2); fp2_sub(&y3, &y3, &e2);
    fp2_mul(&z3, &b, &h);
    T->x = x3; T->y = y3; T->z = z3;
}

static void line_add(g2_proj* T, fp2* l0, fp2* l2, fp2* l3, const g2_aff* Q, const fp* xp, const fp* yp) {
    fp2 theta, lambda, c, d, e, f, g, h, t;
    fp2_mul(&t, &Q->y, &T->z); fp2_sub(&theta, &T->y, &t);
    fp2_mul(&t, &Q->x, &T->z); fp2_sub(&lambda, &T->x, &t);
    fp2_sqr(&c, &theta);
    fp2_sqr(&d, &lambda);
    fp2_mul(&e, &lambda, &d);
    fp2_mul(&f, &T->z, &c);
    fp2_mul(&g, &T->x, &d);
    fp2_add(&h, &e, &f); fp2_sub(&h, &h, &g); fp2_sub(&h, &h, &g);
    fp2 x3, y3, z3;
    fp2_mul(&x3, &lambda, &h);
    fp2_sub(&t, &g, &h); fp2_mul(&y3, &theta, &t); fp2_mul(&t, &e, &T->y); fp2_sub(&y3, &y3, &t);
    fp2_mul(&z3, &T->z, &e);
    T->x = x3; T->y = y3; T->z = z3;
    fp2_mul(l0, &theta, &Q->x); fp2_mul(&t, &lambda, &Q->y); fp2_sub(l0, l0, &t);   /* theta x_Q - lambda y_Q */
    fp2_neg(&t, &theta); fp2_mul_fp(l2, &t, xp);                                    /* -theta x_P */
    fp2_mul_fp(l3, &lambda, yp);                                                    /* lambda y_P */
}

/* prod_k f_{x,Q_k}(P_k), pairs with an infinity point contribute 1 (AMCL ate on O) */
static void miller_multi(fp12* out, const g1_aff* P, const g2_aff* Q, int npairs) {
    g2_proj T[8];
    int live[8];
    fp12 f;
    fp12_set_one(&f);
    for (int k = 0; k < npairs; k++) {
        live[k] = !(P[k].inf || Q[k].inf);
        T[k].x = Q[k].x; T[k].y = Q[k].y; fp2_set_one(&T[k].z);
    }
    for (int i = 62; i >= 0; i--) {
        fp12_sqr(&f, &f);
        for (int k = 0; k < npairs; k++) {
            if (!live[k]) continue;
            fp2 l0, l2, l3;
            line_dbl(&T[k], &l0, &l2, &l3, &P[k].x, &P[k].y);
            fp12_mul_line(&f, &f, &l0, &l2, &l3);
        }
        if ((X_ABS >> i) & 1) {
            for (int k = 0; k < npairs; k++) {
                if (!live[k]) continue;
                fp2 l0, l2, l3;
                line_add(&T[k], &l0, &l2, &l3, &Q[k], &P[k].x, &P[k].y);
                fp12_mul_line(&f, &f, &l0, &l2, &l3);
            }
        }
    }
    fp12_conj(out, &f);
}

/* ============================== codec ============================== */
static void gt_to_bytes(uint8_t* out, const fp12* f) {
    /* AMCL slots a.a, a.b, b.a, b.b, c.a, c.b = W^0, W^3, W^1, W^4, W^2, W^5 */
    const fp2* s[6] = {&f->c0.c0, &f->c1.c1, &f->c1.c0, &f->c0.c2, &f->c0.c1, &f->c1.c2};
    for (int k = 0; k < 6; k++) {
        fp_to_be(out + 96 * k, &s[k]->a);
        fp_to_be(out + 96 * k + 48, &s[k]->b);
    }
}

static void g1_from_bytes(g1_aff* r, const uint8_t* b) {
    if (b[0] != 0x04) { memset(r, 0, sizeof *r); r->inf = 1; return; }
    fp_from_be(&r->x, b + 1);
    fp_from_be(&r->y, b + 49);
    r->inf = 0;
    if (!g1_aff_on_curve(r)) { memset(r, 0, sizeof *r); r->inf = 1; }
}

static void g1_to_bytes(uint8_t* b, const g1_aff* a) {
    b[0] = 0x04;
    if (a->inf) {
        memset(b + 1, 0, 96);
        b[96] = 1;
        return;
    }
    fp_to_be(b + 1, &a->x);
    fp_to_be(b + 49, &a->y);
}

static void g2_from_bytes(g2_aff* r, const uint8_t* b) {
    fp_from_be(&r->x.a, b);
    fp_from_be(&r->x.b, b + 48);
    fp_from_be(&r->y.a, b + 96);
    fp_from_be(&r->y.b, b + 144);
    r->inf = 0;
    if (!g2_aff_on_curve(r)) { memset(r, 0, sizeof *r); r->inf = 1; }
}

static void g2_to_bytes(uint8_t* b, const g2_aff* a) {
    if (a->inf) {
        memset(b, 0, 192);
        b[143] = 1;
        return;
    }
    fp_to_be(b, &a->x.a);
    fp_to_be(b + 48, &a->x.b);
    fp_to_be(b + 96, &a->y.a);
    fp_to_be(b + 144, &a->y.b);
}

/* Fr: 48-byte BE -> canonical little-endian u64[4] mod r */
static void fr_from_be(uint64_t k[4], const uint8_t* b) {
    uint64_t v[6];
    for (int i = 0; i < 6; i++) {
        uint64_t w = 0;
        for (int j = 0; j < 8; j++) w = (w << 8) | b[(5 - i) * 8 + j];
        v[i] = w;
    }
    /* binary long reduction by r << s */
    for (int s = 384 - 255; s >= 0; s--) {
        uint64_t m[6] = {0};
        for (int i = 0; i < 4; i++) {
            int wi = i + s / 64, sh = s % 64;
            if (wi < 6) m[wi] |= RM[i] << sh;
            if (sh && wi + 1 < 6) m[wi + 1] |= RM[i] >> (64 - sh);
        }
        if (geq6(v, m)) sub6(v, v, m);
    }
    memcpy(k, v, 4 * sizeof(uint64_t));
}

static void fr_to_be(uint8_t* b, const uint64_t k[4]) {
    memset(b, 0, 16);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) b[16 + (3 - i) * 8 + j] = (uint8_t)(k[i] >> (56 - 8 * j));
}

/* ============================== init ============================== */
static pthread_once_t init_once = PTHREAD_ONCE_INIT;

static void do_init(void) {
    /* R mod p and R^2 mod p, raw (not Montgomery) */
    static const uint64_t RMODP[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL,
                                      0x77ce585370525745ULL, 0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};
    static const uint64_t R2MODP[6] = {0xf4df1f341c341746ULL, 0x0a76e6a609d104f1ULL, 0x8de5476c4c95b6d5ULL,
                                       0x67eb88a9939d83c0ULL, 0x9a793e85b519952dULL, 0x11988fe592cae3aaULL};
    memcpy(FP_ONE.l, RMODP, sizeof RMODP);
    memcpy(FP_R2.l, R2MODP, sizeof R2MODP);
    {
        fp two;
        fp_add(&two, &FP_ONE, &FP_ONE);
        fp_inv(&FP_INV2, &two);
    }
    static const char* gam[6][2] = {
        {"1", "0"},
        {"1904d3bf02bb0667c231beb4202c0d1f0fd603fd3cbd5f4f7b2443d784bab9c4f67ea53d63e7813d8d0775ed92235fb8",
         "fc3e2b36c4e03288e9e902231f9fb854a14787b6c7b36fec0c8ec971f63c5f282d5ac14d6c7ec22cf78a126ddc4af3"},
        {"0", "1a0111ea397fe699ec02408663d4de85aa0d857d89759ad4897d29650fb85f9b409427eb4f49fffd8bfd00000000aaac"},
        {"6af0e0437ff400b6831e36d6bd17ffe48395dabc2d3435e77f76e17009241c5ee67992f72ec05f4c81084fbede3cc09",
         "6af0e0437ff400b6831e36d6bd17ffe48395dabc2d3435e77f76e17009241c5ee67992f72ec05f4c81084fbede3cc09"},
        {"1a0111ea397fe699ec02408663d4de85aa0d857d89759ad4897d29650fb85f9b409427eb4f49fffd8bfd00000000aaad", "0"},
        {"5b2cfd9013a5fd8df47fa6b48b1e045f39816240c0b8fee8beadf4d8e9c0566c63a3e6e257f87329b18fae980078116",
         "144e4211384586c16bd3ad4afa99cc9170df3560e77982d0db45f3536814f0bd5871c1908bd478cd1ee605167ff82995"}};
    for (int k = 0; k < 6; k++) {
        fp_from_hex(&FROB_G[k].a, gam[k][0]);
        fp_from_hex(&FROB_G[k].b, gam[k][1]);
    }
    fp_from_hex(&g1_B, "4");
    fp_from_hex(&g2_B.a, "4");
    fp_from_hex(&g2_B.b, "4");
    fp2_add(&g2_B3, &g2_B, &g2_B);
    fp2_add(&g2_B3, &g2_B3, &g2_B);
    fp_from_hex(&G1_GEN_A.x, "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb");
    fp_from_hex(&G1_GEN_A.y, "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1");
    G1_GEN_A.inf = 0;
    fp_from_hex(&G2_GEN_A.x.a, "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8");
    fp_from_hex(&G2_GEN_A.x.b, "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e");
    fp_from_hex(&G2_GEN_A.y.a, "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801");
    fp_from_hex(&G2_GEN_A.y.b, "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be");
    G2_GEN_A.inf = 0;
}

static void init(void) { pthread_once(&init_once, do_init); }

/* ============================== PS / Coconut ============================== */
/* mode 0 = SigG2 (reference default: sigma in G2, vk in G1), 1 = SigG1 */
static int sig_bytes(int mode) { return mode == 0 ? 192 : 97; }
static int oth_bytes(int mode) { return mode == 0 ? 97 : 192; }

/* ps_sig ate_2_pairing(s1, o1, s2, o2) with points already decoded into G1/G2 slots */
static void pair2(fp12* gt, const g1_aff* P, const g2_aff* Q) {
    fp12 ml;
    miller_multi(&ml, P, Q, 2);
    final_exp(gt, &ml);
}

/* one Signature::verify; returns verdict (0/1), -1 on length error never (q given) */
static int verify_one(int mode, size_t q, const uint8_t* s1b, const uint8_t* s2b, const uint8_t* msgs,
                      const uint8_t* Xb, const uint8_t* Yb, const uint8_t* gtb, uint8_t* gt_out) {
    uint64_t(*ks)[4] = (uint64_t(*)[4])malloc(sizeof(uint64_t[4]) * (q + 1));
    memset(ks[0], 0, sizeof ks[0]);
    ks[0][0] = 1;
    for (size_t j = 0; j < q; j++) fr_from_be(ks[j + 1], msgs + 48 * j);
    g1_aff P[2];
    g2_aff Q[2];
    int inf1, inf2;
    if (mode == 0) {
        g2_aff s1, s2;
        g2_from_bytes(&s1, s1b);
        g2_from_bytes(&s2, s2b);
        inf1 = s1.inf; inf2 = s2.inf;
        g1_aff* pts = (g1_aff*)malloc(sizeof(g1_aff) * (q + 1));
        g1_from_bytes(&pts[0], Xb);
        for (size_t j = 0; j < q; j++) g1_from_bytes(&pts[j + 1], Yb + 97 * j);
        g1_jac pr;
        g1_msm(&pr, pts, (const uint64_t(*)[4])ks, q + 1);
        free(pts);
        g1_to_aff(&P[0], &pr);
        g1_from_bytes(&P[1], gtb);
        Q[0] = s1;
        Q[1] = s2;
        fp2_neg(&Q[1].y, &s2.y);
    } else {
        g1_aff s1, s2;
        g1_from_bytes(&s1, s1b);
        g1_from_bytes(&s2, s2b);
        inf1 = s1.inf; inf2 = s2.inf;
        g2_aff* pts = (g2_aff*)malloc(sizeof(g2_aff) * (q + 1));
        g2_from_bytes(&pts[0], Xb);
        for (size_t j = 0; j < q; j++) g2_from_bytes(&pts[j + 1], Yb + 192 * j);
        g2_jac pr;
        g2_msm(&pr, pts, (const uint64_t(*)[4])ks, q + 1);
        free(pts);
        g2_to_aff(&Q[0], &pr);
        g2_from_bytes(&Q[1], gtb);
        P[0] = s1;
        P[1] = s2;
        fp_neg(&P[1].y, &s2.y);
    }
    free(ks);
    fp12 gt;
    pair2(&gt, P, Q);
    if (gt_out) gt_to_bytes(gt_out, &gt);
    if (inf1 || inf2) return 0;
    return fp12_is_one(&gt);
}

typedef struct {
    int mode;
    size_t q, lo, hi;
    const uint8_t *s1, *s2, *msgs, *X, *Y, *gtilde;
    int per_cred_vk;
    uint8_t *verdicts, *gts;
} vjob;

static void* vworker(void* arg) {
    vjob* j = (vjob*)arg;
    size_t sb = (size_t)sig_bytes(j->mode), ob = (size_t)oth_bytes(j->mode);
    for (size_t i = j->lo; i < j->hi; i++) {
        const uint8_t* X = j->per_cred_vk ? j->X + i * ob : j->X;
        const uint8_t* Y = j->per_cred_vk ? j->Y + i * ob * j->q : j->Y;
        j->verdicts[i] = (uint8_t)verify_one(j->mode, j->q, j->s1 + i * sb, j->s2 + i * sb, j->msgs + i * 48 * j->q,
                                             X, Y, j->gtilde, j->gts ? j->gts + 576 * i : NULL);
    }
    return NULL;
}

/* Batch of independent Signature::verify calls over nthreads host threads.
 * X/Y: shared verkey (per_cred_vk = 0) or n verkeys (per_cred_vk = 1). */
int oc_verify_batch(int mode, size_t n, size_t q, const uint8_t* s1, const uint8_t* s2, const uint8_t* msgs,
                    const uint8_t* X, const uint8_t* Y, int per_cred_vk, const uint8_t* gtilde,
                    uint8_t* verdicts, uint8_t* gts, int nthreads) {
    init();
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > n) nthreads = (int)(n ? n : 1);
    pthread_t th[256];
    vjob jobs[256];
    int started[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (vjob){mode, q, n * t / nthreads, n * (t + 1) / nthreads, s1, s2, msgs, X, Y, gtilde,
                         per_cred_vk, verdicts, gts};
        started[t] = nthreads > 1 && pthread_create(&th[t], NULL, vworker, &jobs[t]) == 0;
        if (!started[t]) vworker(&jobs[t]);
    }
    for (int t = 0; t < nthreads; t++)
        if (started[t]) pthread_join(th[t], NULL);
    return 0;
}

/* e(P, Q) for one G1 and one G2 encoding (AMCL ate_pairing), GT bytes out */
int oc_pairing(const uint8_t* Pb, const uint8_t* Qb, uint8_t* gt_out) {
    init();
    g1_aff P[1];
    g2_aff Q[1];
    g1_from_bytes(&P[0], Pb);
    g2_from_bytes(&Q[0], Qb);
    fp12 ml, gt;
    miller_multi(&ml, P, Q, 1);
    final_exp(&gt, &ml);
    gt_to_bytes(gt_out, &gt);
    return 0;
}

/* k * generator (group 1 or 2), k as 48-byte BE; output canonical bytes */
int oc_gen_mul(int group, size_t n, const uint8_t* ks, uint8_t* out) {
    init();
    for (size_t i = 0; i < n; i++) {
        uint64_t k[4];
        fr_from_be(k, ks + 48 * i);
        if (group == 1) {
            g1_jac r; g1_aff a;
            g1_mul(&r, &G1_GEN_A, k);
            g1_to_aff(&a, &r);
            g1_to_bytes(out + 97 * i, &a);
        } else {
            g2_jac r; g2_aff a;
            g2_mul(&r, &G2_GEN_A, k);
            g2_to_aff(&a, &r);
            g2_to_bytes(out + 192 * i, &a);
        }
    }
    return 0;
}

typedef struct { int group; size_t lo, hi; const uint8_t* ks; uint8_t* out; } gjob;
static void* gworker(void* arg) {
    gjob* j = (gjob*)arg;
    size_t ob = j->group == 1 ? 97 : 192;
    oc_gen_mul(j->group, j->hi - j->lo, j->ks + 48 * j->lo, j->out + ob * j->lo);
    return NULL;
}

int oc_gen_mul_mt(int group, size_t n, const uint8_t* ks, uint8_t* out, int nthreads) {
    init();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    gjob jobs[256];
    int started[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (gjob){group, n * t / nthreads, n * (t + 1) / nthreads, ks, out};
        started[t] = pthread_create(&th[t], NULL, gworker, &jobs[t]) == 0;
        if (!started[t]) gworker(&jobs[t]);
    }
    for (int t = 0; t < nthreads; t++)
        if (started[t]) pthread_join(th[t], NULL);
    return 0;
}

/* generic MSM on encoded points: group 1/2, n points, 48-B BE scalars, out canonical bytes */
int oc_msm(int group, size_t n, const uint8_t* pts, const uint8_t* ks, uint8_t* out) {
    init();
    uint64_t(*k)[4] = (uint64_t(*)[4])malloc(sizeof(uint64_t[4]) * (n ? n : 1));
    for (size_t i = 0; i < n; i++) fr_from_be(k[i], ks + 48 * i);
    if (group == 1) {
        g1_aff* a = (g1_aff*)malloc(sizeof(g1_aff) * (n ? n : 1));
        for (size_t i = 0; i < n; i++) g1_from_bytes(&a[i], pts + 97 * i);
        g1_jac r; g1_aff ra;
        g1_msm(&r, a, (const uint64_t(*)[4])k, n);
        g1_to_aff(&ra, &r);
        g1_to_bytes(out, &ra);
        free(a);
    } else {
        g2_aff* a = (g2_aff*)malloc(sizeof(g2_aff) * (n ? n : 1));
        for (size_t i = 0; i < n; i++) g2_from_bytes(&a[i], pts + 192 * i);
        g2_jac r; g2_aff ra;
        g2_msm(&r, a, (const uint64_t(*)[4])k, n);
        g2_to_aff(&ra, &r);
        g2_to_bytes(out, &ra);
        free(a);
    }
    free(k);
    return 0;
}

/* Lagrange basis at 0 over the de-duplicated set of the first t ids (secret_sharing [EXT]);
 * out: t x 48-B BE.  Fr arithmetic through Python-free modular ops on 4x64 limbs. */
static void fr_mulmod(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
    /* schoolbook 256x256 -> 512, then reduce by long division (oracle speed is irrelevant) */
    uint64_t t[8] = {0};
    for (int i = 0; i < 4; i++) {
        u128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (u128)a[i] * b[j] + t[i + j];
            t[i + j] = (uint64_t)c;
            c >>= 64;
        }
        t[i + 4] = (uint64_t)c;
    }
    for (int s = 512 - 255; s >= 0; s--) {
        uint64_t m[8] = {0};
        for (int i = 0; i < 4; i++) {
            int wi = i + s / 64, sh = s % 64;
            if (wi < 8) m[wi] |= RM[i] << sh;
            if (sh && wi + 1 < 8) m[wi + 1] |= RM[i] >> (64 - sh);
        }
        int ge = 1;
        for (int i = 7; i >= 0; i--) if (t[i] != m[i]) { ge = t[i] > m[i]; break; }
        if (ge) {
            uint64_t br = 0;
            for (int i = 0; i < 8; i++) { u128 d = (u128)t[i] - m[i] - br; t[i] = (uint64_t)d; br = (uint64_t)(d >> 64) & 1; }
        }
    }
    memcpy(r, t, 32);
}

static void fr_sub(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) {
    uint64_t br = 0, t[4];
    for (int i = 0; i < 4; i++) { u128 d = (u128)a[i] - b[i] - br; t[i] = (uint64_t)d; br = (uint64_t)(d >> 64) & 1; }
    if (br) { uint64_t c = 0; for (int i = 0; i < 4; i++) { u128 s = (u128)t[i] + RM[i] + c; t[i] = (uint64_t)s; c = (uint64_t)(s >> 64); } }
    memcpy(r, t, 32);
}

static void fr_inv(uint64_t r[4], const uint64_t a[4]) {
    uint64_t e[4] = {RM[0] - 2, RM[1], RM[2], RM[3]}, acc[4] = {1, 0, 0, 0}, b[4];
    memcpy(b, a, 32);
    for (int i = 0; i < 256; i++) {
        if ((e[i / 64] >> (i % 64)) & 1) fr_mulmod(acc, acc, b);
        fr_mulmod(b, b, b);
    }
    memcpy(r, acc, 32);
}

int oc_lagrange(size_t t, const uint64_t* ids, uint8_t* out) {
    init();
    for (size_t a = 0; a < t; a++) {
        uint64_t num[4] = {1, 0, 0, 0}, den[4] = {1, 0, 0, 0};
        uint64_t xi[4] = {ids[a], 0, 0, 0};
        for (size_t b = 0; b < t; b++) {
            int dup = 0;
            for (size_t c = 0; c < b; c++) if (ids[c] == ids[b]) dup = 1;
            if (dup || ids[b] == ids[a]) continue;
            uint64_t xj[4] = {ids[b], 0, 0, 0}, d[4];
            fr_mulmod(num, num, xj);
            fr_sub(d, xj, xi);
            fr_mulmod(den, den, d);
        }
        fr_inv(den, den);
        fr_mulmod(num, num, den);
        fr_to_be(out + 48 * a, num);
    }
    return 0;
}

/* Signature::aggregate (signature.rs:448-470) for one credential: sigs = t entries (first t used) */
int oc_signature_aggregate(int mode, size_t len, size_t t, const uint64_t* ids, const uint8_t* s1,
                           const uint8_t* s2, uint8_t* out_s1, uint8_t* out_s2) {
    init();
    if (len < t) return -3;
    size_t sb = (size_t)sig_bytes(mode);
    uint8_t* l = (uint8_t*)malloc(48 * (t ? t : 1));
    oc_lagrange(t, ids, l);
    memcpy(out_s1, s1, sb);
    oc_msm(mode == 0 ? 2 : 1, t, s2, l, out_s2);
    free(l);
    return 0;
}

/* Verkey::aggregate (signature.rs:483-526): X (t entries), Y (t x q) */
int oc_verkey_aggregate(int mode, size_t len, size_t t, size_t q, const uint64_t* ids, const uint8_t* X,
                        const uint8_t* Y, uint8_t* outX, uint8_t* outY) {
    init();
    if (len < t) return -3;
    size_t ob = (size_t)oth_bytes(mode);
    int grp = mode == 0 ? 1 : 2;
    uint8_t* l = (uint8_t*)malloc(48 * (t ? t : 1));
    uint8_t* col = (uint8_t*)malloc(ob * (t ? t : 1));
    oc_lagrange(t, ids, l);
    oc_msm(grp, t, X, l, outX);
    for (size_t j = 0; j < q; j++) {
        for (size_t i = 0; i < t; i++) memcpy(col + ob * i, Y + ob * (i * q + j), ob);
        oc_msm(grp, t, col, l, outY + ob * j);
    }
    free(l);
    free(col);
    return 0;
}

/* PoKOfSignatureProof::verify [EXT] for one proof.
 * revealed_idx/revealed_msgs: r entries; responses: (q - r + 1) x 48 B ordered [g~, hidden Y~ asc].
 * Returns verdict, or -2 on UnequalNoOfBasesExponents. */
int oc_pok_verify(int mode, size_t q, size_t r, const uint8_t* s1b, const uint8_t* s2b, const uint8_t* Jb,
                  const uint8_t* Tb, const uint8_t* responses, size_t nresp, const uint8_t* chal,
                  const uint64_t* revealed_idx, const uint8_t* revealed_msgs, const uint8_t* Xb,
                  const uint8_t* Yb, const uint8_t* gtb, uint8_t* gt_out) {
    init();
    size_t sb = (size_t)sig_bytes(mode), ob = (size_t)oth_bytes(mode);
    int grp = mode == 0 ? 1 : 2;
    /* identity check */
    int inf1, inf2;
    if (mode == 0) { g2_aff a, b; g2_from_bytes(&a, s1b); g2_from_bytes(&b, s2b); inf1 = a.inf; inf2 = b.inf; }
    else { g1_aff a, b; g1_from_bytes(&a, s1b); g1_from_bytes(&b, s2b); inf1 = a.inf; inf2 = b.inf; }
    if (inf1 || inf2) return 0;
    size_t nb = 1;
    uint8_t* bases = (uint8_t*)malloc(ob * (q + 2));
    uint8_t* sc = (uint8_t*)malloc(48 * (q + 2));
    memcpy(bases, gtb, ob);
    for (size_t i = 0; i < q; i++) {
        int rev = 0;
        for (size_t k = 0; k < r; k++) if (revealed_idx[k] == i) rev = 1;
        if (!rev) memcpy(bases + ob * nb++, Yb + ob * i, ob);
    }
    if (nb != nresp) { free(bases); free(sc); return -2; }
    memcpy(sc, responses, 48 * nresp);
    memcpy(bases + ob * nb, Jb, ob);
    memcpy(sc + 48 * nb, chal, 48);
    uint8_t* chk = (uint8_t*)malloc(ob);
    oc_msm(grp, nb + 1, bases, sc, chk);
    int ok_schnorr;
    if (grp == 1) {
        g1_aff a, t; g1_from_bytes(&a, chk); g1_from_bytes(&t, Tb);
        g1_jac ja, jt; g1_from_aff(&ja, &a); g1_from_aff(&jt, &t); g1_neg(&jt, &jt); g1_add(&ja, &ja, &jt);
        ok_schnorr = g1_is_inf(&ja);
    } else {
        g2_aff a, t; g2_from_bytes(&a, chk); g2_from_bytes(&t, Tb);
        g2_jac ja, jt; g2_from_aff(&ja, &a); g2_from_aff(&jt, &t); g2_neg(&jt, &jt); g2_add(&ja, &ja, &jt);
        ok_schnorr = g2_is_inf(&ja);
    }
    if (!ok_schnorr) { free(bases); free(sc); free(chk); return 0; }
    /* J' = X~ + J + sum revealed Y~_i m_i  as an MSM with scalars 1, 1, m_i */
    uint8_t* b2 = (uint8_t*)malloc(ob * (r + 2));
    uint8_t* s2 = (uint8_t*)calloc(r + 2, 48);
    memcpy(b2, Xb, ob); s2[47] = 1;
    memcpy(b2 + ob, Jb, ob); s2[48 + 47] = 1;
    for (size_t k = 0; k < r; k++) {
        memcpy(b2 + ob * (k + 2), Yb + ob * revealed_idx[k], ob);
        memcpy(s2 + 48 * (k + 2), revealed_msgs + 48 * k, 48);
    }
    uint8_t* jp = (uint8_t*)malloc(ob);
    oc_msm(grp, r + 2, b2, s2, jp);
    /* pairing check via verify_one with q = 0 (pr = X = J') */
    int v = verify_one(mode, 0, s1b, s2b, NULL, jp, NULL, gtb, gt_out);
    free(bases); free(sc); free(chk); free(b2); free(s2); free(jp);
    (void)sb;
    return v;
}

int oc_nthreads_hint(void) { return (int)sysconf(_SC_NPROCESSORS_ONLN); }
