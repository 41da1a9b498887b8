/* Elliptic-curve template for the C oracle — TEST INFRASTRUCTURE ONLY.
 * Included twice by bls_oracle.c: G = g1 over F = fp, and G = g2 over F = fp2.
 * Short Weierstrass y^2 = x^3 + b, a = 0, Jacobian coordinates (x = X/Z^2, y = Y/Z^3).
 * Restates the point arithmetic amcl_wrapper/AMCL ECP, ECP2 perform [EXT]; results are group
 * elements, so only the (canonical affine) outputs are compared. */
#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)
#define FN(x) CAT(F, CAT(_, x))
#define GN(x) CAT(G, CAT(_, x))

typedef struct { F x, y, z; } GN(jac);
typedef struct { F x, y; int inf; } GN(aff);

static int GN(is_inf)(const GN(jac) * p) { return FN(is_zero)(&p->z); }

static void GN(set_inf)(GN(jac) * p) {
    FN(set_one)(&p->x);
    FN(set_one)(&p->y);
    FN(set_zero)(&p->z);
}

static void GN(from_aff)(GN(jac) * r, const GN(aff) * a) {
    if (a->inf) { GN(set_inf)(r); return; }
    r->x = a->x; r->y = a->y; FN(set_one)(&r->z);
}

static void GN(to_aff)(GN(aff) * r, const GN(jac) * p) {
    if (GN(is_inf)(p)) { FN(set_zero)(&r->x); FN(set_zero)(&r->y); r->inf = 1; return; }
    F zi, zi2, zi3;
    FN(inv)(&zi, &p->z);
    FN(sqr)(&zi2, &zi);
    FN(mul)(&zi3, &zi2, &zi);
    FN(mul)(&r->x, &p->x, &zi2);
    FN(mul)(&r->y, &p->y, &zi3);
    r->inf = 0;
}

/* dbl-2009-l */
static void GN(dbl)(GN(jac) * r, const GN(jac) * p) {
    if (GN(is_inf)(p)) { *r = *p; return; }
    F A, Bq, C, D, E, Fv, t;
    FN(sqr)(&A, &p->x);
    FN(sqr)(&Bq, &p->y);
    FN(sqr)(&C, &Bq);
    FN(add)(&t, &p->x, &Bq);
    FN(sqr)(&t, &t);
    FN(sub)(&t, &t, &A);
    FN(sub)(&t, &t, &C);
    FN(add)(&D, &t, &t);
    FN(add)(&E, &A, &A);
    FN(add)(&E, &E, &A);
    FN(sqr)(&Fv, &E);
    F z3;
    FN(mul)(&z3, &p->y, &p->z);
    FN(add)(&z3, &z3, &z3);
    F x3;
    FN(sub)(&x3, &Fv, &D);
    FN(sub)(&x3, &x3, &D);
    F y3, c8;
    FN(sub)(&t, &D, &x3);
    FN(mul)(&y3, &E, &t);
    FN(add)(&c8, &C, &C);
    FN(add)(&c8, &c8, &c8);
    FN(add)(&c8, &c8, &c8);
    FN(sub)(&y3, &y3, &c8);
    r->x = x3; r->y = y3; r->z = z3;
}

/* add-2007-bl with the exceptional cases handled */
static void GN(add)(GN(jac) * r, const GN(jac) * p, const GN(jac) * q) {
    if (GN(is_inf)(p)) { *r = *q; return; }
    if (GN(is_inf)(q)) { *r = *p; return; }
    F z1z1, z2z2, u1, u2, s1, s2, h, i, j, rr, v, t;
    FN(sqr)(&z1z1, &p->z);
    FN(sqr)(&z2z2, &q->z);
    FN(mul)(&u1, &p->x, &z2z2);
    FN(mul)(&u2, &q->x, &z1z1);
    FN(mul)(&s1, &p->y, &q->z);
    FN(mul)(&s1, &s1, &z2z2);
    FN(mul)(&s2, &q->y, &p->z);
    FN(mul)(&s2, &s2, &z1z1);
    FN(sub)(&h, &u2, &u1);
    FN(sub)(&rr, &s2, &s1);
    if (FN(is_zero)(&h)) {
        if (FN(is_zero)(&rr)) { GN(dbl)(r, p); return; }
        GN(set_inf)(r);
        return;
    }
    FN(add)(&rr, &rr, &rr);
    FN(add)(&i, &h, &h);
    FN(sqr)(&i, &i);
    FN(mul)(&j, &h, &i);
    FN(mul)(&v, &u1, &i);
    F x3, y3, z3;
    FN(sqr)(&x3, &rr);
    FN(sub)(&x3, &x3, &j);
    FN(sub)(&x3, &x3, &v);
    FN(sub)(&x3, &x3, &v);
    FN(sub)(&t, &v, &x3);
    FN(mul)(&y3, &rr, &t);
    FN(mul)(&t, &s1, &j);
    FN(add)(&t, &t, &t);
    FN(sub)(&y3, &y3, &t);
    FN(add)(&z3, &p->z, &q->z);
    FN(sqr)(&z3, &z3);
    FN(sub)(&z3, &z3, &z1z1);
    FN(sub)(&z3, &z3, &z2z2);
    FN(mul)(&z3, &z3, &h);
    r->x = x3; r->y = y3; r->z = z3;
}

static void GN(neg)(GN(jac) * r, const GN(jac) * p) {
    *r = *p;
    FN(neg)(&r->y, &p->y);
}

static int GN(aff_on_curve)(const GN(aff) * a) {
    if (a->inf) return 1;
    F l, rr;
    FN(sqr)(&l, &a->y);
    FN(sqr)(&rr, &a->x);
    FN(mul)(&rr, &rr, &a->x);
    FN(add)(&rr, &rr, &CAT(G, _B));
    return FN(eq)(&l, &rr);
}

/* width-5 wNAF of a 256-bit scalar (little-endian u64[4]); returns digit count */
static int GN(wnaf)(int8_t* out, const uint64_t k_in[4]) {
    uint64_t k[5] = {k_in[0], k_in[1], k_in[2], k_in[3], 0};
    int n = 0;
    while (k[0] | k[1] | k[2] | k[3] | k[4]) {
        int d = 0;
        if (k[0] & 1) {
            d = (int)(k[0] & 31);
            if (d >= 16) d -= 32;
            /* k -= d */
            if (d > 0) {
                uint64_t b = (uint64_t)d;
                for (int w = 0; w < 5; w++) { uint64_t o = k[w]; k[w] = o - b; b = (o < b); }
            } else {
                uint64_t c = (uint64_t)(-d);
                for (int w = 0; w < 5; w++) { uint64_t o = k[w]; k[w] = o + c; c = (k[w] < o); }
            }
        }
        out[n++] = (int8_t)d;
        for (int w = 0; w < 4; w++) k[w] = (k[w] >> 1) | (k[w + 1] << 63);
        k[4] >>= 1;
    }
    return n;
}

/* amcl_wrapper multi_scalar_mul_var_time restated as interleaved (Straus) width-5 wNAF */
static void GN(msm)(GN(jac) * r, const GN(aff) * pts, const uint64_t (*ks)[4], size_t n) {
    enum { TBL = 8 };
    GN(jac)* tbl = (GN(jac)*)malloc(sizeof(GN(jac)) * TBL * (n ? n : 1));
    int8_t(*naf)[260] = (int8_t(*)[260])calloc(n ? n : 1, 260);
    int maxlen = 0;
    for (size_t i = 0; i < n; i++) {
        GN(jac) p, p2;
        GN(from_aff)(&p, &pts[i]);
        GN(dbl)(&p2, &p);
        tbl[i * TBL] = p;
        for (int j = 1; j < TBL; j++) GN(add)(&tbl[i * TBL + j], &tbl[i * TBL + j - 1], &p2);
        int len = GN(wnaf)(naf[i], ks[i]);
        if (len > maxlen) maxlen = len;
    }
    GN(jac) acc;
    GN(set_inf)(&acc);
    for (int b = maxlen - 1; b >= 0; b--) {
        GN(dbl)(&acc, &acc);
        for (size_t i = 0; i < n; i++) {
            int d = naf[i][b];
            if (!d) continue;
            if (d > 0) {
                GN(add)(&acc, &acc, &tbl[i * TBL + (d >> 1)]);
            } else {
                GN(jac) t;
                GN(neg)(&t, &tbl[i * TBL + ((-d) >> 1)]);
                GN(add)(&acc, &acc, &t);
            }
        }
    }
    *r = acc;
    free(tbl);
    free(naf);
}

static void GN(mul)(GN(jac) * r, const GN(aff) * p, const uint64_t k[4]) {
    GN(msm)(r, p, (const uint64_t(*)[4])k, 1);
}

#undef FN
#undef GN
