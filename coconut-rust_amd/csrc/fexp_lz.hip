// Final-exponentiation kernel for gfx950 on the lazy radix-2^28 field (lazy.h, tower_lz.h) — AMCL
// `pair::fexp` via amcl_wrapper `GT::ate_2_pairing` (reference src/lib.rs:13).
// Same chain as fexp_pl.hip (easy part, hard part 3 + (x-1)^2 [p^3 + x p^2 + (x^2-1) p + x^3 - x]
// = 3 Phi_12(p) / r, compressed cyclotomic squarings with one batched decompression per pow-by-x),
// one credential per lane pair.
//
// Values that only pass through additions from one squaring to the next (the compressed squaring's
// 3u +- 2v, the Fp12 steps' results) are brought back below 0.57 p by lazy.h reduce() (a top-limb
// quotient estimate and one carried subtraction, ~70 simple ops), not by a product.  Between steps
// the Fp12 values rest in the scratch as reduced lazy values, 14 words per Fp (slot-major SoA).
#ifdef CC_HOT_INLINE  // build option (Makefile HOT_INLINE=1): inline every Fp multiplication
#define CC_FP_INLINE 1
#endif
#include <cstdlib>

#include "codec.h"
#include "tower_lz.h"

namespace cc {
namespace lz {
// Build option CC_FEXP_PROF (tools/fexp_phases.py): per-wave shader-clock totals of the kernel's
// phases, written by lane 0 of each wave with plain vector stores to g_fx_prof[wave][slot].
#ifdef CC_FEXP_PROF
constexpr int kProfSlots = 24, kProfWaves = 8192;
__device__ unsigned long long g_fx_prof[kProfWaves][kProfSlots];
#define FXP_DECL unsigned long long fxp[kProfSlots] = {}
#define FXP_T(v) const unsigned long long v = clock64()
#define FXP_ADD(slot, t0) (fxp[slot] += clock64() - (t0))
#else
#define FXP_DECL
#define FXP_T(v)
#define FXP_ADD(slot, t0)
#endif
namespace {

using F2R = F2<AN, 9>;
using FR = F12<AN, 9>;  // at rest: reduced

template <int A, int B>
DEV F4<AN, 9> rest4(const F4<A, B>& x) {
    return {reduce(x.a), reduce(x.b)};
}
template <int A, int B>
DEV FR rest(const F12<A, B>& x) {
    return {{reduce(x.a.a), reduce(x.a.b)}, {reduce(x.b.a), reduce(x.b.b)}, {reduce(x.c.a), reduce(x.c.b)}};
}

// lazy SoA: Fp slot s, limb k of element i at word (s * LN + k) * n + i; an Fp2 in slots (s, s + 1),
// each lane moving its own half
struct Zs {
    int32_t* p;
    size_t n;
};
DEV void st_z(const Zs& s, int slot, size_t i, const F2R& x) {
    int32_t* q = s.p + (size_t)(slot + (int)half_id()) * LN * s.n + i;
#pragma unroll
    for (int k = 0; k < LN; k++) q[(size_t)k * s.n] = x.c.v[k];
}
DEV F2R ld_z(const Zs& s, int slot, size_t i) {
    const int32_t* q = s.p + (size_t)(slot + (int)half_id()) * LN * s.n + i;
    F2R r;
#pragma unroll
    for (int k = 0; k < LN; k++) r.c.v[k] = q[(size_t)k * s.n];
    return r;
}
DEV void st12(const Zs& s, size_t i, const FR& x) {
    const F2R* v = reinterpret_cast<const F2R*>(&x);
#pragma unroll
    for (int k = 0; k < 6; k++) st_z(s, 2 * k, i, v[k]);
}
DEV FR ld12(const Zs& s, size_t i) {
    FR x;
    F2R* v = reinterpret_cast<F2R*>(&x);
#pragma unroll
    for (int k = 0; k < 6; k++) v[k] = ld_z(s, 2 * k, i);
    return x;
}

enum ZOp { OP_ID = 0, OP_CONJ = 1, OP_FROB = 2, OP_FROB2 = 3 };
DEV FR zapply(const FR& x, int op) {
    if (op == OP_CONJ) return f12_conj(x);
    if (op == OP_FROB) return rest(f12_frob(x));
    if (op == OP_FROB2) return rest(f12_frob2(x));
    return x;
}

// ---------------------------------------------------------------- Fp12 products with one operand in LDS
// The multiplier waits in LDS, packed (78 words a lane: the 512 lanes a CU holds fill its 160 KiB),
// and its coefficients are unpacked right before each use: x, the Karatsuba terms and the results
// are then what lives across the out-of-line products (with both operands in registers every call
// site spilled to scratch).  The memory clobber forces the re-read at each use.
constexpr int FB = 256;  // lanes per block
using Park = int32_t (*)[FB];
DEV void park12(Park lds, const FR& y) {
    const F2R* v = reinterpret_cast<const F2R*>(&y);
#pragma unroll
    for (int k = 0; k < 6; k++) pack_fq<FB>(lds, PW * k, v[k].c);
}
DEV F2R unp(Park lds, int k) {
    asm volatile("" ::: "memory");
    return {unpack_fq<FB, 9>(lds, PW * k)};
}
DEV F4<AN, 9> unp4(Park lds, int j) { return {unp(lds, 2 * j), unp(lds, 2 * j + 1)}; }
DEV FR unpark12(Park lds) {
    return {{unp(lds, 0), unp(lds, 1)}, {unp(lds, 2), unp(lds, 3)}, {unp(lds, 4), unp(lds, 5)}};
}
// x * y, y parked (tower.inc f12_mul)
template <int A, int B>
DEV FR f12_mul_lds(const F12<A, B>& x, Park y) {
    const auto t0 = norm(mul(x.a, unp4(y, 0)));
    const auto t1 = norm(mul(x.b, unp4(y, 1)));
    const auto t2 = norm(mul(x.c, unp4(y, 2)));
    const auto rb = rest4(add(sub(sub(mul(norm(add(x.a, x.b)), norm(add(unp4(y, 0), unp4(y, 1)))), t0), t1), mul_s(t2)));
    const auto rc = rest4(add(sub(sub(mul(norm(add(x.a, x.c)), norm(add(unp4(y, 0), unp4(y, 2)))), t0), t2), t1));
    const auto ra = rest4(add(mul_s(norm(sub(sub(mul(norm(add(x.b, x.c)), norm(add(unp4(y, 1), unp4(y, 2)))), t1), t2))), t0));
    return {ra, rb, rc};
}

// F <- the Miller values (fexp_pl.hip's input: 12 x 32 SoA, R form), in R' form
static __device__ __noinline__ void zx_in(const uint32_t* fbuf, size_t n, Zs dst, size_t i) {
    const Soa F{const_cast<uint32_t*>(fbuf), n};
#pragma unroll 1
    for (int k = 0; k < 6; k++) {
        pl::Fp2 v;
        pl::ld_f2(v, F, 2 * k, i);
        st_z(dst, 2 * k, i, reduce(in_r2(v)));
    }
}
static __device__ __noinline__ void zx_inv(Zs src, Zs dst, size_t i) { st12(dst, i, rest(f12_inv(ld12(src, i)))); }
// dst <- op_a(a) * op_b(b)
// (a == b, opb in {id, conj}: a is read back from LDS, not reloaded from the scratch; conj is an
// involution commuting with the Frobenius maps)
DEV void zx_mul(Zs a, int opa, Zs b, int opb, Zs dst, Park lds, size_t i) {
    park12(lds, zapply(ld12(b, i), opb));
    FR y;
    if (a.p == b.p && (opb == OP_ID || opb == OP_CONJ)) {
        y = unpark12(lds);
        if (opb == OP_CONJ) y = f12_conj(y);
    } else {
        y = ld12(a, i);
    }
    const FR x = zapply(y, opa);
    st12(dst, i, f12_mul_lds(x, lds));
}
// dst <- src^3 (cyclotomic)
static __device__ __noinline__ void zx_cube(Zs src, Zs dst, size_t i) {
    const FR x = ld12(src, i);
    st12(dst, i, rest(f12_mul(rest(f12_cyc_sqr(x)), x)));
}
// dst <- src^x by Granger-Scott square-and-multiply: the fallback of zx_pow_x for a zero
// decompression denominator (never reached by honest inputs)
static __device__ __noinline__ void zx_pow_x_gs(Zs src, Zs dst, size_t i) {
    FR acc = ld12(src, i);
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
        acc = rest(f12_cyc_sqr(acc));
        if ((X_ABS >> b) & 1ull) {
            asm volatile("" ::: "memory");
            acc = rest(f12_mul(acc, ld12(src, i)));
        }
    }
    st12(dst, i, f12_conj(acc));
}

// ---------------------------------------------------------------- compressed cyclotomic squaring
// fexp_pl.hip cyc4_sqr (Karabina's compression restated for this tower):
//     b0' = 3 (2 xi c0 c1) + 2 b0    b1' = 3 (c0^2 + xi c1^2) - 2 b1
//     c0' = 3 (b0^2 + xi b1^2) - 2 c0    c1' = 3 (2 b0 b1) + 2 c1
struct Z4 {
    F2R b0, b1, c0, c1;
};
DEV void z4_sqr(Z4& x) {
    const auto s0 = sqrr(x.b0);
    const auto s1 = sqrr(x.b1);
    const auto Xb = norm(sub(sub(sqrr(add(x.b0, x.b1)), s0), s1));  // 2 b0 b1
    const auto Tb = norm(add(s0, xi(s1)));                           // b0^2 + xi b1^2
    const auto u0 = sqrr(x.c0);
    const auto u1 = sqrr(x.c1);
    const auto Xc = norm(xi(sub(sub(sqrr(add(x.c0, x.c1)), u0), u1)));  // 2 xi c0 c1
    const auto Tc = norm(add(u0, xi(u1)));                              // c0^2 + xi c1^2
    // 3u + 2v = u + 2 (u + v), 3u - 2v = u + 2 (u - v)
    x.b0 = reduce(add(Xc, dbl(add(Xc, x.b0))));
    x.b1 = reduce(add(Tc, dbl(sub(Tc, x.b1))));
    x.c0 = reduce(add(Tb, dbl(sub(Tb, x.c0))));
    x.c1 = reduce(add(Xb, dbl(add(Xb, x.c1))));
}
// numerators and denominator of a0, a1 (fexp_pl.hip cyc4_num)
DEV void z4_num(F2R& n0, F2R& n1, F2R& den, const Z4& x) {
    const auto Nb = norm(sub(sqrr(x.b0), xi(sqrr(x.b1))));  // b0^2 - xi b1^2
    const auto Nc = norm(sub(sqrr(x.c0), xi(sqrr(x.c1))));  // c0^2 - xi c1^2
    n0 = reduce(add(mulr(x.b0, Nb), xi(mulr(x.c1, Nc))));
    n1 = reduce(add(mulr(x.c0, Nc), mulr(x.b1, Nb)));
    den = reduce(dbl(sub(mulr(x.b0, x.c0), xi(mulr(x.b1, x.c1)))));
}
template <class I>
DEV FR z4_expand(const Z4& x, const F2R& n0, const F2R& n1, const I& inv) {
    return {{reduce(mulr(n0, inv)), reduce(mulr(n1, inv))}, {x.b0, x.b1}, {x.c0, x.c1}};
}
// a compressed snapshot (4 Fp2 = 52 packed words a lane) in the park rows, while the squaring loops
// leave LDS free
DEV void park4(Park lds, const Z4& x) {
    pack_fq<FB>(lds, 0, x.b0.c);
    pack_fq<FB>(lds, PW, x.b1.c);
    pack_fq<FB>(lds, 2 * PW, x.c0.c);
    pack_fq<FB>(lds, 3 * PW, x.c1.c);
}
DEV Z4 unpark4(Park lds) { return {unp(lds, 0), unp(lds, 1), unp(lds, 2), unp(lds, 3)}; }
DEV void st_z4(const Zs& K, int base, size_t i, const Z4& x) {
    st_z(K, base + 0, i, x.b0);
    st_z(K, base + 2, i, x.b1);
    st_z(K, base + 4, i, x.c0);
    st_z(K, base + 6, i, x.c1);
}
DEV Z4 ld_z4(const Zs& K, int base, size_t i) {
    return {ld_z(K, base + 0, i), ld_z(K, base + 2, i), ld_z(K, base + 4, i), ld_z(K, base + 6, i)};
}

// dst <- src^x (fexp_pl.hip fx_pow_x): 57 compressed squarings with snapshots g^(2^16), g^(2^48) in K,
// one inversion for the three decompressions, 6 Granger-Scott squarings, 5 Fp12 products, conj.
#ifdef CC_FEXP_PROF
#define FXP_ARG , unsigned long long* fxp
#else
#define FXP_ARG
#endif
template <bool kSnapLds>
DEV void zx_pow_x(Zs src, Zs dst, Zs K, Park lds, size_t i FXP_ARG) {
    FXP_T(t_sq);
    Z4 c{ld_z(src, 4, i), ld_z(src, 6, i), ld_z(src, 8, i), ld_z(src, 10, i)};
    // three loops, the snapshot stores between them (a store inside the loop body gets its address
    // arithmetic spilled and reloaded at every iteration)
#pragma unroll 1
    for (int k = 0; k < 16; k++) z4_sqr(c);
    st_z4(K, 0, i, c);
#pragma unroll 1
    for (int k = 16; k < 48; k++) z4_sqr(c);
    if (kSnapLds) park4(lds, c);
    else st_z4(K, 12, i, c);
#pragma unroll 1
    for (int k = 48; k < 57; k++) z4_sqr(c);
    FXP_ADD(18, t_sq);
    FXP_T(t_dc);
    F2R n0, n1, d57, d16, d48;
    {
        Z4 s = ld_z4(K, 0, i);
        z4_num(n0, n1, d16, s);
        st_z(K, 8, i, n0);
        st_z(K, 10, i, n1);
        s = kSnapLds ? unpark4(lds) : ld_z4(K, 12, i);
        z4_num(n0, n1, d48, s);
        if (kSnapLds) {  // the park rows after the snapshot's four
            pack_fq<FB>(lds, 4 * PW, n0.c);
            pack_fq<FB>(lds, 5 * PW, n1.c);
        } else {
            st_z(K, 20, i, n0);
            st_z(K, 22, i, n1);
        }
    }
    z4_num(n0, n1, d57, c);
    const auto p1 = mulr(d16, d48);
    const auto p2 = mulr(p1, d57);
    if (is_zero(p2)) {  // pair-uniform
        zx_pow_x_gs(src, dst, i);
        return;
    }
    const auto iv = inv(p2);
    st12(dst, i, z4_expand(c, n0, n1, mulr(iv, p1)));  // y = g^(2^57), waits in dst
    const auto iv2 = mulr(iv, d57);                   // (d16 d48)^-1
    park12(lds, z4_expand(kSnapLds ? unpark4(lds) : ld_z4(K, 12, i), kSnapLds ? unp(lds, 4) : ld_z(K, 20, i),
                          kSnapLds ? unp(lds, 5) : ld_z(K, 22, i), mulr(iv2, d16)));  // g^(2^48)
    {
        const FR acc = f12_mul_lds(z4_expand(ld_z4(K, 0, i), ld_z(K, 8, i), ld_z(K, 10, i), mulr(iv2, d48)),
                                   lds);  // g^(2^16) g^(2^48)
        FXP_ADD(19, t_dc);
        park12(lds, ld12(dst, i));        // y
        st12(K, i, f12_mul_lds(acc, lds));  // acc waits in K while y squares in LDS
    }
    // then y^2 three times, acc *= y (2^60), y^2 twice, acc *= y (2^62), y^2, acc *= y (2^63)
    constexpr uint32_t kSq = 0b010110111u;  // from bit 0: S S S M S S M S M  (1 = square)
    FXP_T(t_tl);
#pragma unroll 1
    for (int st = 0; st < 9; st++) {
        if ((kSq >> st) & 1u) park12(lds, rest(f12_cyc_sqr(unpark12(lds))));
        else st12(K, i, f12_mul_lds(ld12(K, i), lds));
    }
    st12(dst, i, f12_conj(ld12(K, i)));
    FXP_ADD(20, t_tl);
}

// verdict and GT bytes of the result (fexp_pl.hip fexp_out), through the storage form
DEV void zexp_out(size_t i, const FR& res, const uint32_t* flags, uint8_t* verdicts, uint8_t* gt_out) {
    pl::Fp12 r;
    pl::Fp2* v = reinterpret_cast<pl::Fp2*>(&r);
    const F2R* z = reinterpret_cast<const F2R*>(&res);
#pragma unroll 1
    for (int k = 0; k < 6; k++) v[k] = out_r2(z[k]);
    const uint32_t fl = flags ? flags[i] : 0u;
    const bool ok = pl::f12_is_one(r) && (fl & 11u) == 0;  // sigma_1/sigma_2 = O or PoK Schnorr failure
    if (!half_id()) verdicts[i] = ok ? 1 : 0;
    if (gt_out) {  // each lane writes its halves: Fp slots 2k + h of the AMCL FP12 order
        uint8_t* o = gt_out + i * 576 + 48 * half_id();
        for (int k = 0; k < 6; k++) {
            Fp c;
            fp_from_mont(c, v[k].c);
            store_be48_aligned(o + 96 * k, c);
        }
    }
}

// the chain after the easy part's inversion (fexp_pl.hip fexp_chain); regions F 0, T 1, A 2, S 3, R 4
struct ZStep {
    uint8_t kind, a, opa, b, opb, d;  // kind 0: d = op_a(a) op_b(b); 1: d = a^x; 2: d = a^3
};
__constant__ static const ZStep kChain[16] = {
    {0, 0, OP_CONJ, 1, OP_ID, 0},    // f^(p^6 - 1)
    {0, 0, OP_FROB2, 0, OP_ID, 0},   // ^(p^2 + 1)
    {2, 0, 0, 0, 0, 4},              // res = f^3
    {1, 0, 0, 0, 0, 1},              // t = f^x
    {0, 1, OP_ID, 0, OP_CONJ, 1},    // t = f^(x-1)
    {1, 1, 0, 0, 0, 2},              // a = t^x
    {0, 2, OP_ID, 1, OP_CONJ, 2},    // a = f^((x-1)^2)
    {0, 2, OP_FROB2, 2, OP_CONJ, 3},
    {0, 3, OP_FROB, 4, OP_ID, 4},    // res *= (a^(p^2) a^-1)^p
    {1, 2, 0, 0, 0, 1},              // b = a^x
    {0, 1, OP_FROB2, 1, OP_CONJ, 3},
    {0, 3, OP_ID, 4, OP_ID, 4},      // res *= b^(p^2) b^-1
    {1, 1, 0, 0, 0, 2},              // c = b^x
    {0, 2, OP_FROB, 4, OP_ID, 4},    // res *= c^p
    {1, 2, 0, 0, 0, 1},              // d = c^x
    {0, 1, OP_ID, 4, OP_ID, 4},      // res *= d
};

}  // namespace

// fbuf: Miller output f (12 x 32 SoA, 12 slots); scratch: 84 lazy Fp slots (F, T, A, S, R, K)
template <bool kSnapLds>
__global__ __launch_bounds__(256, 2) void k_fexp_lz(size_t n, const uint32_t* __restrict__ fbuf,
                                                 int32_t* __restrict__ scratch, const uint32_t* __restrict__ flags,
                                                 uint8_t* __restrict__ verdicts, uint8_t* __restrict__ gt_out) {
    __shared__ int32_t lds[6 * PW][FB];
    const size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 1;  // credential of this lane pair
    if (i >= n) return;  // pair-uniform
    const size_t sl = (size_t)LN * n;
    const Zs F{scratch, n}, T{scratch + 12 * sl, n}, A{scratch + 24 * sl, n}, S{scratch + 36 * sl, n},
        R{scratch + 48 * sl, n}, K{scratch + 60 * sl, n};
    FXP_DECL;
    FXP_T(t_in);
    zx_in(fbuf, n, F, i);
    FXP_ADD(0, t_in);
    FXP_T(t_inv);
    zx_inv(F, T, i);
    FXP_ADD(1, t_inv);
    // The rest of the chain as ONE loop over its steps with the product and the pow-by-x inlined once
    // each: an out-of-line step function saves and restores every callee-saved register it touches
    // (~330 scratch instructions a call, ~20 calls a lane pair).
#pragma unroll 1
    for (int s = 0; s < 16; s++) {
        const ZStep z = kChain[s];
        const Zs a{scratch + z.a * 12 * sl, n}, b{scratch + z.b * 12 * sl, n}, d{scratch + z.d * 12 * sl, n};
        FXP_T(t_st);
        if (z.kind == 0) zx_mul(a, z.opa, b, z.opb, d, lds, i);
#ifdef CC_FEXP_PROF
        else if (z.kind == 1) zx_pow_x<kSnapLds>(a, d, K, lds, i, fxp);
#else
        else if (z.kind == 1) zx_pow_x<kSnapLds>(a, d, K, lds, i);
#endif
        else zx_cube(a, d, i);
        FXP_ADD(2 + s, t_st);
    }
    FXP_T(t_out);
    zexp_out(i, ld12(R, i), flags, verdicts, gt_out);
    FXP_ADD(21, t_out);
#ifdef CC_FEXP_PROF
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0 && wave < (size_t)kProfWaves)
        for (int k = 0; k < kProfSlots; k++) g_fx_prof[wave][k] = fxp[k];
#endif
}

}  // namespace lz
}  // namespace cc

// scratch: 84 x 14 words per element (cc_ctx sizes it for this kernel)
#ifdef CC_FEXP_PROF
extern "C" int cck_fexp_prof_read(unsigned long long* out, size_t nwaves) {
    if (nwaves > (size_t)cc::lz::kProfWaves) nwaves = cc::lz::kProfWaves;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(cc::lz::g_fx_prof), nwaves * cc::lz::kProfSlots * 8, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int cck_fexp_lz(size_t n, const uint32_t* d_f, uint32_t* d_scratch, const uint32_t* d_flags,
                           uint8_t* d_verdicts, uint8_t* d_gt, hipStream_t st) {
    if (!n) return 0;
    hipLaunchKernelGGL(cc::lz::k_fexp_lz<true>, dim3((unsigned)((2 * n + 255) / 256)), dim3(256), 0, st, n, d_f,
                       reinterpret_cast<int32_t*>(d_scratch), d_flags, d_verdicts, d_gt);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
