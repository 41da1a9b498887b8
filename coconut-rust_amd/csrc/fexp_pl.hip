// Final-exponentiation kernel for gfx950 (AMCL `pair::fexp` via amcl_wrapper `GT::ate_2_pairing`,
// reference src/lib.rs:13), pair-lane form (tower_pl.h): one credential per
// pair of adjacent lanes, each lane holding one half of every Fp2 value.
//
// CC_FP_INLINE: the multiplications are inlined inside each step function; the steps themselves are
// out of line and exchange Fp12 values through a per-lane SoA scratch (one load/store per step,
// against thousands of Fp multiplications per step), so each step's code exists once.
#ifdef CC_HOT_INLINE  // build option (Makefile HOT_INLINE=1): inline every Fp multiplication
#define CC_FP_INLINE 1
#endif
#include "codec.h"
#include "tower_pl.h"

namespace cc {
namespace pl {

// ================================================================ final exponentiation
// f^((p^6-1)(p^2+1)) then the hard part 3 + (x-1)^2 [p^3 + x p^2 + (x^2-1) p + x^3 - x]
// (= 3*Phi_12(p)/r, AMCL's exponent).  Each step below is one out-of-line function reading its
// Fp12 operands from, and writing its result to, a per-lane SoA slot (12 Fp slots each).
enum FxOp { OP_ID = 0, OP_CONJ = 1, OP_FROB = 2, OP_FROB2 = 3 };

DEV void fx_apply(Fp12& x, int op) {
    if (op == OP_CONJ) {
        f12_conj(x, x);
    } else if (op == OP_FROB) {
        Fp12 t = x;
        f12_frob(x, t);
    } else if (op == OP_FROB2) {
        Fp12 t = x;
        f12_frob2(x, t);
    }
}

// dst <- src^-1
static __device__ __noinline__ void fx_inv(Soa src, Soa dst, size_t i) {
    Fp12 f, t;
    ld_f12(f, src, i);
    f12_inv(t, f);
    st_f12(dst, i, t);
}

// dst <- src^3 (cyclotomic)
static __device__ __noinline__ void fx_cube(Soa src, Soa dst, size_t i) {
    Fp12 f, r;
    ld_f12(f, src, i);
    f12_cyc_sqr(r, f);
    f12_mul(r, r, f);
    st_f12(dst, i, r);
}

// dst <- src^x, x = -|x| (cyclotomic square-and-multiply, then conj).  The base is re-read from src at
// each of the 5 multiplications instead of being held in registers across the 63 squarings.
static __device__ __noinline__ void fx_pow_x(Soa src, Soa dst, size_t i) {
    Fp12 acc;
    ld_f12(acc, src, i);
    for (int b = 62; b >= 0; b--) {
        f12_cyc_sqr(acc, acc);
        if ((X_ABS >> b) & 1ull) {
            asm volatile("" ::: "memory");  // keep the reload inside the loop
            Fp12 y;
            ld_f12(y, src, i);
            f12_mul(acc, acc, y);
        }
    }
    f12_conj(acc, acc);
    st_f12(dst, i, acc);
}

// dst <- op_a(a) * op_b(b)
static __device__ __noinline__ void fx_mul(Soa a, int opa, Soa b, int opb, Soa dst, size_t i) {
    Fp12 x, y;
    ld_f12(x, a, i);
    fx_apply(x, opa);
    ld_f12(y, b, i);
    fx_apply(y, opb);
    f12_mul(x, x, y);
    st_f12(dst, i, x);
}

// fbuf: Miller output f (12 slots); scratch: 4 x 12 slots (T, A, S, R)
__global__ __launch_bounds__(256, 2) void k_fexp(size_t n, uint32_t* __restrict__ fbuf, uint32_t* __restrict__ scratch,
                                              const uint32_t* __restrict__ flags, uint8_t* __restrict__ verdicts,
                                              uint8_t* __restrict__ gt_out) {
    const size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 1;  // credential of this lane pair
    if (i >= n) return;  // pair-uniform
    const Soa F{fbuf, n};
    const Soa T{scratch, n}, A{scratch + (size_t)12 * NL * n, n}, S{scratch + (size_t)24 * NL * n, n},
        R{scratch + (size_t)36 * NL * n, n};
    fx_inv(F, T, i);
    fx_mul(F, OP_CONJ, T, OP_ID, F, i);  // f^(p^6 - 1)
    fx_mul(F, OP_FROB2, F, OP_ID, F, i); // ^(p^2 + 1)
    fx_cube(F, R, i);                    // res = f^3
    fx_pow_x(F, T, i);
    fx_mul(T, OP_ID, F, OP_CONJ, T, i);  // t = f^(x-1)
    fx_pow_x(T, A, i);
    fx_mul(A, OP_ID, T, OP_CONJ, A, i);  // a = f^((x-1)^2)
    fx_mul(A, OP_FROB2, A, OP_CONJ, S, i);
    fx_mul(S, OP_FROB, R, OP_ID, R, i);  // res *= (a^(p^2) a^-1)^p
    fx_pow_x(A, T, i);                   // b = a^x
    fx_mul(T, OP_FROB2, T, OP_CONJ, S, i);
    fx_mul(S, OP_ID, R, OP_ID, R, i);    // res *= b^(p^2) b^-1
    fx_pow_x(T, A, i);                   // c = b^x
    fx_mul(A, OP_FROB, R, OP_ID, R, i);  // res *= c^p
    fx_pow_x(A, T, i);                   // d = c^x
    fx_mul(T, OP_ID, R, OP_ID, R, i);    // res *= d
    Fp12 res;
    ld_f12(res, R, i);
    const uint32_t fl = flags ? flags[i] : 0u;
    const bool ok = f12_is_one(res) && (fl & 11u) == 0;  // sigma_1/sigma_2 = O or PoK Schnorr failure
    if (!half_id()) verdicts[i] = ok ? 1 : 0;
    if (gt_out) {  // each lane writes its halves: Fp slots 2k + h of the AMCL FP12 order
        const Fp2* v = reinterpret_cast<const Fp2*>(&res);
        uint8_t* o = gt_out + i * 576 + 48 * half_id();
        for (int k = 0; k < 6; k++) {
            Fp c;
            fp_from_mont(c, v[k].c);
            store_be48_aligned(o + 96 * k, c);
        }
    }
}

}  // namespace pl
}  // namespace cc

static inline unsigned nblocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

extern "C" int cck_fexp_pl(size_t n, uint32_t* d_f, uint32_t* d_scratch, const uint32_t* d_flags, uint8_t* d_verdicts,
                        uint8_t* d_gt, hipStream_t st) {
    if (!n) return 0;
    hipLaunchKernelGGL(cc::pl::k_fexp, dim3(nblocks(2 * n, 256)), dim3(256), 0, st, n, d_f, d_scratch, d_flags, d_verdicts,
                       d_gt);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
