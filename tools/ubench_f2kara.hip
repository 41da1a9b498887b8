// Pair-lane Fp2 product prototypes on the lazy radix-2^28 field: the
// product lazy.h ships (lz_f2_mul_v: per lane a c + b d as two 14 x 14 product scans under one
// Montgomery reduction, 392 + 196 mads) against a one-level limb Karatsuba of the same two-product sum
// (7 + 7 split, subtractive form: a c = L + (M' + L + H) X + H X^2 with M' = (a_lo - a_hi)(c_hi - c_lo),
// 3 x 49 product mads per product, 294 + 196 mads; L[j] and H[j] are each needed in two columns, so they
// are formed in temporaries and added twice).  Both are out-of-line calls as in the kernels, at 2
// waves/SIMD (the Miller loop's occupancy).  Prints products/s per variant and a bit-exactness check of
// the two variants' outputs over 2^20 random normalised operand pairs.
//   build: hipcc --offload-arch=gfx950 -O3 -I coconut-rust_amd/csrc tools/ubench_f2kara.hip -o tools/ubench_f2kara
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "lazy.h"

using namespace cc;
using namespace cc::lz;

// the same sum as lz_mont<2>, columns formed by one-level Karatsuba
DEV W14 lz_mont2_kara(const int32_t a[LN], const int32_t c[LN], const int32_t b[LN], const int32_t d[LN]) {
    constexpr int H = LN / 2;
    int32_t sa[H], sc[H], sb[H], sd[H];
#pragma unroll
    for (int i = 0; i < H; i++) {
        sa[i] = a[i] - a[H + i];
        sc[i] = c[H + i] - c[i];
        sb[i] = b[i] - b[H + i];
        sd[i] = d[H + i] - d[i];
    }
    int64_t Ls[2 * H - 1], Hs[2 * H - 1];
    int32_t m[LN];
    W14 r;
    int64_t acc = 0;
#pragma unroll
    for (int col = 0; col < 2 * LN - 1; col++) {
        if (col < 2 * H - 1) {  // L[col]: into its own temporary (used again at col + 7)
            int64_t t = 0;
#pragma unroll
            for (int i = 0; i < H; i++) {
                const int j = col - i;
                if (j < 0 || j >= H) continue;
                t += (int64_t)a[i] * c[j];
                t += (int64_t)b[i] * d[j];
            }
            Ls[col] = t;
            acc += t;
        }
        if (col >= H && col - H < 2 * H - 1) {
            const int k = col - H;
            int64_t h = 0;  // H[k]: used again at col + 7
#pragma unroll
            for (int i = 0; i < H; i++) {
                const int j = k - i;
                if (j < 0 || j >= H) continue;
                h += (int64_t)a[H + i] * c[H + j];
                h += (int64_t)b[H + i] * d[H + j];
            }
            Hs[k] = h;
            int64_t mm = Ls[k];  // M'[k] chained onto L[k]
#pragma unroll
            for (int i = 0; i < H; i++) {
                const int j = k - i;
                if (j < 0 || j >= H) continue;
                mm += (int64_t)sa[i] * sc[j];
                mm += (int64_t)sb[i] * sd[j];
            }
            acc += mm + h;
        }
        if (col >= 2 * H && col - 2 * H < 2 * H - 1) acc += Hs[col - 2 * H];
        lz_redc_col(col, acc, m, r.v);
    }
    r.v[LN - 1] = (int32_t)acc;
    return r;
}


// variant 2: S = U (1 + X) + X M' with U = L + X H: one temporary chain per column (L[c] and H[c-7]
// together), reused once 7 columns later as the start of the M' chain: 7 stashed 64-bit values, two
// 64-bit additions a middle column
DEV W14 lz_mont2_kara2(const int32_t a[LN], const int32_t c[LN], const int32_t b[LN], const int32_t d[LN]) {
    constexpr int H = LN / 2;
    int32_t sa[H], sc[H], sb[H], sd[H];
#pragma unroll
    for (int i = 0; i < H; i++) {
        sa[i] = a[i] - a[H + i];
        sc[i] = c[H + i] - c[i];
        sb[i] = b[i] - b[H + i];
        sd[i] = d[H + i] - d[i];
    }
    int64_t U[3 * H - 1];
    int32_t m[LN];
    W14 r;
    int64_t acc = 0;
#pragma unroll
    for (int col = 0; col < 2 * LN - 1; col++) {
        if (col < 3 * H - 1) {
            int64_t u = 0;
#pragma unroll
            for (int i = 0; i < H; i++) {
                const int j = col - i;
                if (j >= 0 && j < H) {
                    u += (int64_t)a[i] * c[j];
                    u += (int64_t)b[i] * d[j];
                }
                const int k = col - H - i;
                if (k >= 0 && k < H) {
                    u += (int64_t)a[H + i] * c[H + k];
                    u += (int64_t)b[H + i] * d[H + k];
                }
            }
            U[col] = u;
            acc += u;
        }
        if (col >= H) {
            const int k = col - H;
            int64_t mm = U[k];
#pragma unroll
            for (int i = 0; i < H; i++) {
                const int j = k - i;
                if (j < 0 || j >= H) continue;
                mm += (int64_t)sa[i] * sc[j];
                mm += (int64_t)sb[i] * sd[j];
            }
            acc += mm;
        }
        lz_redc_col(col, acc, m, r.v);
    }
    r.v[LN - 1] = (int32_t)acc;
    return r;
}


// variant 3: the shipped product scan with both products on ONE accumulator chain (lz_mont<2> keeps the
// c d products on a second chain and adds it per column)
DEV W14 lz_mont2_1chain(const int32_t a[LN], const int32_t b[LN], const int32_t c[LN], const int32_t d[LN]) {
    int32_t m[LN];
    W14 r;
    int64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * LN - 1; k++) {
#pragma unroll
        for (int i = 0; i < LN; i++) {
            const int j = k - i;
            if (j < 0 || j >= LN) continue;
            acc += (int64_t)a[i] * b[j];
            acc += (int64_t)c[i] * d[j];
        }
        lz_redc_col(k, acc, m, r.v);
    }
    r.v[LN - 1] = (int32_t)acc;
    return r;
}

template <int KV>
DEV W14 f2_mul_kara_v(const W14& x, const W14& y) {
    int32_t xs[LN], b[LN], d[LN];
#pragma unroll
    for (int k = 0; k < LN; k++) {
        xs[k] = swp(x.v[k]);
        b[k] = bc_re(y.v[k]);
        d[k] = bc_im(y.v[k]);
    }
    neg_re14(d);
    if (KV == 3) return lz_mont2_1chain(x.v, b, xs, d);
    return KV == 1 ? lz_mont2_kara(x.v, b, xs, d) : lz_mont2_kara2(x.v, b, xs, d);
}
static __device__ __noinline__ W14 f2_mul_kara_call(LZ_L14(a), LZ_L14(b)) {
    const W14 A = {{LZ_V14(a)}}, B = {{LZ_V14(b)}};
    return f2_mul_kara_v<1>(A, B);
}
static __device__ __noinline__ W14 f2_mul_kara2_call(LZ_L14(a), LZ_L14(b)) {
    const W14 A = {{LZ_V14(a)}}, B = {{LZ_V14(b)}};
    return f2_mul_kara_v<2>(A, B);
}
static __device__ __noinline__ W14 f2_mul_1chain_call(LZ_L14(a), LZ_L14(b)) {
    const W14 A = {{LZ_V14(a)}}, B = {{LZ_V14(b)}};
    return f2_mul_kara_v<3>(A, B);
}
template <int KV>
DEV W14 f2_mul_kara_c(const W14& x, const W14& y) {
    if (KV == 3) return f2_mul_1chain_call(LZ_E14(x), LZ_E14(y));
    return KV == 1 ? f2_mul_kara_call(LZ_E14(x), LZ_E14(y)) : f2_mul_kara2_call(LZ_E14(x), LZ_E14(y));
}

DEV W14 seed_w(uint32_t s) {
    W14 x;
#pragma unroll
    for (int k = 0; k < LN; k++) {
        s = s * 1664525u + 1013904223u;
        x.v[k] = (int32_t)(s >> 4);  // [0, 2^28)
    }
    x.v[LN - 1] &= 0x1ffff;
    return x;
}

template <int V>
__global__ __launch_bounds__(256, 2) void k_bench(int32_t* out, int iters) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    W14 a = seed_w(s), b = seed_w(s ^ 0x9e3779b9u);
    for (int it = 0; it < iters; it++) {
#pragma unroll 1
        for (int k = 0; k < 16; k++) {
            if (V == 0) {
                a = lz_f2_mul_c(a, b);
                b = lz_f2_mul_c(b, a);
            } else {
                a = f2_mul_kara_c<V>(a, b);
                b = f2_mul_kara_c<V>(b, a);
            }
        }
    }
    int32_t x = 0;
#pragma unroll
    for (int k = 0; k < LN; k++) x ^= a.v[k] ^ b.v[k];
    out[s] = x;
}

// both variants on the same operands: every output limb equal
__global__ void k_check(uint32_t* bad, int n) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if ((int)(s >> 1) >= n) return;
    const W14 a = seed_w(s * 7 + 1), b = seed_w(s * 13 + 5);
    const W14 r0 = lz_f2_mul_c(a, b), r1 = f2_mul_kara_c<1>(a, b), r2 = f2_mul_kara_c<2>(a, b),
              r3 = f2_mul_kara_c<3>(a, b);
    uint32_t diff = 0;
#pragma unroll
    for (int k = 0; k < LN; k++) diff |= (uint32_t)(r0.v[k] ^ r1.v[k]) | (uint32_t)(r0.v[k] ^ r2.v[k]) | (uint32_t)(r0.v[k] ^ r3.v[k]);
    if (diff) atomicAdd(bad, 1u);
}

template <int V>
static double run(int32_t* d, int cus, int iters) {
    const int blocks = cus * 8;  // 2 waves/SIMD x 4 SIMDs... 256 lanes a block: 2 blocks a CU at 2 waves/SIMD, 4 rounds
    hipLaunchKernelGGL(k_bench<V>, dim3(blocks), dim3(256), 0, 0, d, 1);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_bench<V>, dim3(blocks), dim3(256), 0, 0, d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    // one Fp2 product per lane PAIR per call
    const double prods = (double)blocks * 128 * iters * 32;
    return prods / (ms * 1e-3);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    int32_t* d;
    uint32_t* bad;
    hipMalloc(&d, (size_t)cus * 8 * 256 * 4);
    hipMalloc(&bad, 4);
    hipMemset(bad, 0, 4);
    const int n = 1 << 20;
    hipLaunchKernelGGL(k_check, dim3((2 * n + 255) / 256), dim3(256), 0, 0, bad, n);
    uint32_t nb = 0;
    hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost);
    printf("{\"device\": \"%s\", \"cus\": %d, \"check_pairs\": %d, \"mismatches\": %u}\n", p.gcnArchName, cus, n, nb);
    for (int rep = 0; rep < 3; rep++) {
        const double v0 = run<0>(d, cus, 256), v1 = run<1>(d, cus, 256), v2 = run<2>(d, cus, 256), v3 = run<3>(d, cus, 256);
        printf("{\"rep\": %d, \"f2_mul_shipped_per_s\": %.4e, \"karatsuba_LH_per_s\": %.4e, \"karatsuba_U_per_s\": %.4e, "
               "\"one_chain_per_s\": %.4e, \"ratio_LH\": %.4f, \"ratio_U\": %.4f, \"ratio_one_chain\": %.4f}\n", rep, v0, v1,
               v2, v3, v1 / v0, v2 / v0, v3 / v0);
    }
    hipFree(d);
    hipFree(bad);
    return nb != 0;
}
