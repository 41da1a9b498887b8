// Device self-test of the lazy radix-2^28 field core (lazy.h) and of the divstep inversions (field.h
// fp_inv_int, tower_q.h fp_inv_int_quad) — test infrastructure exported through the C ABI
// (cc_selftest_lazy) so tests/test_gpu_lazy.py can drive the kernels' exact code on the device with
// inputs at the limits the compile-time bounds allow and check them against Python big integers.
// Not on any verification path.
#include "tower_q.h"

namespace {

// op 0: (a b + c d) / R' (lz_mont<2>); op 1: a b / R' (lz_mont<1>); op 2: reduce(a); op 3: squeeze(a);
// op 4: fp_inv_int(a) and op 5: fp_inv_int_quad(a) on a plain integer a < p in limbs 0..11 (op 5: the
// four lanes of each quad must hold the same a).
// One kernel per op: with a runtime op the four paths shared one exit block and hipcc (ROCm 7.2)
// left limb 0 of the squeeze path in an undefined register (an implicit-def merged at the shared
// store) — separate instantiations keep each path's control flow trivial.
template <int op>
__global__ __launch_bounds__(256) void k_lz_selftest(size_t n, const int32_t* __restrict__ a,
                                                     const int32_t* __restrict__ b, const int32_t* __restrict__ c,
                                                     const int32_t* __restrict__ d, int32_t* __restrict__ out) {
    using namespace cc::lz;
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t x[LN], y[LN], u[LN], v[LN];
#pragma unroll
    for (int k = 0; k < LN; k++) {
        x[k] = a[i * LN + k];
        y[k] = b[i * LN + k];
        u[k] = c[i * LN + k];
        v[k] = d[i * LN + k];
    }
    W14 r;
    if constexpr (op == 4 || op == 5) {
        cc::Fp fa, fr;
#pragma unroll
        for (int k = 0; k < cc::NL; k++) fa.v[k] = (uint32_t)x[k];
        if constexpr (op == 4) cc::fp_inv_int(fr, fa);
        else fp_inv_int_quad(fr, fa);
#pragma unroll
        for (int k = 0; k < LN; k++) r.v[k] = k < cc::NL ? (int32_t)fr.v[k] : 0;
    } else if constexpr (op == 0) {
        r = lz_mont<2>(x, y, u, v);
    } else if constexpr (op == 1) {
        r = lz_mont<1>(x, y, x, y);
    } else {
        Fq<2047, 32768> q;
#pragma unroll
        for (int k = 0; k < LN; k++) q.v[k] = x[k];
        if constexpr (op == 2) {
            const auto z = reduce(q);
#pragma unroll
            for (int k = 0; k < LN; k++) r.v[k] = z.v[k];
        } else {
            const auto z = squeeze(q);
#pragma unroll
            for (int k = 0; k < LN; k++) r.v[k] = z.v[k];
        }
    }
#pragma unroll
    for (int k = 0; k < LN; k++) out[i * LN + k] = r.v[k];
}

}  // namespace

// host buffers of n x 14 int32 limbs each; returns 0 on success, -1 on a HIP error or bad op
extern "C" int cc_selftest_lazy(int op, size_t n, const int32_t* h_a, const int32_t* h_b, const int32_t* h_c,
                                const int32_t* h_d, int32_t* h_out) {
    if (op < 0 || op > 5 || !n) return -1;
    const size_t bytes = n * cc::lz::LN * sizeof(int32_t);
    int32_t* dv[5] = {};
    int rc = 0;
    for (int k = 0; k < 5 && !rc; k++)
        if (hipMalloc(&dv[k], bytes) != hipSuccess) rc = -1;
    const int32_t* hs[4] = {h_a, h_b ? h_b : h_a, h_c ? h_c : h_a, h_d ? h_d : h_a};
    for (int k = 0; k < 4 && !rc; k++)
        if (hipMemcpy(dv[k], hs[k], bytes, hipMemcpyHostToDevice) != hipSuccess) rc = -1;
    if (!rc) {
        const dim3 g((unsigned)((n + 255) / 256)), b(256);
        if (op == 0) hipLaunchKernelGGL(k_lz_selftest<0>, g, b, 0, 0, n, dv[0], dv[1], dv[2], dv[3], dv[4]);
        else if (op == 1) hipLaunchKernelGGL(k_lz_selftest<1>, g, b, 0, 0, n, dv[0], dv[1], dv[2], dv[3], dv[4]);
        else if (op == 2) hipLaunchKernelGGL(k_lz_selftest<2>, g, b, 0, 0, n, dv[0], dv[1], dv[2], dv[3], dv[4]);
        else if (op == 3) hipLaunchKernelGGL(k_lz_selftest<3>, g, b, 0, 0, n, dv[0], dv[1], dv[2], dv[3], dv[4]);
        else if (op == 4) hipLaunchKernelGGL(k_lz_selftest<4>, g, b, 0, 0, n, dv[0], dv[1], dv[2], dv[3], dv[4]);
        else hipLaunchKernelGGL(k_lz_selftest<5>, g, b, 0, 0, n, dv[0], dv[1], dv[2], dv[3], dv[4]);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = -1;
    }
    if (!rc && hipMemcpy(h_out, dv[4], bytes, hipMemcpyDeviceToHost) != hipSuccess) rc = -1;
    for (int k = 0; k < 5; k++)
        if (dv[k]) (void)hipFree(dv[k]);
    return rc;
}
