// Fp Montgomery-multiplication throughput micro-benchmark for gfx950 (design input for the
// field layer): compares the CIOS 12x32-bit multiply with the radix-2^29
// product-scanning multiply, out-of-line vs inlined, at 1/2/4 waves per SIMD, and measures
// what a large straight-line body (instruction-cache pressure) and live state across calls cost.
//   build: hipcc --offload-arch=gfx950 -O3 tools/ubench_fpmul.hip -o tools/ubench_fpmul
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int NL = 12;
struct Fp {
    uint32_t v[NL];
};
constexpr uint32_t P32[NL] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                              0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
constexpr uint32_t N0 = 0xfffcfffdu;

__device__ __forceinline__ Fp cios(const Fp& a, const Fp& b) {
    uint32_t t[NL];
#pragma unroll
    for (int i = 0; i < NL; i++) {
        const uint32_t bi = b.v[i];
        uint64_t A = (uint64_t)a.v[0] * bi + (i ? t[0] : 0u);
        const uint32_t t0 = (uint32_t)A;
        const uint32_t m = t0 * N0;
        uint64_t C = (uint64_t)m * P32[0] + t0;
#pragma unroll
        for (int j = 1; j < NL; j++) {
            A = (uint64_t)a.v[j] * bi + (uint64_t)(i ? t[j] : 0u) + (A >> 32);
            C = (uint64_t)m * P32[j] + (uint64_t)(uint32_t)A + (C >> 32);
            t[j - 1] = (uint32_t)C;
        }
        t[NL - 1] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
    }
    Fp r;
    for (int j = 0; j < NL; j++) r.v[j] = t[j];
    return r;
}

constexpr int L = 14;
constexpr uint32_t M29 = (1u << 29) - 1;
constexpr uint32_t Q[L] = {0x1fffaaab, 0xff7ffff, 0x14ffffee, 0x17fffd62, 0xf6241ea, 0x9507b58, 0xafd9cc3,
                           0x109e70a2, 0x1764774b, 0x121a5d66, 0x12c6e9ed, 0x12ffcd34, 0x111ea3, 0xd};
constexpr uint32_t NQ = 0x1ffcfffd;

__device__ __forceinline__ void to29(uint32_t o[L], const uint32_t v[NL]) {
#pragma unroll
    for (int k = 0; k < L; k++) {
        int bit = 29 * k, w = bit >> 5, s = bit & 31;
        uint32_t x = s ? __builtin_amdgcn_alignbit((w + 1 < NL) ? v[w + 1] : 0u, v[w], s) : v[w];
        o[k] = x & M29;
    }
}
__device__ __forceinline__ Fp m29(const Fp& A, const Fp& B) {
    uint32_t a[L], b[L], m[L], r[L];
    to29(a, A.v);
    to29(b, B.v);
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * L - 1; k++) {
#pragma unroll
        for (int i = 0; i < L; i++) {
            int j = k - i;
            if (j < 0 || j >= L) continue;
            acc += (uint64_t)a[i] * b[j];
        }
#pragma unroll
        for (int i = 0; i < L; i++) {
            int j = k - i;
            if (i >= k || j < 0 || j >= L) continue;
            acc += (uint64_t)m[i] * Q[j];
        }
        if (k < L) {
            m[k] = ((uint32_t)acc * NQ) & M29;
            acc += (uint64_t)m[k] * Q[0];
        } else {
            r[k - L] = (uint32_t)acc & M29;
        }
        acc >>= 29;
    }
    r[L - 1] = (uint32_t)acc;
    Fp o;
#pragma unroll
    for (int w = 0; w < NL; w++) {
        int bit = 32 * w, k = bit / 29, s = bit % 29;
        uint32_t x = r[k] >> s;
        if (k + 1 < L) x |= r[k + 1] << (29 - s);
        if (s > 26 && k + 2 < L) x |= r[k + 2] << (58 - s);
        o.v[w] = x;
    }
    return o;
}

__device__ __noinline__ Fp cios_call(Fp a, Fp b) { return cios(a, b); }
__device__ __noinline__ Fp m29_call(Fp a, Fp b) { return m29(a, b); }

__device__ __forceinline__ Fp seed_fp(uint32_t s) {
    Fp x;
    for (int j = 0; j < NL; j++) x.v[j] = (s * 2654435761u + j * 0x9e3779b9u) ^ (j << 7);
    x.v[NL - 1] &= 0x0fffffffu;
    return x;
}

// MODE 0: CIOS out-of-line, 1: m29 out-of-line, 2: m29 inlined (2 sites in a rolled loop),
// 3: m29 out-of-line with 16 extra live Fp (192 VGPRs) across the calls,
// 4: m29 inlined, 48 distinct straight-line sites per iteration (~200 KB of code), 5: 288 sites (~1.2 MB)
template <int MODE>
__global__ __launch_bounds__(256) void k_bench(uint32_t* out, int iters) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    Fp a = seed_fp(s), b = seed_fp(s ^ 0x5555u);
    if (MODE == 3) {
        Fp live[16];
#pragma unroll
        for (int k = 0; k < 16; k++) live[k] = seed_fp(s + k * 77);
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int k = 0; k < 16; k++) {
                a = m29_call(a, live[k]);
                live[k].v[k % NL] ^= a.v[0];
            }
        }
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) x ^= live[k].v[3];
        out[s] = a.v[0] ^ a.v[11] ^ x;
        return;
    }
    if (MODE == 4) {
        Fp c = seed_fp(s ^ 0x777u);
        for (int it = 0; it < iters; it++) {
#define CC_S3 a = m29(a, b); b = m29(b, c); c = m29(c, a);
#define CC_S12 CC_S3 CC_S3 CC_S3 CC_S3
            CC_S12 CC_S12 CC_S12 CC_S12
        }
        out[s] = a.v[0] ^ b.v[5] ^ c.v[11];
        return;
    }
    if (MODE == 5) {
        Fp c = seed_fp(s ^ 0x777u);
        for (int it = 0; it < iters; it++) {
#define CC_S48 CC_S12 CC_S12 CC_S12 CC_S12
            CC_S48 CC_S48 CC_S48 CC_S48 CC_S48 CC_S48
        }
        out[s] = a.v[0] ^ b.v[5] ^ c.v[11];
        return;
    }
    for (int it = 0; it < iters; it++) {
#pragma unroll 1
        for (int k = 0; k < 24; k++) {
            if (MODE == 0) {
                a = cios_call(a, b);
                b = cios_call(b, a);
            } else if (MODE == 1) {
                a = m29_call(a, b);
                b = m29_call(b, a);
            } else {
                a = m29(a, b);
                b = m29(b, a);
            }
        }
    }
    out[s] = a.v[0] ^ b.v[11];
}

template <int MODE>
static void run(const char* name, int muls_per_iter, uint32_t* d, int cus) {
    const int iters = 8;
    for (int w = 1; w <= 4; w *= 2) {
        int blocks = cus * w;  // 256 threads = 1 wave per SIMD per block
        hipLaunchKernelGGL(k_bench<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1);
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_bench<MODE>, dim3(blocks), dim3(256), 0, 0, d, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        double muls = (double)blocks * 256 * iters * muls_per_iter;
        printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"fp_mul_per_s\": %.4e}\n", name, w, ms,
               muls / (ms * 1e-3));
        hipEventDestroy(e0);
        hipEventDestroy(e1);
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount;
    uint32_t* d;
    hipMalloc(&d, (size_t)cus * 4 * 256 * 4);
    printf("{\"device\": \"%s\", \"cus\": %d}\n", p.gcnArchName, cus);
    run<0>("cios_call", 48, d, cus);
    run<1>("m29_call", 48, d, cus);
    run<2>("m29_inline_rolled", 48, d, cus);
    run<3>("m29_call_192_live", 16, d, cus);
    run<4>("m29_inline_48_sites", 48, d, cus);
    run<5>("m29_inline_288_sites", 288, d, cus);
    hipFree(d);
    return 0;
}
