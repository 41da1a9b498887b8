// Integer-multiply issue-rate micro-benchmark for gfx950 (sets the roofline denominator,
// SURVEY.md §8d "Peak").  Each lane runs K independent dependency chains of one instruction
// kind; throughput = instructions issued / elapsed, reported per CU per cycle and chip-wide.
//   build: hipcc --offload-arch=gfx950 -O3 tools/ubench_int.hip -o tools/ubench_int
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHAINS 8
#define ITERS 4096

__global__ void k_mad64(uint64_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x * 2654435761u + seed;
    uint64_t acc[CHAINS];
    uint32_t b[CHAINS];
    for (int c = 0; c < CHAINS; c++) { acc[c] = a + c; b[c] = a ^ (c * 0x9e3779b9u); }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
            uint64_t r;
            uint64_t cy;
            asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cy) : "v"(b[c]), "v"((uint32_t)acc[c]), "v"(acc[c]));
            acc[c] = r;
        }
    }
    uint64_t s = 0;
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint64_t* out, uint32_t seed) {
    uint32_t acc[CHAINS], b[CHAINS];
    uint32_t a = threadIdx.x * 2654435761u + seed;
    for (int c = 0; c < CHAINS; c++) { acc[c] = a + c; b[c] = a ^ (c * 0x9e3779b9u) | 1; }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b[c]));
    }
    uint64_t s = 0;
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi(uint64_t* out, uint32_t seed) {
    uint32_t acc[CHAINS], b[CHAINS];
    uint32_t a = threadIdx.x * 2654435761u + seed;
    for (int c = 0; c < CHAINS; c++) { acc[c] = a + c; b[c] = a ^ (c * 0x9e3779b9u) | 1; }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b[c]));
    }
    uint64_t s = 0;
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addco(uint64_t* out, uint32_t seed) {
    uint32_t acc[CHAINS], b[CHAINS];
    uint32_t a = threadIdx.x * 2654435761u + seed;
    for (int c = 0; c < CHAINS; c++) { acc[c] = a + c; b[c] = a ^ (c * 0x9e3779b9u); }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
            uint64_t cy;
            asm volatile("v_add_co_u32 %0, %1, %0, %2\n\tv_addc_co_u32 %0, %1, %0, %2, %1" : "+v"(acc[c]), "=&s"(cy) : "v"(b[c]));
        }
    }
    uint64_t s = 0;
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_fma64(uint64_t* out, uint32_t seed) {
    double acc[CHAINS], b[CHAINS];
    double a = (double)(threadIdx.x + seed) * 1e-3;
    for (int c = 0; c < CHAINS; c++) { acc[c] = a + c; b[c] = 0.999999 + c * 1e-9; }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(acc[c]) : "v"(b[c]));
    }
    double s = 0;
    for (int c = 0; c < CHAINS; c++) s += acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ void k_add(uint64_t* out, uint32_t seed) {
    uint32_t acc[CHAINS], b[CHAINS];
    uint32_t a = threadIdx.x * 2654435761u + seed;
    for (int c = 0; c < CHAINS; c++) { acc[c] = a + c; b[c] = a ^ (c * 0x9e3779b9u); }
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b[c]));
    }
    uint64_t s = 0;
    for (int c = 0; c < CHAINS; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// plain-C multiply-add chains, as the field code writes them (c + (u64)a * b): the compiler's own
// v_mad_u64_u32 with a dead carry-out, no asm hazard padding.  NC independent chains per lane.
template <int NC>
__global__ void k_mad64_c(uint64_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x * 2654435761u + seed;
    uint64_t acc[NC];
    uint32_t b[NC];
    for (int c = 0; c < NC; c++) { acc[c] = a + c; b[c] = a ^ (c * 0x9e3779b9u); }
    for (int it = 0; it < ITERS * CHAINS / NC; it++) {
#pragma unroll
        for (int c = 0; c < NC; c++) acc[c] = acc[c] + (uint64_t)b[c] * (uint32_t)acc[c];
    }
    uint64_t s = 0;
    for (int c = 0; c < NC; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// dependent chain latency: one chain only
__global__ void k_mad64_lat(uint64_t* out, uint32_t seed) {
    uint32_t b = threadIdx.x * 2654435761u + seed;
    uint64_t acc = b;
    for (int it = 0; it < ITERS * CHAINS; it++) {
        uint64_t r, cy;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cy) : "v"(b), "v"((uint32_t)acc), "v"(acc));
        acc = r;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static double run(kfn k, int blocks, int threads, uint64_t* d, int instr_per_chain_iter) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double waves = (double)blocks * threads / 64.0 * 5;
    double winstr = waves * (double)ITERS * CHAINS * instr_per_chain_iter;
    return winstr / (ms * 1e-3);  // wave-instructions per second
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount;
    printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.gcnArchName, cus, p.clockRate);
    uint64_t* d;
    hipMalloc(&d, sizeof(uint64_t) * 4096 * 1024);
    struct { const char* name; kfn k; int ipc; } ks[] = {
        {"v_mad_u64_u32", k_mad64, 1}, {"v_mul_lo_u32", k_mullo, 1}, {"v_mul_hi_u32", k_mulhi, 1},
        {"v_add_co+v_addc_co", k_addco, 2}, {"v_add_u32", k_add, 1}, {"v_fma_f64", k_fma64, 1}, {"v_mad_u64_u32_latency_1chain", k_mad64_lat, 1},
        {"v_mad_u64_u32_plainC_2chains", k_mad64_c<2>, 1}, {"v_mad_u64_u32_plainC_4chains", k_mad64_c<4>, 1},
        {"v_mad_u64_u32_plainC_8chains", k_mad64_c<8>, 1}, {"v_mad_u64_u32_plainC_16chains", k_mad64_c<16>, 1}};
    for (auto& e : ks) {
        for (int wps = 1; wps <= 8; wps *= 2) {
            int threads = 256;  // 4 waves per block -> one per SIMD
            int blocks = cus * wps;
            double wi = run(e.k, blocks, threads, d, e.ipc);
            double per_cu_cycle = wi / cus / (p.clockRate * 1e3);
            printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"wave_instr_per_s\": %.4g, \"lane_ops_per_s\": %.4g, "
                   "\"wave_instr_per_cu_per_clk\": %.3f}\n",
                   e.name, wps, wi, wi * 64, per_cu_cycle);
        }
    }
    hipFree(d);
    return 0;
}
