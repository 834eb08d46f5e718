// ubench_int.hip — throughput of the integer instructions the modmul chain
// can be built from, on gfx950.  Not part of the product; informs DESIGN.md §3.
// Each thread runs 8 independent chains (throughput, not latency), full chip.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);    \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

constexpr int L = 2048; // iterations per thread
constexpr int C = 8;    // independent chains

__global__ void k_add(uint32_t *out, uint32_t b) {
    uint32_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
    uint32_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_lo(uint32_t *out, uint32_t b) {
    uint32_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
    uint32_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_hi(uint32_t *out, uint32_t b) {
    uint32_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
    uint32_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mul_u24(uint32_t *out, uint32_t b) {
    uint32_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(b));
    uint32_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mad64(uint32_t *out, uint32_t b) {
    uint64_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c)
            asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(a[c]) : "v"(b), "v"(b + c) : "s40", "s41");
    uint64_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
__global__ void k_lshl_add64(uint32_t *out, uint32_t b) {
    uint64_t a[C];
    const uint64_t bb = b;
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a[c]) : "v"(bb));
    uint64_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}
__global__ void k_addc(uint32_t *out, uint32_t b) {
    uint32_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c)
            asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, 0, vcc" : "+v"(a[c]) : "v"(b) : "vcc");
    uint32_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma64(uint32_t *out, uint32_t b) {
    double a[C];
    const double bb = 1.0000001 + b * 1e-12;
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a[c]) : "v"(bb));
    double s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_mad_u24(uint32_t *out, uint32_t b) {
    uint32_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[c]) : "v"(b));
    uint32_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_cndmask(uint32_t *out, uint32_t b) {
    uint32_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c)
            asm volatile("v_cmp_lt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[c]) : "v"(b) : "vcc");
    uint32_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kern_t)(uint32_t *, uint32_t);

int main() {
    int dev = 0;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, dev));
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 8, threads = 256;
    uint32_t *out;
    CHK(hipMalloc(&out, (size_t)blocks * threads * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    struct { const char *name; kern_t k; int insts; } ks[] = {
        {"v_add_u32", k_add, 1},         {"v_mul_lo_u32", k_mul_lo, 1}, {"v_mul_hi_u32", k_mul_hi, 1},
        {"v_mul_u32_u24", k_mul_u24, 1}, {"v_mad_u32_u24", k_mad_u24, 1}, {"v_mad_u64_u32", k_mad64, 1},
        {"v_lshl_add_u64", k_lshl_add64, 1}, {"v_add_co+v_addc_co", k_addc, 2}, {"v_cmp+v_cndmask", k_cndmask, 2},
        {"v_fma_f64", k_fma64, 1},
    };
    printf("{\"cus\": %d, \"clock_mhz\": %d, \"results\": [\n", cus, prop.clockRate / 1000);
    for (size_t i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
        hipLaunchKernelGGL(ks[i].k, dim3(blocks), dim3(threads), 0, 0, out, 3u); // warm
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0, 0));
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ks[i].k, dim3(blocks), dim3(threads), 0, 0, out, 3u);
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        const double waveinst = 5.0 * blocks * (threads / 64) * (double)L * C * ks[i].insts;
        const double per_s = waveinst / (ms * 1e-3);
        // wave-instructions per CU per cycle at the nominal clock
        const double per_cu_clk = per_s / cus / (prop.clockRate * 1e3);
        printf("  {\"op\": \"%s\", \"ms\": %.3f, \"wave_inst_per_s\": %.4e, \"wave_inst_per_cu_per_clk\": %.3f}%s\n",
               ks[i].name, ms, per_s, per_cu_clk, i + 1 < sizeof(ks) / sizeof(ks[0]) ? "," : "");
    }
    printf("]}\n");
    return 0;
}
