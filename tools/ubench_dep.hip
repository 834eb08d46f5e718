// ubench_dep.hip — issue rate of DEPENDENT integer chains vs waves per SIMD
// on gfx950 (not part of the product; informs DESIGN.md §3).  Each thread runs
// C independent chains of dependent instructions; the grid puts W workgroups
// of 256 threads (one wave per SIMD each) on every CU, so W = waves/SIMD.
// Sequences: v_add_u32; v_mad_u64_u32; and the lazy modmul of the BSGS
// encode (field.h mulfold32_fast, as compiled: 2 x v_mad_u64_u32 + 3 simple).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../sidekick_amd/csrc/field.h"

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);    \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

constexpr int L = 4096;

template <int C>
__global__ __launch_bounds__(256) void k_add(uint32_t *out, uint32_t b) {
    uint32_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(b));
    uint32_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int C>
__global__ __launch_bounds__(256) void k_mad(uint32_t *out, uint32_t b) {
    uint64_t a[C];
    for (int c = 0; c < C; ++c) a[c] = threadIdx.x + c;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) {
            uint64_t k;
            asm volatile("v_mad_u64_u32 %0, %1, %2, %2, %0" : "+v"(a[c]), "=s"(k) : "v"(b));
        }
    uint64_t s = 0;
    for (int c = 0; c < C; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s ^ (s >> 32));
}

// C chains y <- mulfold32_fast(y, x); 5 VALU per step
template <int C>
__global__ __launch_bounds__(256) void k_mulfold(uint32_t *out, uint32_t b) {
    uint32_t y[C];
    uint32_t w = 0;
    for (int c = 0; c < C; ++c) y[c] = threadIdx.x * 977u + c + b;
    const uint32_t x = 0x9E3779B1u ^ b;
    for (int i = 0; i < L; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) y[c] = qk::mulfold32_fast(y[c], x, w);
    uint32_t s = w;
    for (int c = 0; c < C; ++c) s += y[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kern_t)(uint32_t *, uint32_t);

int main() {
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t *out;
    CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    struct { const char *name; kern_t k; int chains; int insts; } ks[] = {
        {"v_add_u32", k_add<1>, 1, 1},     {"v_add_u32", k_add<2>, 2, 1},     {"v_add_u32", k_add<4>, 4, 1},
        {"v_add_u32", k_add<8>, 8, 1},     {"v_mad_u64_u32", k_mad<1>, 1, 1}, {"v_mad_u64_u32", k_mad<2>, 2, 1},
        {"v_mad_u64_u32", k_mad<4>, 4, 1}, {"v_mad_u64_u32", k_mad<8>, 8, 1}, {"mulfold32_fast", k_mulfold<1>, 1, 5},
        {"mulfold32_fast", k_mulfold<2>, 2, 5}, {"mulfold32_fast", k_mulfold<4>, 4, 5},
    };
    const int waves[] = {1, 2, 3, 4, 8};
    printf("{\"cus\": %d, \"clock_mhz\": %d, \"note\": \"wave-instructions per CU per clock at the nominal clock; "
           "W = waves per SIMD, C = independent chains per lane\", \"results\": [\n",
           cus, prop.clockRate / 1000);
    bool first = true;
    for (size_t i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
        for (int W : waves) {
            const int blocks = cus * W, threads = 256;
            hipLaunchKernelGGL(ks[i].k, dim3(blocks), dim3(threads), 0, 0, out, 3u); // warm
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(e0, 0));
            for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(ks[i].k, dim3(blocks), dim3(threads), 0, 0, out, 3u);
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            const double waveinst = 3.0 * blocks * (threads / 64) * (double)L * ks[i].chains * ks[i].insts;
            const double per_cu_clk = waveinst / (ms * 1e-3) / cus / (prop.clockRate * 1e3);
            printf("%s  {\"seq\": \"%s\", \"C\": %d, \"W\": %d, \"ms\": %.3f, \"wave_inst_per_cu_per_clk\": %.3f}",
                   first ? "" : ",\n", ks[i].name, ks[i].chains, W, ms, per_cu_clk);
            first = false;
        }
    }
    printf("\n]}\n");
    return 0;
}
