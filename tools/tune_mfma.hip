// tune_mfma.hip — A/B harness for the matrix-core u32 encode body
// (sidekick_amd/csrc/mfma8.h; not product code).  Interleaved rounds over 1e9
// device-resident u32 ids; ms per launch for each shape and ablation (LDS
// stores off, transposed reads off, MFMAs off, modmuls off) plus the shader
// clock (s_memtime vs s_memrealtime).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../sidekick_amd/csrc/mfma8.h"

using namespace qk;

#define CHK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);           \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

__global__ void k_fill(uint32_t *out, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)(splitmix_mix(seed + (i + 1) * GAMMA) >> 32);
}

template <int NM, int NN, int ABL, int PIPE = 1, int OCC = 1>
__global__ __launch_bounds__(256, OCC) void k_var(const uint32_t *ids, uint64_t n, uint64_t *partials, uint64_t *clk) {
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    mf8::body<NM, NN, ABL, PIPE>(ids, n, partials);
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

struct Var {
    const char *name;
    void (*fn)(const uint32_t *, uint64_t, uint64_t *, uint64_t *);
};

int main(int argc, char **argv) {
    const uint64_t n = 1000000000ull;
    uint32_t *ids;
    uint64_t *part, *clk;
    CHK(hipMalloc(&ids, n * 4));
    CHK(hipMalloc(&part, 256 * 8192 * 8));
    CHK(hipMalloc(&clk, 2 * 8192 * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, ids, n, 0x5EED0001ull);
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<Var> vars = {
        {"t32 (1,2)", k_var<1, 2, 0>},
        {"t32 (1,2) no pipe", k_var<1, 2, 0, 0>},
        {"t32 ablate: no LDS stores", k_var<1, 2, 1>},
        {"t32 ablate: no tr reads", k_var<1, 2, 2>},
        {"t32 ablate: no MFMA", k_var<1, 2, 3>},
        {"t32 ablate: no modmuls", k_var<1, 2, 4>},
        {"t32 ablate: no stores, no reads", k_var<1, 2, 5>},
        {"t32 ablate: VALU only (modmuls, xor)", k_var<1, 2, 6>},
        {"t32 ablate: loads + MFMA only", k_var<1, 2, 7>},
        {"t32 (1,2) occ4", k_var<1, 2, 0, 1, 4>},
        {"t32 VALU only occ4", k_var<1, 2, 6, 1, 4>},
        {"t16 (1,1)", k_var<1, 1, 0>},
        {"t64 (2,2)", k_var<2, 2, 0>},
        {"t64 (2,2) no pipe", k_var<2, 2, 0, 0>},
        {"t64 ablate: no modmuls", k_var<2, 2, 4>},
        {"t128 (2,4)", k_var<2, 4, 0>},
        {"t256 (4,4)", k_var<4, 4, 0>},
    };
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    std::vector<double> best(vars.size(), 1e30), ghz(vars.size(), 0);
    const int wgpc = argc > 1 ? atoi(argv[1]) : 8;
    for (int round = 0; round < 4; ++round) {
        for (size_t v = 0; v < vars.size(); ++v) {
            int occ = 0;
            CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vars[v].fn, 256, 0));
            const uint32_t grid = cus * (occ < wgpc ? occ : wgpc);
            if (round == 0 && v < 1) printf("# occupancy (workgroups/CU) of variant 0: %d\n", occ);
            CHK(hipEventRecord(a));
            hipLaunchKernelGGL(vars[v].fn, dim3(grid), dim3(256), 0, 0, ids, n, part, clk);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, a, b));
            std::vector<uint64_t> h(2 * grid);
            CHK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
            double c = 0, r = 0;
            for (uint32_t i = 0; i < grid; ++i) { c += h[2 * i]; r += h[2 * i + 1]; }
            if (ms < best[v]) { best[v] = ms; ghz[v] = c / r * 0.1; }   // s_memrealtime runs at 100 MHz
        }
    }
    printf("{\"n\": %llu, \"variants\": [", (unsigned long long)n);
    for (size_t v = 0; v < vars.size(); ++v)
        printf("%s\n {\"name\": \"%s\", \"ms\": %.3f, \"ids_per_s\": %.4g, \"shader_ghz\": %.3f}", v ? "," : "",
               vars[v].name, best[v], n / (best[v] * 1e-3), ghz[v]);
    printf("]}\n");
    return 0;
}
