// tune_u64.hip — A/B harness for the u64 baby-step/giant-step encode body
// (sidekick_amd/csrc/bsgs64.h; not product code).  One process, interleaved
// rounds over 1e9 device-resident u64 ids at t = 80; reports ms per launch
// for each variant (carry-counting modes, occupancy, ablations: MACs off,
// modmuls off) and the shader clock (s_memtime vs s_memrealtime).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../sidekick_amd/csrc/bsgs64.h"

using namespace qk;

#define CHK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);           \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

__global__ void k_fill(uint64_t *out, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = splitmix_mix(seed + (i + 1) * GAMMA);
}

template <int NA, int MODE, int SG, int ABL, int OCC, int PF = 0, bool BSH = false, int LD = 0, int PRIO = 0,
          int TR = 0>
__global__ __launch_bounds__(256, OCC) void k_var(const uint64_t *ids, uint64_t n, uint32_t T, uint64_t *partials,
                                                  uint64_t *clk) {
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    bsgs64::body<NA, MODE, SG, ABL, PF, false, BSH, LD, 0, bsgs64::NB, PRIO, TR>(ids, n, T, partials);
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
        clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

struct Var {
    const char *name;
    void (*fn)(const uint64_t *, uint64_t, uint32_t, uint64_t *, uint64_t *);
    int occ;
    int abl = 0;   // ablation: results not compared
};

int main() {
    const uint64_t n = 1000000000ull;
    uint64_t *ids, *part, *clk;
    CHK(hipMalloc(&ids, n * 8));
    CHK(hipMalloc(&part, 2 * 80 * 4096 * 8));
    CHK(hipMalloc(&clk, 2 * 4096 * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, ids, n, 0x5EED0003ull);
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // (the round-3/4 layout and carry-mode variants are in the git history and
    // profiles/r03/tune_u64*.json, profiles/r04/u64/)
    std::vector<Var> vars = {
        {"product: mode3 sg14, row-0 sums at prio 1, MACs at 2", k_var<10, 3, 14, 0, 4, 0, true, 1, 3>, 4},
        {"product-tree step 1 (paired products)", k_var<10, 3, 14, 0, 4, 0, true, 1, 3, 1>, 4},
        {"product-tree step 1, sg16", k_var<10, 3, 16, 0, 4, 0, true, 1, 3, 1>, 4},
        {"product again", k_var<10, 3, 14, 0, 4, 0, true, 1, 3>, 4},
        {"product-tree step 1 (again)", k_var<10, 3, 14, 0, 4, 0, true, 1, 3, 1>, 4},
    };
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    std::vector<double> best(vars.size(), 1e30), ghz(vars.size(), 0);
    std::vector<uint64_t> ref;
    std::vector<bool> ok(vars.size(), true);
    for (int round = 0; round < 4; ++round) {
        for (size_t v = 0; v < vars.size(); ++v) {
            const uint32_t grid = cus * vars[v].occ;
            CHK(hipEventRecord(a));
            hipLaunchKernelGGL(vars[v].fn, dim3(grid), dim3(256), 0, 0, ids, n, 80u, part, clk);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, a, b));
            {   // per power: (sum of lo limbs, sum of hi limbs) over the blocks, folded mod p
                std::vector<uint64_t> pp((size_t)2 * 80 * grid);
                CHK(hipMemcpy(pp.data(), part, pp.size() * 8, hipMemcpyDeviceToHost));
                std::vector<uint64_t> sums(80);
                for (int m = 0; m < 80; ++m) {
                    unsigned __int128 lo = 0, hi = 0;
                    for (uint32_t b = 0; b < grid; ++b) {
                        lo += pp[(size_t)(2 * m) * grid + b];
                        hi += pp[(size_t)(2 * m + 1) * grid + b];
                    }
                    const unsigned __int128 P = (unsigned __int128)0xFFFFFFFFFFFFFFC5ull;
                    sums[m] = (uint64_t)(((lo % P) + ((hi % P) << 32) % P) % P);
                }
                if (v == 0 && round == 0) ref = sums;
                if (vars[v].abl == 0 && sums != ref) ok[v] = false;
            }
            std::vector<uint64_t> h(2 * grid);
            CHK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
            double c = 0, r = 0;
            for (uint32_t i = 0; i < grid; ++i) { c += h[2 * i]; r += h[2 * i + 1]; }
            if (ms < best[v]) { best[v] = ms; ghz[v] = c / r * 0.1; }   // s_memrealtime runs at 100 MHz
        }
    }
    printf("{\"n\": %llu, \"t\": 80, \"variants\": [", (unsigned long long)n);
    for (size_t v = 0; v < vars.size(); ++v)
        printf("%s{\"name\": \"%s\", \"ms\": %.3f, \"ids_per_s\": %.4g, \"shader_ghz\": %.3f, \"bit_exact\": %s}",
               v ? ", " : "", vars[v].name, best[v], n / (best[v] * 1e-3), ghz[v],
               vars[v].abl ? "null" : ok[v] ? "true" : "false");
    printf("]}\n");
    return 0;
}
