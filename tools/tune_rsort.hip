// tune_rsort.hip — where the time of one grouping-sort pass (radix.h) goes.
// 1e8 (key, value) pairs, one process, best of R interleaved rounds:
//   copy        sequential uint2 copy (the bandwidth of a pass's 16 B/item)
//   count       k_rs_count over the keys
//   scatter_u   k_rs_scatter, keys with uniform random 8-bit digits (a real pass)
//   scatter_1   the same with every key's digit 0 (one run per sub-tile: the
//               ranking / staging cost without the scattered write pattern)
//   scatter_16  digits uniform over 16 values (16 runs per sub-tile)
//   scatter_ro  the real pass's reads and ranking, writes of the staged items
//               to the chunk's own range (sequential)
//   scatter_direct  a real pass without LDS staging (each lane writes its item)
// Writes one JSON line per (variant, round-best).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../sidekick_amd/csrc tune_rsort.hip -o tune_rsort
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "radix.h"

using namespace qk;

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

__global__ void k_copy(const uint2 *__restrict__ a, uint2 *__restrict__ b, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

__global__ void k_fill(uint32_t *k, uint32_t *v, uint64_t n, uint32_t mask, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        k[i] = (uint32_t)z & mask;
        v[i] = (uint32_t)(z >> 32);
    }
}

// exclusive scan of cnt (small: R x nwg) on one workgroup
__global__ void k_scan(const uint32_t *cnt, uint32_t *base, uint32_t m) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (m + 1023) / 1024, t = threadIdx.x;
    uint32_t s = 0;
    for (uint32_t j = t * per; j < std::min(m, t * per + per); ++j) s += cnt[j];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        uint32_t a = 0;
        for (int j = 0; j < 1024; ++j) { const uint32_t x = part[j]; part[j] = a; a += x; }
    }
    __syncthreads();
    uint32_t a = part[t];
    for (uint32_t j = t * per; j < std::min(m, t * per + per); ++j) { base[j] = a; a += cnt[j]; }
}

// chunk-local base: every digit's run starts where the chunk starts (writes
// stay inside the chunk's own range: sequential-ish, no global scatter)
__global__ void k_local_base(const uint32_t *cnt, uint32_t *base, uint32_t nwg, uint64_t chunk) {
    const uint32_t w = blockIdx.x;
    if (threadIdx.x == 0) {
        uint32_t a = (uint32_t)(w * chunk);
        for (uint32_t d = 0; d < rsort::R; ++d) { base[d * nwg + w] = a; a += cnt[d * nwg + w]; }
    }
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? (uint64_t)atof(argv[1]) : 100000000ull;
    const int rounds = argc > 2 ? atoi(argv[2]) : 4;
    int dev = 0, ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    uint32_t *k0, *v0, *k1, *v1, *cnt, *base;
    CK(hipMalloc(&k0, n * 8));   // pairs region = k0 .. (k0 + 2n)
    CK(hipMalloc(&k1, n * 8));
    v0 = k0 + n;
    v1 = k1 + n;
    const uint32_t nwg4 = (uint32_t)std::min<uint64_t>((uint64_t)ncu * 4, (n + 4095) / 4096);
    CK(hipMalloc(&cnt, (size_t)rsort::R * nwg4 * 4));
    CK(hipMalloc(&base, (size_t)rsort::R * nwg4 * 4));
    uint32_t *zdp = nullptr;   // k_rs_scatter digit totals: 0 (base holds the full scan)
    CK(hipMalloc(&zdp, rsort::RMAX * 4));
    CK(hipMemset(zdp, 0, rsort::RMAX * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V {
        const char *name;
        uint32_t mask;   // key mask of the input (digit distribution)
        int kind;        // 0 copy, 1 count, 2 scatter (global base), 3 scatter (chunk-local base), 4 direct
        int blk, wgpc;
    };
    const V vs[] = {{"copy", 0xFF, 0, 256, 4},        {"count", 0xFF, 1, 256, 4},
                    {"scatter_u", 0xFF, 2, 256, 4},   {"scatter_u_1024", 0xFF, 2, 1024, 1},
                    {"scatter_1", 0x0, 2, 256, 4},    {"scatter_16", 0xF, 2, 256, 4},
                    {"scatter_ro", 0xFF, 3, 256, 4},  {"scatter_direct", 0xFF, 4, 256, 4}};
    const int nv = sizeof(vs) / sizeof(vs[0]);
    std::vector<float> best(nv, 1e30f);
    for (int r = 0; r < rounds; ++r) {
        for (int i = 0; i < nv; ++i) {
            const V &v = vs[i];
            hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, k0, v0, n, v.mask, 12345ull + r);
            const uint32_t nwg = (uint32_t)std::min<uint64_t>((uint64_t)ncu * v.wgpc, (n + 4095) / 4096);
            const uint64_t chunk = (((n + nwg - 1) / nwg) + 3) & ~(uint64_t)3;
            hipLaunchKernelGGL((rsort::k_rs_count<8, false>), dim3(nwg), dim3(256), 0, 0, k0, n, chunk, 0u, 0xFFu, nwg,
                               cnt);
            if (v.kind == 3) hipLaunchKernelGGL(k_local_base, dim3(nwg), dim3(64), 0, 0, cnt, base, nwg, chunk);
            else hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, 0, cnt, base, rsort::R * nwg);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            switch (v.kind) {
            case 0: hipLaunchKernelGGL(k_copy, dim3(ncu * 8), dim3(256), 0, 0, (const uint2 *)k0, (uint2 *)k1, n); break;
            case 1:
                hipLaunchKernelGGL((rsort::k_rs_count<8, false>), dim3(nwg), dim3(256), 0, 0, k0, n, chunk, 0u, 0xFFu, nwg,
                                   cnt);
                break;
            default:
                if (v.kind == 4)
                    hipLaunchKernelGGL((rsort::k_rs_scatter<8, 256, 16, false, true, true>), dim3(nwg), dim3(256), 0, 0,
                                       k0, v0, n, chunk, 0u, 0xFFu, nwg, base, zdp, k1, v1);
                else if (v.blk == 1024)
                    hipLaunchKernelGGL((rsort::k_rs_scatter<8, 1024, 16, false, true>), dim3(nwg), dim3(1024), 0, 0, k0, v0,
                                       n, chunk, 0u, 0xFFu, nwg, base, zdp, k1, v1);
                else
                    hipLaunchKernelGGL((rsort::k_rs_scatter<8, 256, 16, false, true>), dim3(nwg), dim3(256), 0, 0, k0, v0,
                                       n, chunk, 0u, 0xFFu, nwg, base, zdp, k1, v1);
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best[i] = std::min(best[i], ms);
        }
    }
    for (int i = 0; i < nv; ++i)
        printf("{\"variant\": \"%s\", \"n\": %llu, \"best_ms\": %.4f, \"GBps_16B_per_item\": %.1f}\n", vs[i].name,
               (unsigned long long)n, best[i], 16.0 * n / (best[i] * 1e-3) / 1e9);
    return 0;
}
