// tune_bsgs.hip — A/B harness for the t = 32 BSGS encode body (not product
// code).  One process, interleaved rounds, 1e9 device-resident ids; every
// variant's power sums are checked against the first variant's.  Each
// workgroup's thread 0 records s_memtime (shader clock) and s_memrealtime
// (constant wall clock) around its body, so the harness also reports the
// shader clock the body actually ran at.
//
// Variants: bsgs::body<8, 4, SG> (sidekick_amd/csrc/bsgs.h) for several SG =
// number of 4-wide accumulator groups whose wraps are counted on the scalar
// unit (groups 0-1: the a = 0 add row, 2-7: MAC rows), plus the previous
// product kernel (compiler-generated a = 0 row, canon of each id).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../sidekick_amd/csrc/bsgs.h"

using namespace qk;

#define CHK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);           \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr int T = 32;
constexpr int BLOCK = 256;

__global__ void k_fill(uint32_t *out, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)(splitmix_mix(seed + (i + 1) * GAMMA) >> 32);
}

// ---- the previous product kernel (round-1 commit 5cc9059), for reference --
namespace legacy {
__device__ __forceinline__ void mac4(uint64_t &a0, uint64_t &a1, uint64_t &a2, uint64_t &a3, uint32_t &c0,
                                     uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t A, uint32_t b0,
                                     uint32_t b1, uint32_t b2, uint32_t b3) {
    uint64_t k0, k1, k2, k3;
    asm("v_mad_u64_u32 %0, %8, %12, %13, %0\n\t"
        "v_mad_u64_u32 %1, %9, %12, %14, %1\n\t"
        "v_mad_u64_u32 %2, %10, %12, %15, %2\n\t"
        "v_mad_u64_u32 %3, %11, %12, %16, %3\n\t"
        "v_addc_co_u32_e64 %4, %8, %4, 0, %8\n\t"
        "v_addc_co_u32_e64 %5, %9, %5, 0, %9\n\t"
        "v_addc_co_u32_e64 %6, %10, %6, 0, %10\n\t"
        "v_addc_co_u32_e64 %7, %11, %7, 0, %11"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "=&s"(k0),
          "=&s"(k1), "=&s"(k2), "=&s"(k3)
        : "v"(A), "v"(b0), "v"(b1), "v"(b2), "v"(b3));
}
template <int NB, int NA>
struct BsgsAcc {
    uint64_t a0[NB];
    uint64_t m[NA - 1][NB];
    uint32_t c[NA - 1][NB];
};
template <int NB, int NA>
__device__ __forceinline__ uint32_t powers(uint32_t id, uint32_t (&B)[NB], uint32_t (&A)[NA - 1]) {
    uint32_t wrapped = 0;
    B[0] = canon32(id);
#pragma unroll
    for (int b = 1; b < NB; ++b) B[b] = mulfold32_fast(B[b - 1], B[0], wrapped);
    A[0] = B[NB - 1];
#pragma unroll
    for (int a = 1; a < NA - 1; ++a) A[a] = mulfold32_fast(A[a - 1], A[0], wrapped);
    return wrapped;
}
template <int NB, int NA>
__device__ __forceinline__ void powers_exact(uint32_t (&B)[NB], uint32_t (&A)[NA - 1]) {
#pragma unroll
    for (int b = 1; b < NB; ++b) B[b] = mulfold32_exact(B[b - 1], B[0]);
    A[0] = B[NB - 1];
#pragma unroll
    for (int a = 1; a < NA - 1; ++a) A[a] = mulfold32_exact(A[a - 1], A[0]);
}
__device__ void body(const uint32_t *__restrict__ ids, uint64_t n, uint64_t *__restrict__ partials) {
    constexpr int NB = 8, NA = 4;
    __shared__ uint64_t sm[4 * 32];
    BsgsAcc<NB, NA> S;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        S.a0[b] = 0;
#pragma unroll
        for (int a = 0; a < NA - 1; ++a) { S.m[a][b] = 0; S.c[a][b] = 0; }
    }
    const uint64_t gtid = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * BLOCK;
    const uint64_t body = n >> 2;
    const uint4 *__restrict__ v = reinterpret_cast<const uint4 *>(ids);
    const uint32_t iters = gtid < body ? (uint32_t)((body - gtid + nthr - 1) / nthr) : 0u;
    const uint4 *__restrict__ p = v + gtid;
    uint4 nxt = iters ? *p : make_uint4(0, 0, 0, 0);
    for (uint32_t it = 0; it < iters; ++it) {
        const uint4 w = nxt;
        p += nthr;
        if (it + 1 < iters) nxt = *p;
        const uint32_t wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            uint32_t B[NB], A[NA - 1];
            const uint32_t wrapped = powers<NB, NA>(wv[c], B, A);
            if (__builtin_expect(__any(wrapped), 0)) {
                if (wrapped) powers_exact<NB, NA>(B, A);
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) S.a0[b] += B[b];
#pragma unroll
            for (int a = 0; a < NA - 1; ++a)
#pragma unroll
                for (int b = 0; b < NB; b += 4)
                    mac4(S.m[a][b], S.m[a][b + 1], S.m[a][b + 2], S.m[a][b + 3], S.c[a][b], S.c[a][b + 1],
                         S.c[a][b + 2], S.c[a][b + 3], A[a], B[b], B[b + 1], B[b + 2], B[b + 3]);
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            uint64_t x;
            if (a == 0) x = fold64_32(S.a0[b]);
            else x = (uint64_t)fold64_32(S.m[a - 1][b]) + fold64_32((uint64_t)S.c[a - 1][b] * 25u);
            x = fold64_32(x);
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) x += bsgs::shfl_xor_u64(x, off);
            if (lane == 0) sm[wave * 32 + a * NB + b] = x;
        }
    }
    __syncthreads();
    if (threadIdx.x < 32) {
        uint64_t s = 0;
        for (int w = 0; w < 4; ++w) s += sm[w * 32 + threadIdx.x];
        partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = s;
    }
}
} // namespace legacy

__device__ __forceinline__ void clk_begin(uint64_t &c0, uint64_t &r0) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void clk_end(uint64_t *clk, uint64_t c0, uint64_t r0) {
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = c1 - c0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

__global__ __launch_bounds__(BLOCK, 3) void k_legacy(const uint32_t *ids, uint64_t n, uint64_t *partials,
                                                     uint64_t *clk) {
    uint64_t c0, r0;
    clk_begin(c0, r0);
    legacy::body(ids, n, partials);
    clk_end(clk, c0, r0);
}

template <int SG, int ROW0, int FOLD, bool PAIR = false, int MINW = 3>
__global__ __launch_bounds__(BLOCK, MINW) void k_sg(const uint32_t *ids, uint64_t n, uint64_t *partials,
                                                    uint64_t *clk) {
    uint64_t c0, r0;
    clk_begin(c0, r0);
    bsgs::body<bsgs::Cfg<8, 4, SG, ROW0, FOLD, PAIR>>(ids, n, 0, T, partials);
    clk_end(clk, c0, r0);
}

// s_setprio around the MAC phase (bsgs.h Cfg PRIO)
template <int PRIO, int SG = 8, int MINW = 5, bool TREE = false, bool PAIR = false>
__global__ __launch_bounds__(BLOCK, MINW) void k_prio(const uint32_t *ids, uint64_t n, uint64_t *partials,
                                                      uint64_t *clk) {
    uint64_t c0, r0;
    clk_begin(c0, r0);
    bsgs::body<bsgs::Cfg<8, 4, SG, 1, 1, PAIR, false, 0, TREE, PRIO>>(ids, n, 0, T, partials);
    clk_end(clk, c0, r0);
}

// product-tree babies (bsgs.h Cfg TREE): same modmuls, dependency depth 3
template <int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void k_tree(const uint32_t *ids, uint64_t n, uint64_t *partials,
                                                      uint64_t *clk) {
    uint64_t c0, r0;
    clk_begin(c0, r0);
    bsgs::body<bsgs::Cfg<8, 4, 8, 1, 1, false, false, 0, true>>(ids, n, 0, T, partials);
    clk_end(clk, c0, r0);
}

__global__ void k_fin(const uint64_t *partials, uint32_t nb, uint32_t *out) {
    const uint32_t m = threadIdx.x;
    if (m >= T) return;
    uint64_t s = 0;
    for (uint32_t b = 0; b < nb; ++b) s += fold64_32(partials[(size_t)m * nb + b]);
    out[m] = canon32(fold64_32(s));
}

typedef void (*KFn)(const uint32_t *, uint64_t, uint64_t *, uint64_t *);
struct Var {
    std::string name;
    KFn k;
};

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1000000000ull;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    int wall_khz = 0;
    CHK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
    uint32_t *ids;
    uint64_t *partials, *clk;
    uint32_t *out;
    CHK(hipMalloc(&ids, n * 4));
    CHK(hipMalloc(&partials, 64ull << 20));
    CHK(hipMalloc(&clk, 1ull << 20));
    CHK(hipMalloc(&out, T * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, ids, n, 0x5EED0002ull);
    CHK(hipDeviceSynchronize());

    // SG counts row-0 groups (0-1) only when ROW0 == 0; with ROW0 == 1 the
    // scalar groups start at the first MAC group (g = 2)
    // round-1 measurements: legacy 3.13 ms; row 0 as mads +
    // min-tracked folds + all MAC wraps scalar (r1f1_sg8) 2.73 ms at 4 waves,
    // 2.67 ms at 5 waves; burst-free interleaved scalar counting 3.12 ms;
    // compiler-scheduled popcounts spill SGPRs; the whole accumulate as one
    // asm statement (no asm-boundary nops) 2.71 vs 2.71 ms.  Ablations (wrong sums): no
    // scalar counting 2.58 ms, no MACs 1.69 ms.
    // round 4 (profiles/r04/check2/tune_bsgs_prio.json): s_setprio around the
    // MAC phase 2.56 vs 2.62-2.63 ms (the product since), around the modmuls
    // 2.68; with priority (profiles/r04/prio/tune_bsgs_prio_sweep.json): 4
    // waves/SIMD 2.73 vs 2.63-2.66, 7 / 6 scalar-counted groups 3.42 / 4.05,
    // product-tree babies 2.57; again (tune_bsgs_prio_tree.json) tree 2.559 /
    // 2.569 vs product 2.559 / 2.587: even, not adopted; two ids interleaved
    // (PAIR) under priority 2.72 (w4) vs 2.64-2.71 (tune_bsgs_prio_pair.json).
    // The priority window without row 0 2.67 / 2.67, row 0 at 1 and the MAC
    // rows at 2 2.652 / 2.654 vs 2.720 / 2.733 (tune_bsgs_prio_levels.json).
    // More schemes (tune_bsgs_prio_levels2.json): rows rising 2 -> 3 2.68,
    // row 0 above the rows 2.70, 4 waves 2.75.  This set: row 0 after the MAC
    // rows
    std::vector<Var> vars = {{"prio_row0_1_macrows_2_w5 (product)", k_prio<4>},
                             {"prio_macrows_2_then_row0_1_w5", k_prio<7>},
                             {"prio_mac_w5 (one level)", k_prio<1>},
                             {"prio_row0_1_macrows_2_w5_again", k_prio<4>},
                             {"prio_macrows_2_then_row0_1_w5_again", k_prio<7>}};
    uint32_t ref[T], got[T];
    std::vector<std::vector<float>> times(vars.size());
    std::vector<double> mhz(vars.size(), 0.0);
    std::vector<int> grids(vars.size()), bad(vars.size(), 0);
    for (size_t v = 0; v < vars.size(); ++v) {
        int occ = 0;
        CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vars[v].k, BLOCK, 0));
        grids[v] = occ * prop.multiProcessorCount;
    }
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    std::vector<uint64_t> hclk;
    for (int r = 0; r < rounds + 1; ++r) {
        for (size_t v = 0; v < vars.size(); ++v) {
            CHK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(vars[v].k, dim3(grids[v]), dim3(BLOCK), 0, 0, ids, n, partials, clk);
            CHK(hipEventRecord(e1, 0));
            hipLaunchKernelGGL(k_fin, dim3(1), dim3(64), 0, 0, partials, (uint32_t)grids[v], out);
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            CHK(hipMemcpy(got, out, sizeof(got), hipMemcpyDeviceToHost));
            if (r == 0 && v == 0) memcpy(ref, got, sizeof(ref));
            if (memcmp(ref, got, sizeof(ref))) {
                printf("MISMATCH %s round %d\n", vars[v].name.c_str(), r);
                bad[v] = 1;
            }
            if (r) {
                times[v].push_back(ms);
                hclk.resize(2 * grids[v]);
                CHK(hipMemcpy(hclk.data(), clk, hclk.size() * 8, hipMemcpyDeviceToHost));
                double cs = 0, rs = 0;
                for (int b = 0; b < grids[v]; ++b) { cs += hclk[2 * b]; rs += hclk[2 * b + 1]; }
                mhz[v] += (cs / rs) * wall_khz / 1e3 / rounds;
            }
        }
    }
    printf("{\"n\": %llu, \"wall_khz\": %d, \"variants\": [\n", (unsigned long long)n, wall_khz);
    for (size_t v = 0; v < vars.size(); ++v) {
        std::vector<float> t = times[v];
        std::sort(t.begin(), t.end());
        const float med = t[t.size() / 2];
        printf("  {\"name\": \"%s\", \"grid\": %d, \"median_ms\": %.4f, \"min_ms\": %.4f, \"ids_per_s\": %.4e, "
               "\"shader_mhz\": %.0f, \"ok\": %s}%s\n",
               vars[v].name.c_str(), grids[v], med, t[0], n / (med * 1e-3), mhz[v], bad[v] ? "false" : "true",
               v + 1 < vars.size() ? "," : "");
    }
    printf("]}\n");
    return 0;
}
