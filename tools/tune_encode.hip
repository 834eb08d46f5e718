// tune_encode.hip — A/B harness for u32 encode kernel variants (not product
// code).  One process, interleaved rounds (cdna_hip_programming.md §5.4 rule
// 24), 1e9 device-resident ids, every variant's sums checked against V0.
//
// Variants: CH independent chains per lane (ids per lane per iteration),
// G lanes per id (G = 2: the lane pair splits odd/even powers with step x^2,
// halving accumulator VGPRs), MINW = __launch_bounds__ min waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../sidekick_amd/csrc/field.h"

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

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// G lanes per id group; K = T/G accumulators; CH ids per lane per iteration.
template <int CH, int G, int MINW, int PF = 0>
__global__ __launch_bounds__(BLOCK, MINW) void k_var(const uint32_t *__restrict__ ids, uint64_t n,
                                                    uint64_t *__restrict__ partials) {
    constexpr int K = T / G;
    __shared__ uint64_t sm[BLOCK / 64][T];
    uint64_t acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0;
    const int j = threadIdx.x % G;
    const uint64_t grp = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) / G;
    const uint64_t ngrp = (uint64_t)gridDim.x * BLOCK / G;
    const uint64_t units = n / CH; // n multiple of CH assumed (1e9)
    for (uint64_t u = grp; u < units; u += ngrp) {
        uint32_t w[CH];
        if constexpr (CH == 4) {
            const uint4 v = reinterpret_cast<const uint4 *>(ids)[u];
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else if constexpr (CH == 2) {
            const uint2 v = reinterpret_cast<const uint2 *>(ids)[u];
            w[0] = v.x; w[1] = v.y;
        } else if constexpr (CH == 8) {
            const uint4 a = reinterpret_cast<const uint4 *>(ids)[2 * u];
            const uint4 b = reinterpret_cast<const uint4 *>(ids)[2 * u + 1];
            w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
        } else {
            w[0] = ids[u];
        }
        uint32_t x[CH], f[CH];
        uint64_t t[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const uint32_t xc = canon32(w[c]);
            if constexpr (G == 1) {
                x[c] = xc;
                t[c] = xc;
            } else { // G == 2: step x^2, lane 0 starts at x, lane 1 at x^2
                const uint32_t x2 = canon32(mul32_lazy(xc, xc));
                x[c] = x2;
                t[c] = j ? x2 : xc;
            }
            f[c] = times5_32(x[c]);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int c = 0; c < CH; ++c) acc[k] += t[c];
            if (k + 1 < K) {
#pragma unroll
                for (int c = 0; c < CH; ++c) t[c] = tstep32p(t[c], x[c], f[c], 0u);
            }
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint64_t v = fold64_32(acc[k]);
#pragma unroll
        for (int off = 32; off >= G; off >>= 1) v += shfl_xor_u64(v, off);
        if (lane < G) sm[wave][lane + k * G] = v;
    }
    __syncthreads();
    if (threadIdx.x < T) {
        uint64_t s = 0;
        for (int w = 0; w < BLOCK / 64; ++w) s += sm[w][threadIdx.x];
        partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = s;
    }
}

// CH = 4, G = 1 with the next 16-byte load issued before the current chains
template <int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void k_pf(const uint32_t *__restrict__ ids, uint64_t n,
                                                   uint64_t *__restrict__ partials) {
    constexpr int K = T;
    __shared__ uint64_t sm[BLOCK / 64][T];
    uint64_t acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0;
    const uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t ng = (uint64_t)gridDim.x * BLOCK;
    const uint64_t units = n / 4;
    const uint4 *v = reinterpret_cast<const uint4 *>(ids);
    uint4 cur = g < units ? v[g] : make_uint4(0, 0, 0, 0);
    for (uint64_t u = g; u < units; u += ng) {
        const uint64_t un = u + ng;
        const uint4 nxt = un < units ? v[un] : make_uint4(0, 0, 0, 0);
        uint32_t x[4], f[4];
        uint64_t t[4];
        const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) { x[c] = canon32(w[c]); t[c] = x[c]; f[c] = times5_32(x[c]); }
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[k] += t[c];
            if (k + 1 < K) {
#pragma unroll
                for (int c = 0; c < 4; ++c) t[c] = tstep32p(t[c], x[c], f[c], 0u);
            }
        }
        cur = nxt;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint64_t vv = fold64_32(acc[k]);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) vv += shfl_xor_u64(vv, off);
        if (lane == 0) sm[wave][k] = vv;
    }
    __syncthreads();
    if (threadIdx.x < T) {
        uint64_t s = 0;
        for (int w = 0; w < BLOCK / 64; ++w) s += sm[w][threadIdx.x];
        partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = s;
    }
}

// ---- baby-step / giant-step: S_{8a+b} = sum_i A_a(x_i) * B_b(x_i) -------
// B_b = x^b (b = 1..8), A_a = x^(8a) (a = 0..3); 9 modmuls per id, then a
// 3x8 multiply-accumulate with carry counting plus the a = 0 row of adds.
__device__ __forceinline__ uint32_t mulfold32(uint32_t y, uint32_t x) {
    const uint64_t P = (uint64_t)y * x;
    const uint32_t Ph = (uint32_t)(P >> 32);
    const uint64_t Q = P + (uint64_t)Ph * 5u;
    const uint32_t tl = (uint32_t)Q, th = (uint32_t)(Q >> 32) - Ph;   // t = tl + th*2^32, th <= 5
    const uint32_t m = th * 5u;
    uint32_t r = tl + m;
    if (r < m) r += 5u;   // wrapped: 2^32 == 5 (mod p); r < 25 here, no second wrap
    return r;
}

__device__ __forceinline__ void mac_carry(uint64_t &acc, uint32_t &cnt, uint32_t a, uint32_t b) {
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "v"(b));
    asm("v_addc_co_u32_e64 %0, %1, %0, 0, %2" : "+v"(cnt), "=s"(c) : "s"(c));
}

// variant 2: VCC-carried MAC (no SGPR hazard padding) and a fold whose rare
// wrap (prob ~25/2^32) is only flagged; a wave with a flagged lane recomputes
// that lane's powers with the exact fold before accumulating.
__device__ __forceinline__ uint32_t mulfold32_flag(uint32_t y, uint32_t x, uint32_t &flag) {
    const uint64_t P = (uint64_t)y * x;
    const uint32_t Ph = (uint32_t)(P >> 32);
    const uint64_t Q = P + (uint64_t)Ph * 5u;
    const uint32_t tl = (uint32_t)Q, th = (uint32_t)(Q >> 32) - Ph;
    const uint32_t m = th * 5u;
    const uint32_t r = tl + m;
    flag |= (r < m);
    return r;
}
__device__ __forceinline__ void mac_vcc(uint64_t &acc, uint32_t &cnt, uint32_t a, uint32_t b) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(cnt) : "v"(a), "v"(b) : "vcc");
}

__device__ __forceinline__ void mac_vcc_nop(uint64_t &acc, uint32_t &cnt, uint32_t a, uint32_t b) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(cnt) : "v"(a), "v"(b) : "vcc");
}
__device__ __forceinline__ void add_vcc(uint64_t &acc, uint32_t b) {
    uint32_t lo = (uint32_t)acc, hi = (uint32_t)(acc >> 32);
    asm("v_add_co_u32_e32 %0, vcc, %0, %2\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
        : "+v"(lo), "+v"(hi) : "v"(b) : "vcc");
    acc = ((uint64_t)hi << 32) | lo;
}

// 4 MACs sharing A, carries in 4 distinct SGPR pairs: every v_addc reads a
// carry written >= 3 VALU instructions earlier (>= 2 wait states, no s_nop).
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
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3),
          "=&s"(k0), "=&s"(k1), "=&s"(k2), "=&s"(k3)
        : "v"(A), "v"(b0), "v"(b1), "v"(b2), "v"(b3));
}

template <int MINW, int CHN, int MAC = 0, int PF = 0>
__global__ __launch_bounds__(BLOCK, MINW) void k_bsgs2(const uint32_t *__restrict__ ids, uint64_t n,
                                                      uint64_t *__restrict__ partials) {
    __shared__ uint64_t sm[BLOCK / 64][T];
    uint64_t acc0[8], acc[3][8];
    uint32_t cnt[MAC == 2 ? 1 : 3][8];
    uint64_t accH[MAC == 2 ? 3 : 1][8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        acc0[b] = 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            acc[a][b] = 0;
            if constexpr (MAC == 2) accH[a][b] = 0; else cnt[a][b] = 0;
        }
    }
    const uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t ng = (uint64_t)gridDim.x * BLOCK;
    const uint64_t units = n / CHN;
    uint4 nxt = make_uint4(0, 0, 0, 0);
    if (PF && g < units) nxt = reinterpret_cast<const uint4 *>(ids)[g];
    for (uint64_t u = g; u < units; u += ng) {
        uint32_t w[CHN];
        if constexpr (CHN == 4 && PF) {
            const uint4 v = nxt;
            if (u + ng < units) nxt = reinterpret_cast<const uint4 *>(ids)[u + ng];
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else if constexpr (CHN == 4) {
            const uint4 v = reinterpret_cast<const uint4 *>(ids)[u];
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else if constexpr (CHN == 2) {
            const uint2 v = reinterpret_cast<const uint2 *>(ids)[u];
            w[0] = v.x; w[1] = v.y;
        } else {
            w[0] = ids[u];
        }
#pragma unroll
        for (int c = 0; c < CHN; ++c) {
            uint32_t B[8], A[3], flag = 0;
            B[0] = canon32(w[c]);
#pragma unroll
            for (int b = 1; b < 8; ++b) B[b] = mulfold32_flag(B[b - 1], B[0], flag);
            A[0] = B[7];
            A[1] = mulfold32_flag(A[0], A[0], flag);
            A[2] = mulfold32_flag(A[1], A[0], flag);
            if (__builtin_expect(__any(flag), 0)) {
                if (flag) {
#pragma unroll
                    for (int b = 1; b < 8; ++b) B[b] = mulfold32(B[b - 1], B[0]);
                    A[0] = B[7];
                    A[1] = mulfold32(A[0], A[0]);
                    A[2] = mulfold32(A[1], A[0]);
                }
            }
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                if constexpr (MAC == 4) add_vcc(acc0[b], B[b]);
                else acc0[b] += B[b];
            }
            if constexpr (MAC == 5) {
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                    for (int b = 0; b < 8; b += 4)
                        mac4(acc[a][b], acc[a][b + 1], acc[a][b + 2], acc[a][b + 3], cnt[a][b], cnt[a][b + 1],
                             cnt[a][b + 2], cnt[a][b + 3], A[a], B[b], B[b + 1], B[b + 2], B[b + 3]);
            } else
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    if constexpr (MAC == 0) mac_vcc(acc[a][b], cnt[a][b], A[a], B[b]);
                    else if constexpr (MAC == 3 || MAC == 4) mac_vcc_nop(acc[a][b], cnt[a][b], A[a], B[b]);
                    else if constexpr (MAC == 1) mac_carry(acc[a][b], cnt[a][b], A[a], B[b]);
                    else {
                        // B = Bh*2^16 + Bl: A*Bl, A*Bh < 2^48, no carry for 2^16 ids per lane;
                        // acc holds sum A*Bl, acc2 (reusing cnt as storage is not possible) -> accH
                        acc[a][b] += (uint64_t)A[a] * (B[b] & 0xFFFFu);
                        accH[a][b] += (uint64_t)A[a] * (B[b] >> 16);
                    }
                }
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < T; ++k) {
        const int a = k / 8, b = k % 8;
        uint64_t vv;
        if (a == 0) vv = fold64_32(acc0[b]);
        else if constexpr (MAC == 2)
            vv = (uint64_t)fold64_32(acc[a - 1][b]) + (uint64_t)mul32(canon32(fold64_32(accH[a - 1][b])), 65536u);
        else vv = (uint64_t)fold64_32(acc[a - 1][b]) + (uint64_t)fold64_32((uint64_t)cnt[a - 1][b] * 25u);
        vv = fold64_32(vv);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) vv += shfl_xor_u64(vv, off);
        if (lane == 0) sm[wave][k] = vv;
    }
    __syncthreads();
    if (threadIdx.x < T) {
        uint64_t s = 0;
        for (int w = 0; w < BLOCK / 64; ++w) s += sm[w][threadIdx.x];
        partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = s;
    }
}

template <int MINW, int CHN>
__global__ __launch_bounds__(BLOCK, MINW) void k_bsgs(const uint32_t *__restrict__ ids, uint64_t n,
                                                     uint64_t *__restrict__ partials) {
    __shared__ uint64_t sm[BLOCK / 64][T];
    uint64_t acc0[8], acc[3][8];
    uint32_t cnt[3][8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        acc0[b] = 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) { acc[a][b] = 0; cnt[a][b] = 0; }
    }
    const uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t ng = (uint64_t)gridDim.x * BLOCK;
    const uint64_t units = n / CHN;
    for (uint64_t u = g; u < units; u += ng) {
        uint32_t w[CHN];
        if constexpr (CHN == 4) {
            const uint4 v = reinterpret_cast<const uint4 *>(ids)[u];
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
        } else if constexpr (CHN == 2) {
            const uint2 v = reinterpret_cast<const uint2 *>(ids)[u];
            w[0] = v.x; w[1] = v.y;
        } else {
            w[0] = ids[u];
        }
#pragma unroll
        for (int c = 0; c < CHN; ++c) {
            uint32_t B[8];
            B[0] = canon32(w[c]);
#pragma unroll
            for (int b = 1; b < 8; ++b) B[b] = mulfold32(B[b - 1], B[0]);
            uint32_t A[3];
            A[0] = B[7];
            A[1] = mulfold32(A[0], A[0]);
            A[2] = mulfold32(A[1], A[0]);
#pragma unroll
            for (int b = 0; b < 8; ++b) acc0[b] += B[b];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 8; ++b) mac_carry(acc[a][b], cnt[a][b], A[a], B[b]);
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < T; ++k) {
        const int a = k / 8, b = k % 8;   // power k+1 = 8a + b + 1
        uint64_t vv;
        if (a == 0) vv = fold64_32(acc0[b]);
        else        // value = cnt*2^64 + acc, 2^64 == 25 (mod p)
            vv = (uint64_t)fold64_32(acc[a - 1][b]) + (uint64_t)fold64_32((uint64_t)cnt[a - 1][b] * 25u);
        vv = fold64_32(vv);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) vv += shfl_xor_u64(vv, off);
        if (lane == 0) sm[wave][k] = vv;
    }
    __syncthreads();
    if (threadIdx.x < T) {
        uint64_t s = 0;
        for (int w = 0; w < BLOCK / 64; ++w) s += sm[w][threadIdx.x];
        partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = s;
    }
}

__global__ void k_fin(const uint64_t *partials, uint32_t nb, uint32_t *out) {
    const uint32_t m = threadIdx.x;
    if (m >= T) return;
    uint64_t s = 0;
    for (uint32_t b = 0; b < nb; ++b) s += fold64_32(partials[(size_t)m * nb + b]);
    out[m] = canon32(fold64_32(s));
}

struct Var {
    const char *name;
    void (*k)(const uint32_t *, uint64_t, uint64_t *);
    int G;
};

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1000000000ull;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    uint32_t *ids;
    uint64_t *partials;
    uint32_t *out;
    CHK(hipMalloc(&ids, n * 4));
    CHK(hipMalloc(&partials, 64ull << 20));
    CHK(hipMalloc(&out, T * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, ids, n, 0x5EED0002ull);
    CHK(hipDeviceSynchronize());

    std::vector<Var> vars = {
        {"BSGS2_C4", k_bsgs2<1, 4, 0>, 1}, {"BSGS2_C4_NOP", k_bsgs2<1, 4, 3>, 1}, {"BSGS_MAC4", k_bsgs2<1, 4, 5>, 1},
        {"BSGS_PF", k_bsgs2<1, 4, 0, 1>, 1}, {"BSGS_MAC4_PF", k_bsgs2<1, 4, 5, 1>, 1}, {"BSGS_NOP_PF", k_bsgs2<1, 4, 3, 1>, 1},
    };
    uint32_t ref[T], got[T];
    std::vector<std::vector<float>> times(vars.size());
    std::vector<int> grids(vars.size());
    for (size_t v = 0; v < vars.size(); ++v) {
        int occ = 0;
        CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vars[v].k, BLOCK, 0));
        grids[v] = occ * prop.multiProcessorCount;
    }
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int r = 0; r < rounds + 1; ++r) {
        for (size_t v = 0; v < vars.size(); ++v) {
            CHK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(vars[v].k, dim3(grids[v]), dim3(BLOCK), 0, 0, ids, n, partials);
            CHK(hipEventRecord(e1, 0));
            hipLaunchKernelGGL(k_fin, dim3(1), dim3(64), 0, 0, partials, (uint32_t)grids[v], out);
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            CHK(hipMemcpy(got, out, sizeof(got), hipMemcpyDeviceToHost));
            if (r == 0 && v == 0) memcpy(ref, got, sizeof(ref));
            if (memcmp(ref, got, sizeof(ref))) printf("MISMATCH %s round %d\n", vars[v].name, r);
            if (r) times[v].push_back(ms);
        }
    }
    printf("{\"n\": %llu, \"variants\": [\n", (unsigned long long)n);
    for (size_t v = 0; v < vars.size(); ++v) {
        std::vector<float> t = times[v];
        std::sort(t.begin(), t.end());
        const float med = t[t.size() / 2];
        printf("  {\"name\": \"%s\", \"grid\": %d, \"median_ms\": %.4f, \"min_ms\": %.4f, \"ids_per_s\": %.4e}%s\n",
               vars[v].name, grids[v], med, t[0], n / (med * 1e-3), v + 1 < vars.size() ? "," : "");
    }
    printf("]}\n");
    return 0;
}
