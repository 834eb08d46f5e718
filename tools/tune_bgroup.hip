// tune_bgroup.hip — by-slot grouping of 1e8 (slot, id) pairs over 1e6 flows
// in a 22-bit slot space (the 1e6-flow batch of DESIGN.md §3.6): the radix.h
// sort (three 8-bit passes) against one 8-bit pass on the top bits followed by
// a per-bucket counting placement in LDS (k_bgroup: 2^14 slot counters + last
// positions per bucket, one workgroup per bucket).  Checks that both give the
// same segments (count, sum and xor of ids, last id per slot), then prints the
// best of R interleaved rounds per variant as JSON lines.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../sidekick_amd/csrc tune_bgroup.hip -o tune_bgroup
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "radix.h"

using namespace qk;

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr uint32_t NONE = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// packet i: flow f uniform over nf, slot = the flow's hashed slot (C - 1 never
// used), id random; every 50th packet is not an insert (NONE)
__global__ void k_fill(uint32_t *k, uint32_t *v, uint64_t n, uint32_t nf, uint32_t cmask, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t z = mix(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
        const uint32_t f = (uint32_t)((z & 0xFFFFFFFFull) * nf >> 32);
        uint32_t s = (uint32_t)mix(0x1234567ull + f) & cmask;
        if (s == cmask) s = 0;
        k[i] = (z >> 58) == 0 ? NONE : s;
        v[i] = (uint32_t)(z >> 20);
    }
}

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

// one workgroup per top-bits bucket b: items [base[b * nwg], base[(b + 1) * nwg])
// of the bucket-sorted pairs (the last bucket ends at n).  Per slot of the
// bucket (LB low bits): count and last position in LDS, a block scan, then
// each id goes to its slot's run (any order inside it).  Writes start[slot]
// (global position of the slot's run) and last[slot] (its last packet's id)
// for the nonempty slots.
template <int LB, int BLK, int U>
__global__ __launch_bounds__(BLK) void k_bgroup(const uint2 *__restrict__ pairs, const uint32_t *__restrict__ base,
                                                uint32_t nwg, uint64_t n, uint32_t *__restrict__ out,
                                                uint32_t *__restrict__ start, uint32_t *__restrict__ last) {
    constexpr uint32_t L = 1u << LB, PER = L / BLK, NW = BLK / 64;
    extern __shared__ uint32_t lds[];
    uint32_t *cnt = lds, *lst = lds + L;
    __shared__ uint32_t ws[NW];
    const uint32_t b = blockIdx.x;
    const uint64_t b0 = base[(size_t)b * nwg], b1 = b + 1 < gridDim.x ? base[(size_t)(b + 1) * nwg] : n;
    for (uint32_t j = threadIdx.x; j < 2 * L; j += BLK) lds[j] = 0;
    __syncthreads();
    // U independent loads in flight per thread (one per thread the loop is
    // latency-bound: one workgroup per CU)
    for (uint64_t i0 = b0 + threadIdx.x; i0 < b1; i0 += (uint64_t)U * BLK) {
        uint2 p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = i0 + (uint64_t)u * BLK < b1 ? pairs[i0 + (uint64_t)u * BLK] : make_uint2(NONE, 0u);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (p[u].x != NONE) {
                const uint32_t l = p[u].x & (L - 1);
                atomicAdd(&cnt[l], 1u);
                atomicMax(&lst[l], (uint32_t)(i0 + (uint64_t)u * BLK - b0) + 1u);
            }
    }
    __syncthreads();
    uint32_t c[PER], s = 0;
#pragma unroll
    for (int j = 0; j < (int)PER; ++j) {
        c[j] = cnt[threadIdx.x * PER + j];
        s += c[j];
    }
    uint32_t tot;
    uint32_t a = rsort::block_excl<NW>(s, ws, &tot);
#pragma unroll
    for (int j = 0; j < (int)PER; ++j) {
        const uint32_t l = threadIdx.x * PER + j;
        if (c[j]) {
            const uint32_t slot = (b << LB) | l;
            start[slot] = (uint32_t)b0 + a;
            last[slot] = pairs[b0 + lst[l] - 1].y;
        }
        cnt[l] = a;
        a += c[j];
    }
    __syncthreads();
    for (uint64_t i0 = b0 + threadIdx.x; i0 < b1; i0 += (uint64_t)U * BLK) {
        uint2 p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = i0 + (uint64_t)u * BLK < b1 ? pairs[i0 + (uint64_t)u * BLK] : make_uint2(NONE, 0u);
        uint32_t d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = p[u].x != NONE ? atomicAdd(&cnt[p[u].x & (L - 1)], 1u) : NONE;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (d[u] != NONE) out[b0 + d[u]] = p[u].y;
    }
}

// segment starts / last ids of slot-sorted keys (the baseline's k_slot_offsets + last)
__global__ void k_starts(const uint32_t *key, const uint32_t *val, uint64_t n, uint32_t *start, uint32_t *last) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = key[i];
        if (k == NONE) continue;
        if (i == 0 || key[i - 1] != k) start[k] = (uint32_t)i;
        if (i + 1 == n || key[i + 1] != k) last[k] = val[i];
    }
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? (uint64_t)atof(argv[1]) : 100000000ull;
    const int rounds = argc > 2 ? atoi(argv[2]) : 4;
    const uint32_t nf = argc > 3 ? (uint32_t)atof(argv[3]) : 1000000u;
    constexpr int CB = 22, LB = CB - 8;
    const uint32_t C = 1u << CB;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *k0, *k1, *k2, *cnt, *base, *st0, *la0, *st1, *la1;
    CK(hipMalloc(&k0, n * 8));   // (keys, vals) of the input
    CK(hipMalloc(&k1, n * 8));
    CK(hipMalloc(&k2, n * 8));   // the input copy each round sorts (radix passes ping-pong k2 <-> k1)
    uint32_t *v0 = k0 + n, *v1 = k1 + n, *v2 = k2 + n;
    const uint32_t nwg = (uint32_t)std::min<uint64_t>((uint64_t)ncu * 4, (n + 4095) / 4096);
    const uint64_t chunk = (((n + nwg - 1) / nwg) + 3) & ~(uint64_t)3;
    CK(hipMalloc(&cnt, (size_t)256 * nwg * 4));
    CK(hipMalloc(&base, (size_t)256 * nwg * 4));
    uint32_t *zdp = nullptr;   // k_rs_scatter digit totals: 0 (base holds the full scan)
    CK(hipMalloc(&zdp, rsort::RMAX * 4));
    CK(hipMemset(zdp, 0, rsort::RMAX * 4));
    CK(hipMalloc(&st0, (size_t)C * 4));
    CK(hipMalloc(&la0, (size_t)C * 4));
    CK(hipMalloc(&st1, (size_t)C * 4));
    CK(hipMalloc(&la1, (size_t)C * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, k0, v0, n, nf, C - 1, 777ull);
    constexpr int BLK = 1024;
    const size_t lds = (size_t)2 * (1u << LB) * 4;
    CK(hipFuncSetAttribute((const void *)k_bgroup<LB, BLK, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // one pass: count + scan + scatter of digit (shift, 8 bits); ip/op: pair arrays
    auto pass = [&](const uint32_t *ki, const uint32_t *vi, uint32_t *ko, uint32_t *vo, uint32_t shift, bool ip, bool op) {
        if (ip) hipLaunchKernelGGL((rsort::k_rs_count<8, true>), dim3(nwg), dim3(256), 0, 0, ki, n, chunk, shift, 0xFFu, nwg, cnt);
        else hipLaunchKernelGGL((rsort::k_rs_count<8, false>), dim3(nwg), dim3(256), 0, 0, ki, n, chunk, shift, 0xFFu, nwg, cnt);
        hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, 0, cnt, base, 256 * nwg);
        auto kern = ip ? (op ? rsort::k_rs_scatter<8, 256, 16, true, true> : rsort::k_rs_scatter<8, 256, 16, true, false>)
                       : (op ? rsort::k_rs_scatter<8, 256, 16, false, true> : rsort::k_rs_scatter<8, 256, 16, false, false>);
        hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), 0, 0, ki, vi, n, chunk, shift, 0xFFu, nwg, base, zdp, ko, vo);
    };
    float best[3] = {1e30f, 1e30f, 1e30f};   // radix3 + starts, bucket pass + group, bucket pass alone
    for (int r = 0; r < rounds; ++r) {
        for (int variant = 0; variant < 3; ++variant) {
            CK(hipMemcpy(k2, k0, n * 8, hipMemcpyDeviceToDevice));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            if (variant == 0) {
                pass(k2, v2, k1, v1, 0, false, true);    // k2 -> pairs in k1
                pass(k1, v1, k2, v2, 8, true, true);     // pairs k1 -> pairs k2
                pass(k2, v2, k1, v1, 16, true, false);   // pairs k2 -> arrays (k1, v1)
                hipLaunchKernelGGL(k_starts, dim3(ncu * 8), dim3(256), 0, 0, k1, v1, n, st0, la0);
            } else {
                pass(k2, v2, k1, v1, LB, false, true);   // top 8 bits -> pairs in k1 (base: bucket starts)
                if (variant == 1)
                    hipLaunchKernelGGL((k_bgroup<LB, BLK, 8>), dim3(256), dim3(BLK), lds, 0, (const uint2 *)k1, base, nwg, n,
                                       v2, st1, la1);
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best[variant] = std::min(best[variant], ms);
            if (r == 0 && variant == 1) {
                // compare segments: counts from starts (both orderings are by slot), sums / xors, last
                std::vector<uint32_t> ko(n), vo(n), vb(n), s0(C), s1(C), l0(C), l1(C);
                // baseline result: keys k1/vals v1 after variant 0 ran earlier this round? recompute
                CK(hipMemcpy(k2, k0, n * 8, hipMemcpyDeviceToDevice));
                pass(k2, v2, k1, v1, 0, false, true);
                pass(k1, v1, k2, v2, 8, true, true);
                pass(k2, v2, k1, v1, 16, true, false);
                CK(hipMemset(st0, 0xFF, (size_t)C * 4));
                hipLaunchKernelGGL(k_starts, dim3(ncu * 8), dim3(256), 0, 0, k1, v1, n, st0, la0);
                CK(hipMemcpy(ko.data(), k1, n * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(vo.data(), v1, n * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(s0.data(), st0, (size_t)C * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(l0.data(), la0, (size_t)C * 4, hipMemcpyDeviceToHost));
                // bucket path again (v2 was overwritten above)
                CK(hipMemcpy(k2, k0, n * 8, hipMemcpyDeviceToDevice));
                pass(k2, v2, k1, v1, LB, false, true);
                CK(hipMemset(st1, 0xFF, (size_t)C * 4));
                hipLaunchKernelGGL((k_bgroup<LB, BLK, 8>), dim3(256), dim3(BLK), lds, 0, (const uint2 *)k1, base, nwg, n, v2,
                                   st1, la1);
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(vb.data(), v2, n * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(s1.data(), st1, (size_t)C * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(l1.data(), la1, (size_t)C * 4, hipMemcpyDeviceToHost));
                uint64_t bad = 0, segs = 0, ins = 0;
                for (uint64_t i = 0; i < n; ++i) ins += ko[i] != NONE;
                for (uint64_t i = 0; i < ins;) {
                    const uint32_t s = ko[i];
                    uint64_t j = i;
                    uint32_t sum0 = 0, x0 = 0, sum1 = 0, x1 = 0;
                    for (; j < ins && ko[j] == s; ++j) { sum0 += vo[j]; x0 ^= vo[j] * 2654435761u; }
                    if (s0[s] != i || s1[s] != i || l0[s] != l1[s] || l0[s] != vo[j - 1]) ++bad;
                    for (uint64_t q = i; q < j; ++q) { sum1 += vb[q]; x1 ^= vb[q] * 2654435761u; }
                    if (sum0 != sum1 || x0 != x1) ++bad;
                    ++segs;
                    i = j;
                }
                printf("{\"check\": \"segments\", \"inserted\": %llu, \"segments\": %llu, \"mismatches\": %llu}\n",
                       (unsigned long long)ins, (unsigned long long)segs, (unsigned long long)bad);
                fflush(stdout);
                if (bad) return 1;
            }
        }
    }
    const char *names[3] = {"radix3_plus_starts", "bucket8_plus_group", "bucket8_pass_only"};
    for (int i = 0; i < 3; ++i)
        printf("{\"variant\": \"%s\", \"n\": %llu, \"flows\": %u, \"best_ms\": %.4f}\n", names[i], (unsigned long long)n,
               nf, best[i]);
    return 0;
}
