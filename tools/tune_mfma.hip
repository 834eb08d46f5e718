// tune_mfma.hip — feasibility of the t = 32 power-sum encode on the i8
// matrix cores (prototype; not product code).
//
// The headline kernel (bsgs.h, NB = 8 babies x NA = 4 giants) spends ~47 % of
// its VALU issue on the 24 multiply-accumulates + 8 row-0 adds per id:
// S[8a + b] += g_a h_b with g_a = x^(8a), h_b = x^b (lazy residues < 2^32).
// That is a matrix product summed over ids.  Split every residue into bytes
// (u = s + 128 with s a signed i8): with rows (a, i) (16) and columns (b, j)
// (32), M[(a,i)][(b,j)] = sum_ids s_{a,i} s_{b,j} is two
// v_mfma_i32_16x16x64_i8 per 64 ids, and
//   sum_ids (g_a - 128K)(h_b - 128K) = Z_ab = sum_{i,j} 2^(8(i+j)) M,  K = 0x01010101,
// so T_ab = sum g_a h_b = Z_ab + 128K (sum h_b + sum g_a) - 16384 K^2 N, where
// sum h_b = T_0b and sum g_a = T_(a-1),8 (mod p): T_0b = Z_0b / (1 - 128K) + 128 K N,
// then T_ab for a = 1..3 in order.  Each lane computes the 11 residues of its
// id (9 lazy modmuls, the headline's), writes its 48 bytes as one row into LDS
// ([id][16] and [id][32]), and the operands come back column-major with
// ds_read_b64_tr_b8 (8 ids x 16 byte-columns per 16-lane group).  i32
// accumulators are flushed to i64 every 1024 steps (|sum| < 2^30).
//
// Modes: check (small n vs a CPU power-sum loop), bench (n ids: this kernel
// vs the library's qk_u32_encode_device, same ids, sums compared).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../sidekick_amd/csrc tune_mfma.hip
//         -L../sidekick_amd -lquack_hip -Wl,-rpath,'$ORIGIN/../sidekick_amd' -o tune_mfma
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "field.h"
#include "quack_hip.h"

using namespace qk;

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
#define LDS_PTR(p) ((__attribute__((address_space(3))) v2i *)(p))

constexpr int BLK = 256, NWV = BLK / 64;
constexpr uint32_t WAVE_LDS = 64 * 48;   // per wave: three [64 ids][16 B] arrays: g, h1..4, h5..8
constexpr int PART = 512 + 8;             // per wave: M (512 i64, lane-major), entries processed, pad

// tr8 probe: LDS byte q = q & 255 (+ 256-byte pages tagged in a second run);
// lane l reads 8 bytes at address addr(l); out[l] = the 8 bytes
__global__ void k_probe(int page, const uint32_t *addr, uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2048];
    for (int j = threadIdx.x; j < 2048; j += 64) lds[j] = page ? (uint8_t)(j >> 8) : (uint8_t)j;
    __syncthreads();
    v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32(LDS_PTR(lds + addr[threadIdx.x]));
    out[2 * threadIdx.x] = (uint32_t)r.x;
    out[2 * threadIdx.x + 1] = (uint32_t)r.y;
}

__device__ __forceinline__ void powers(uint32_t x, uint32_t h[8], uint32_t g[4], bool exact) {
    uint32_t mn = 0xFFFFFFFFu;
    auto mul = [&](uint32_t a, uint32_t b) { return exact ? mulfold32_exact(a, b) : mulfold32_min(a, b, mn); };
    h[0] = x;
    h[1] = mul(x, x);
    h[2] = mul(h[1], x);
    h[3] = mul(h[1], h[1]);
    h[4] = mul(h[3], x);
    h[5] = mul(h[2], h[2]);
    h[6] = mul(h[3], h[2]);
    h[7] = mul(h[3], h[3]);
    g[0] = 1u;
    g[1] = h[7];
    g[2] = mul(h[7], h[7]);
    g[3] = mul(g[2], h[7]);
    if (!exact && __ballot(mn < 25u)) {   // a lazy fold may have wrapped: redo those ids exactly (rare)
        if (mn < 25u) {
            uint32_t mn2;
            (void)mn2;
            h[1] = mulfold32_exact(x, x);
            h[2] = mulfold32_exact(h[1], x);
            h[3] = mulfold32_exact(h[1], h[1]);
            h[4] = mulfold32_exact(h[3], x);
            h[5] = mulfold32_exact(h[2], h[2]);
            h[6] = mulfold32_exact(h[3], h[2]);
            h[7] = mulfold32_exact(h[3], h[3]);
            g[1] = h[7];
            g[2] = mulfold32_exact(h[7], h[7]);
            g[3] = mulfold32_exact(g[2], h[7]);
        }
    }
}

// one wave: ids [i0, i1) in steps of 256 ids (4 per lane: one 16-byte load),
// four 64-id MFMA steps per load
__global__ __launch_bounds__(BLK) void k_mfma32(const uint32_t *__restrict__ ids, uint64_t n, uint64_t per_wave,
                                               long long *__restrict__ part) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[NWV * WAVE_LDS];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *la = lds + wv * WAVE_LDS, *lb = la + 64 * 16, *lc = lb + 64 * 16;
    const uint64_t gw = (uint64_t)blockIdx.x * NWV + wv;
    const uint64_t i0 = gw * per_wave, i1 = std::min<uint64_t>(i0 + per_wave, n);
    const int q = lane & 15, grp = lane >> 4;
    // tr8 read addresses: rows (ids) 16 grp + (q >> 1) [+ 8], byte half 8 (q & 1)
    const uint32_t ra0 = (uint32_t)(16 * grp + (q >> 1)) * 16 + 8 * (q & 1), ra1 = ra0 + 8 * 16;
    v4i c0 = {0, 0, 0, 0}, c1 = {0, 0, 0, 0};
    long long a64[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t done = 0;
    uint32_t steps = 0;
    for (uint64_t b = i0; b < i1; b += 256) {
        uint4 v;
        const uint64_t p = b + 4 * (uint64_t)lane;
        if (p + 3 < i1) v = *reinterpret_cast<const uint4 *>(ids + p);
        else {
            v.x = p < i1 ? ids[p] : 0u;
            v.y = p + 1 < i1 ? ids[p + 1] : 0u;
            v.z = p + 2 < i1 ? ids[p + 2] : 0u;
            v.w = p + 3 < i1 ? ids[p + 3] : 0u;
        }
        done += 256;
        const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint32_t h[8], g[4];
            powers(xs[u], h, g, false);
            const uint32_t B = 0x80808080u;
            *reinterpret_cast<uint4 *>(la + lane * 16) = make_uint4(g[0] ^ B, g[1] ^ B, g[2] ^ B, g[3] ^ B);
            *reinterpret_cast<uint4 *>(lb + lane * 16) = make_uint4(h[0] ^ B, h[1] ^ B, h[2] ^ B, h[3] ^ B);
            *reinterpret_cast<uint4 *>(lc + lane * 16) = make_uint4(h[4] ^ B, h[5] ^ B, h[6] ^ B, h[7] ^ B);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const v2i A0 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(LDS_PTR(la + ra0));
            const v2i A1 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(LDS_PTR(la + ra1));
            const v2i B00 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(LDS_PTR(lb + ra0));
            const v2i B01 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(LDS_PTR(lb + ra1));
            const v2i B10 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(LDS_PTR(lc + ra0));
            const v2i B11 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(LDS_PTR(lc + ra1));
            const v4i A = {A0.x, A0.y, A1.x, A1.y};
            const v4i Bm0 = {B00.x, B00.y, B01.x, B01.y};
            const v4i Bm1 = {B10.x, B10.y, B11.x, B11.y};
            c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, Bm0, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, Bm1, c1, 0, 0, 0);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (++steps == 256) {   // 1024 MFMA steps: flush before the i32 sums can reach 2^31
            steps = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                a64[r] += c0[r];
                a64[4 + r] += c1[r];
            }
            c0 = v4i{0, 0, 0, 0};
            c1 = v4i{0, 0, 0, 0};
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        a64[r] += c0[r];
        a64[4 + r] += c1[r];
    }
    // the workgroup's 4 waves summed through LDS (reusing the staging area:
    // 4 x 512 i64 = 16 KB > 12 KB, so two halves), one partial per workgroup
    __syncthreads();
    long long *red = reinterpret_cast<long long *>(lds);   // [NWV][256]
    long long *o = part + (uint64_t)blockIdx.x * PART;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wv * 256 + lane * 4 + r] = a64[4 * h + r];
        __syncthreads();
        const long long s = red[threadIdx.x] + red[256 + threadIdx.x] + red[512 + threadIdx.x] + red[768 + threadIdx.x];
        // entry e = lane * 8 + 4 h + r  <-  threadIdx.x = lane * 4 + r
        o[(threadIdx.x >> 2) * 8 + 4 * h + (threadIdx.x & 3)] = s;
        __syncthreads();
    }
    __shared__ unsigned long long ldone;
    if (threadIdx.x == 0) ldone = 0;
    __syncthreads();
    if (lane == 0) atomicAdd(&ldone, (unsigned long long)done);
    __syncthreads();
    if (threadIdx.x == 0) o[512] = (long long)ldone;
}

// stage 1: block b sums partials [b * per, (b + 1) * per) -> part2[b]
__global__ __launch_bounds__(PART) void k_mfma_sum(const long long *__restrict__ part, uint32_t np, uint32_t per,
                                                  long long *__restrict__ part2) {
    const uint32_t e = threadIdx.x;
    long long s = 0;
    const uint32_t w0 = blockIdx.x * per, w1 = std::min(np, w0 + per);
    for (uint32_t w = w0; w < w1; ++w) s += part[(size_t)w * PART + e];
    part2[(size_t)blockIdx.x * PART + e] = s;
}

__device__ uint32_t modp_i64(long long v) {
    long long m = v % (long long)P32;
    if (m < 0) m += P32;
    return (uint32_t)m;
}
__device__ uint32_t mulp(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) % P32); }
__device__ uint32_t addp(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + b) % P32); }
__device__ uint32_t subp(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + P32 - b) % P32); }
__device__ uint32_t powp(uint32_t a, uint64_t e) {
    uint32_t r = 1;
    while (e) {
        if (e & 1) r = mulp(r, a);
        a = mulp(a, a);
        e >>= 1;
    }
    return r;
}

// one workgroup of 512 threads: sum the waves' partials, then the 32 sums
__global__ __launch_bounds__(512) void k_mfma_epilogue(const long long *__restrict__ part, uint32_t nwaves,
                                                      uint32_t *__restrict__ sums) {
    __shared__ uint32_t mres[16][32];   // M mod p by [(a,i)][(b-1,j)]
    __shared__ unsigned long long ntot;
    const uint32_t e = threadIdx.x;   // lane * 8 + nb * 4 + r
    long long s = 0;
    for (uint32_t w = 0; w < nwaves; ++w) s += part[(size_t)w * PART + e];
    if (e == 0) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < nwaves; ++w) t += (unsigned long long)part[(size_t)w * PART + 512];
        ntot = t;
    }
    const uint32_t lane = e >> 3, nb = (e >> 2) & 1, r = e & 3;
    const uint32_t row = (lane >> 4) * 4 + r, col = 16 * nb + (lane & 15);
    mres[row][col] = modp_i64(s);
    __syncthreads();
    if (e == 0) {
        const uint32_t K = 0x01010101u % P32, N = (uint32_t)(ntot % P32);
        const uint32_t k128 = mulp(128, K), k2 = mulp(16384, mulp(K, K));
        uint32_t Z[4][8], T[4][8];
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 8; ++b) {
                uint32_t z = 0;
                for (int i = 0; i < 4; ++i)
                    for (int j = 0; j < 4; ++j)
                        z = addp(z, mulp(mres[4 * a + i][4 * b + j], powp(256, (uint64_t)(i + j))));
                Z[a][b] = z;
            }
        const uint32_t inv = powp(subp(1, k128), P32 - 2);
        for (int b = 0; b < 8; ++b) T[0][b] = addp(mulp(Z[0][b], inv), mulp(k128, N));
        for (int a = 1; a < 4; ++a)
            for (int b = 0; b < 8; ++b)
                T[a][b] = subp(addp(Z[a][b], mulp(k128, addp(T[0][b], T[a - 1][7]))), mulp(k2, N));
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 8; ++b) sums[8 * a + b] = T[a][b];   // S_(8a + b + 1)
    }
}

__global__ void k_fill(uint32_t *ids, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        ids[i] = (uint32_t)splitmix_mix(seed + i);
}

static uint32_t cpu_mul(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) % P32); }

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "check";
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    if (!strcmp(mode, "probe")) {
        // lane l reads at 8 l (two runs: low byte, page) -> print source addresses of lanes 0..31
        uint32_t *d_addr, *d_out;
        CK(hipMalloc(&d_addr, 64 * 4));
        CK(hipMalloc(&d_out, 128 * 4));
        std::vector<uint32_t> addr(64), o0(128), o1(128);
        for (int l = 0; l < 64; ++l) addr[l] = 8 * l;
        CK(hipMemcpy(d_addr, addr.data(), 256, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, 0, d_addr, d_out);
        CK(hipMemcpy(o0.data(), d_out, 512, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, 1, d_addr, d_out);
        CK(hipMemcpy(o1.data(), d_out, 512, hipMemcpyDeviceToHost));
        for (int l = 0; l < 32; ++l) {
            printf("lane %2d:", l);
            for (int j = 0; j < 8; ++j) {
                const uint32_t w0 = o0[2 * l + j / 4], w1 = o1[2 * l + j / 4];
                printf(" %4u", ((w1 >> (8 * (j % 4))) & 255) * 256 + ((w0 >> (8 * (j % 4))) & 255));
            }
            printf("\n");
        }
        return 0;
    }
    const bool check = !strcmp(mode, "check");
    const uint64_t n = argc > 2 ? (uint64_t)atof(argv[2]) : (check ? 1000003ull : 1000000000ull);
    const uint32_t wgpc = argc > 3 ? (uint32_t)atoi(argv[3]) : 8;
    const int reps = argc > 4 ? atoi(argv[4]) : 10;
    uint32_t *ids, *d_sums;
    long long *part, *part2;
    CK(hipMalloc(&ids, n * 4 + 64));
    const uint32_t nwg = (uint32_t)ncu * wgpc, nwaves = nwg * NWV;
    const uint64_t per_wave = ((n + nwaves - 1) / nwaves + 255) / 256 * 256;
    CK(hipMalloc(&part, (size_t)nwg * PART * 8));
    CK(hipMalloc(&part2, (size_t)64 * PART * 8));
    CK(hipMalloc(&d_sums, 32 * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, ids, n, 0x5eed0002ull);
    const uint32_t nsum = 64, sper = (nwg + nsum - 1) / nsum;
    auto epilogue = [&]() {
        hipLaunchKernelGGL(k_mfma_sum, dim3(nsum), dim3(PART), 0, 0, part, nwg, sper, part2);
        hipLaunchKernelGGL(k_mfma_epilogue, dim3(1), dim3(512), 0, 0, part2, nsum, d_sums);
    };
    auto run = [&]() {
        hipLaunchKernelGGL(k_mfma32, dim3(nwg), dim3(BLK), 0, 0, ids, n, per_wave, part);
        epilogue();
    };
    run();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> got(32), want(32, 0);
    CK(hipMemcpy(got.data(), d_sums, 128, hipMemcpyDeviceToHost));
    if (check) {
        std::vector<uint32_t> h(n);
        CK(hipMemcpy(h.data(), ids, n * 4, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t x = h[i] % P32;
            uint32_t pw = 1;
            for (int k = 0; k < 32; ++k) {
                pw = cpu_mul(pw, x);
                want[k] = (uint32_t)(((uint64_t)want[k] + pw) % P32);
            }
        }
    } else {
        qk_ctx *ctx = nullptr;
        if (qk_ctx_create(0, &ctx) != 0) return 2;
        std::vector<uint8_t> qb(qk_u32_size(32));
        qk_u32 *q = reinterpret_cast<qk_u32 *>(qb.data());
        qk_u32_init(q, 32);
        if (qk_u32_encode_device(ctx, ids, n, q, nullptr) != 0) return 3;
        for (int k = 0; k < 32; ++k) want[k] = q->power_sums[k];
        // timing: kernel + epilogue vs the library call, interleaved
        hipEvent_t e0, e1, em;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventCreate(&em));
        std::vector<float> tm, tl, te;
        for (int r = 0; r < reps; ++r) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(k_mfma32, dim3(nwg), dim3(BLK), 0, 0, ids, n, per_wave, part);
            CK(hipEventRecord(em, 0));
            epilogue();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, em));
            tm.push_back(ms);
            CK(hipEventElapsedTime(&ms, em, e1));
            te.push_back(ms);
            qk_u32_init(q, 32);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            if (qk_u32_encode_device(ctx, ids, n, q, nullptr) != 0) return 3;
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            tl.push_back(ms);
        }
        std::sort(tm.begin(), tm.end());
        std::sort(tl.begin(), tl.end());
        std::sort(te.begin(), te.end());
        printf("{\"n\": %llu, \"wgpc\": %u, \"mfma_kernel_ms_median\": %.4f, \"mfma_kernel_ms_min\": %.4f, "
               "\"mfma_kernel_ids_per_s\": %.4g, \"epilogue_ms\": %.4f, "
               "\"library_wall_ms_median\": %.4f, \"library_ids_per_s\": %.4g}\n",
               (unsigned long long)n, wgpc, tm[tm.size() / 2], tm[0], n / (tm[tm.size() / 2] * 1e-3), te[te.size() / 2],
               tl[tl.size() / 2], n / (tl[tl.size() / 2] * 1e-3));
        qk_ctx_destroy(ctx);
    }
    int bad = 0;
    for (int k = 0; k < 32; ++k) bad += got[k] != want[k];
    printf("{\"mode\": \"%s\", \"n\": %llu, \"sums_equal\": %s, \"mismatches\": %d, \"S1\": [%u, %u], \"S32\": [%u, %u]}\n",
           mode, (unsigned long long)n, bad ? "false" : "true", bad, got[0], want[0], got[31], want[31]);
    return bad ? 1 : 0;
}
