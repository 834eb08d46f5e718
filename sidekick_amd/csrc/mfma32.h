// mfma32.h — u32 power sums S_1..S_32 on the i8 matrix cores (encode.hip,
// 25 <= t <= 32 by default; knob u32_mfma).
//
// Replaces PowerSumQuack::insert (sidekick.rs:42, sidekick_multi.rs:82,
// media_client.rs:249) over a batch like the baby-step/giant-step kernels
// (bsgs.h) and shares their decomposition S[8a + b] = sum_ids g_a h_b with
// g_a = x^(8a) (a = 0..3) and h_b = x^b (b = 1..8), all lazy residues < 2^32
// (9 modmuls per id).  The 32 products per id and their sums are a matrix
// product over the ids, which the bsgs kernels run as 24 VALU
// multiply-accumulates + 8 adds per id.  Here every residue is split into
// bytes, u = s + 128 with s a signed i8 (one XOR with 0x80808080), so that
//   M[(a,i)][(b,j)] = sum_ids s_{a,i}(id) s_{b,j}(id)      16 x 32, i32
// is two v_mfma_i32_16x16x64_i8 per 64 ids, and with K = 0x01010101
//   Z_ab = sum_{i,j} 2^(8(i+j)) M[(a,i)][(b,j)] = sum_ids (g_a - 128K)(h_b - 128K)
//   T_ab = sum_ids g_a h_b = Z_ab + 128K (sum h_b + sum g_a) - 16384 K^2 N.
// Mod p, sum h_b = T_0b (g_0 = 1) and sum g_a = T_(a-1)8 (= S_8a), so
//   T_0b = Z_0b / (1 - 128K) + 128K N,   then T_ab for a = 1, 2, 3 in order.
// That relation is linear, so each workgroup turns its own M and entry count
// N into its 32 partial sums (canonical, < p) and the bsgs kernels' partial
// layout [power][block] and k_finalize_u32 take it from there.
//
// Data flow per wave and 64-id step: each lane computes the residues of one
// id and writes them as three 16-byte rows ([64 ids][16 B] each: g_0..g_3,
// h_1..h_4, h_5..h_8) into the wave's LDS; ds_read_b64_tr_b8 returns them
// column-major — per 16-lane group 8 ids x 16 byte-columns, lane q getting
// byte-column q — which is the operand layout (lane l: row / column l & 15,
// ids 16 (l >> 4) + 0..15 over two reads).  The i32 accumulators stay below
// 2^30 for 1024 steps (|s s'| <= 2^14, 64 ids a step) and are flushed into
// i64 every 1024 steps.  A lazy product that may have wrapped (min < 25,
// probability ~25 / 2^32, bsgs.h) sends its wave through the exact products
// for that step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.h"

namespace qk {
namespace mfma32 {

constexpr int BLK = 256, NWV = BLK / 64;
constexpr uint32_t WAVE_LDS = 3 * 64 * 16;   // g, h1..4, h5..8: [64 ids][16 B] each

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr uint32_t mulc(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) % P32); }
constexpr uint32_t powc(uint32_t a, uint64_t e) {
    uint32_t r = 1;
    while (e) {
        if (e & 1) r = mulc(r, a);
        a = mulc(a, a);
        e >>= 1;
    }
    return r;
}
constexpr uint32_t KB = 0x01010101u;                          // < p
constexpr uint32_t K128 = mulc(128u, KB);                     // 128 K mod p
constexpr uint32_t K2 = mulc(16384u, mulc(KB, KB));           // 16384 K^2 mod p
constexpr uint32_t INV = powc((1u + P32 - K128) % P32, P32 - 2);   // (1 - 128K)^-1 mod p
static_assert(mulc(INV, (1u + P32 - K128) % P32) == 1u, "1 - 128K is invertible mod p");

__device__ __forceinline__ uint32_t mulp(uint32_t a, uint32_t b) { return canon32(mul32_lazy(a, b)); }
__device__ __forceinline__ uint32_t addp(uint32_t a, uint32_t b) { return add32(a, b); }
__device__ __forceinline__ uint32_t subp(uint32_t a, uint32_t b) { return sub32(a, b); }
// a signed 64-bit sum -> its residue in [0, p)
__device__ __forceinline__ uint32_t resid(long long v) {
    const uint32_t m = canon32(fold64_32((uint64_t)(v < 0 ? -v : v)));
    return v < 0 ? neg32(m) : m;
}

// residues of x: h[b - 1] = x^b (b = 1..8), g[a] = x^(8a); lazy products, with
// the exact ones for the whole wave when a lane's may have wrapped
__device__ __forceinline__ void powers(uint32_t x, uint32_t (&h)[8], uint32_t (&g)[4]) {
    uint32_t mn = 0xFFFFFFFFu;
    h[0] = x;
    h[1] = mulfold32_min(x, x, mn);
    h[2] = mulfold32_min(h[1], x, mn);
    h[3] = mulfold32_min(h[1], h[1], mn);
    h[4] = mulfold32_min(h[3], x, mn);
    h[5] = mulfold32_min(h[2], h[2], mn);
    h[6] = mulfold32_min(h[3], h[2], mn);
    h[7] = mulfold32_min(h[3], h[3], mn);
    g[0] = 1u;
    g[1] = h[7];
    g[2] = mulfold32_min(h[7], h[7], mn);
    g[3] = mulfold32_min(g[2], h[7], mn);
    if (__ballot(mn < 25u)) {
        if (mn < 25u) {
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

#define QK_LDS_V2(p) ((__attribute__((address_space(3))) v2i *)(p))

// one 64-id step of a wave: x = this lane's id (0 for padding)
__device__ __forceinline__ void step(uint32_t x, uint8_t *la, uint8_t *lb, uint8_t *lc, int lane, uint32_t ra0,
                                     uint32_t ra1, v4i &c0, v4i &c1) {
    uint32_t h[8], g[4];
    powers(x, h, g);
    constexpr uint32_t B = 0x80808080u;
    *reinterpret_cast<uint4 *>(la + lane * 16) = make_uint4(g[0] ^ B, g[1] ^ B, g[2] ^ B, g[3] ^ B);
    *reinterpret_cast<uint4 *>(lb + lane * 16) = make_uint4(h[0] ^ B, h[1] ^ B, h[2] ^ B, h[3] ^ B);
    *reinterpret_cast<uint4 *>(lc + lane * 16) = make_uint4(h[4] ^ B, h[5] ^ B, h[6] ^ B, h[7] ^ B);
    // the wave's own rows: LDS runs one wave's DS operations in order; the
    // fences only keep the compiler from moving the reads above the writes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const v2i a0 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(QK_LDS_V2(la + ra0));
    const v2i a1 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(QK_LDS_V2(la + ra1));
    const v2i b0 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(QK_LDS_V2(lb + ra0));
    const v2i b1 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(QK_LDS_V2(lb + ra1));
    const v2i d0 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(QK_LDS_V2(lc + ra0));
    const v2i d1 = __builtin_amdgcn_ds_read_tr8_b64_v2i32(QK_LDS_V2(lc + ra1));
    const v4i A = {a0.x, a0.y, a1.x, a1.y};
    const v4i B0 = {b0.x, b0.y, b1.x, b1.y};
    const v4i B1 = {d0.x, d0.y, d1.x, d1.y};
    c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B0, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B1, c1, 0, 0, 0);
    // the next step's writes stay below these reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup w takes ids [w per_wg, (w + 1) per_wg) (per_wg a multiple of
// 1024), wave v of it the v-th quarter; `head` ids before the first 16-byte
// boundary go to workgroup 0's wave 0 as one extra step.  partials[m * grid +
// w] = this workgroup's S_(m+1) for m < T (canonical).
__global__ __launch_bounds__(BLK) void k_encode_u32_mfma(const uint32_t *__restrict__ ids, uint64_t n, uint32_t head,
                                                         uint32_t T, uint64_t per_wg,
                                                         uint64_t *__restrict__ partials) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[NWV * WAVE_LDS];
    __shared__ long long mfin[512];
    __shared__ unsigned long long ldone;
    __shared__ uint32_t Tv[32];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *la = lds + wv * WAVE_LDS, *lb = la + 64 * 16, *lc = lb + 64 * 16;
    const int q = lane & 15, grp = lane >> 4;
    // tr8 rows (ids) 16 grp + (q >> 1) [+ 8], byte half 8 (q & 1)
    const uint32_t ra0 = (uint32_t)(16 * grp + (q >> 1)) * 16 + 8 * (q & 1), ra1 = ra0 + 8 * 16;
    const uint32_t *al = ids + head;   // 16-byte aligned
    const uint64_t na = n - head;
    const uint64_t per_wave = per_wg / NWV;
    const uint64_t i0 = (uint64_t)blockIdx.x * per_wg + (uint64_t)wv * per_wave;
    const uint64_t i1 = i0 + per_wave < na ? i0 + per_wave : na;
    v4i c0 = {0, 0, 0, 0}, c1 = {0, 0, 0, 0};
    long long a64[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t done = 0;
    if (threadIdx.x == 0) ldone = 0;
    if (head && blockIdx.x == 0 && wv == 0) {
        step((uint32_t)lane < head ? ids[lane] : 0u, la, lb, lc, lane, ra0, ra1, c0, c1);
        done += 64;
    }
    uint32_t steps = 0;
    for (uint64_t b = i0; b < i1; b += 256) {
        uint4 v;
        const uint64_t p = b + 4 * (uint64_t)lane;
        if (p + 3 < i1) {
            v = *reinterpret_cast<const uint4 *>(al + p);
        } else {
            v.x = p < i1 ? al[p] : 0u;
            v.y = p + 1 < i1 ? al[p + 1] : 0u;
            v.z = p + 2 < i1 ? al[p + 2] : 0u;
            v.w = p + 3 < i1 ? al[p + 3] : 0u;
        }
        done += 256;
        step(v.x, la, lb, lc, lane, ra0, ra1, c0, c1);
        step(v.y, la, lb, lc, lane, ra0, ra1, c0, c1);
        step(v.z, la, lb, lc, lane, ra0, ra1, c0, c1);
        step(v.w, la, lb, lc, lane, ra0, ra1, c0, c1);
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
    // the 4 waves' M summed through LDS (the staging area, in two halves);
    // entry e = lane * 8 + 4 nb + r holds M[row (lane >> 4) * 4 + r][column 16 nb + (lane & 15)]
    __syncthreads();
    long long *red = reinterpret_cast<long long *>(lds);   // [NWV][256]
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wv * 256 + lane * 4 + r] = a64[4 * hf + r];
        __syncthreads();
        const long long s = red[threadIdx.x] + red[256 + threadIdx.x] + red[512 + threadIdx.x] + red[768 + threadIdx.x];
        mfin[(threadIdx.x >> 2) * 8 + 4 * hf + (threadIdx.x & 3)] = s;
        __syncthreads();
    }
    if (lane == 0) atomicAdd(&ldone, (unsigned long long)done);
    __syncthreads();
    // Z_ab, one thread per (a, b): 16 entries weighted by 2^(8(i+j))
    if (threadIdx.x < 32) {
        const int a = threadIdx.x >> 3, bb = threadIdx.x & 7;
        uint32_t z = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = 4 * a + i;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = 4 * bb + j;
                const int l = (row >> 2) * 16 + (col & 15);
                const long long m = mfin[l * 8 + (col >> 4) * 4 + (row & 3)];
                z = addp(z, mulp(resid(m), powc(256u, (uint64_t)(i + j))));
            }
        }
        Tv[threadIdx.x] = z;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t N = canon32(fold64_32(ldone));
        const uint32_t kn = mulp(K128, N), k2n = mulp(K2, N);
        uint32_t t0[8];
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) Tv[bb] = t0[bb] = addp(mulp(Tv[bb], INV), kn);
        for (int a = 1; a < 4; ++a) {
            const uint32_t ga = Tv[8 * (a - 1) + 7];   // sum g_a = S_8a
#pragma unroll
            for (int bb = 0; bb < 8; ++bb)
                Tv[8 * a + bb] = subp(addp(Tv[8 * a + bb], mulp(K128, addp(t0[bb], ga))), k2n);
        }
    }
    __syncthreads();
    if (threadIdx.x < T) partials[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = Tv[threadIdx.x];
}

#undef QK_LDS_V2

} // namespace mfma32
} // namespace qk
