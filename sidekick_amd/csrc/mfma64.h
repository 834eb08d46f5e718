// mfma64.h — u64 encode (p64 = 2^64 - 59) with the baby-step/giant-step
// products on the matrix cores, DESIGN.md §3.3b.  The u32 form (mfma8.h)
// with 8-byte values: power P = NB*a + b is S_P = sum_i A_a(x_i) B_b(x_i)
// with babies B_b = x^b (b = 1..NB) and giants A_a = x^(NB a) (A_0 = 1), and
//     A B = sum_{j,k < 8} 256^(j+k) u_{a,j} u_{b,k}
// an int8 GEMM over the ids with M = NA giants x 8 limbs (an MFMA tile's 16
// rows are two giants) and N = NB babies x 8 limbs (two babies per tile).
// Bytes are stored u ^ 0x80 (signed), and with R = sum_{j<8} 256^j the same
// corrections as the u32 form hold (k_mfma64_fix in encode.hip):
//     S_P = Cw(a,b) + 128 R (sum_i A_a + sum_i B_b) - 16384 R^2 N   (mod p)
//
// Per wave and K-block of 64 ids: the lane's NB - 1 + NA - 2 modmuls are the
// exact hand-scheduled p64 step of bsgs64.h (mulv), two XORs per value, one
// 16-byte LDS segment per two values, two ds_read_b64_tr_b8 per fragment,
// NM x NN MFMAs.  Every FLUSH K-blocks the int32 tiles are folded (mod p,
// weighted 256^(j+k), reduced over the lanes of a power) into the wave's
// LDS row of canonical power sums, so no per-tile 64-bit state stays in
// registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bsgs64.h"
#include "field.h"
#include "mfma8.h"

namespace qk {
namespace mf64 {

using mf8::BLOCK;
using mf8::FLUSH;
using mf8::OFS;
using mf8::tr8;
using mf8::v2i;
using mf8::v4i;
using mf8::WAVES;

// 256^d mod p64 for d = 0..14 (2^64 == 59)
__device__ __forceinline__ uint64_t wpow(int d) { return d < 8 ? (1ull << (8 * d)) : (59ull << (8 * (d - 8))); }

__device__ __forceinline__ uint64_t shfl_add64(uint64_t v, int m) {   // canonical in, canonical out
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return add64(v, ((uint64_t)hi << 32) | lo);
}

// NM tiles of 2 giants (NA = 2 NM), NN tiles of 2 babies (NB = 2 NN)
template <int NM, int NN>
struct Shape {
    static constexpr int NA = 2 * NM, NB = 2 * NN, SEGS = NM + NN, NP = 4 * NM * NN;
};

// Writes partials[(power - 1) * gridDim.x + blockIdx.x] = the block's Cw mod
// p (canonical) for powers 1 .. NB*NA; super-blocks of 256 ids as mfma8.h.
// OFF: an offset pass (T > NB * NA): giants x^(base + NB a), a = 0..NA-1
// (base a multiple of NB, wave-uniform), powers base + 1 .. base + NB * NA.
template <int NM, int NN, int ABL = 0, bool OFF = false>
__device__ __forceinline__ void body(const uint64_t *__restrict__ ids, uint64_t n, uint64_t *__restrict__ partials,
                                     uint32_t base = 0) {
    using S = Shape<NM, NN>;
    constexpr int NA = S::NA, NB = S::NB, SEGS = S::SEGS, NP = S::NP;
    __shared__ __attribute__((aligned(16))) uint8_t img[WAVES][SEGS][1024];
    __shared__ uint64_t red[WAVES][NP];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *my = &img[wave][0][0];
    const uint32_t rd = 8 * (lane & 15) + 128 * (lane >> 4);
    for (int p = lane; p < NP; p += 64) red[wave][p] = 0;

    v4i acc[NM][NN];
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int c = 0; c < NN; ++c) acc[m][c] = v4i{0, 0, 0, 0};

    // tile (m, c), lane l, register r: giant 2m + (l >> 5), limb j = 4 ((l >> 4) & 1) + r;
    // baby 2c + ((l & 15) >> 3), limb k = l & 7.  The 16 lanes of one (giant,
    // baby) pair differ in bits 0-2 and 4.
    auto flush = [&]() {
        const int k = lane & 7, jh = 4 * ((lane >> 4) & 1);
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int c = 0; c < NN; ++c) {
                uint64_t v = 0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int32_t a = acc[m][c][r];
                    const uint64_t am = a < 0 ? P64 - (uint64_t)(-(int64_t)a) : (uint64_t)a;   // canonical
                    v = add64(v, mul64(am, wpow(jh + r + k)));
                }
                v = shfl_add64(v, 1);
                v = shfl_add64(v, 2);
                v = shfl_add64(v, 4);
                v = shfl_add64(v, 16);
                if ((lane & 0x17) == 0) {
                    const int p = (2 * m + (lane >> 5)) * NB + 2 * c + ((lane & 15) >> 3);
                    red[wave][p] = add64(red[wave][p], v);
                }
                acc[m][c] = v4i{0, 0, 0, 0};
                // one tile at a time: hoisting the other tiles' reads would
                // hold all of them in VGPRs beside the accumulators
                __builtin_amdgcn_sched_barrier(0);
            }
    };

    const uint64_t nsb = (n + 255) / 256;
    const uint64_t W = (uint64_t)gridDim.x * WAVES;
    uint64_t sb = (uint64_t)blockIdx.x * WAVES + wave;
    uint64_t nx[4];
    auto load = [&](uint64_t s) {
        if (s * 256 + 256 <= n) {
            const uint64_t *base = ids + s * 256 + lane;
#pragma unroll
            for (int q = 0; q < 4; ++q) nx[q] = base[64 * q];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t i = s * 256 + 64 * q + lane;
                const uint64_t v = ids[i < n ? i : n - 1];
                nx[q] = i < n ? v : 0ull;
            }
        }
    };
    auto put = [&](int seg, uint64_t lo, uint64_t hi) {   // two values -> one 16-byte segment row
        if constexpr (ABL != 1)
            *reinterpret_cast<uint4 *>(my + seg * 1024 + lane * 16) =
                make_uint4((uint32_t)lo ^ OFS, (uint32_t)(lo >> 32) ^ OFS, (uint32_t)hi ^ OFS,
                           (uint32_t)(hi >> 32) ^ OFS);
    };
    auto kblock = [&](uint64_t x) {
        const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32);
        uint64_t B[NB];
        uint64_t V = x;
        B[0] = x;
#pragma unroll
        for (int b = 1; b < NB; ++b) {
            if constexpr (ABL != 4) bsgs64::mulv(V, x0, x1);
            else V += b;
            B[b] = V;
        }
#pragma unroll
        for (int c = 0; c < NN; ++c) put(NM + c, B[2 * c], B[2 * c + 1]);
        const uint32_t g0 = (uint32_t)V, g1 = (uint32_t)(V >> 32);   // x^NB
        uint64_t prev;                                                // G_(a-1) of an odd a
        if constexpr (OFF) {
            // G_0 = (x^NB)^(base / NB): square-and-multiply over the wave-uniform exponent
            uint32_t q = base / NB;
            uint64_t r = 0, sq = V;
            bool have = false;
            for (;;) {
                if (q & 1) {
                    if (have) bsgs64::mulv(r, (uint32_t)sq, (uint32_t)(sq >> 32));
                    else r = sq;
                    have = true;
                }
                q >>= 1;
                if (!q) break;
                const uint32_t s0 = (uint32_t)sq, s1 = (uint32_t)(sq >> 32);
                bsgs64::mulv(sq, s0, s1);
            }
            V = r;
            prev = r;
        } else {
            prev = 1;                                                 // G_0
        }
#pragma unroll
        for (int a = 1; a < NA; ++a) {
            if (OFF || a > 1) {
                if constexpr (ABL != 4) bsgs64::mulv(V, g0, g1);
                else V ^= a;
            }
            if (a & 1) put(a >> 1, prev, V);
            else prev = V;
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        v4i af[NM], bf[NN];
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            const v2i lo = tr8(my + m * 1024 + rd), hi = tr8(my + m * 1024 + rd + 512);
            af[m] = v4i{lo.x, lo.y, hi.x, hi.y};
        }
#pragma unroll
        for (int c = 0; c < NN; ++c) {
            const v2i lo = tr8(my + (NM + c) * 1024 + rd), hi = tr8(my + (NM + c) * 1024 + rd + 512);
            bf[c] = v4i{lo.x, lo.y, hi.x, hi.y};
        }
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int c = 0; c < NN; ++c)
                acc[m][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[m], bf[c], acc[m][c], 0, 0, 0);
    };
    if (sb < nsb) load(sb);
    while (sb < nsb) {
        const uint64_t stop = sb + (uint64_t)(FLUSH / 4) * W;
        for (; sb < nsb && sb < stop; sb += W) {
            uint64_t x4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) x4[q] = nx[q];
            if (sb + W < nsb) load(sb + W);
            // one K-block at a time (unrolled, the four K-blocks' values and
            // fragments stay live together)
#pragma unroll 1
            for (int q = 0; q < 4; ++q) kblock(x4[q]);
        }
        flush();
    }
    __syncthreads();
    for (int p = threadIdx.x; p < NP; p += BLOCK) {
        uint64_t s = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s = add64(s, red[w][p]);
        partials[(size_t)p * gridDim.x + blockIdx.x] = s;
    }
}

} // namespace mf64
} // namespace qk
