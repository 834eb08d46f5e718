// mfma8.h — u32 encode with the baby-step/giant-step products on the matrix
// cores (v_mfma_i32_16x16x64_i8), DESIGN.md §3.2b.
//
// Power P = NB*a + b (a = 0..NA-1, b = 1..NB) is S_P = sum_i A_a(x_i) B_b(x_i)
// with babies B_b = x^b and giants A_a = x^(NB a) (A_0 = 1): over a tile of
// ids that is a matrix product, giants (rows) x babies (columns) contracted
// over the ids.  A 32-bit value is four bytes u_j, so
//     A B = sum_{j,k} 256^(j+k) u_{a,j} u_{b,k}
// and the integer limb products sum_i u_{a,j}(i) u_{b,k}(i) are an int8 GEMM
// with K = ids: M = NA giants x 4 limbs, N = NB babies x 4 limbs.  The MFMA
// multiplies SIGNED bytes, so each byte is stored as s = u - 128 (u ^ 0x80):
//     sum_i u_a u_b = C + 128 sum_i s_a + 128 sum_i s_b + 16384 N
// and, weighted by 256^(j+k) and summed (R = 0x01010101, N = id slots):
//     S_P = Cw(a,b) + 128 R (sum_i A_a + sum_i B_b) - 16384 R^2 N   (mod p)
// where sum_i A_a = S_(NB a) for a >= 1 (= N for a = 0) and sum_i B_b = S_b,
// so the a = 0 row solves to S_b = Cw(0,b) / (1 - 128 R) + 128 R N and each
// later row uses powers already resolved (k_mfma32_fix in encode.hip).
//
// Per wave and K-block of 64 ids (one per lane): the lane computes its id's
// NB - 1 + NA - 2 lazy modmuls (field.h mulfold32_min, exact redo on a
// possible wrap), XORs 0x80 into every byte and writes 16-byte segments (4
// giants, or 4 babies) to the wave's LDS image [segment][64 slots][16 B].
// ds_read_b64_tr_b8 then hands each lane one byte column of 8 slots — for
// lanes 16g .. 16g+15, lane 2q+p addresses row q, bytes 8p .. 8p+7, and lane
// i receives byte i of the 8 rows (tools/probe_i8.hip pins this and the MFMA
// lane maps on the hardware) — which is exactly the MFMA operand fragment
// A[row = byte][k = slot].  Two reads per fragment, NM + NN fragments and
// NM x NN MFMAs per K-block; no cross-wave traffic, no barrier.
//
// The int32 accumulators take at most 64 * 2^14 per K-block, so every
// FLUSH = 1024 K-blocks they are folded (mod p, weighted 256^(j+k)) into one
// 64-bit value per tile and lane.  The integer work per id is the modmuls
// plus one XOR per stored word; the products cost the matrix pipe
// 16 cycles per MFMA per 64 ids.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bsgs.h"
#include "field.h"

namespace qk {
namespace mf8 {

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;
constexpr uint32_t FLUSH = 1024;       // K-blocks between int32 folds: 1024 * 64 * 2^14 = 2^30
constexpr uint32_t OFS = 0x80808080u;  // u -> s = u - 128 per byte

__device__ __forceinline__ v2i tr8(const uint8_t *p) {
    return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i *)(p));
}

// 256^d mod p for d = 0..6 (2^32 == 5)
__device__ __forceinline__ uint32_t wpow(int d) { return d < 4 ? (1u << (8 * d)) : (5u << (8 * (d - 4))); }

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// NM tiles of 4 giant rows, NN tiles of 4 baby columns; NA <= 4 NM giants and
// NB <= 4 NN babies are used (powers 1 .. NA*NB; the spare rows/columns of a
// tile hold zero and their products are dropped)
template <int NM, int NN, int NBU = 4 * NN, int NAU = 4 * NM>
struct Shape {
    static_assert(NBU <= 4 * NN && NAU <= 4 * NM && NBU >= 2 && NAU >= 2, "used rows fit the tiles");
    static constexpr int NA = NAU, NB = NBU, SEGS = NM + NN, NP = NAU * NBU;
};

// int32 tile -> V += sum_r 256^(r + k) (acc_r mod p), k = this lane's baby limb
__device__ __forceinline__ void fold_tile(v4i &acc, uint64_t &V, int k) {
    uint64_t s = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int32_t c = acc[r];
        const uint32_t cm = c < 0 ? (uint32_t)((int64_t)c + (int64_t)P32) : (uint32_t)c;   // < p
        s += (uint64_t)cm * wpow(r + k);                                                    // < 2^57 each
    }
    V = fold64_32(V + fold64_32(s));
    acc = v4i{0, 0, 0, 0};
}

// Writes partials[(power - 1) * gridDim.x + blockIdx.x] = the block's Cw
// (sum of canonical lane values, < 2^40) for powers 1 .. NB*NA.  The ids are
// walked in super-blocks of 256 (4 K-blocks per wave), grid-stride over
// waves; slots past n hold id 0 (N = 256 * ceil(n / 256) slots in all).
// ABL (ablations for tools/tune_mfma.hip only; the product uses 0): 1 skips
// the LDS stores, 2 the transposed reads (operands from registers), 3 the
// MFMAs (the fragments are XORed into the accumulators), 4 the modmuls,
// 5 both the stores and the reads, 6 stores, reads and MFMAs (VALU only),
// 7 everything but the loads and the MFMAs.
// PIPE 1: each K-block's MFMAs take the fragments read one K-block earlier,
// so the transposed reads' latency hides behind the next id's modmuls
// instead of stalling the wave (in-order issue) at the MFMA.
// OFF: an offset pass of a multi-pass encode (T > NB * NA): the giants are
// x^(base + NB a) for a = 0..NA-1 (base a multiple of NB, wave-uniform), so
// the pass yields powers base + 1 .. base + NB * NA.
template <int NM, int NN, int ABL = 0, int PIPE = 1, bool OFF = false, int NBU = 4 * NN, int NAU = 4 * NM>
__device__ __forceinline__ void body(const uint32_t *__restrict__ ids, uint64_t n, uint64_t *__restrict__ partials,
                                     uint32_t base = 0) {
    using S = Shape<NM, NN, NBU, NAU>;
    constexpr int NA = S::NA, NB = S::NB, SEGS = S::SEGS, NP = S::NP;
    __shared__ __attribute__((aligned(16))) uint8_t img[WAVES][SEGS][1024];
    __shared__ uint64_t red[WAVES][NP];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int k = lane & 3;
    uint8_t *my = &img[wave][0][0];
    // tr read: lane group g = lane >> 4 takes slots 8 (4h + g) .. +7 for
    // fragment half h (the two groups of a 32-lane half sit in different
    // bank halves); lane i of the group addresses row i >> 1, byte 8 (i & 1)
    const uint32_t rd = 8 * (lane & 15) + 128 * (lane >> 4);

    v4i acc[NM][NN];
    uint64_t V[NM][NN];
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int c = 0; c < NN; ++c) { acc[m][c] = v4i{0, 0, 0, 0}; V[m][c] = 0; }
    // fragments read but not yet multiplied (PIPE): zero bytes add nothing
    v4i paf[NM], pbf[NN];
#pragma unroll
    for (int m = 0; m < NM; ++m) paf[m] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < NN; ++c) pbf[c] = v4i{0, 0, 0, 0};
    auto mma = [&](const v4i (&fa)[NM], const v4i (&fb)[NN], uint32_t mn) {
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int c = 0; c < NN; ++c) {
                if constexpr (ABL == 3 || ABL == 6)
                    acc[m][c] ^= fa[m] ^ fb[c];
                else if constexpr (ABL == 1)
                    acc[m][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[m] ^ (int)mn, fb[c], acc[m][c], 0, 0, 0);
                else
                    acc[m][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[m], fb[c], acc[m][c], 0, 0, 0);
            }
    };

    const uint64_t nsb = (n + 255) / 256;
    const uint64_t W = (uint64_t)gridDim.x * WAVES;
    uint64_t sb = (uint64_t)blockIdx.x * WAVES + wave;
    uint32_t nx[4];
    // a whole super-block in range: four loads off one wave-uniform base;
    // the last one: clamped indices (unconditional loads either way, so the
    // wait for this super-block's ids leaves the next one's in flight)
    auto load = [&](uint64_t s) {
        if (s * 256 + 256 <= n) {
            const uint32_t *base = ids + s * 256 + lane;
#pragma unroll
            for (int q = 0; q < 4; ++q) nx[q] = base[64 * q];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t i = s * 256 + 64 * q + lane;
                const uint32_t v = ids[i < n ? i : n - 1];
                nx[q] = i < n ? v : 0u;
            }
        }
    };
    // one K-block: store the id's segments, read the fragments transposed,
    // multiply (PIPE: the previous K-block's fragments)
    auto bw = [](const uint32_t (&B)[NB], int b) { return b < NB ? B[b] ^ OFS : 0u; };   // stored baby word
    auto emit = [&](const uint32_t (&B)[NB], const uint32_t (&G)[NA], uint32_t mn) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            uint32_t g[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) g[c] = 4 * m + c < NA ? G[4 * m + c] ^ OFS : 0u;
            if constexpr (ABL != 1 && ABL < 5)
                *reinterpret_cast<uint4 *>(my + m * 1024 + lane * 16) = make_uint4(g[0], g[1], g[2], g[3]);
            else
                mn ^= g[0] ^ g[1] ^ g[2] ^ g[3];
        }
#pragma unroll
        for (int c = 0; c < NN; ++c) {
            if constexpr (ABL != 1 && ABL < 5)
                *reinterpret_cast<uint4 *>(my + (NM + c) * 1024 + lane * 16) =
                    make_uint4(bw(B, 4 * c), bw(B, 4 * c + 1), bw(B, 4 * c + 2), bw(B, 4 * c + 3));
            else
                mn ^= bw(B, 4 * c) ^ bw(B, 4 * c + 1) ^ bw(B, 4 * c + 2) ^ bw(B, 4 * c + 3);
        }
        // the wave's own stores, then transposed reads of them: a wave's LDS
        // instructions execute in order, so only code motion is fenced here
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        v4i af[NM], bf[NN];
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            if constexpr (ABL == 2 || ABL >= 5) {
                af[m] = v4i{(int)B[0], (int)(B[1] ^ mn), (int)B[2], (int)B[3]};
            } else {
                const v2i lo = tr8(my + m * 1024 + rd), hi = tr8(my + m * 1024 + rd + 512);
                af[m] = v4i{lo.x, lo.y, hi.x, hi.y};
            }
        }
#pragma unroll
        for (int c = 0; c < NN; ++c) {
            if constexpr (ABL == 2 || ABL >= 5) {
                bf[c] = v4i{(int)bw(B, 4 * c), (int)bw(B, 4 * c + 1), (int)bw(B, 4 * c + 2), (int)(bw(B, 4 * c + 3) ^ mn)};
            } else {
                const v2i lo = tr8(my + (NM + c) * 1024 + rd), hi = tr8(my + (NM + c) * 1024 + rd + 512);
                bf[c] = v4i{lo.x, lo.y, hi.x, hi.y};
            }
        }
        if constexpr (PIPE) {
            mma(paf, pbf, mn);
#pragma unroll
            for (int m = 0; m < NM; ++m) paf[m] = af[m];
#pragma unroll
            for (int c = 0; c < NN; ++c) pbf[c] = bf[c];
        } else {
            mma(af, bf, mn);
        }
    };
    // one id per lane: babies x^1..x^NB, giants G_a (G_0 = 1, or x^base for
    // an offset pass), lazy modmuls with an exact redo when a fold may have
    // wrapped (field.h mulfold32_min), then the K-block
    auto kblock = [&](uint32_t x) {
        uint32_t B[NB], G[NA];
        uint32_t mn = 0xFFFFFFFFu;
        B[0] = x;
        if constexpr (ABL == 4 || ABL == 7) {
#pragma unroll
            for (int b = 1; b < NB; ++b) B[b] = x + b;
#pragma unroll
            for (int a = 0; a < NA; ++a) G[a] = x ^ a;
            mn = 99;
        } else {
#pragma unroll
            for (int b = 1; b < NB; ++b) B[b] = mulfold32_min(B[b - 1], x, mn);
            const uint32_t xn = B[NB - 1];
            if constexpr (OFF) {
                G[0] = bsgs::pow_uniform(xn, base / NB, [&](uint32_t u, uint32_t v) { return mulfold32_min(u, v, mn); });
#pragma unroll
                for (int a = 1; a < NA; ++a) G[a] = mulfold32_min(G[a - 1], xn, mn);
            } else {
                G[0] = 1;
                G[1] = xn;
#pragma unroll
                for (int a = 2; a < NA; ++a) G[a] = mulfold32_min(G[a - 1], xn, mn);
            }
        }
        if (__builtin_expect(__any(mn < 25u), 0)) {
            if (mn < 25u) {
#pragma unroll
                for (int b = 1; b < NB; ++b) B[b] = mulfold32_exact(B[b - 1], x);
                const uint32_t xn = B[NB - 1];
                if constexpr (OFF) {
                    G[0] = bsgs::pow_uniform(xn, base / NB, [](uint32_t u, uint32_t v) { return mulfold32_exact(u, v); });
#pragma unroll
                    for (int a = 1; a < NA; ++a) G[a] = mulfold32_exact(G[a - 1], xn);
                } else {
                    G[1] = xn;
#pragma unroll
                    for (int a = 2; a < NA; ++a) G[a] = mulfold32_exact(G[a - 1], xn);
                }
            }
        }
        emit(B, G, mn);
    };
    if (sb < nsb) load(sb);
    // flush periods of FLUSH / 4 super-blocks: no branch inside the inner loop
    while (sb < nsb) {
        const uint64_t stop = sb + (uint64_t)(FLUSH / 4) * W;
        for (; sb < nsb && sb < stop; sb += W) {
            uint32_t x4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) x4[q] = nx[q];
            if (sb + W < nsb) load(sb + W);   // next super-block in flight during this one
#pragma unroll
            for (int q = 0; q < 4; ++q) kblock(x4[q]);
        }
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int c = 0; c < NN; ++c) fold_tile(acc[m][c], V[m][c], k);
    }
    if constexpr (PIPE) {   // the last K-block's fragments
        mma(paf, pbf, 0u);
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int c = 0; c < NN; ++c) fold_tile(acc[m][c], V[m][c], k);
    }
    // epilogue: lane (g = lane >> 4, col = lane & 15) holds rows 4g + r of
    // tile (m, c): giant 4m + g, limb r; baby 4c + (col >> 2), limb k
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int c = 0; c < NN; ++c) {
            uint64_t v = V[m][c];                       // < 2^32
            v += shfl_xor_u64(v, 1);
            v += shfl_xor_u64(v, 2);                    // the four baby limbs: < 2^34
            const int a = 4 * m + (lane >> 4), b = 4 * c + ((lane & 15) >> 2);
            if (k == 0 && a < NA && b < NB) red[wave][a * NB + b] = v;
        }
    __syncthreads();
    for (int p = threadIdx.x; p < NP; p += BLOCK) {
        uint64_t s = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s += red[w][p];   // < 2^36
        partials[(size_t)p * gridDim.x + blockIdx.x] = s;
    }
}

} // namespace mf8
} // namespace qk
