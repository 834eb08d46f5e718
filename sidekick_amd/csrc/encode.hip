// encode.hip — batch power-sum encode on gfx950 (the hot path).
//
// Replaces the reference's per-id loop `for id in ids { quack.insert(id) }`
// (sidekick/src/sidekick.rs:42 inside the sniff loop :76-124; quack's
// benchmark_construct, figures/fig2_microbenchmarks.py:220-228) for an id
// array resident in HBM.
//
// Kernels and dispatch (`enc32` / `enc64` below):
//   * 5 <= t <= 80 (u32) — the headline kernel k_encode_u32_bsgs<NB,NA,SG>
//     (bsgs.h): baby steps x^1..x^NB and giant steps x^(NB a) per id, lane
//     private, then S_(NB a + b) += A_a * B_b as 64-bit multiply-accumulates
//     whose wraps are counted per wave on the scalar unit.  t = 32 is
//     (NB, NA) = (8, 4): 9 lazy modmuls + 24 MACs + 8 row-0 mads per id =
//     4.47 SIMD-cycles of VALU issue per id (the algorithmic anchor,
//     tools/issue_model.py); the kernel issues 1.19 VALU + 0.76 SALU
//     wave-instructions per id, each id's MAC phase at raised wave priority
//     (s_setprio, knob bsgs_prio), over encode grids of three rounds of
//     resident workgroups (knob grid_mult), and runs at 0.86-0.89 of the
//     anchor at the bench run's own shader clock (bench.py roofline.valu,
//     DESIGN.md §4) and ~0.20-0.21 of the HBM read roofline (4 B/id; the
//     line moves with the box's shader clock, 2.0-2.1 GHz).
//   * 14 <= t <= 80 (u64) — k_encode_u64_bsgs<NA,SG,F> (bsgs64.h): the
//     same split with the babies/giants of a 256-id tile shared through LDS,
//     each wave owning two babies' MAC rows (paired, at raised priority).
//   * t > 80 — passes of the BSGS kernels (offset giants x^(base + 8a)).
//   * small t (u32 t <= 4, u64 t <= 13) — power chains: a lane group of G
//     lanes owns one id, lane j computes powers j+1, j+1+G, ... with step
//     x^G and K lazy accumulators (G K >= t).
//   The ids are never reduced mod p up front (x^k is congruent either way).
//   Lane partials -> wavefront butterfly -> LDS across the waves -> one
//   partial per (power, block), stored [power][block] -> a finalize kernel
//   (one workgroup per power) writes the canonical partial vector.
// Integer-issue bound; no MFMA (north_star).  (The int8 matrix-core variant
// measured in rounds 2-3, DESIGN.md §3.9, was removed from the sources in
// round 4; it lives in the git history.)
#include "ctx.h"
#include "field.h"
#include "bsgs.h"
#include "bsgs64.h"

// scalar-counted wrap groups of the t = 25..32 BSGS kernel (tools/tune_bsgs.hip)
#ifndef QK_BSGS_SG_T32
#define QK_BSGS_SG_T32 8
#endif
#ifndef QK_BSGS_ROW0
#define QK_BSGS_ROW0 1
#endif
#ifndef QK_BSGS_FOLD
#define QK_BSGS_FOLD 1
#endif

namespace qk {

QK_WARM_KERNEL(encode)

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// ------------------------------------------------------------------ u32
// Power chain in t-form (field.h: tstep32): per power three v_mad_u64_u32,
// one v_sub_u32 and one 64-bit accumulate; x and x5 = 5x are canonical.

template <int K>
__device__ __forceinline__ void chain32(uint64_t (&acc)[K], uint32_t start, uint32_t step) {
    // start: any value < 2^32 (t-form with hi = 0); step canonical
    const uint32_t step5 = times5_32(step);
    uint64_t t = start;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        acc[k] += t;
        if (k + 1 < K) t = tstep32p(t, step, step5, 0u);
    }
}

// four independent ids in lockstep (ILP for the dependent modmul chains);
// the four t-form values of a power are summed before the accumulate
// (each < 6*2^32, so the sum and the lane accumulator stay far below 2^64).
template <int K>
__device__ __forceinline__ void chain32x4(uint64_t (&acc)[K], uint4 w) {
    const uint32_t x0 = canon32(w.x), x1 = canon32(w.y), x2 = canon32(w.z), x3 = canon32(w.w);
    const uint32_t f0 = times5_32(x0), f1 = times5_32(x1), f2 = times5_32(x2), f3 = times5_32(x3);
    uint64_t t0 = x0, t1 = x1, t2 = x2, t3 = x3;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        acc[k] += t0;
        acc[k] += t1;
        acc[k] += t2;
        acc[k] += t3;
        if (k + 1 < K) {
            t0 = tstep32p(t0, x0, f0, 0u);
            t1 = tstep32p(t1, x1, f1, 0u);
            t2 = tstep32p(t2, x2, f2, 0u);
            t3 = tstep32p(t3, x3, f3, 0u);
        }
    }
}

// ---- baby-step / giant-step encode for 9 <= t <= 32 (bsgs.h)
// waves per SIMD the register budget is sized for (tools/tune_bsgs.hip: 5 for
// (8,4) beat 4 by 2-3 %; its three spilled VGPRs live outside the loop)
// PRIO (knob bsgs_prio): wave priority over each id's accumulation — row 0
// at 1, the MAC rows at 2, the powers at 0 (bsgs.h Cfg PRIO 4; t = 32: 2.60 /
// 2.67 vs 2.66 / 2.73 ms for the MAC phase at 1, vs 2.77 ms for none,
// profiles/r04/prio/tune_bsgs_prio_levels*.json)
template <int NB, int NA, int SG, int PRIO = 1>
__global__ __launch_bounds__(BLOCK, (NB * NA == 32 ? 5 : NB * NA > 64 ? 2 : NB * NA > 40 ? 3 : 4)) void k_encode_u32_bsgs(const uint32_t *__restrict__ ids,
                                                                                  uint64_t n, uint32_t head,
                                                                                  uint32_t T,
                                                                                  uint64_t *__restrict__ partials) {
    bsgs::body<bsgs::Cfg<NB, NA, SG, QK_BSGS_ROW0, QK_BSGS_FOLD, false, false, 0, false, PRIO ? 4 : 0>>(ids, n, head,
                                                                                                        T, partials);
}


// Pass 0 of a multi-pass encode (powers 1..80) that also writes x^80 per id
// for pass 1 (the x^base cache, enc32_passes)
template <int SG, int PRIO = 1>
__global__ __launch_bounds__(BLOCK, 2) void k_encode_u32_bsgs_x80(const uint32_t *__restrict__ ids, uint64_t n,
                                                                 uint32_t head, uint32_t T,
                                                                 uint64_t *__restrict__ partials,
                                                                 const uint32_t *xin,
                                                                 uint32_t *xout) {
    (void)xin;
    bsgs::body<bsgs::Cfg<8, 10, SG, 1, 1, false, false, 2, false, PRIO ? 4 : 0>>(ids, n, head, T, partials, 0, nullptr,
                                                                                 xout);
}

// Offset pass for thresholds > 80 (several passes over the ids): powers
// base+1 .. base+8*NA with giants x^(base + 8a), a = 0..NA-1 (bsgs.h OFF).
// XC: x^base from the previous pass's per-id cache (bit 0) / x^(base + 8 NA)
// to the next pass's (bit 1) instead of square-and-multiply per pass.
template <int NA, int SG, int XC = 0, int PRIO = 1>
__global__ __launch_bounds__(BLOCK, (NA > 6 ? 2 : NA > 5 ? 3 : 4)) void k_encode_u32_bsgs_off(
    const uint32_t *__restrict__ ids, uint64_t n, uint32_t head, uint32_t T, uint32_t base,
    uint64_t *__restrict__ partials, const uint32_t *xin, uint32_t *xout) {
    bsgs::body<bsgs::Cfg<8, NA, SG, 1, 1, false, true, XC, false, PRIO ? 4 : 0>>(ids, n, head, T, partials, base, xin,
                                                                                 xout);
}

// lane j of a G-group: start = x^(j+1), step = x^G (square-and-multiply).
template <int G>
__device__ __forceinline__ void group_powers32(uint32_t x, int j, uint32_t &start, uint32_t &step) {
    uint32_t b = x, r = 1;
    const uint32_t e = (uint32_t)j + 1;
#pragma unroll
    for (int bit = 0; (1 << bit) <= G; ++bit) {
        const uint32_t rb = mul32_lazy(r, b);
        r = ((e >> bit) & 1) ? rb : r;
        if ((1 << bit) < G) b = mul32_lazy(b, b);
    }
    start = r;
    step = canon32(b); // after log2(G) squarings b = x^G; the chain needs it canonical
}

// Reduce per-lane accumulators to one partial per (power, block).
// acc[k] of lane with (lane % G) == j belongs to power m = j + k*G (0-based).
template <int G, int K, typename Fold>
__device__ __forceinline__ void block_store(const uint64_t (&acc)[K], uint32_t T, uint64_t *partials,
                                            uint64_t *sm, Fold fold) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint64_t v = fold(acc[k]);                   // < 2^32
#pragma unroll
        for (int off = 32; off >= G; off >>= 1) v += shfl_xor_u64(v, off); // < 2^38
        if (lane < G) sm[wave * (G * K) + lane + k * G] = v;
    }
    __syncthreads();
    for (uint32_t m = threadIdx.x; m < T; m += BLOCK) {
        uint64_t s = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s += sm[w * (G * K) + m];   // < 2^40
        partials[(size_t)m * gridDim.x + blockIdx.x] = s;
    }
}

struct Fold32 {
    __device__ uint64_t operator()(uint64_t a) const { return fold64_32(a); }
};

// G == 1: each lane streams ids with 16-byte loads.
template <int K>
__global__ __launch_bounds__(BLOCK) void k_encode_u32_g1(const uint32_t *__restrict__ ids, uint64_t n,
                                                         uint32_t head, uint32_t T,
                                                         uint64_t *__restrict__ partials) {
    __shared__ uint64_t sm[WAVES * K];
    uint64_t acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0;

    const uint64_t gtid = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * BLOCK;
    const uint64_t h = head < n ? head : n;
    const uint64_t body = (n - h) >> 2;
    const uint4 *__restrict__ v = reinterpret_cast<const uint4 *>(ids + h);

    for (uint64_t i = gtid; i < body; i += nthr) chain32x4<K>(acc, v[i]);
    // unaligned head (< 4 ids) and tail (< 4 ids)
    const uint64_t tail0 = h + (body << 2);
    if (gtid < h) chain32<K>(acc, ids[gtid], canon32(ids[gtid]));
    if (gtid < n - tail0) chain32<K>(acc, ids[tail0 + gtid], canon32(ids[tail0 + gtid]));

    block_store<1, K>(acc, T, partials, sm, Fold32{});
}

// G > 1: lane groups share one id (scalar loads; G lanes read one address).
template <int G, int K>
__global__ __launch_bounds__(BLOCK) void k_encode_u32_gn(const uint32_t *__restrict__ ids, uint64_t n,
                                                         uint32_t head, uint32_t T,
                                                         uint64_t *__restrict__ partials) {
    (void)head;
    __shared__ uint64_t sm[WAVES * G * K];
    uint64_t acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0;
    const int j = threadIdx.x % G;
    const uint64_t grp = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) / G;
    const uint64_t ngrp = (uint64_t)gridDim.x * BLOCK / G;
    for (uint64_t i = grp; i < n; i += ngrp) {
        uint32_t start, step;
        group_powers32<G>(ids[i], j, start, step);
        chain32<K>(acc, start, step);
    }
    block_store<G, K>(acc, T, partials, sm, Fold32{});
}

// Sum block partials of power m = blockIdx.x; write canonical S_m (or add it
// into out when accumulate), count and last id.
__global__ __launch_bounds__(BLOCK) void k_finalize_u32(const uint64_t *__restrict__ partials,
                                                        uint32_t nblocks, uint32_t T,
                                                        const uint32_t *__restrict__ ids, uint64_t n,
                                                        uint64_t *__restrict__ out, int accumulate) {
    __shared__ uint64_t sm[WAVES];
    const uint32_t m = blockIdx.x;
    uint64_t s = 0;
    for (uint32_t b = threadIdx.x; b < nblocks; b += BLOCK) s += partials[(size_t)m * nblocks + b]; // < 2^60
    s = fold64_32(s);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += shfl_xor_u64(s, off);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t tot = 0;
        for (int w = 0; w < WAVES; ++w) tot += sm[w];
        uint32_t c = canon32(fold64_32(tot));
        out[m] = accumulate ? (uint64_t)add32((uint32_t)out[m], c) : (uint64_t)c;
        if (m == 0) {
            out[T] = accumulate ? out[T] + n : n;
            if (n) out[T + 1] = ids[n - 1];
            else if (!accumulate) out[T + 1] = 0;
        }
    }
}

// One pass of a multi-pass encode: powers m < T of this pass go to
// out[m] (out = the partial vector + the pass's base); the pass with
// meta != nullptr also writes count and last id there (meta[0], meta[1]).
__global__ __launch_bounds__(BLOCK) void k_finalize_u32_pass(const uint64_t *__restrict__ partials,
                                                             uint32_t nblocks, uint32_t T,
                                                             const uint32_t *__restrict__ ids, uint64_t n,
                                                             uint64_t *__restrict__ out,
                                                             uint64_t *__restrict__ meta, int accumulate) {
    __shared__ uint64_t sm[WAVES];
    const uint32_t m = blockIdx.x;
    uint64_t s = 0;
    for (uint32_t b = threadIdx.x; b < nblocks; b += BLOCK) s += partials[(size_t)m * nblocks + b];
    s = fold64_32(s);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += shfl_xor_u64(s, off);
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t tot = 0;
        for (int w = 0; w < WAVES; ++w) tot += sm[w];
        const uint32_t c = canon32(fold64_32(tot));
        out[m] = accumulate ? (uint64_t)add32((uint32_t)out[m], c) : (uint64_t)c;
        if (m == 0 && meta) {
            meta[0] = accumulate ? meta[0] + n : n;
            if (n) meta[1] = ids[n - 1];
            else if (!accumulate) meta[1] = 0;
        }
    }
}

// ------------------------------------------------------------------ u64
// Power chain over p64 = 2^64 - 59, hand-scheduled (gfx950 ISA).  State:
// t = t0 + t1*2^32 + th*2^64 (th <= 59; t0:t1 pinned in v[2:3] so the step can
// address the halves of its 64-bit pairs).  One step, for a step value x < 2^64:
//   V  = (t0:t1) + 59*th            v_mad_u64_u32; wraps past 2^64 only when
//                                   V < 59*60, then V += 59 (2^64 == 59) exactly
//   P  = V*x < 2^128                four v_mad_u64_u32:
//        A = V.lo*x0, B = V.hi*x0 + A.hi, C = V.lo*x1 + B (carry cc),
//        PH = V.hi*x1 + C.hi + cc*2^32, P_L = A.lo + C.lo*2^32
//   t' = P_L + 59*PH  (< 60*2^64)   two v_mad_u64_u32: E = P_L + 59*PH.lo
//                                   (carry ce), F = E.hi + ce*2^32 + 59*PH.hi;
//                                   t0' = E.lo, t1' = F.lo, th' = F.hi
// and the previous power's value is added into its 96-bit accumulator
// (a0, a1, a2) with a carry chain in the same block: 7 multiplies + 14 simple
// ops per power (the compiler's rendering of field.h tstep64 plus the
// accumulate spends 8 multiplies and ~20 moves/adds/compares).  Every
// VALU-written carry is read >= 2 wait states later (gfx950 VALU SGPR-write ->
// VALU read hazard).
#define QK_U64_STEP_ASM                                                                            \
    "v_add_co_u32_e64 %[a0], %[sc], %[a0], v2\n\t"                                                   \
    "v_mad_u64_u32 v[4:5], %[cw], %[th], 59, v[2:3]\n\t"                                             \
    "v_mov_b32_e32 v11, 0\n\t"                                                                     \
    "v_addc_co_u32_e64 %[a1], %[sc], %[a1], v3, %[sc]\n\t"                                           \
    "v_cndmask_b32_e64 %[tmp], 0, 59, %[cw]\n\t"                                                     \
    "v_add_u32_e32 v4, v4, %[tmp]\n\t"                                                               \
    "v_addc_co_u32_e64 %[a2], %[cx], %[a2], %[th], %[sc]\n\t"                                        \
    "v_mad_u64_u32 v[6:7], %[cx], v4, %[x0], 0\n\t"                                                  \
    "v_mov_b32_e32 v10, v7\n\t"                                                                    \
    "v_mad_u64_u32 v[8:9], %[cx], v5, %[x0], v[10:11]\n\t"                                           \
    "v_mad_u64_u32 v[8:9], %[cc], v4, %[x1], v[8:9]\n\t"                                             \
    "v_mov_b32_e32 v7, v8\n\t"                                                                     \
    "v_mov_b32_e32 v10, v9\n\t"                                                                    \
    "v_cndmask_b32_e64 v11, 0, 1, %[cc]\n\t"                                                         \
    "v_mad_u64_u32 v[4:5], %[cx], v5, %[x1], v[10:11]\n\t"                                           \
    "v_mad_u64_u32 v[2:3], %[ce], v4, 59, v[6:7]\n\t"                                                \
    "v_mov_b32_e32 v8, v3\n\t"                                                                     \
    "s_nop 0\n\t"                                                                                  \
    "v_cndmask_b32_e64 v9, 0, 1, %[ce]\n\t"                                                          \
    "v_mad_u64_u32 v[8:9], %[cx], v5, 59, v[8:9]\n\t"                                                \
    "v_mov_b32_e32 v3, v8\n\t"                                                                     \
    "v_mov_b32_e32 %[th], v9\n\t"

template <int K>
__device__ __forceinline__ void chain64(uint32_t (&a0)[K], uint32_t (&a1)[K], uint32_t (&a2)[K], uint64_t start,
                                        uint64_t step) {
    // start, step: any values < 2^64 (t-form with th = 0)
    uint64_t t = start;
    uint32_t th = 0;
    const uint32_t x0 = (uint32_t)step, x1 = (uint32_t)(step >> 32);
#pragma unroll
    for (int k = 0; k + 1 < K; ++k) {
        uint64_t sc, cw, cx, cc, ce;
        uint32_t tmp;
        asm volatile(QK_U64_STEP_ASM
                     : [a0] "+v"(a0[k]), [a1] "+v"(a1[k]), [a2] "+v"(a2[k]), "+{v[2:3]}"(t), [th] "+v"(th),
                       [sc] "=&s"(sc), [cw] "=&s"(cw), [cx] "=&s"(cx), [cc] "=&s"(cc), [ce] "=&s"(ce),
                       [tmp] "=&v"(tmp)
                     : [x0] "v"(x0), [x1] "v"(x1)
                     : "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11");
    }
    uint64_t sc, cx;
    asm volatile("v_add_co_u32_e64 %[a0], %[sc], %[a0], v2\n\t"
                 "s_nop 1\n\t"
                 "v_addc_co_u32_e64 %[a1], %[sc], %[a1], v3, %[sc]\n\t"
                 "s_nop 1\n\t"
                 "v_addc_co_u32_e64 %[a2], %[cx], %[a2], %[th], %[sc]\n\t"
                 : [a0] "+v"(a0[K - 1]), [a1] "+v"(a1[K - 1]), [a2] "+v"(a2[K - 1]), [sc] "=&s"(sc), [cx] "=&s"(cx)
                 : "{v[2:3]}"(t), [th] "v"(th));
}

// (lo, hi) -> a 64-bit value through an opaque move, so the 32-bit
// accumulators are not kept as zero-extended / shifted 64-bit pairs
__device__ __forceinline__ uint64_t pack64(uint32_t lo, uint32_t hi) {
    uint64_t v;
    asm volatile("v_mov_b32_e32 v12, %1\n\tv_mov_b32_e32 v13, %2" : "={v[12:13]}"(v) : "v"(lo), "v"(hi));
    return v;
}

// t-form value -> a value < 2^64 congruent to it (chain starts and steps)
__device__ __forceinline__ uint64_t vfold64(uint32_t t0, uint32_t t1, uint32_t th) {
    const uint64_t t = ((uint64_t)t1 << 32) | t0;
    const uint64_t v = t + (uint64_t)th * C64;
    return v < t ? v + C64 : v; // wrapped: v < 59*60 and 2^64 == 59
}

// The step without an accumulate (chain setup): t <- t*x, t-form in/out.
#define QK_U64_MUL_ASM                                                                             \
    "v_mad_u64_u32 v[4:5], %[cw], %[th], 59, v[2:3]\n\t"                                             \
    "v_mov_b32_e32 v11, 0\n\t"                                                                     \
    "s_nop 0\n\t"                                                                                  \
    "v_cndmask_b32_e64 %[tmp], 0, 59, %[cw]\n\t"                                                     \
    "v_add_u32_e32 v4, v4, %[tmp]\n\t"                                                               \
    "v_mad_u64_u32 v[6:7], %[cx], v4, %[x0], 0\n\t"                                                  \
    "v_mov_b32_e32 v10, v7\n\t"                                                                    \
    "v_mad_u64_u32 v[8:9], %[cx], v5, %[x0], v[10:11]\n\t"                                           \
    "v_mad_u64_u32 v[8:9], %[cc], v4, %[x1], v[8:9]\n\t"                                             \
    "v_mov_b32_e32 v7, v8\n\t"                                                                     \
    "v_mov_b32_e32 v10, v9\n\t"                                                                    \
    "v_cndmask_b32_e64 v11, 0, 1, %[cc]\n\t"                                                         \
    "v_mad_u64_u32 v[4:5], %[cx], v5, %[x1], v[10:11]\n\t"                                           \
    "v_mad_u64_u32 v[2:3], %[ce], v4, 59, v[6:7]\n\t"                                                \
    "v_mov_b32_e32 v8, v3\n\t"                                                                     \
    "s_nop 0\n\t"                                                                                  \
    "v_cndmask_b32_e64 v9, 0, 1, %[ce]\n\t"                                                          \
    "v_mad_u64_u32 v[8:9], %[cx], v5, 59, v[8:9]\n\t"                                                \
    "v_mov_b32_e32 v3, v8\n\t"                                                                     \
    "v_mov_b32_e32 %[th], v9\n\t"

__device__ __forceinline__ void tmul64_asm(uint64_t &t, uint32_t &th, uint32_t x0, uint32_t x1) {
    uint64_t cw, cx, cc, ce;
    uint32_t tmp;
    asm volatile(QK_U64_MUL_ASM
                 : "+{v[2:3]}"(t), [th] "+v"(th), [cw] "=&s"(cw), [cx] "=&s"(cx), [cc] "=&s"(cc), [ce] "=&s"(ce),
                   [tmp] "=&v"(tmp)
                 : [x0] "v"(x0), [x1] "v"(x1)
                 : "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11");
}

// Lane j of a group of G starts at x^(j+1) and steps by x^G: x^2 .. x^G by
// the same step, each folded below 2^64.
template <int G>
__device__ __forceinline__ void group_powers64(uint64_t x, int j, uint64_t &start, uint64_t &step) {
    const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32);
    uint64_t t = x;
    uint32_t th = 0;
    start = x;
    step = x;
#pragma unroll
    for (int g = 1; g < G; ++g) {
        tmul64_asm(t, th, x0, x1);
        const uint64_t v = vfold64((uint32_t)t, (uint32_t)(t >> 32), th);
        if (g == j) start = v;
        step = v; // after the last iteration: x^G
    }
}

// u64 partials: two 32-bit limbs per power, stored [2m + limb][block].
template <int G, int K>
__device__ __forceinline__ void block_store64(const uint32_t (&a0)[K], const uint32_t (&a1)[K],
                                              const uint32_t (&a2)[K], uint32_t T, uint64_t *partials,
                                              uint64_t *sm) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t f = fold96_64(a2[k], pack64(a0[k], a1[k]));
        uint64_t a = (uint32_t)f, b = f >> 32;
#pragma unroll
        for (int off = 32; off >= G; off >>= 1) {
            a += shfl_xor_u64(a, off);
            b += shfl_xor_u64(b, off);
        }
        if (lane < G) {
            sm[wave * (2 * G * K) + 2 * (lane + k * G)] = a;
            sm[wave * (2 * G * K) + 2 * (lane + k * G) + 1] = b;
        }
    }
    __syncthreads();
    for (uint32_t m = threadIdx.x; m < 2 * T; m += BLOCK) {
        uint64_t s = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s += sm[w * (2 * G * K) + m];
        partials[(size_t)m * gridDim.x + blockIdx.x] = s;
    }
}

template <int K>
__global__ __launch_bounds__(BLOCK) void k_encode_u64_g1(const uint64_t *__restrict__ ids, uint64_t n,
                                                         uint32_t head, uint32_t T,
                                                         uint64_t *__restrict__ partials) {
    __shared__ uint64_t sm[WAVES * 2 * K];
    uint32_t a0[K], a1[K], a2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) { a0[k] = 0; a1[k] = 0; a2[k] = 0; }
    const uint64_t gtid = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * BLOCK;
    const uint64_t h = head < n ? head : n;
    const uint64_t body = (n - h) >> 1;
    const ulonglong2 *__restrict__ v = reinterpret_cast<const ulonglong2 *>(ids + h);
    for (uint64_t i = gtid; i < body; i += nthr) {
        const ulonglong2 w = v[i];
        chain64<K>(a0, a1, a2, w.x, w.x);
        chain64<K>(a0, a1, a2, w.y, w.y);
    }
    const uint64_t tail0 = h + (body << 1);
    if (gtid < h) chain64<K>(a0, a1, a2, ids[gtid], ids[gtid]);
    if (gtid < n - tail0) chain64<K>(a0, a1, a2, ids[tail0 + gtid], ids[tail0 + gtid]);
    block_store64<1, K>(a0, a1, a2, T, partials, sm);
}

template <int G, int K>
__global__ __launch_bounds__(BLOCK) void k_encode_u64_gn(const uint64_t *__restrict__ ids, uint64_t n,
                                                         uint32_t head, uint32_t T,
                                                         uint64_t *__restrict__ partials) {
    (void)head;
    __shared__ uint64_t sm[WAVES * 2 * G * K];
    uint32_t a0[K], a1[K], a2[K];
#pragma unroll
    for (int k = 0; k < K; ++k) { a0[k] = 0; a1[k] = 0; a2[k] = 0; }
    const int j = threadIdx.x % G;
    const uint64_t grp = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) / G;
    const uint64_t ngrp = (uint64_t)gridDim.x * BLOCK / G;
    for (uint64_t i = grp; i < n; i += ngrp) {
        uint64_t start, step;
        group_powers64<G>(ids[i], j, start, step);
        chain64<K>(a0, a1, a2, start, step);
    }
    block_store64<G, K>(a0, a1, a2, T, partials, sm);
}

// Sum block limb partials of power m = blockIdx.x; write canonical S_m as
// two 32-bit limbs out[2m], out[2m+1] (or add it in when accumulate); the
// launch with meta != nullptr also writes count and last id (meta[0..1]).
__device__ __forceinline__ void finalize_u64_body(const uint64_t *__restrict__ partials, uint32_t nblocks,
                                                  uint32_t T, const uint64_t *__restrict__ ids, uint64_t n,
                                                  uint64_t *__restrict__ out, uint64_t *__restrict__ meta,
                                                  int accumulate) {
    __shared__ uint64_t sm[2][WAVES];
    const uint32_t m = blockIdx.x; // power index
    uint64_t a = 0, b = 0;         // limb sums, each < nblocks * 2^40
    for (uint32_t i = threadIdx.x; i < nblocks; i += BLOCK) {
        a += partials[(size_t)(2 * m) * nblocks + i];
        b += partials[(size_t)(2 * m + 1) * nblocks + i];
    }
    // fold each limb sum to < 2^64 congruent, then re-split to limbs so the
    // cross-lane sums cannot overflow: value = a + b*2^32.
    {
        const uint64_t av = canon64(a), bv = mul64_lazy(canon64(b), 1ull << 32);
        const uint64_t vv = canon64(add64(canon64(av), canon64(bv)));
        a = (uint32_t)vv;
        b = vv >> 32;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        a += shfl_xor_u64(a, off);
        b += shfl_xor_u64(b, off);
    }
    if ((threadIdx.x & 63) == 0) { sm[0][threadIdx.x >> 6] = a; sm[1][threadIdx.x >> 6] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t sa = 0, sb = 0;
        for (int w = 0; w < WAVES; ++w) { sa += sm[0][w]; sb += sm[1][w]; } // < 2^40
        uint64_t v = add64(canon64(sa), mul64(canon64(sb), 1ull << 32));
        if (accumulate) v = add64(canon64(out[2 * m] | (out[2 * m + 1] << 32)), v);
        out[2 * m] = (uint32_t)v;
        out[2 * m + 1] = v >> 32;
        if (m == 0 && meta) {
            meta[0] = accumulate ? meta[0] + n : n;
            if (n) meta[1] = ids[n - 1];
            else if (!accumulate) meta[1] = 0;
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_finalize_u64_pass(const uint64_t *__restrict__ partials,
                                                             uint32_t nblocks, uint32_t T,
                                                             const uint64_t *__restrict__ ids, uint64_t n,
                                                             uint64_t *__restrict__ out,
                                                             uint64_t *__restrict__ meta, int accumulate) {
    finalize_u64_body(partials, nblocks, T, ids, n, out, meta, accumulate);
}

// single-pass form: count and last id right after the T limb pairs
__global__ __launch_bounds__(BLOCK) void k_finalize_u64(const uint64_t *__restrict__ partials,
                                                        uint32_t nblocks, uint32_t T,
                                                        const uint64_t *__restrict__ ids, uint64_t n,
                                                        uint64_t *__restrict__ out, int accumulate) {
    finalize_u64_body(partials, nblocks, T, ids, n, out, out + 2 * T, accumulate);
}

// u64 baby-step / giant-step (bsgs64.h): 256-id tiles, babies and giants
// shared through LDS, the MAC powers split over the 4 waves.  The babies'
// B * 2^32 are recomputed by their owner wave instead of stored (BSH) and x^8
// is read from baby 8: 32 KB of LDS per workgroup at t = 80, 4 per CU
// (tools/tune_u64.hip: 24.1 vs 25.6 ms per 1e9 ids with 50 KB at 3 per CU).
// The first SG MACs of a wave's tile count their carries on the scalar unit.
// F (knob bsgs64_prio): 1 — wave priority in the MAC step (the row-0 sums
// at 1, the MACs at 2: bsgs64.h PRIO 3, ~1 % over one level) and, with two
// babies per wave, the two MACs of a giant row issued as one interleaved
// block (MODE 3); 0 — the round-3 form (MODE 0, no priority changes)
template <int NA, int SG, int F = 1>
__global__ __launch_bounds__(bsgs64::BLOCK, 4) void k_encode_u64_bsgs(const uint64_t *__restrict__ ids, uint64_t n,
                                                                      uint32_t head, uint32_t T,
                                                                      uint64_t *__restrict__ partials) {
    (void)head;
    bsgs64::body<NA, F ? 3 : 0, SG, 0, 0, false, true, 1, 0, bsgs64::NB, F ? 3 : 0>(ids, n, T, partials);
}

// the same with four babies per id (one per wave) and NA giant rows of 4
// powers: t <= 40 (bsgs64.h NBT)
template <int NA, int F = 1>
__global__ __launch_bounds__(bsgs64::BLOCK, 4) void k_encode_u64_bsgs4(const uint64_t *__restrict__ ids, uint64_t n,
                                                                       uint32_t head, uint32_t T,
                                                                       uint64_t *__restrict__ partials) {
    (void)head;
    bsgs64::body<NA, 0, 16, 0, 0, false, true, 1, 0, 4, F ? 3 : 0>(ids, n, T, partials);
}

// Pass 0 of a u64 multi-pass encode that also writes x^80 per id for pass 1
template <int F = 1>
__global__ __launch_bounds__(bsgs64::BLOCK, 4) void k_encode_u64_bsgs_x80(const uint64_t *__restrict__ ids,
                                                                          uint64_t n, uint32_t head, uint32_t T,
                                                                          uint64_t *__restrict__ partials,
                                                                          uint64_t *xout) {
    (void)head;
    bsgs64::body<10, F ? 3 : 0, 16, 0, 0, false, true, 1, 2, bsgs64::NB, F ? 3 : 0>(ids, n, T, partials, 0, nullptr,
                                                                                 xout);
}

// Offset pass for u64 thresholds > 80: powers base+1 .. base+8NA with giants
// x^(base + 8a) (bsgs64.h OFF); the ids are read once per pass.
// XC: the per-id x^base cache between passes (bsgs64.h)
template <int NA, int XC = 0, int F = 1>
__global__ __launch_bounds__(bsgs64::BLOCK, 4) void k_encode_u64_bsgs_off(const uint64_t *__restrict__ ids,
                                                                          uint64_t n, uint32_t head, uint32_t T,
                                                                          uint32_t base,
                                                                          uint64_t *__restrict__ partials,
                                                                          const uint64_t *xin,
                                                                          uint64_t *xout) {
    (void)head;
    bsgs64::body<NA, F ? 3 : 0, 16, 0, 0, true, true, 1, XC, bsgs64::NB, F ? 3 : 0>(ids, n, T, partials, base, xin,
                                                                                     xout);
}

// ------------------------------------------------------------- dispatch
template <typename KernelT>
static uint32_t grid_for(qk_ctx *ctx, KernelT kern, uint64_t units, uint32_t per_block, int mult = 0) {
    if (ctx->grid_override) return ctx->grid_override;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, BLOCK, 0) != hipSuccess || occ < 1) occ = 1;
    // knob grid_mult: resident workgroups x this.  The encode kernels take
    // one contiguous run per workgroup; with one round of workgroups the
    // launch ends with the slowest CU's run, with three the runs are a third
    // as long and the CUs that finish early take the later ones
    // (mult > 0: fixed by the caller — u32 t > 48 and the u32 passes measured
    // 0.4-2.3 % slower at three rounds, profiles/r04/grid_mult/)
    const uint64_t full = (uint64_t)ctx->num_cus * (uint64_t)occ * (uint64_t)(mult > 0 ? mult : ctx->knobs.grid_mult);
    uint64_t need = (units + per_block - 1) / per_block;
    if (need < 1) need = 1;
    return (uint32_t)(need < full ? need : full);
}

// An upper bound on grid_for over every kernel a multi-pass encode may
// launch, whatever its occupancy: the device's resident threads per CU
// (hipDeviceAttributeMaxThreadsPerMultiProcessor, read at context creation)
// in workgroups of BLOCK threads.  The x^base cache is placed after the
// largest partials this allows.
static uint32_t grid_cap(const qk_ctx *ctx, uint64_t units, uint32_t per_block, int mult = 0) {
    if (ctx->grid_override) return ctx->grid_override;
    const uint64_t full = (uint64_t)ctx->num_cus * (uint64_t)ctx->max_blocks_per_cu(BLOCK) *
                          (uint64_t)(mult > 0 ? mult : ctx->knobs.grid_mult);
    uint64_t need = (units + per_block - 1) / per_block;
    if (need < 1) need = 1;
    return (uint32_t)(need < full ? need : full);
}

// Launch main kernel (+profiling events) then finalize.
template <typename IdT, typename KernelT, typename FinT>
static int run_encode(qk_ctx *ctx, KernelT kern, FinT fin, uint32_t GK, uint32_t words_per_power,
                      const IdT *d_ids, size_t n, uint32_t head, uint32_t T, uint64_t units,
                      uint32_t per_block, uint64_t *d_partial, int accumulate, hipStream_t s, int mult = 0) {
    const uint32_t nb = grid_for(ctx, kern, units, per_block, mult);
    const size_t need = (size_t)nb * words_per_power * GK * sizeof(uint64_t);
    int rc = ensure_scratch(ctx, need, s);
    if (rc) return rc;
    uint64_t *partials = (uint64_t *)ctx->d_scratch;
    rc = scratch_acquire(ctx, s);
    if (rc) return rc;
    hipEvent_t e0 = prof_begin(ctx, s);
    hipLaunchKernelGGL(kern, dim3(nb), dim3(BLOCK), 0, s, d_ids, (uint64_t)n, head, T, partials);
    prof_end(ctx, s, e0);
    QK_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(fin, dim3(T), dim3(BLOCK), 0, s, partials, nb, T, d_ids, (uint64_t)n, d_partial,
                       accumulate);
    QK_HIP_TRY(hipGetLastError());
    return scratch_release(ctx, s);
}

// sums of per-block partials [power][block] -> canonical S_1..S_T in out[0..T)
int launch_finalize_powers_u32(const uint64_t *partials, uint32_t nblocks, uint32_t T, uint64_t *out,
                               hipStream_t s) {
    hipLaunchKernelGGL(k_finalize_u32_pass, dim3(T), dim3(BLOCK), 0, s, partials, nblocks, T,
                       (const uint32_t *)nullptr, (uint64_t)0, out, (uint64_t *)nullptr, 0);
    return hipGetLastError() == hipSuccess ? QK_OK : QK_E_HIP;
}

// Thresholds 81..1024 by baby-step/giant-step passes: pass 0 is the (8,10)
// kernel (powers 1..80), each further pass the offset kernel with giants
// from x^base (the ids are read once per pass; HBM has the bandwidth, the
// passes are integer-issue bound like the single-pass kernels).
// xcache (offset passes): the per-id x^base cache (xin / xout), placed in
// the scratch after the partials (run_pass32_cached sizes the scratch once)
// KIND 0: a plain kernel (ids, n, head, T, partials); 1: an offset pass
// (+ base, xin, xout); 2: a plain kernel that writes the x^base cache
// (+ xin, xout)
template <int KIND, class KernelT>
static int run_pass(qk_ctx *ctx, KernelT kern, uint32_t GK, const uint32_t *d_ids, size_t n,
                    uint32_t head, uint32_t Tp, uint32_t base, uint64_t *out, uint64_t *meta, int acc,
                    hipStream_t s, const uint32_t *xin = nullptr, uint32_t *xout = nullptr) {
    const uint32_t nb = grid_for(ctx, kern, (n + 3) / 4, BLOCK, 1);
    if (int rc = ensure_scratch(ctx, (size_t)nb * GK * sizeof(uint64_t), s)) return rc;
    uint64_t *partials = (uint64_t *)ctx->d_scratch;
    if (int rc = scratch_acquire(ctx, s)) return rc;
    hipEvent_t e0 = prof_begin(ctx, s);
    if constexpr (KIND == 1)
        hipLaunchKernelGGL(kern, dim3(nb), dim3(BLOCK), 0, s, d_ids, (uint64_t)n, head, Tp, base, partials, xin,
                           xout);
    else if constexpr (KIND == 2)
        hipLaunchKernelGGL(kern, dim3(nb), dim3(BLOCK), 0, s, d_ids, (uint64_t)n, head, Tp, partials, xin, xout);
    else
        hipLaunchKernelGGL(kern, dim3(nb), dim3(BLOCK), 0, s, d_ids, (uint64_t)n, head, Tp, partials);
    prof_end(ctx, s, e0);
    QK_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_finalize_u32_pass, dim3(Tp), dim3(BLOCK), 0, s, partials, nb, Tp, d_ids, (uint64_t)n, out,
                       meta, acc);
    QK_HIP_TRY(hipGetLastError());
    return scratch_release(ctx, s);
}


static int enc32_passes_chunk(qk_ctx *ctx, const uint32_t *ids, size_t n, uint32_t head, uint32_t T, uint64_t *out,
                              int acc, hipStream_t s) {
    // pass 0: powers 1..80 with the single-pass (8,10) kernel; then passes of
    // <= 48 powers with the offset (8,6) kernel (142 VGPRs, 3 waves/SIMD;
    // every row of an offset pass is a MAC row: the 80-power form spills, a
    // 64-power (8,8) form at 2 waves/SIMD measured the same as 48)
    //
    // Each pass hands x^(next base) to the next one through a per-id cache
    // (4 B per id read + 4 B written per pass) instead of every offset pass
    // raising x^8 to base/8 (~4-8 of its ~16-22 modmuls per id): pass 0
    // writes x^80, the middle passes read and write, the last one reads.  The
    // cache lives in the scratch after the partials, sized once for every
    // pass (a regrow between passes would drop it), with the ids' address
    // modulo 16 so that both are read in the same 16-byte groups.
    const uint32_t npass = T <= 80 ? 0 : (T - 80 + 47) / 48;   // offset passes
    uint32_t *xc = nullptr;
    if (npass >= 1) {
        const uint32_t nbmax = grid_cap(ctx, (n + 3) / 4, BLOCK, 1);   // run_pass: one round
        const size_t poff = ((size_t)nbmax * 80 * sizeof(uint64_t) + 255) & ~(size_t)255;
        if (ensure_scratch(ctx, poff + 16 + (size_t)n * 4, s) == QK_OK)
            xc = (uint32_t *)((char *)ctx->d_scratch + poff + ((uintptr_t)ids & 15));
        // else: no room for the cache, each pass raises x^8 itself
    }
    uint32_t pass = 0;
    for (uint32_t base = 0; base < T; ++pass) {
        const uint32_t Tp = std::min<uint32_t>(base == 0 ? 80 : 48, T - base);
        uint64_t *meta = base == 0 ? out + T : nullptr;
        // XC: pass 0 writes the cache, the middle passes read and write it, the last reads it
        const int xcm = !xc ? 0 : (pass > 0 ? 1 : 0) | (pass < npass ? 2 : 0);
        int rc;
        if (base == 0 && xc)
            rc = run_pass<2>(ctx, k_encode_u32_bsgs_x80<16, 1>, 80, ids, n, head, Tp, 0, out, meta, acc, s, nullptr,
                             xc);
        else if (base == 0)
            rc = run_pass<0>(ctx, k_encode_u32_bsgs<8, 10, 16, 1>, 80, ids, n, head, Tp, 0, out, meta, acc, s);
        else if (Tp <= 40) {   // the last pass (npass >= 1): NA = ceil(Tp / 8) giant rows
#define QK_OFF32(NA_, XC_) k_encode_u32_bsgs_off<NA_, 2 * NA_, XC_, 1>
#define QK_LAST32(NA_)                                                                                       \
    (xcm & 1 ? run_pass<1>(ctx, QK_OFF32(NA_, 1), 8 * NA_, ids, n, head, Tp, base,                            \
                              out + base, meta, acc, s, xc, nullptr)                                          \
             : run_pass<1>(ctx, QK_OFF32(NA_, 0), 8 * NA_, ids, n, head, Tp, base,                            \
                              out + base, meta, acc, s))
            switch ((Tp + 7) / 8) {
            case 1: rc = QK_LAST32(1); break;   // <= 8 powers: one giant row (x^base)
            case 2: rc = QK_LAST32(2); break;
            case 3: rc = QK_LAST32(3); break;
            case 4: rc = QK_LAST32(4); break;
            default: rc = QK_LAST32(5); break;
            }
#undef QK_LAST32
        } else {
            switch (xcm) {
            case 1: rc = run_pass<1>(ctx, QK_OFF32(6, 1), 48, ids, n, head, Tp, base, out + base,
                                        meta, acc, s, xc, nullptr); break;
            case 2: rc = run_pass<1>(ctx, QK_OFF32(6, 2), 48, ids, n, head, Tp, base, out + base,
                                        meta, acc, s, nullptr, xc); break;
            case 3: rc = run_pass<1>(ctx, QK_OFF32(6, 3), 48, ids, n, head, Tp, base, out + base,
                                        meta, acc, s, xc, xc); break;
            default: rc = run_pass<1>(ctx, QK_OFF32(6, 0), 48, ids, n, head, Tp, base, out + base,
                                         meta, acc, s); break;
            }
#undef QK_OFF32
        }
        if (rc) return rc;
        base += Tp;
    }
    return QK_OK;
}

// The x^base cache holds 4 B per id for the whole array: above XC_CHUNK32 ids
// the passes run chunk by chunk (each chunk all its passes, the later chunks
// accumulating into out), so the scratch stays <= 1 GiB.
constexpr size_t XC_CHUNK32 = (size_t)1 << 28;
static int enc32_passes(qk_ctx *ctx, const uint32_t *ids, size_t n, uint32_t head, uint32_t T, uint64_t *out,
                        int acc, hipStream_t s) {
    if (n <= XC_CHUNK32) return enc32_passes_chunk(ctx, ids, n, head, T, out, acc, s);
    for (size_t c0 = 0; c0 < n; c0 += XC_CHUNK32) {
        const uint32_t *p = ids + c0;
        const uint32_t hd = (uint32_t)(((16 - ((uintptr_t)p & 15)) & 15) / 4);
        if (int rc = enc32_passes_chunk(ctx, p, std::min(XC_CHUNK32, n - c0), hd, T, out, c0 ? 1 : acc, s)) return rc;
    }
    return QK_OK;
}

// u64 thresholds > 80: pass 0 is the single-pass (8 babies, 10 giants)
// kernel for powers 1..80, then offset passes of <= 80 powers (giants
// x^(base + 8a), every row a MAC row; NA = ceil(Tp / 8)).  Each pass reads the
// 8-byte ids once more: at ~25 ms of integer issue per pass over 1e9 ids, the
// extra 1 ms of HBM reads is noise.
template <int NA, int XC = 0>
static int run_pass64(qk_ctx *ctx, const uint64_t *ids, size_t n, uint32_t head, uint32_t Tp, uint32_t base,
                      uint64_t *out, uint64_t *meta, int acc, hipStream_t s, uint64_t *xc = nullptr) {
    auto kern = k_encode_u64_bsgs_off<NA, XC, 1>;
    const uint32_t nb = grid_for(ctx, kern, (n + bsgs64::BLOCK - 1) / bsgs64::BLOCK, 1);
    if (int rc = ensure_scratch(ctx, (size_t)nb * 2 * 8 * NA * sizeof(uint64_t), s)) return rc;
    uint64_t *partials = (uint64_t *)ctx->d_scratch;
    if (int rc = scratch_acquire(ctx, s)) return rc;
    hipEvent_t e0 = prof_begin(ctx, s);
    hipLaunchKernelGGL(kern, dim3(nb), dim3(BLOCK), 0, s, ids, (uint64_t)n, head, Tp, base, partials,
                       (const uint64_t *)xc, xc);
    prof_end(ctx, s, e0);
    QK_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_finalize_u64_pass, dim3(Tp), dim3(BLOCK), 0, s, partials, nb, Tp, ids, (uint64_t)n, out,
                       meta, acc);
    QK_HIP_TRY(hipGetLastError());
    return scratch_release(ctx, s);
}

static int enc64_passes_chunk(qk_ctx *ctx, const uint64_t *ids, size_t n, uint32_t head, uint32_t T, uint64_t *out,
                              int acc, hipStream_t s) {
    uint64_t *meta = out + 2 * T;
    // x^(next base) goes from pass to pass through a per-id cache (8 B read +
    // 8 B written per id and pass; pass 0 writes x^80) instead of each offset
    // pass raising x^8 to base/8 (as enc32_passes).  The cache follows the
    // partials in the scratch, sized once.
    const uint32_t npass = (T - 80 + 79) / 80;
    uint64_t *xc = nullptr;
    if (npass >= 1) {
        const uint64_t tiles = (n + bsgs64::BLOCK - 1) / bsgs64::BLOCK;
        const uint32_t nbmax = grid_cap(ctx, tiles, 1);
        const size_t poff = ((size_t)nbmax * 2 * 80 * sizeof(uint64_t) + 255) & ~(size_t)255;
        if (ensure_scratch(ctx, poff + (size_t)n * 8, s) == QK_OK) xc = (uint64_t *)((char *)ctx->d_scratch + poff);
    }
    {   // pass 0: powers 1..80 (+ x^80 per id for pass 1 when the cache is on)
        auto kern = k_encode_u64_bsgs<10, 14, 1>;
        auto kx80 = k_encode_u64_bsgs_x80<1>;
        const uint32_t nb = grid_for(ctx, kern, (n + bsgs64::BLOCK - 1) / bsgs64::BLOCK, 1);
        if (int rc = ensure_scratch(ctx, (size_t)nb * 2 * 80 * sizeof(uint64_t), s)) return rc;
        uint64_t *partials = (uint64_t *)ctx->d_scratch;
        if (int rc = scratch_acquire(ctx, s)) return rc;
        hipEvent_t e0 = prof_begin(ctx, s);
        if (xc)
            hipLaunchKernelGGL(kx80, dim3(nb), dim3(BLOCK), 0, s, ids, (uint64_t)n, head, 80u, partials, xc);
        else
            hipLaunchKernelGGL(kern, dim3(nb), dim3(BLOCK), 0, s, ids, (uint64_t)n, head, 80u, partials);
        prof_end(ctx, s, e0);
        QK_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(k_finalize_u64_pass, dim3(80), dim3(BLOCK), 0, s, partials, nb, 80u, ids, (uint64_t)n,
                           out, meta, acc);
        QK_HIP_TRY(hipGetLastError());
        if (int rc = scratch_release(ctx, s)) return rc;
    }
    uint32_t pass = 1;
    for (uint32_t base = 80; base < T; ++pass) {
        const uint32_t Tp = std::min<uint32_t>(80, T - base);
        uint64_t *o = out + 2 * base;
        // pass 0 wrote the cache; the middle passes read and write it (all
        // full 80-power passes), the last one reads it
        const int xcm = !xc ? 0 : 1 | (pass < npass ? 2 : 0);
        int rc;
#define QK_PASS64(NA_)                                                                              \
    (xcm & 1 ? run_pass64<NA_, 1>(ctx, ids, n, head, Tp, base, o, nullptr, acc, s, xc)           \
             : run_pass64<NA_, 0>(ctx, ids, n, head, Tp, base, o, nullptr, acc, s))
        if (xcm & 2) {   // a middle pass: Tp = 80
            rc = run_pass64<10, 3>(ctx, ids, n, head, Tp, base, o, nullptr, acc, s, xc);
        } else {
            switch ((Tp + 7) / 8) {   // a last pass of <= 8 powers: one giant row (x^base)
            case 1: rc = QK_PASS64(1); break;
            case 2: rc = QK_PASS64(2); break;
            case 3: rc = QK_PASS64(3); break;
            case 4: rc = QK_PASS64(4); break;
            case 5: rc = QK_PASS64(5); break;
            case 6: rc = QK_PASS64(6); break;
            case 7: rc = QK_PASS64(7); break;
            case 8: rc = QK_PASS64(8); break;
            case 9: rc = QK_PASS64(9); break;
            default: rc = QK_PASS64(10); break;
            }
        }
#undef QK_PASS64
        if (rc) return rc;
        base += Tp;
    }
    return QK_OK;
}

// as enc32_passes: 8 B of cache per id, chunks of XC_CHUNK64 ids (1 GiB)
constexpr size_t XC_CHUNK64 = (size_t)1 << 27;
static int enc64_passes(qk_ctx *ctx, const uint64_t *ids, size_t n, uint32_t head, uint32_t T, uint64_t *out,
                        int acc, hipStream_t s) {
    if (n <= XC_CHUNK64) return enc64_passes_chunk(ctx, ids, n, head, T, out, acc, s);
    for (size_t c0 = 0; c0 < n; c0 += XC_CHUNK64) {
        const uint64_t *p = ids + c0;
        const uint32_t hd = (uint32_t)(((16 - ((uintptr_t)p & 15)) & 15) / 8);
        if (int rc = enc64_passes_chunk(ctx, p, std::min(XC_CHUNK64, n - c0), hd, T, out, c0 ? 1 : acc, s)) return rc;
    }
    return QK_OK;
}

// Choose (G, K): the smallest G whose K = ceil(T/G) fits the register
// budget, then the smallest instantiated K >= ceil(T/G).
static const int K32_G1[] = {1, 2, 4, 8, 12, 16, 20, 24, 28, 32};
static const int K32_GN[] = {20, 24, 28, 32};
static const int K64_G1[] = {1, 2, 4, 8, 12, 16, 20, 24, 32, 40};
static const int K64_GN[] = {12, 16, 20, 24, 32, 40};

template <int G, int K>
static int enc32_gk(qk_ctx *ctx, const uint32_t *ids, size_t n, uint32_t head, uint32_t T, uint64_t *out,
                    int acc, hipStream_t s) {
    if constexpr (G == 1)
        return run_encode<uint32_t>(ctx, k_encode_u32_g1<K>, k_finalize_u32, K, 1, ids, n, head, T,
                                    (n + 3) / 4, BLOCK, out, acc, s);
    else
        return run_encode<uint32_t>(ctx, k_encode_u32_gn<G, K>, k_finalize_u32, G * K, 1, ids, n, head, T,
                                    n, BLOCK / G, out, acc, s);
}

template <int G>
static int enc32_g(qk_ctx *ctx, int K, const uint32_t *ids, size_t n, uint32_t head, uint32_t T, uint64_t *out,
                   int acc, hipStream_t s) {
    if constexpr (G == 1) {
        switch (K) {
        case 1: return enc32_gk<1, 1>(ctx, ids, n, head, T, out, acc, s);
        case 2: return enc32_gk<1, 2>(ctx, ids, n, head, T, out, acc, s);
        case 4: return enc32_gk<1, 4>(ctx, ids, n, head, T, out, acc, s);
        case 8: return enc32_gk<1, 8>(ctx, ids, n, head, T, out, acc, s);
        case 12: return enc32_gk<1, 12>(ctx, ids, n, head, T, out, acc, s);
        case 16: return enc32_gk<1, 16>(ctx, ids, n, head, T, out, acc, s);
        case 20: return enc32_gk<1, 20>(ctx, ids, n, head, T, out, acc, s);
        case 24: return enc32_gk<1, 24>(ctx, ids, n, head, T, out, acc, s);
        case 28: return enc32_gk<1, 28>(ctx, ids, n, head, T, out, acc, s);
        case 32: return enc32_gk<1, 32>(ctx, ids, n, head, T, out, acc, s);
        }
    } else {
        switch (K) {
        case 20: return enc32_gk<G, 20>(ctx, ids, n, head, T, out, acc, s);
        case 24: return enc32_gk<G, 24>(ctx, ids, n, head, T, out, acc, s);
        case 28: return enc32_gk<G, 28>(ctx, ids, n, head, T, out, acc, s);
        case 32: return enc32_gk<G, 32>(ctx, ids, n, head, T, out, acc, s);
        }
    }
    return QK_E_THRESHOLD;
}

template <int G, int K>
static int enc64_gk(qk_ctx *ctx, const uint64_t *ids, size_t n, uint32_t head, uint32_t T, uint64_t *out,
                    int acc, hipStream_t s) {
    if constexpr (G == 1)
        return run_encode<uint64_t>(ctx, k_encode_u64_g1<K>, k_finalize_u64, K, 2, ids, n, head, T,
                                    (n + 1) / 2, BLOCK, out, acc, s);
    else
        return run_encode<uint64_t>(ctx, k_encode_u64_gn<G, K>, k_finalize_u64, G * K, 2, ids, n, head, T,
                                    n, BLOCK / G, out, acc, s);
}

template <int G>
static int enc64_g(qk_ctx *ctx, int K, const uint64_t *ids, size_t n, uint32_t head, uint32_t T, uint64_t *out,
                   int acc, hipStream_t s) {
    if constexpr (G == 1) {
        switch (K) {
        case 1: return enc64_gk<1, 1>(ctx, ids, n, head, T, out, acc, s);
        case 2: return enc64_gk<1, 2>(ctx, ids, n, head, T, out, acc, s);
        case 4: return enc64_gk<1, 4>(ctx, ids, n, head, T, out, acc, s);
        case 8: return enc64_gk<1, 8>(ctx, ids, n, head, T, out, acc, s);
        case 12: return enc64_gk<1, 12>(ctx, ids, n, head, T, out, acc, s);
        case 16: return enc64_gk<1, 16>(ctx, ids, n, head, T, out, acc, s);
        case 20: return enc64_gk<1, 20>(ctx, ids, n, head, T, out, acc, s);
        case 24: return enc64_gk<1, 24>(ctx, ids, n, head, T, out, acc, s);
        case 32: return enc64_gk<1, 32>(ctx, ids, n, head, T, out, acc, s);
        case 40: return enc64_gk<1, 40>(ctx, ids, n, head, T, out, acc, s);
        }
    } else {
        switch (K) {
        case 12: return enc64_gk<G, 12>(ctx, ids, n, head, T, out, acc, s);
        case 16: return enc64_gk<G, 16>(ctx, ids, n, head, T, out, acc, s);
        case 20: return enc64_gk<G, 20>(ctx, ids, n, head, T, out, acc, s);
        case 24: return enc64_gk<G, 24>(ctx, ids, n, head, T, out, acc, s);
        case 32: return enc64_gk<G, 32>(ctx, ids, n, head, T, out, acc, s);
        case 40: return enc64_gk<G, 40>(ctx, ids, n, head, T, out, acc, s);
        }
    }
    return QK_E_THRESHOLD;
}

static void choose_gk(uint32_t T, int kmax, const int *kg1, int nkg1, const int *kgn, int nkgn, int &G, int &K) {
    G = 1;
    while ((T + G - 1) / G > (uint32_t)kmax) G *= 2;
    const uint32_t kneed = (T + G - 1) / G;
    const int *ks = G == 1 ? kg1 : kgn;
    const int nk = G == 1 ? nkg1 : nkgn;
    K = ks[nk - 1];
    for (int i = 0; i < nk; ++i)
        if ((uint32_t)ks[i] >= kneed) { K = ks[i]; break; }
}


static int enc32(qk_ctx *ctx, const uint32_t *ids, size_t n, uint32_t T, uint64_t *out, int acc, hipStream_t s) {
    if (T == 0 || T > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    const uintptr_t a = (uintptr_t)ids;
    if (a & 3) return QK_E_INVAL;
    const uint32_t head = (uint32_t)(((16 - (a & 15)) & 15) / 4);
    if (n >= (1ull << 40)) return QK_E_INVAL; // 4 TB of ids: beyond any HBM; keeps per-lane trip counts 32-bit
    // baby-step / giant-step for 9 <= T <= 32 (fewer modmuls per id); the
    // power chain otherwise
    // Scalar-counted BSGS groups (bsgs.h) keep per-wave 32-bit wrap totals: a
    // wave sees at most 64 * (4 * trips + 2) wraps per accumulator, so trips
    // must stay < 2^24 - 1 — true for any n < 2^40 at >= 1 workgroup per CU;
    // a tiny override grid over a huge n takes the all-VALU form.
    const uint64_t min_grid = ctx->grid_override ? ctx->grid_override : (uint64_t)ctx->num_cus;
    const bool sc_ok = n / (4ull * BLOCK * min_grid) < (1ull << 24) - 2;
#define QK_BSGS(NB_, NA_, G_)                                                                                 \
    run_encode<uint32_t>(ctx, k_encode_u32_bsgs<NB_, NA_, G_, 1>, k_finalize_u32, NB_ * NA_, 1, ids, n, head, T, \
                         (n + 3) / 4, BLOCK, out, acc, s, NB_ * NA_ > 48 ? 1 : 0)
    if (T >= 5 && T <= 8 && sc_ok) return QK_BSGS(4, 2, 1);
    if (T >= 9 && T <= 12) return sc_ok ? QK_BSGS(4, 3, 3) : QK_BSGS(4, 3, 0);
    if (T >= 13 && T <= 16) return sc_ok ? QK_BSGS(4, 4, 4) : QK_BSGS(4, 4, 0);
    // Round-3 shapes: the (NB, NA) with the fewest issue cycles for the
    // powers actually needed — modmuls NB - 1 + NA - 2 at ~17 cycles, MACs
    // NB (NA - 1) and row-0 adds NB at ~4.2, measured: 17..28
    // four babies and ceil(T / 4) giant rows (every group 4 wide,
    // scalar-counted; (6,4) / (8,4) computed 24 / 32 powers), 29..30 (6,5),
    // 33..36 (6,6), 41..42 (6,7), 65..72 (8,9)
    if (sc_ok) {
        if (T >= 17 && T <= 20) return QK_BSGS(4, 5, 5);
        if (T >= 21 && T <= 24) return QK_BSGS(4, 6, 6);
        if (T >= 25 && T <= 28) return QK_BSGS(4, 7, 7);
        if (T >= 29 && T <= 30) return QK_BSGS(6, 5, 5);
        if (T >= 31 && T <= 32) return QK_BSGS(8, 4, QK_BSGS_SG_T32);
        if (T >= 33 && T <= 36) return QK_BSGS(6, 6, 6);
        if (T >= 37 && T <= 40) return QK_BSGS(8, 5, 10);
        if (T >= 41 && T <= 42) return QK_BSGS(6, 7, 7);
        if (T >= 43 && T <= 48) return QK_BSGS(8, 6, 12);
        if (T >= 49 && T <= 56) return QK_BSGS(8, 7, 14);
        if (T >= 57 && T <= 64) return QK_BSGS(8, 8, 16);
        if (T >= 65 && T <= 72) return QK_BSGS(8, 9, 14);
        if (T >= 73 && T <= 80) return QK_BSGS(8, 10, 16);
        if (T > 80) return enc32_passes(ctx, ids, n, head, T, out, acc, s);
    } else {
        // the all-VALU forms that fit the registers; t 33..80 would spill, so
        // a grid too small for scalar counts takes the power chain there
        if (T >= 17 && T <= 24) return QK_BSGS(6, 4, 0);
        if (T >= 25 && T <= 32) return QK_BSGS(8, 4, 0);
    }
#undef QK_BSGS
    int G, K;
    choose_gk(T, 32, K32_G1, 10, K32_GN, 4, G, K);
    switch (G) {
    case 1: return enc32_g<1>(ctx, K, ids, n, head, T, out, acc, s);
    case 2: return enc32_g<2>(ctx, K, ids, n, head, T, out, acc, s);
    case 4: return enc32_g<4>(ctx, K, ids, n, head, T, out, acc, s);
    case 8: return enc32_g<8>(ctx, K, ids, n, head, T, out, acc, s);
    case 16: return enc32_g<16>(ctx, K, ids, n, head, T, out, acc, s);
    case 32: return enc32_g<32>(ctx, K, ids, n, head, T, out, acc, s);
    }
    return QK_E_THRESHOLD;
}

static int enc64(qk_ctx *ctx, const uint64_t *ids, size_t n, uint32_t T, uint64_t *out, int acc, hipStream_t s) {
    if (T == 0 || T > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    const uintptr_t a = (uintptr_t)ids;
    if (a & 7) return QK_E_INVAL;
    const uint32_t head = (uint32_t)(((16 - (a & 15)) & 15) / 8);
    // baby-step / giant-step for 14 <= T <= 80 (configs[2] is T = 80; below
    // 14 powers the 8 modmuls of the babies and x^8 cost more than the chain
    // they save: profiles/r03/shapes/sweep64_tmin_ab.jsonl — 21 before round
    // 3, BSGS +3..9 % at t = 14..20): NA = ceil(T / 8) giant rows; its
    // per-wave 32-bit carry totals need < 2^31 ids per workgroup.  Every form
    // runs with s_setprio around the MACs and paired MACs (F = 1).
    const uint64_t min_grid64 = ctx->grid_override ? ctx->grid_override : (uint64_t)ctx->num_cus;
    const bool bsgs_ok = n / min_grid64 < (1ull << 30);
    if (T >= 14 && T <= 80 && bsgs_ok) {
#define QK_BSGS64(NA_, SG_)                                                                           \
    run_encode<uint64_t>(ctx, k_encode_u64_bsgs<NA_, SG_, 1>, k_finalize_u64, 8 * NA_, 2, ids, n, head, T,   \
                         (n + bsgs64::BLOCK - 1) / bsgs64::BLOCK, 1, out, acc, s)
#define QK_BSGS64_4(NA_)                                                                              \
    run_encode<uint64_t>(ctx, k_encode_u64_bsgs4<NA_, 1>, k_finalize_u64, 4 * NA_, 2, ids, n, head, T,      \
                         (n + bsgs64::BLOCK - 1) / bsgs64::BLOCK, 1, out, acc, s)
        // four babies per id and ceil(T/4) giant rows where 8 babies would
        // compute 4+ powers more: t = 14..20, 25..28, 33..36 (+8..17 %,
        // profiles/r03/shapes/sweep64_four_babies_ab.jsonl; at t = 21..24,
        // 29..32 even, at 37..40 7 % slower: not used)
        if (T <= 36) switch ((T + 3) / 4) {
            case 4: return QK_BSGS64_4(4);
            case 5: return QK_BSGS64_4(5);
            case 7: return QK_BSGS64_4(7);
            case 9: return QK_BSGS64_4(9);
            default: break;
            }
#undef QK_BSGS64_4
        switch ((T + 7) / 8) {   // NA <= 9: a wave's <= 16 MACs all scalar-counted
        case 2: return QK_BSGS64(2, 16);
        case 3: return QK_BSGS64(3, 16);
        case 4: return QK_BSGS64(4, 16);
        case 5: return QK_BSGS64(5, 16);
        case 6: return QK_BSGS64(6, 16);
        case 7: return QK_BSGS64(7, 16);
        case 8: return QK_BSGS64(8, 16);
        case 9: return QK_BSGS64(9, 16);
        // NA = 10: 14 of the 18 MACs scalar-counted with the paired-MAC form
        // (22.65 vs 23.19 ms at 16, twice, profiles/r04/prio/tune_u64_prio.json)
        default: return QK_BSGS64(10, 14);
        }
#undef QK_BSGS64
    }
    if (T > 80 && bsgs_ok) return enc64_passes(ctx, ids, n, head, T, out, acc, s);
    int G, K;
    // K <= 40 accumulators per lane (120 VGPRs, 3 waves/SIMD) beat K <= 20 at
    // 5 waves by needing fewer lanes per id (t = 80: 2 x (39 + 1) steps vs
    // 4 x (19 + 3)).
    choose_gk(T, 40, K64_G1, 10, K64_GN, 6, G, K);
    switch (G) {
    case 1: return enc64_g<1>(ctx, K, ids, n, head, T, out, acc, s);
    case 2: return enc64_g<2>(ctx, K, ids, n, head, T, out, acc, s);
    case 4: return enc64_g<4>(ctx, K, ids, n, head, T, out, acc, s);
    case 8: return enc64_g<8>(ctx, K, ids, n, head, T, out, acc, s);
    case 16: return enc64_g<16>(ctx, K, ids, n, head, T, out, acc, s);
    case 32: return enc64_g<32>(ctx, K, ids, n, head, T, out, acc, s);
    case 64: return enc64_g<64>(ctx, K, ids, n, head, T, out, acc, s);
    }
    return QK_E_THRESHOLD;
}

int launch_encode_u32(qk_ctx *ctx, const uint32_t *d_ids, size_t n, uint32_t t, uint64_t *d_partial, hipStream_t s) {
    return enc32(ctx, d_ids, n, t, d_partial, 0, s);
}
int launch_encode_u64(qk_ctx *ctx, const uint64_t *d_ids, size_t n, uint32_t t, uint64_t *d_partial, hipStream_t s) {
    return enc64(ctx, d_ids, n, t, d_partial, 0, s);
}
int launch_encode_u32_acc(qk_ctx *ctx, const uint32_t *d_ids, size_t n, uint32_t t, uint64_t *d_partial,
                          hipStream_t s) {
    return enc32(ctx, d_ids, n, t, d_partial, 1, s);
}
int launch_encode_u64_acc(qk_ctx *ctx, const uint64_t *d_ids, size_t n, uint32_t t, uint64_t *d_partial,
                          hipStream_t s) {
    return enc64(ctx, d_ids, n, t, d_partial, 1, s);
}

} // namespace qk
