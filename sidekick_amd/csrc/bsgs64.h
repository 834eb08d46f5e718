// bsgs64.h — baby-step / giant-step u64 encode over p64 = 2^64 - 59 for
// 41 <= t <= 80 (configs[2] is t = 80).
//
// Power 8a + b (a = 0..NA-1, b = 1..8) is S = sum_i A_a(x_i) * B_b(x_i) with
// babies B_b = x^b and giants A_a = x^(8a) (A_0 = 1): 7 + (NA - 2) modmuls
// per id instead of t - 1, and (NA - 1) * 8 multiply-accumulates.  A 64x64
// MAC is four 32x32 v_mad_u64_u32 into two 64-bit column accumulators: with
// A = a0 + a1 2^32 and the per-baby precomputed Bsh = B * 2^32 mod p,
//     A * B == B * a0 + Bsh * a1 (mod p)
//     C0 += B.lo a0 + Bsh.lo a1      (weight 1)
//     C1 += B.hi a0 + Bsh.hi a1      (weight 2^32)
// and each mad's carry-out (a wrap of 2^64, i.e. 2^64 == 59 for C0 and 2^96
// == 59 * 2^32 for C1) is counted: per wave on the scalar unit (only the sum
// over lanes of a power matters) for the first SG MACs of a wave's tile,
// per lane with v_addc for the rest.
//
// One MAC per power needs all lanes of a wave on the same power, and a wave
// can hold about 20 powers' accumulators (5 VGPRs + 2 SGPR counters each),
// so the powers are split over the 4 waves of a workgroup and the babies and
// giants of an id are computed ONCE and shared through LDS:
//   step 1  each thread takes one id of the 256-id tile: 7 baby and NA - 2
//           giant modmuls (exact, hand-scheduled p64 step), and writes B per
//           baby and A per giant (x^8 = baby 8 is not stored twice) to LDS
//   step 3  wave w takes babies 2w+1, 2w+2: computes their Bsh, runs their
//           a = 0 row (S_b += B_b) and their MACs with every giant, over all
//           256 ids of the tile (4 per lane), reading the operands from LDS
// LDS: 256 ids x (8 + 8) x 8 B = 32 KB per workgroup at t = 80, 4 workgroups
// per CU (the product form, BSH; storing Bsh too takes 50 KB, 3 per CU, and
// measured 6 % slower).  Integer-VALU (+SALU) bound; the ids are read once.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bsgs.h"
#include "field.h"

namespace qk {
namespace bsgs64 {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;
constexpr int NB = 8;

// V <- V * x mod p, V and the result < 2^64 (not necessarily canonical),
// exact.  V pinned in v[2:3] (the asm addresses its halves):
//   A = V.lo x0;  B = V.hi x0 + A.hi;  C = V.lo x1 + B (carry cc);
//   ((A.hi:0) as one v_pk_mov_b32 instead of two moves: 1 % slower at t = 80,
//   profiles/r05/u64_step1/)
//   PH = V.hi x1 + C.hi + cc 2^32;  P_L = A.lo + C.lo 2^32          (P = V x)
//   E = P_L + 59 PH.lo (carry ce);  F = E.hi + ce 2^32 + 59 PH.hi   (t-form)
//   V' = (F.lo:E.lo) + 59 F.hi; a wrap past 2^64 leaves V' < 59*60, so +59
// Every VALU-written carry is read >= 2 wait states after its write.
#define QK_U64_MULV_ASM                                                                            \
    "v_mov_b32_e32 v11, 0\n\t"                                                                     \
    "v_mad_u64_u32 v[6:7], %[cx], v2, %[x0], 0\n\t"                                                  \
    "v_mov_b32_e32 v10, v7\n\t"                                                                    \
    "v_mad_u64_u32 v[8:9], %[cx], v3, %[x0], v[10:11]\n\t"                                           \
    "v_mad_u64_u32 v[8:9], %[cc], v2, %[x1], v[8:9]\n\t"                                             \
    "v_mov_b32_e32 v7, v8\n\t"                                                                     \
    "v_mov_b32_e32 v10, v9\n\t"                                                                    \
    "v_cndmask_b32_e64 v11, 0, 1, %[cc]\n\t"                                                         \
    "v_mad_u64_u32 v[4:5], %[cx], v3, %[x1], v[10:11]\n\t"                                           \
    "v_mad_u64_u32 v[2:3], %[ce], v4, 59, v[6:7]\n\t"                                                \
    "v_mov_b32_e32 v8, v3\n\t"                                                                     \
    "s_nop 0\n\t"                                                                                  \
    "v_cndmask_b32_e64 v9, 0, 1, %[ce]\n\t"                                                          \
    "v_mad_u64_u32 v[8:9], %[cx], v5, 59, v[8:9]\n\t"                                                \
    "v_mov_b32_e32 v3, v8\n\t"                                                                     \
    "v_mad_u64_u32 v[2:3], %[cw], v9, 59, v[2:3]\n\t"                                                \
    "s_nop 1\n\t"                                                                                  \
    "v_cndmask_b32_e64 %[tmp], 0, 59, %[cw]\n\t"                                                     \
    "v_add_u32_e32 v2, v2, %[tmp]\n\t"

__device__ __forceinline__ void mulv(uint64_t &V, uint32_t x0, uint32_t x1) {
    uint64_t cw, cx, cc, ce;
    uint32_t tmp;
    asm volatile(QK_U64_MULV_ASM
                 : "+{v[2:3]}"(V), [cw] "=&s"(cw), [cx] "=&s"(cx), [cc] "=&s"(cc), [ce] "=&s"(ce),
                   [tmp] "=&v"(tmp)
                 : [x0] "v"(x0), [x1] "v"(x1)
                 : "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11");
}

// Two independent products V <- V * x, W <- W * y in one block, the two
// instruction streams interleaved (W in v[12:13], its scratch v14..v21): each
// stream's carries get their wait states from the other stream's
// instructions, and the two dependency chains overlap in one wave.
#define QK_U64_MULV2_ASM                                                                           \
    "v_mov_b32_e32 v11, 0\n\t"                                                                     \
    "v_mov_b32_e32 v21, 0\n\t"                                                                     \
    "v_mad_u64_u32 v[6:7], %[cx], v2, %[x0], 0\n\t"                                                  \
    "v_mad_u64_u32 v[16:17], %[dx], v12, %[y0], 0\n\t"                                               \
    "v_mov_b32_e32 v10, v7\n\t"                                                                    \
    "v_mov_b32_e32 v20, v17\n\t"                                                                   \
    "v_mad_u64_u32 v[8:9], %[cx], v3, %[x0], v[10:11]\n\t"                                           \
    "v_mad_u64_u32 v[18:19], %[dx], v13, %[y0], v[20:21]\n\t"                                        \
    "v_mad_u64_u32 v[8:9], %[cc], v2, %[x1], v[8:9]\n\t"                                             \
    "v_mad_u64_u32 v[18:19], %[dc], v12, %[y1], v[18:19]\n\t"                                        \
    "v_mov_b32_e32 v7, v8\n\t"                                                                     \
    "v_mov_b32_e32 v17, v18\n\t"                                                                   \
    "v_mov_b32_e32 v10, v9\n\t"                                                                    \
    "v_mov_b32_e32 v20, v19\n\t"                                                                   \
    "v_cndmask_b32_e64 v11, 0, 1, %[cc]\n\t"                                                         \
    "v_cndmask_b32_e64 v21, 0, 1, %[dc]\n\t"                                                         \
    "v_mad_u64_u32 v[4:5], %[cx], v3, %[x1], v[10:11]\n\t"                                           \
    "v_mad_u64_u32 v[14:15], %[dx], v13, %[y1], v[20:21]\n\t"                                        \
    "v_mad_u64_u32 v[2:3], %[ce], v4, 59, v[6:7]\n\t"                                                \
    "v_mad_u64_u32 v[12:13], %[de], v14, 59, v[16:17]\n\t"                                           \
    "v_mov_b32_e32 v8, v3\n\t"                                                                     \
    "v_mov_b32_e32 v18, v13\n\t"                                                                   \
    "v_cndmask_b32_e64 v9, 0, 1, %[ce]\n\t"                                                          \
    "v_cndmask_b32_e64 v19, 0, 1, %[de]\n\t"                                                         \
    "v_mad_u64_u32 v[8:9], %[cx], v5, 59, v[8:9]\n\t"                                                \
    "v_mad_u64_u32 v[18:19], %[dx], v15, 59, v[18:19]\n\t"                                           \
    "v_mov_b32_e32 v3, v8\n\t"                                                                     \
    "v_mov_b32_e32 v13, v18\n\t"                                                                   \
    "v_mad_u64_u32 v[2:3], %[cw], v9, 59, v[2:3]\n\t"                                                \
    "v_mad_u64_u32 v[12:13], %[dw], v19, 59, v[12:13]\n\t"                                           \
    "s_nop 0\n\t"                                                                                  \
    "v_cndmask_b32_e64 %[tmp], 0, 59, %[cw]\n\t"                                                     \
    "v_cndmask_b32_e64 %[tmq], 0, 59, %[dw]\n\t"                                                     \
    "v_add_u32_e32 v2, v2, %[tmp]\n\t"                                                             \
    "v_add_u32_e32 v12, v12, %[tmq]\n\t"

__device__ __forceinline__ void mulv2(uint64_t &V, uint32_t x0, uint32_t x1, uint64_t &W, uint32_t y0, uint32_t y1) {
    uint64_t cw, cx, cc, ce, dw, dx, dc, de;
    uint32_t tmp, tmq;
    asm volatile(QK_U64_MULV2_ASM
                 : "+{v[2:3]}"(V), "+{v[12:13]}"(W), [cw] "=&s"(cw), [cx] "=&s"(cx), [cc] "=&s"(cc),
                   [ce] "=&s"(ce), [dw] "=&s"(dw), [dx] "=&s"(dx), [dc] "=&s"(dc), [de] "=&s"(de),
                   [tmp] "=&v"(tmp), [tmq] "=&v"(tmq)
                 : [x0] "v"(x0), [x1] "v"(x1), [y0] "v"(y0), [y1] "v"(y1)
                 : "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v14", "v15", "v16", "v17", "v18", "v19",
                   "v20", "v21");
}

// P[1..M] = u^1 .. u^M from P[1] = u in 1 + ceil((M - 2) / 2) dependent
// steps instead of M - 1: P[2] = P[1]^2, then (P[2j-1], P[2j]) =
// (P[j] P[j-1], P[j]^2) as one mulv2 block.  store(k, P[k]) after each.
template <int M, typename St>
__device__ __forceinline__ void pow_tree(uint64_t (&P)[M + 1], St &&store) {
    if constexpr (M >= 2) {
        P[2] = P[1];
        mulv(P[2], (uint32_t)P[1], (uint32_t)(P[1] >> 32));
        store(2, P[2]);
    }
#pragma unroll
    for (int j = 2; 2 * j - 1 <= M; ++j) {
        const uint64_t pj = P[j], pm = P[j - 1];
        if (2 * j <= M) {
            uint64_t a = pj, b = pj;
            mulv2(a, (uint32_t)pm, (uint32_t)(pm >> 32), b, (uint32_t)pj, (uint32_t)(pj >> 32));
            P[2 * j - 1] = a;
            P[2 * j] = b;
            store(2 * j - 1, a);
            store(2 * j, b);
        } else {
            uint64_t a = pj;
            mulv(a, (uint32_t)pm, (uint32_t)(pm >> 32));
            P[2 * j - 1] = a;
            store(2 * j - 1, a);
        }
    }
}

// B * 2^32 mod p for B < 2^64: B.lo 2^32 + 59 B.hi (+59 after a wrap, which
// leaves < 59 2^32: the second mad cannot wrap)
__device__ __forceinline__ uint64_t shift32(uint64_t B) {
    uint64_t r, cw, cx;
    uint32_t f;
    asm volatile("v_mad_u64_u32 %[r], %[cw], %[bh], 59, %[sh]\n\t"
                 "s_nop 1\n\t"
                 "v_cndmask_b32_e64 %[f], 0, 1, %[cw]\n\t"
                 "v_mad_u64_u32 %[r], %[cx], %[f], 59, %[r]"
                 : [r] "=&v"(r), [cw] "=&s"(cw), [cx] "=&s"(cx), [f] "=&v"(f)
                 : [bh] "v"((uint32_t)(B >> 32)), [sh] "v"(B << 32));
    return r;
}

// ---- MAC of one power, carries counted ------------------------------------
// operands: %0 C0, %1 C1 (64-bit), %2 k0, %3 k1 (counters), %4 a0, %5 a1,
// %6 B.lo, %7 B.hi, %8 Bsh.lo, %9 Bsh.hi
#define QK_MAC64S(P0, P1, P2, P3, T)                                                                    \
    "v_mad_u64_u32 %0, " P0 ", %6, %4, %0\n\t"                                                        \
    "v_mad_u64_u32 %1, " P1 ", %7, %4, %1\n\t"                                                        \
    "v_mad_u64_u32 %0, " P2 ", %8, %5, %0\n\t"                                                        \
    "v_mad_u64_u32 %1, " P3 ", %9, %5, %1\n\t"                                                        \
    "s_bcnt1_i32_b64 " T ", " P0 "\n\ts_add_u32 %2, %2, " T "\n\t"                                          \
    "s_bcnt1_i32_b64 " T ", " P1 "\n\ts_add_u32 %3, %3, " T "\n\t"                                          \
    "s_bcnt1_i32_b64 " T ", " P2 "\n\ts_add_u32 %2, %2, " T "\n\t"                                          \
    "s_bcnt1_i32_b64 " T ", " P3 "\n\ts_add_u32 %3, %3, " T
#define QK_MAC64V(P0, P1, P2, P3)                                                                       \
    "v_mad_u64_u32 %0, " P0 ", %6, %4, %0\n\t"                                                        \
    "v_mad_u64_u32 %1, " P1 ", %7, %4, %1\n\t"                                                        \
    "v_mad_u64_u32 %0, " P2 ", %8, %5, %0\n\t"                                                        \
    "v_mad_u64_u32 %1, " P3 ", %9, %5, %1\n\t"                                                        \
    "v_addc_co_u32_e64 %2, " P0 ", %2, 0, " P0 "\n\t"                                                 \
    "v_addc_co_u32_e64 %3, " P1 ", %3, 0, " P1 "\n\t"                                                 \
    "v_addc_co_u32_e64 %2, " P2 ", %2, 0, " P2 "\n\t"                                                 \
    "v_addc_co_u32_e64 %3, " P3 ", %3, 0, " P3

// mixed: P0..P2 on the scalar unit, P3 (a C1 carry) per lane into kv —
// the scalar unit issues one instruction per SIMD every 4 cycles, so a MAC
// with all four carries scalar (8 SALU) outlasts its 4 mads.  The per-lane
// v_addc reads P3 after six scalar instructions (>= 2 wait states).
#define QK_MAC64M(P0, P1, P2, P3, T)                                                                    \
    "v_mad_u64_u32 %[C0], " P0 ", %[bl], %[a0], %[C0]\n\t"                                             \
    "v_mad_u64_u32 %[C1], " P1 ", %[bh], %[a0], %[C1]\n\t"                                             \
    "v_mad_u64_u32 %[C0], " P2 ", %[sl], %[a1], %[C0]\n\t"                                             \
    "v_mad_u64_u32 %[C1], " P3 ", %[sh], %[a1], %[C1]\n\t"                                             \
    "s_bcnt1_i32_b64 " T ", " P0 "\n\ts_add_u32 %[k0], %[k0], " T "\n\t"                                \
    "s_bcnt1_i32_b64 " T ", " P1 "\n\ts_add_u32 %[k1], %[k1], " T "\n\t"                                \
    "s_bcnt1_i32_b64 " T ", " P2 "\n\ts_add_u32 %[k0], %[k0], " T "\n\t"                                \
    "v_addc_co_u32_e64 %[kv], " P3 ", %[kv], 0, " P3

// Both MACs of a wave's giant row (its two babies) in one block, the eight
// mads ordered so that a mad reading an accumulator follows the one writing
// it by four instructions (in a single MAC the second product into C0 / C1
// follows the first by two), all eight carries counted on the scalar unit.
// Operands: %0 C0[0], %1 C0[1], %2 C1[0], %3 C1[1], %4-%7 counters
// (k0[0], k0[1], k1[0], k1[1]), %8-%11 baby 0 (B.lo, B.hi, Bsh.lo, Bsh.hi),
// %12-%15 baby 1, %16 a0, %17 a1
#define QK_MAC64P(Q0, Q1, Q2, Q3, Q4, Q5, Q6, Q7, T)                                                   \
    "v_mad_u64_u32 %0, " Q0 ", %8, %16, %0\n\t"                                                        \
    "v_mad_u64_u32 %1, " Q1 ", %12, %16, %1\n\t"                                                       \
    "v_mad_u64_u32 %2, " Q2 ", %9, %16, %2\n\t"                                                        \
    "v_mad_u64_u32 %3, " Q3 ", %13, %16, %3\n\t"                                                       \
    "v_mad_u64_u32 %0, " Q4 ", %10, %17, %0\n\t"                                                       \
    "v_mad_u64_u32 %1, " Q5 ", %14, %17, %1\n\t"                                                       \
    "v_mad_u64_u32 %2, " Q6 ", %11, %17, %2\n\t"                                                       \
    "v_mad_u64_u32 %3, " Q7 ", %15, %17, %3\n\t"                                                       \
    "s_bcnt1_i32_b64 " T ", " Q0 "\n\ts_add_u32 %4, %4, " T "\n\t"                                       \
    "s_bcnt1_i32_b64 " T ", " Q1 "\n\ts_add_u32 %5, %5, " T "\n\t"                                       \
    "s_bcnt1_i32_b64 " T ", " Q2 "\n\ts_add_u32 %6, %6, " T "\n\t"                                       \
    "s_bcnt1_i32_b64 " T ", " Q3 "\n\ts_add_u32 %7, %7, " T "\n\t"                                       \
    "s_bcnt1_i32_b64 " T ", " Q4 "\n\ts_add_u32 %4, %4, " T "\n\t"                                       \
    "s_bcnt1_i32_b64 " T ", " Q5 "\n\ts_add_u32 %5, %5, " T "\n\t"                                       \
    "s_bcnt1_i32_b64 " T ", " Q6 "\n\ts_add_u32 %6, %6, " T "\n\t"                                       \
    "s_bcnt1_i32_b64 " T ", " Q7 "\n\ts_add_u32 %7, %7, " T
#define QK_SETP0 "s[40:41]", "s[42:43]", "s[44:45]", "s[46:47]", "s[48:49]", "s[50:51]", "s[52:53]", "s[54:55]", "s72"
#define QK_SETP1 "s[56:57]", "s[58:59]", "s[60:61]", "s[62:63]", "s[64:65]", "s[66:67]", "s[68:69]", "s[70:71]", "s73"
#define QK_CLOBP0 "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", \
                  "s54", "s55", "s72"
#define QK_CLOBP1 "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", \
                  "s70", "s71", "s73"
template <int SET>
__device__ __forceinline__ void mac_pair_s(uint64_t (&C0)[2], uint64_t (&C1)[2], uint32_t (&K0)[2], uint32_t (&K1)[2],
                                           uint32_t a0, uint32_t a1, uint4 b0, uint4 b1) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_MAC64P, QK_SETP0)
                     : "+v"(C0[0]), "+v"(C0[1]), "+v"(C1[0]), "+v"(C1[1]), "+s"(K0[0]), "+s"(K0[1]), "+s"(K1[0]),
                       "+s"(K1[1])
                     : "v"(b0.x), "v"(b0.y), "v"(b0.z), "v"(b0.w), "v"(b1.x), "v"(b1.y), "v"(b1.z), "v"(b1.w),
                       "v"(a0), "v"(a1)
                     : "scc", QK_CLOBP0);
    else
        asm volatile(QK_EXPAND(QK_MAC64P, QK_SETP1)
                     : "+v"(C0[0]), "+v"(C0[1]), "+v"(C1[0]), "+v"(C1[1]), "+s"(K0[0]), "+s"(K0[1]), "+s"(K1[0]),
                       "+s"(K1[1])
                     : "v"(b0.x), "v"(b0.y), "v"(b0.z), "v"(b0.w), "v"(b1.x), "v"(b1.y), "v"(b1.z), "v"(b1.w),
                       "v"(a0), "v"(a1)
                     : "scc", QK_CLOBP1);
}

template <int SET>
__device__ __forceinline__ void mac_m(uint64_t &C0, uint64_t &C1, uint32_t &k0, uint32_t &k1, uint32_t &kv,
                                      uint32_t a0, uint32_t a1, uint4 b) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_MAC64M, QK_SET0T)
                     : [C0] "+v"(C0), [C1] "+v"(C1), [k0] "+s"(k0), [k1] "+s"(k1), [kv] "+v"(kv)
                     : [a0] "v"(a0), [a1] "v"(a1), [bl] "v"(b.x), [bh] "v"(b.y), [sl] "v"(b.z), [sh] "v"(b.w)
                     : "scc", "s56", QK_CLOB0);
    else
        asm volatile(QK_EXPAND(QK_MAC64M, QK_SET1T)
                     : [C0] "+v"(C0), [C1] "+v"(C1), [k0] "+s"(k0), [k1] "+s"(k1), [kv] "+v"(kv)
                     : [a0] "v"(a0), [a1] "v"(a1), [bl] "v"(b.x), [bh] "v"(b.y), [sl] "v"(b.z), [sh] "v"(b.w)
                     : "scc", "s57", QK_CLOB1);
}

template <int SET>
__device__ __forceinline__ void mac_s(uint64_t &C0, uint64_t &C1, uint32_t &k0, uint32_t &k1, uint32_t a0,
                                      uint32_t a1, uint4 b) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_MAC64S, QK_SET0T)
                     : "+v"(C0), "+v"(C1), "+s"(k0), "+s"(k1)
                     : "v"(a0), "v"(a1), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w)
                     : "scc", "s56", QK_CLOB0);
    else
        asm volatile(QK_EXPAND(QK_MAC64S, QK_SET1T)
                     : "+v"(C0), "+v"(C1), "+s"(k0), "+s"(k1)
                     : "v"(a0), "v"(a1), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w)
                     : "scc", "s57", QK_CLOB1);
}
template <int SET>
__device__ __forceinline__ void mac_v(uint64_t &C0, uint64_t &C1, uint32_t &k0, uint32_t &k1, uint32_t a0,
                                      uint32_t a1, uint4 b) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_MAC64V, QK_SET0)
                     : "+v"(C0), "+v"(C1), "+v"(k0), "+v"(k1)
                     : "v"(a0), "v"(a1), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w)
                     : QK_CLOB0);
    else
        asm volatile(QK_EXPAND(QK_MAC64V, QK_SET1)
                     : "+v"(C0), "+v"(C1), "+v"(k0), "+v"(k1)
                     : "v"(a0), "v"(a1), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w)
                     : QK_CLOB1);
}

// ---- the a = 0 row: S_b += B_b as two 64-bit sums of 32-bit halves --------
// lo_j += B_j.lo and hi_j += B_j.hi (weight 2^32) with v_mad_u64_u32 (x 1):
// < 2^32 adds of 32-bit values cannot wrap a 64-bit sum, so no carry is
// counted; the mads' carry-outs go to a dead SGPR set.
#define QK_ROW64M(P0, P1, P2, P3)                                                                       \
    "v_mad_u64_u32 %0, " P0 ", %4, 1, %0\n\t"                                                          \
    "v_mad_u64_u32 %1, " P1 ", %5, 1, %1\n\t"                                                          \
    "v_mad_u64_u32 %2, " P2 ", %6, 1, %2\n\t"                                                          \
    "v_mad_u64_u32 %3, " P3 ", %7, 1, %3"
template <int SET>
__device__ __forceinline__ void row2(uint64_t (&lo)[2], uint64_t (&hi)[2], const uint4 (&b)[2]) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_ROW64M, QK_SET0)
                     : "+v"(lo[0]), "+v"(lo[1]), "+v"(hi[0]), "+v"(hi[1])
                     : "v"(b[0].x), "v"(b[1].x), "v"(b[0].y), "v"(b[1].y)
                     : QK_CLOB0);
    else
        asm volatile(QK_EXPAND(QK_ROW64M, QK_SET1)
                     : "+v"(lo[0]), "+v"(lo[1]), "+v"(hi[0]), "+v"(hi[1])
                     : "v"(b[0].x), "v"(b[1].x), "v"(b[0].y), "v"(b[1].y)
                     : QK_CLOB1);
}

// one baby's a = 0 row (a wave owning one baby, NBT = 4)
__device__ __forceinline__ void row1(uint64_t &lo, uint64_t &hi, uint4 b) {
    uint64_t c0, c1;
    asm volatile("v_mad_u64_u32 %0, %2, %4, 1, %0\n\t"
                 "v_mad_u64_u32 %1, %3, %5, 1, %1"
                 : "+v"(lo), "+v"(hi), "=&s"(c0), "=&s"(c1)
                 : "v"(b.x), "v"(b.y));
}

// (u128 value) mod p, canonical
__device__ __forceinline__ uint64_t mod_p128(unsigned __int128 v) {
    // v = H 2^64 + L == 59 H + L; twice brings it below 2^64 + 59^2
    unsigned __int128 t = (unsigned __int128)(uint64_t)(v >> 64) * C64 + (uint64_t)v;
    t = (unsigned __int128)(uint64_t)(t >> 64) * C64 + (uint64_t)t;
    uint64_t r = (uint64_t)t + C64 * (uint64_t)(t >> 64);
    r = canon64(r);
    return r >= P64 ? r - P64 : r;
}

// The workgroup's operands of one tile in LDS, [value][id] so that lanes read
// consecutive ids: babies (B.lo, B.hi, Bsh.lo, Bsh.hi) and giants (a0, a1).
// BSH: the babies' B * 2^32 are not stored but recomputed by the wave that
// owns the baby (each baby has one owner, so the VALU work is the same), and
// the first giant x^8 is not stored twice (it is baby 8) — 32 KB instead of
// 50 KB per workgroup at t = 80: 4 workgroups per CU instead of 3.
// NG = giant rows stored.
template <int NG, bool BSH = false, int NBB = NB>
struct Smem {
    uint4 bb[NBB][BLOCK];
    uint2 ga[NG][BLOCK];
};
template <int NG, int NBB>
struct Smem<NG, true, NBB> {
    uint2 bb[NBB][BLOCK];
    uint2 ga[NG > 0 ? NG : 1][BLOCK];
};

// The kernel body.  Tiles of 256 consecutive ids, grid-stride over tiles;
// ids past n feed 0 (every power 0).  T <= 8 * NA.  Wave w owns babies 2w
// and 2w+1: the a = 0 row of both and their MACs with every giant row, so
// the four waves do equal work (a wave of a workgroup shares its SIMD with
// the same wave of the other workgroups: an unbalanced split idles SIMDs at
// the barriers).
//   MODE 0  the first SG MACs of a wave's tile count all four carries on the
//           scalar unit, the rest per lane (v_addc)
//   MODE 1  every MAC: three carries on the scalar unit, one per lane
//   MODE 3  as MODE 0, the two MACs of a giant row issued as one interleaved
//           block (mac_pair_s) while both are scalar-counted (CW = 2)
// Writes, per block, partials[(2 m + limb) * gridDim.x + blockIdx.x] for
// powers m < T (32-bit limbs of canonical lane values summed: < 2^40).
// ABL (ablations for tools/tune_u64.hip only; the product uses 0): 1 skips
// the MACs, 2 skips the modmuls (the id itself stands for every power).
//   OFF     offset pass of a multi-pass encode (t > 80): powers base+1 ..
//           base+8NA with giants x^(base+8a), a = 0..NA-1 — every row a MAC
//           row, no a = 0 row; x^base by square-and-multiply from x^8 over
//           the uniform exponent base/8 (base a multiple of 8)
//   BSH     B * 2^32 recomputed by the owner wave in step 3 (see Smem)
//   LD      giant operands read one row ahead instead of all rows at once
//   XC      bit 0 (offset passes) — x^base per id from the previous pass's
//           cache xin (no square-and-multiply); bit 1 — the next pass's
//           x^base per id written to xout: x^(base + 8 NA) after an offset
//           pass, x^(8 NA) after pass 0
//   NBT     babies per id: 8 (two per wave), or 4 (one per wave: thresholds
//           t <= 40 waste fewer powers in 4-wide rows, and the babies and
//           giants of an id cost 3 + NA - 2 products instead of 7 + NA - 2)
//   PRIO    s_setprio 1 for a wave in its MAC step (1), or in its babies /
//           giants step (2); 3: the row-0 sums at 1 and the MACs at 2 (per
//           64-id chunk); 0: no priority changes
template <int NA, int MODE, int SG, int ABL = 0, int PF = 0, bool OFF = false, bool BSH = false, int LD = 0,
          int XC = 0, int NBT = NB, int PRIO = 0, int TR = 0>
__device__ __forceinline__ void body(const uint64_t *__restrict__ ids, uint64_t n, uint32_t T,
                                     uint64_t *__restrict__ partials, uint32_t base = 0,
                                     const uint64_t *xin = nullptr, uint64_t *xout = nullptr) {
    static_assert(OFF || (XC & 1) == 0, "only an offset pass reads x^base");
    static_assert((NA >= 2 || (OFF && NA == 1)) && NA <= 10, "giant rows");
    static_assert(!(BSH && PF) && !(LD && PF), "prefetch form: stored B * 2^32, all rows");
    static_assert(NBT == 8 || (NBT == 4 && BSH && !PF && XC == 0), "babies per id: 8, or 4 (plain BSH form)");
    static_assert(!TR || (BSH && !OFF && ABL == 0), "product-tree step 1: pass-0 BSH form");
    constexpr int CW = NBT / 4;                  // babies per wave
    constexpr int NR = OFF ? NA : NA - 1;        // MAC rows (giants x^8 .. x^(8 NR), or x^base ..)
    constexpr bool G8 = BSH && !OFF;             // giant row 0 (x^8) read from baby 8
    constexpr int NG = G8 ? NR - 1 : NR;
    __shared__ Smem<NG, BSH, NBT> sm;
    auto giant = [&](int r, int j) -> uint2 {
        if constexpr (G8) return r ? sm.ga[r - 1][j] : sm.bb[NBT - 1][j];
        else return sm.ga[r][j];
    };
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cb = CW * wave;                    // this wave's babies (b = cb+1 .. cb+CW)

    // a = 0 row: 64-bit sums of the halves; MAC tile: C0/C1 + carry counters
    uint64_t r0lo[2] = {0, 0}, r0hi[2] = {0, 0};
    uint64_t C0[NR][CW], C1[NR][CW];
    uint32_t K0[NR][CW], K1[NR][CW], KV[NR][CW];
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int c = 0; c < CW; ++c) { C0[r][c] = 0; C1[r][c] = 0; K0[r][c] = 0; K1[r][c] = 0; KV[r][c] = 0; }

    const uint64_t ntiles = (n + BLOCK - 1) / BLOCK;
    uint64_t tile = blockIdx.x;
    uint64_t nxt = 0, nxc = 0;
    if (tile < ntiles && tile * BLOCK + tid < n) {
        nxt = ids[tile * BLOCK + tid];
        if constexpr ((XC & 1) != 0) nxc = xin[tile * BLOCK + tid];
    }
    for (; tile < ntiles; tile += gridDim.x) {
        // ---- step 1: this thread's id -> babies (+ B * 2^32), giants -> LDS
        if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
        if constexpr (TR != 0) {
            uint64_t Pb[NBT + 1], Pg[NR + 1];
            Pb[1] = nxt;
            sm.bb[0][tid] = make_uint2((uint32_t)nxt, (uint32_t)(nxt >> 32));
            pow_tree<NBT>(Pb, [&](int k, uint64_t v) { sm.bb[k - 1][tid] = make_uint2((uint32_t)v, (uint32_t)(v >> 32)); });
            Pg[1] = Pb[NBT];   // giant row r = x^(NBT (r + 1)) = Pg[r + 1], rows >= 1 in ga[r - 1]
            pow_tree<NR>(Pg, [&](int k, uint64_t v) { sm.ga[k - 2][tid] = make_uint2((uint32_t)v, (uint32_t)(v >> 32)); });
            if constexpr ((XC & 2) != 0) {
                uint64_t V = Pg[NR];
                mulv(V, (uint32_t)Pb[NBT], (uint32_t)(Pb[NBT] >> 32));
                if (tile * BLOCK + tid < n) xout[tile * BLOCK + tid] = V;
            }
        } else {
            const uint64_t x = nxt;
            const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32);
            uint64_t V = x;
#pragma unroll
            for (int b = 0; b < NBT; ++b) {
                if (b && ABL != 2) mulv(V, x0, x1);
                if constexpr (BSH) {
                    sm.bb[b][tid] = make_uint2((uint32_t)V, (uint32_t)(V >> 32));
                } else {
                    const uint64_t sh = shift32(V);
                    sm.bb[b][tid] = make_uint4((uint32_t)V, (uint32_t)(V >> 32), (uint32_t)sh, (uint32_t)(sh >> 32));
                }
            }
            const uint32_t g0 = (uint32_t)V, g1 = (uint32_t)(V >> 32);   // x^NBT
            if constexpr ((XC & 1) != 0) {
                V = nxc;   // x^base from the previous pass
            } else if constexpr (OFF) {
                // x^base = (x^8)^(base/8): square-and-multiply, uniform exponent
                uint32_t q = base / NBT;
                uint64_t r = 0, sq = V;
                bool have = false;
                for (;;) {
                    if (q & 1) {
                        if (have) mulv(r, (uint32_t)sq, (uint32_t)(sq >> 32));
                        else r = sq;
                        have = true;
                    }
                    q >>= 1;
                    if (!q) break;
                    const uint32_t s0 = (uint32_t)sq, s1 = (uint32_t)(sq >> 32);
                    mulv(sq, s0, s1);
                }
                V = r;
            }
            if constexpr (!G8) sm.ga[0][tid] = make_uint2((uint32_t)V, (uint32_t)(V >> 32));
#pragma unroll
            for (int a = 1; a < NR; ++a) {
                if (ABL != 2) mulv(V, g0, g1);
                sm.ga[G8 ? a - 1 : a][tid] = make_uint2((uint32_t)V, (uint32_t)(V >> 32));
            }
            if constexpr ((XC & 2) != 0) {   // x^(base + 8 NR), or x^(8 NA) after pass 0, for the next pass
                mulv(V, g0, g1);
                if (tile * BLOCK + tid < n) xout[tile * BLOCK + tid] = V;
            }
        }
        if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
        __syncthreads();
        if constexpr (PRIO == 1 || PRIO == 3) __builtin_amdgcn_s_setprio(1);
        // next tile's id in flight during step 3
        const uint64_t tn = tile + gridDim.x;
        nxt = 0;
        if (tn < ntiles && tn * BLOCK + tid < n) {
            nxt = ids[tn * BLOCK + tid];
            if constexpr ((XC & 1) != 0) nxc = xin[tn * BLOCK + tid];
        }
        // ---- step 3: this wave's 2 x NR MACs over the 256 ids (4 per lane)
        // PF: the next chunk's operands are read from LDS while this chunk's
        // MACs run (double-buffered registers, the chunk loop unrolled)
        uint4 nbv[CW];
        uint2 ng[NR];
        if constexpr (PF) {
            nbv[0] = sm.bb[cb][lane];
            nbv[1] = sm.bb[cb + 1][lane];
#pragma unroll
            for (int r = 0; r < NR; ++r) ng[r] = sm.ga[r][lane];
        }
        constexpr int UNR = PF ? BLOCK / 64 : 1;
#pragma unroll UNR
        for (int q = 0; q < BLOCK / 64; ++q) {
            const int j = q * 64 + lane;
            uint4 bv[CW];
            uint2 g[NR];
            if constexpr (PF) {
                bv[0] = nbv[0];
                bv[1] = nbv[1];
#pragma unroll
                for (int r = 0; r < NR; ++r) g[r] = ng[r];
                if (q + 1 < BLOCK / 64) {
                    nbv[0] = sm.bb[cb][j + 64];
                    nbv[1] = sm.bb[cb + 1][j + 64];
#pragma unroll
                    for (int r = 0; r < NR; ++r) ng[r] = sm.ga[r][j + 64];
                }
            } else {
                if constexpr (BSH) {
#pragma unroll
                    for (int c = 0; c < CW; ++c) {
                        const uint2 B = sm.bb[cb + c][j];
                        const uint64_t sh = shift32(((uint64_t)B.y << 32) | B.x);
                        bv[c] = make_uint4(B.x, B.y, (uint32_t)sh, (uint32_t)(sh >> 32));
                    }
                } else {
                    bv[0] = sm.bb[cb][j];
                    bv[1] = sm.bb[cb + 1][j];
                }
                if constexpr (!LD) {
#pragma unroll
                    for (int r = 0; r < NR; ++r) g[r] = giant(r, j);
                }
            }
            if constexpr (!OFF && CW == 2) row2<1>(r0lo, r0hi, bv);
            if constexpr (!OFF && CW == 1) row1(r0lo[0], r0hi[0], bv[0]);
            if constexpr (PRIO == 3) __builtin_amdgcn_s_setprio(2);   // the MACs above the row-0 sums
            // LD: one giant row's operands in flight while the previous row's
            // MACs run (2 rows live instead of NR: fewer VGPRs)
            uint2 gn;
            if constexpr (LD) gn = giant(0, j);
            if (ABL != 1) {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    if constexpr (LD) {
                        g[r] = gn;
                        if (r + 1 < NR) gn = giant(r + 1, j);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    if constexpr (MODE == 3 && CW == 2) {
                        if (r * CW + 1 < SG) {
                            uint64_t c0[2] = {C0[r][0], C0[r][1]}, c1[2] = {C1[r][0], C1[r][1]};
                            uint32_t k0[2] = {K0[r][0], K0[r][1]}, k1[2] = {K1[r][0], K1[r][1]};
                            // (row 0's block follows row2<1>'s SGPRs: start with the disjoint set)
                            if (r % 2 == 0) mac_pair_s<1>(c0, c1, k0, k1, g[r].x, g[r].y, bv[0], bv[1]);
                            else mac_pair_s<0>(c0, c1, k0, k1, g[r].x, g[r].y, bv[0], bv[1]);
                            C0[r][0] = c0[0]; C0[r][1] = c0[1]; C1[r][0] = c1[0]; C1[r][1] = c1[1];
                            K0[r][0] = k0[0]; K0[r][1] = k0[1]; K1[r][0] = k1[0]; K1[r][1] = k1[1];
                            continue;
                        }
                    }
#pragma unroll
                    for (int c = 0; c < CW; ++c) {
                        const int m = r * CW + c;   // MAC index in the tile: parity picks the SGPR set
                        if constexpr (MODE == 1) {
                            if (m % 2 == 0) mac_m<0>(C0[r][c], C1[r][c], K0[r][c], K1[r][c], KV[r][c], g[r].x, g[r].y, bv[c]);
                            else mac_m<1>(C0[r][c], C1[r][c], K0[r][c], K1[r][c], KV[r][c], g[r].x, g[r].y, bv[c]);
                        } else if (m < SG && MODE != 3) {
                            if (m % 2 == 0) mac_s<0>(C0[r][c], C1[r][c], K0[r][c], K1[r][c], g[r].x, g[r].y, bv[c]);
                            else mac_s<1>(C0[r][c], C1[r][c], K0[r][c], K1[r][c], g[r].x, g[r].y, bv[c]);
                        } else {
                            if (m % 2 == 0) mac_v<0>(C0[r][c], C1[r][c], K0[r][c], K1[r][c], g[r].x, g[r].y, bv[c]);
                            else mac_v<1>(C0[r][c], C1[r][c], K0[r][c], K1[r][c], g[r].x, g[r].y, bv[c]);
                        }
                    }
                }
            }
        }
        if constexpr (PRIO == 1 || PRIO == 3) __builtin_amdgcn_s_setprio(0);
        __syncthreads();
    }

    // ---- reduction: canonical lane values, limb sums over lanes, LDS over waves
    // the tile operands are dead after the loop's last barrier: the reduction
    // reuses their LDS (a separate array pushes the offset pass with NA = 10
    // past 1/3 of the CU's LDS, i.e. to 2 workgroups per CU)
    static_assert(sizeof(Smem<NG, BSH, NBT>) >= 2 * NBT * NA * sizeof(unsigned long long), "reduction space");
    unsigned long long *red = reinterpret_cast<unsigned long long *>(&sm);
    for (int i = tid; i < 2 * NBT * NA; i += BLOCK) red[i] = 0;
    __syncthreads();
    auto put = [&](int m, uint64_t v) {   // v canonical; m = power - 1
        uint64_t lo = (uint32_t)v, hi = v >> 32;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            lo += bsgs::shfl_xor_u64(lo, off);
            hi += bsgs::shfl_xor_u64(hi, off);
        }
        if (lane == 0) {
            atomicAdd(&red[2 * m], lo);
            atomicAdd(&red[2 * m + 1], hi);
        }
    };
    const uint64_t W1 = 59ull << 32;   // 2^96 mod p
#pragma unroll
    for (int c = 0; c < CW; ++c)
        if constexpr (!OFF) put(cb + c, mod_p128((unsigned __int128)r0lo[c] + ((unsigned __int128)r0hi[c] << 32)));
#pragma unroll
    for (int r = 0; r < NR; ++r) {
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            const int m = r * CW + c;
            unsigned __int128 v = (unsigned __int128)C0[r][c] + ((unsigned __int128)C1[r][c] << 32);
            // scalar counts are the wave's totals: added once, by lane 0
            const bool sc = MODE == 3 ? r * CW + 1 < SG : m < SG;   // this MAC's carries counted per wave
            const bool s0 = MODE == 1 || sc, s1 = (MODE == 0 || MODE == 3) && sc;
            const uint32_t k0 = s0 ? (lane == 0 ? K0[r][c] : 0u) : K0[r][c];
            uint64_t k1 = s1 ? (lane == 0 ? K1[r][c] : 0u) : K1[r][c];
            if (MODE == 1) k1 = (lane == 0 ? (uint64_t)K1[r][c] : 0ull) + KV[r][c];
            v += (unsigned __int128)k0 * C64 + (unsigned __int128)k1 * W1;
            put((r + (OFF ? 0 : 1)) * NBT + cb + c, mod_p128(v));
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < 2 * T; i += BLOCK) partials[(size_t)i * gridDim.x + blockIdx.x] = red[i];
}

} // namespace bsgs64
} // namespace qk
