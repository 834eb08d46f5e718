// bsgs.h — baby-step / giant-step u32 encode body for 9 <= t <= 32 (the
// headline kernel).  Shared by encode.hip (product kernel)
// and tools/tune_bsgs.hip (A/B harness), so the tuned code is the shipped code.
//
// Power m+1 = a*NB + b + 1 with B_b = x^(b+1) (b < NB) and A_a = x^(a*NB)
// (a < NA; A_0 = 1), so S_{m+1} = sum_i A_a(x_i) * B_b(x_i): NB-1 + NA-2
// lazy modmuls per id, then (NA-1)*NB 32x32->64 multiply-accumulates into
// 64-bit accumulators whose wraps are counted (2^64 == 25 mod p), plus NB
// 32-bit adds for the a = 0 row whose wraps are counted (2^32 == 5 mod p).
//
// Wrap counting, per accumulator group of four (template knobs):
//   VALU form   v_mad_u64_u32 / v_add_co_u32 writes its carry to an SGPR pair,
//               v_addc_co_u32 adds it into a per-lane 32-bit counter.  gfx950
//               needs two wait states between a VALU SGPR write and a VALU
//               carry-in read (hipcc pads with s_nop), so four ops with four
//               distinct carry pairs are issued back to back first: every
//               v_addc reads a carry written >= 3 VALU instructions earlier.
//   SALU form   only the SUM over lanes of a power's wraps matters (the block
//               reduction adds every lane), so the carry mask is counted per
//               wave on the scalar unit (s_bcnt1 + s_add, issued beside the
//               VALU stream).  Needs EXEC = all lanes at the op (wave-uniform
//               control flow; lanes past their range feed id 0).
//
// Ids are not reduced mod p first: every product below is exact for any
// 32-bit operand and x == id (mod p) either way.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "field.h"

namespace qk {
namespace bsgs {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// ---- multiply-accumulate and add groups, carries counted ------------------
// The carry masks live in explicitly named SGPR pairs, and consecutive groups
// alternate between two disjoint sets (SET 0: s[40:47] + temp s56, SET 1:
// s[48:55] + temp s57).  hipcc treats an inline-asm block's SGPR definitions
// conservatively and pads "s_nop 0" between two blocks that define the same
// SGPRs (8 nops per id with compiler-allocated pairs; 3-5 remain at blocks
// with "+s" operands — one fused asm statement per id measured no faster).
// The blocks are volatile so the compiler keeps them in this alternating
// order.  Inside a block every VALU carry-in read is >= 3 VALU instructions
// after its write.
#define QK_MAC4V(P0, P1, P2, P3)                                                                       \
    "v_mad_u64_u32 %0, " P0 ", %8, %9, %0\n\t"                                                         \
    "v_mad_u64_u32 %1, " P1 ", %8, %10, %1\n\t"                                                        \
    "v_mad_u64_u32 %2, " P2 ", %8, %11, %2\n\t"                                                        \
    "v_mad_u64_u32 %3, " P3 ", %8, %12, %3\n\t"                                                        \
    "v_addc_co_u32_e64 %4, " P0 ", %4, 0, " P0 "\n\t"                                                  \
    "v_addc_co_u32_e64 %5, " P1 ", %5, 0, " P1 "\n\t"                                                  \
    "v_addc_co_u32_e64 %6, " P2 ", %6, 0, " P2 "\n\t"                                                  \
    "v_addc_co_u32_e64 %7, " P3 ", %7, 0, " P3
#define QK_MAC4S(P0, P1, P2, P3, T)                                                                       \
    "v_mad_u64_u32 %0, " P0 ", %8, %9, %0\n\t"                                                         \
    "v_mad_u64_u32 %1, " P1 ", %8, %10, %1\n\t"                                                        \
    "v_mad_u64_u32 %2, " P2 ", %8, %11, %2\n\t"                                                        \
    "v_mad_u64_u32 %3, " P3 ", %8, %12, %3\n\t"                                                        \
    "s_bcnt1_i32_b64 " T ", " P0 "\n\ts_add_u32 %4, %4, " T "\n\t"                                          \
    "s_bcnt1_i32_b64 " T ", " P1 "\n\ts_add_u32 %5, %5, " T "\n\t"                                          \
    "s_bcnt1_i32_b64 " T ", " P2 "\n\ts_add_u32 %6, %6, " T "\n\t"                                          \
    "s_bcnt1_i32_b64 " T ", " P3 "\n\ts_add_u32 %7, %7, " T
#define QK_ADD4V(P0, P1, P2, P3)                                                                       \
    "v_add_co_u32_e64 %0, " P0 ", %0, %8\n\t"                                                          \
    "v_add_co_u32_e64 %1, " P1 ", %1, %9\n\t"                                                          \
    "v_add_co_u32_e64 %2, " P2 ", %2, %10\n\t"                                                         \
    "v_add_co_u32_e64 %3, " P3 ", %3, %11\n\t"                                                         \
    "v_addc_co_u32_e64 %4, " P0 ", %4, 0, " P0 "\n\t"                                                  \
    "v_addc_co_u32_e64 %5, " P1 ", %5, 0, " P1 "\n\t"                                                  \
    "v_addc_co_u32_e64 %6, " P2 ", %6, 0, " P2 "\n\t"                                                  \
    "v_addc_co_u32_e64 %7, " P3 ", %7, 0, " P3
#define QK_ADD4S(P0, P1, P2, P3, T)                                                                       \
    "v_add_co_u32_e64 %0, " P0 ", %0, %8\n\t"                                                          \
    "v_add_co_u32_e64 %1, " P1 ", %1, %9\n\t"                                                          \
    "v_add_co_u32_e64 %2, " P2 ", %2, %10\n\t"                                                         \
    "v_add_co_u32_e64 %3, " P3 ", %3, %11\n\t"                                                         \
    "s_bcnt1_i32_b64 " T ", " P0 "\n\ts_add_u32 %4, %4, " T "\n\t"                                          \
    "s_bcnt1_i32_b64 " T ", " P1 "\n\ts_add_u32 %5, %5, " T "\n\t"                                          \
    "s_bcnt1_i32_b64 " T ", " P2 "\n\ts_add_u32 %6, %6, " T "\n\t"                                          \
    "s_bcnt1_i32_b64 " T ", " P3 "\n\ts_add_u32 %7, %7, " T
#define QK_SET0 "s[40:41]", "s[42:43]", "s[44:45]", "s[46:47]"
#define QK_SET1 "s[48:49]", "s[50:51]", "s[52:53]", "s[54:55]"
// scalar-form temps: one per set, so adjacent blocks never share a definition
#define QK_SET0T QK_SET0, "s56"
#define QK_SET1T QK_SET1, "s57"
#define QK_CLOB0 "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47"
#define QK_CLOB1 "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55"
#define QK_EXPAND(M, ...) M(__VA_ARGS__)

// acc_j += A * b_j (64-bit), wraps counted per lane (c_j) or per wave (s_j)
template <int SET>
__device__ __forceinline__ void mac4v(uint64_t &a0, uint64_t &a1, uint64_t &a2, uint64_t &a3, uint32_t &c0,
                                      uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t A, uint32_t b0,
                                      uint32_t b1, uint32_t b2, uint32_t b3) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_MAC4V, QK_SET0)
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
            : "v"(A), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : QK_CLOB0);
    else
        asm volatile(QK_EXPAND(QK_MAC4V, QK_SET1)
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
            : "v"(A), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : QK_CLOB1);
}
template <int SET>
__device__ __forceinline__ void mac4s(uint64_t &a0, uint64_t &a1, uint64_t &a2, uint64_t &a3, uint32_t &s0,
                                      uint32_t &s1, uint32_t &s2, uint32_t &s3, uint32_t A, uint32_t b0,
                                      uint32_t b1, uint32_t b2, uint32_t b3) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_MAC4S, QK_SET0T)
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
            : "v"(A), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : "scc", "s56", QK_CLOB0);
    else
        asm volatile(QK_EXPAND(QK_MAC4S, QK_SET1T)
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
            : "v"(A), "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : "scc", "s57", QK_CLOB1);
}
// lo_j += b_j (32-bit), wraps counted per lane (c_j) or per wave (s_j)
template <int SET>
__device__ __forceinline__ void add4v(uint32_t &l0, uint32_t &l1, uint32_t &l2, uint32_t &l3, uint32_t &c0,
                                      uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t b0, uint32_t b1,
                                      uint32_t b2, uint32_t b3) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_ADD4V, QK_SET0)
            : "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
            : "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : QK_CLOB0);
    else
        asm volatile(QK_EXPAND(QK_ADD4V, QK_SET1)
            : "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3), "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
            : "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : QK_CLOB1);
}
template <int SET>
__device__ __forceinline__ void add4s(uint32_t &l0, uint32_t &l1, uint32_t &l2, uint32_t &l3, uint32_t &s0,
                                      uint32_t &s1, uint32_t &s2, uint32_t &s3, uint32_t b0, uint32_t b1,
                                      uint32_t b2, uint32_t b3) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_ADD4S, QK_SET0T)
            : "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
            : "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : "scc", "s56", QK_CLOB0);
    else
        asm volatile(QK_EXPAND(QK_ADD4S, QK_SET1T)
            : "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
            : "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : "scc", "s57", QK_CLOB1);
}
// leftovers for NB % 4 != 0 (t = 17..24 uses NB = 6): compiler-allocated
// carries with explicit wait states
__device__ __forceinline__ void mac2v(uint64_t &a0, uint64_t &a1, uint32_t &c0, uint32_t &c1, uint32_t A,
                                      uint32_t b0, uint32_t b1) {
    uint64_t k0, k1;
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"
        "v_mad_u64_u32 %1, %5, %6, %8, %1\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %2, %4, %2, 0, %4\n\t"
        "v_addc_co_u32_e64 %3, %5, %3, 0, %5"
        : "+v"(a0), "+v"(a1), "+v"(c0), "+v"(c1), "=&s"(k0), "=&s"(k1)
        : "v"(A), "v"(b0), "v"(b1));
}
__device__ __forceinline__ void add2v(uint32_t &l0, uint32_t &l1, uint32_t &c0, uint32_t &c1, uint32_t b0,
                                      uint32_t b1) {
    uint64_t k0, k1;
    asm("v_add_co_u32_e64 %0, %4, %0, %6\n\t"
        "v_add_co_u32_e64 %1, %5, %1, %7\n\t"
        "s_nop 0\n\t"
        "v_addc_co_u32_e64 %2, %4, %2, 0, %4\n\t"
        "v_addc_co_u32_e64 %3, %5, %3, 0, %5"
        : "+v"(l0), "+v"(l1), "+v"(c0), "+v"(c1), "=&s"(k0), "=&s"(k1)
        : "v"(b0), "v"(b1));
}

// ---- a = 0 row as 64-bit multiply-adds: acc_j += b_j * 1 ------------------
// acc < 2^64 for < 2^32 adds of 32-bit values, so no carry is counted: one
// VALU per add (its carry-out is dead) instead of an add + add-with-carry pair
// (both SGPR-writing VALU ops, ~4 SIMD cycles each on gfx950: tools/ubench_issue.hip).
#define QK_ROW4M(P0, P1, P2, P3)                                                                       \
    "v_mad_u64_u32 %0, " P0 ", %4, 1, %0\n\t"                                                          \
    "v_mad_u64_u32 %1, " P1 ", %5, 1, %1\n\t"                                                          \
    "v_mad_u64_u32 %2, " P2 ", %6, 1, %2\n\t"                                                          \
    "v_mad_u64_u32 %3, " P3 ", %7, 1, %3"
template <int SET>
__device__ __forceinline__ void row4m(uint64_t &a0, uint64_t &a1, uint64_t &a2, uint64_t &a3, uint32_t b0,
                                      uint32_t b1, uint32_t b2, uint32_t b3) {
    if constexpr (SET == 0)
        asm volatile(QK_EXPAND(QK_ROW4M, QK_SET0)
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
            : "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : QK_CLOB0);
    else
        asm volatile(QK_EXPAND(QK_ROW4M, QK_SET1)
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
            : "v"(b0), "v"(b1), "v"(b2), "v"(b3)
            : QK_CLOB1);
}
__device__ __forceinline__ void row2m(uint64_t &a0, uint64_t &a1, uint32_t b0, uint32_t b1) {
    uint64_t k0, k1;
    asm("v_mad_u64_u32 %0, %2, %4, 1, %0\n\t"
        "v_mad_u64_u32 %1, %3, %5, 1, %1"
        : "+v"(a0), "+v"(a1), "=&s"(k0), "=&s"(k1)
        : "v"(b0), "v"(b1));
}

// ---- configuration ----------------------------------------------------------
//  NB, NA  baby / giant steps (NB even)
//  SG      the first SG 4-wide accumulator groups count their wraps on the
//          scalar unit.  Group numbering: the a = 0 row's groups are
//          g = 0 .. NB/4-1 (only when ROW0 == 0), MAC row a (1..NA-1) has
//          g = a*(NB/4) + b/4.  NB % 4 leftovers always use the VALU form.
//  ROW0    0: a = 0 row as 32-bit adds with counted wraps; 1: 64-bit mads
//  FOLD    0: lazy fold with an SGPR-writing add (wrap = its carry, ORed on the
//          scalar unit); 1: plain add, wraps caught by a per-lane minimum of
//          the fold results (a wrapped fold leaves a value < 25, field.h)
//  PAIR    interleave the power chains of two ids
//  OFF     offset pass (thresholds > 80, several passes over the ids): the
//          giants are x^(base + a*NB) for a = 0..NA-1 with a runtime base
//          (a multiple of NB), so every row is a MAC row (no a = 0 sum row)
//          and the pass yields powers base+1 .. base+NB*NA
//  XC      bit 0 (offset passes) — x^base per id read from the previous
//          pass's cache instead of square-and-multiply; bit 1 — the next
//          pass's x^base written per id (one more product): x^(base + NB*NA)
//          after an offset pass, x^(NB*NA) after a plain one (pass 0)
//  TREE    babies by a product tree (x^(h+l) = x^h x^l, h the highest power
//          of two below): the same NB - 1 lazy modmuls at dependency depth
//          log2(NB) instead of NB - 1 (plain passes with min-tracked folds)
template <int NB_, int NA_, int SG_, int ROW0_ = 1, int FOLD_ = 1, bool PAIR_ = false, bool OFF_ = false,
          int XC_ = 0, bool TREE_ = false, int PRIO_ = 0>
struct Cfg {
    // PRIO  wave priority (s_setprio) over the accumulation: 4 (the product)
    //       row 0 at 1 and the MAC rows with their scalar wrap counts at 2,
    //       the powers at 0; (measurements) 1 the whole accumulation at 1,
    //       2 the powers raised instead, 3 the MAC rows only, 5 / 6 other levels
    static constexpr int PRIO = PRIO_;
    static constexpr int NB = NB_, NA = NA_, SG = SG_, ROW0 = ROW0_, FOLD = FOLD_, XC = XC_;
    static constexpr bool TREE = TREE_;
    static_assert(!TREE_ || (!OFF_ && FOLD_ == 1), "product-tree babies: plain passes, min-tracked folds");
    static constexpr bool PAIR = PAIR_, OFF = OFF_;
    static_assert(OFF_ || (XC_ & 1) == 0, "only an offset pass reads x^base");
    static_assert(!XC_ || FOLD_ == 1, "the x^base cache goes with min-tracked folds");
    static constexpr int ROWS = OFF_ ? NA_ : NA_ - 1;   // MAC rows
    static constexpr int ROW1 = OFF_ ? 0 : 1;           // group-row number of the first MAC row
    static_assert(NB % 2 == 0 && (NA >= 2 || (OFF_ && NA == 1)), "NB even, NA >= 2 (1: offset pass)");
    static_assert(!OFF_ || FOLD_ == 1, "offset passes use min-tracked folds");
};

template <int NB, int NA, int ROWS = NA - 1>
struct Acc {
    uint32_t lo0[NB];         // a = 0 row (ROW0 == 0): sum of B_b mod 2^32
    uint32_t c0[NB];          // ... its wraps (lane count, or wave total if scalar)
    uint64_t r0[NB];          // a = 0 row (ROW0 == 1): sum of B_b, 64-bit
    uint64_t m[ROWS][NB];     // MAC rows: sum of A_a * B_b mod 2^64
    uint32_t c[ROWS][NB];     // ... its wraps (lane count, or wave total if scalar)
};

// group rows: 0 = the a = 0 sum row, ROW1.. = the MAC rows (an offset pass
// has no sum row: its MAC rows start at 0)
template <class C>
__host__ __device__ constexpr bool scalar_group(int row, int b) {
    return b / 4 * 4 + 4 <= C::NB && (row > 0 || C::ROW0 == 0 || C::OFF) && row * (C::NB / 4) + b / 4 < C::SG;
}

// x^(NB*q) from xn = x^NB by square-and-multiply over the (wave-uniform) q >= 1
template <class MUL>
__device__ __forceinline__ uint32_t pow_uniform(uint32_t xn, uint32_t q, MUL mul) {
    uint32_t r = 0, sq = xn;
    bool have = false;
    for (;;) {
        if (q & 1) {
            r = have ? mul(r, sq) : sq;
            have = true;
        }
        q >>= 1;
        if (!q) break;
        sq = mul(sq, sq);
    }
    return r;
}

// powers of one id; returns nonzero if a lazy fold may have wrapped (the
// caller then recomputes exactly).  OFF: A[a] = x^(base + a*NB).
template <class C>
__device__ __forceinline__ uint32_t powers(uint32_t id, uint32_t (&B)[C::NB], uint32_t (&A)[C::ROWS],
                                           uint32_t base = 0, uint32_t xb = 0, uint32_t *xnext = nullptr) {
    constexpr int NB = C::NB, NA = C::NA;
    B[0] = id;
    if constexpr (C::OFF) {
        uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
        for (int b = 1; b < NB; ++b) B[b] = mulfold32_min(B[b - 1], B[0], mn);
        const uint32_t xn = B[NB - 1];                                   // x^NB (B[b] = x^(b+1))
        if constexpr (C::XC & 1) A[0] = xb;
        else A[0] = pow_uniform(xn, base / NB, [&](uint32_t u, uint32_t v) { return mulfold32_min(u, v, mn); });
#pragma unroll
        for (int a = 1; a < NA; ++a) A[a] = mulfold32_min(A[a - 1], xn, mn);
        if constexpr ((C::XC & 2) != 0) *xnext = mulfold32_min(A[NA - 1], xn, mn);
        return mn < 25u;
    } else if constexpr (C::FOLD == 0) {
        uint32_t wrapped = 0;
#pragma unroll
        for (int b = 1; b < NB; ++b) B[b] = mulfold32_fast(B[b - 1], B[0], wrapped);
        A[0] = B[NB - 1];
#pragma unroll
        for (int a = 1; a < NA - 1; ++a) A[a] = mulfold32_fast(A[a - 1], A[0], wrapped);
        return wrapped;
    } else {
        uint32_t mn = 0xFFFFFFFFu;
        if constexpr (C::TREE) {
#pragma unroll
            for (int b = 1; b < NB; ++b) {   // B[b] = x^(b+1) = x^h * x^(b+1-h)
                const int h = 1 << (31 - __builtin_clz((unsigned)(b + 1) - 1u));
                B[b] = (b + 1) == 2 * h ? mulfold32_min(B[h - 1], B[h - 1], mn)
                                        : mulfold32_min(B[h - 1], B[b - h], mn);
            }
        } else {
#pragma unroll
            for (int b = 1; b < NB; ++b) B[b] = mulfold32_min(B[b - 1], B[0], mn);
        }
        A[0] = B[NB - 1];
#pragma unroll
        for (int a = 1; a < NA - 1; ++a) A[a] = mulfold32_min(A[a - 1], A[0], mn);
        if constexpr ((C::XC & 2) != 0) *xnext = mulfold32_min(A[NA - 2], A[0], mn);   // x^(NB NA)
        return mn < 25u;
    }
}
template <class C>
__device__ __forceinline__ void powers_exact(uint32_t (&B)[C::NB], uint32_t (&A)[C::ROWS], uint32_t base = 0,
                                             uint32_t xb = 0, uint32_t *xnext = nullptr) {
#pragma unroll
    for (int b = 1; b < C::NB; ++b) B[b] = mulfold32_exact(B[b - 1], B[0]);
    if constexpr (C::OFF) {
        const uint32_t xn = B[C::NB - 1];
        if constexpr (C::XC & 1) A[0] = xb;
        else A[0] = pow_uniform(xn, base / C::NB, [](uint32_t u, uint32_t v) { return mulfold32_exact(u, v); });
#pragma unroll
        for (int a = 1; a < C::NA; ++a) A[a] = mulfold32_exact(A[a - 1], xn);
        if constexpr ((C::XC & 2) != 0) *xnext = mulfold32_exact(A[C::NA - 1], xn);
        return;
    }
    A[0] = B[C::NB - 1];
#pragma unroll
    for (int a = 1; a < C::NA - 1; ++a) A[a] = mulfold32_exact(A[a - 1], A[0]);
    if constexpr ((C::XC & 2) != 0) *xnext = mulfold32_exact(A[C::NA - 2], A[0]);
}

// Groups are issued in the order row 0, row 1, ... and alternate carry-SGPR
// sets (group index parity), so no two adjacent blocks share SGPRs.
template <class C>
__device__ __forceinline__ void accumulate(Acc<C::NB, C::NA, C::ROWS> &S, const uint32_t (&B)[C::NB],
                                           const uint32_t (&A)[C::ROWS]) {
    constexpr int NB = C::NB;
    auto row0 = [&]() {
    #pragma unroll
        for (int b = 0; b + 4 <= NB; b += 4) {
            if constexpr (C::OFF) break;   // no sum row in an offset pass
            const bool s0 = (b / 4) % 2 == 0;
            if constexpr (C::ROW0 == 1) {
                if (s0) row4m<0>(S.r0[b], S.r0[b + 1], S.r0[b + 2], S.r0[b + 3], B[b], B[b + 1], B[b + 2], B[b + 3]);
                else row4m<1>(S.r0[b], S.r0[b + 1], S.r0[b + 2], S.r0[b + 3], B[b], B[b + 1], B[b + 2], B[b + 3]);
            } else if (scalar_group<C>(0, b)) {
                if (s0)
                    add4s<0>(S.lo0[b], S.lo0[b + 1], S.lo0[b + 2], S.lo0[b + 3], S.c0[b], S.c0[b + 1], S.c0[b + 2],
                             S.c0[b + 3], B[b], B[b + 1], B[b + 2], B[b + 3]);
                else
                    add4s<1>(S.lo0[b], S.lo0[b + 1], S.lo0[b + 2], S.lo0[b + 3], S.c0[b], S.c0[b + 1], S.c0[b + 2],
                             S.c0[b + 3], B[b], B[b + 1], B[b + 2], B[b + 3]);
            } else {
                if (s0)
                    add4v<0>(S.lo0[b], S.lo0[b + 1], S.lo0[b + 2], S.lo0[b + 3], S.c0[b], S.c0[b + 1], S.c0[b + 2],
                             S.c0[b + 3], B[b], B[b + 1], B[b + 2], B[b + 3]);
                else
                    add4v<1>(S.lo0[b], S.lo0[b + 1], S.lo0[b + 2], S.lo0[b + 3], S.c0[b], S.c0[b + 1], S.c0[b + 2],
                             S.c0[b + 3], B[b], B[b + 1], B[b + 2], B[b + 3]);
            }
        }
        if constexpr (NB % 4 == 2 && !C::OFF) {
            if constexpr (C::ROW0 == 1) row2m(S.r0[NB - 2], S.r0[NB - 1], B[NB - 2], B[NB - 1]);
            else add2v(S.lo0[NB - 2], S.lo0[NB - 1], S.c0[NB - 2], S.c0[NB - 1], B[NB - 2], B[NB - 1]);
        }
    };
    if constexpr (C::PRIO != 7) row0();
    if constexpr (C::PRIO == 3) __builtin_amdgcn_s_setprio(1);   // (measurements: the MAC rows only)
    if constexpr (C::PRIO == 4) __builtin_amdgcn_s_setprio(2);   // row 0 at 1, the MAC rows at 2
    if constexpr (C::PRIO == 6) __builtin_amdgcn_s_setprio(2);   // (measurements: row 0 at 3, the rows at 2)
#pragma unroll
    for (int a = 0; a < C::ROWS; ++a) {
        // (measurements) 5: row 0 at 1, MAC row a at min(3, 2 + a)
        if constexpr (C::PRIO == 5) {
            if (a == 0) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(3);
        }
#pragma unroll
        for (int b = 0; b + 4 <= NB; b += 4) {
            const int g = (a + C::ROW1) * (NB / 4) + b / 4;   // group index: parity picks the SGPR set
            if (scalar_group<C>(a + C::ROW1, b)) {
                if (g % 2 == 0)
                    mac4s<0>(S.m[a][b], S.m[a][b + 1], S.m[a][b + 2], S.m[a][b + 3], S.c[a][b], S.c[a][b + 1],
                             S.c[a][b + 2], S.c[a][b + 3], A[a], B[b], B[b + 1], B[b + 2], B[b + 3]);
                else
                    mac4s<1>(S.m[a][b], S.m[a][b + 1], S.m[a][b + 2], S.m[a][b + 3], S.c[a][b], S.c[a][b + 1],
                             S.c[a][b + 2], S.c[a][b + 3], A[a], B[b], B[b + 1], B[b + 2], B[b + 3]);
            } else {
                if (g % 2 == 0)
                    mac4v<0>(S.m[a][b], S.m[a][b + 1], S.m[a][b + 2], S.m[a][b + 3], S.c[a][b], S.c[a][b + 1],
                             S.c[a][b + 2], S.c[a][b + 3], A[a], B[b], B[b + 1], B[b + 2], B[b + 3]);
                else
                    mac4v<1>(S.m[a][b], S.m[a][b + 1], S.m[a][b + 2], S.m[a][b + 3], S.c[a][b], S.c[a][b + 1],
                             S.c[a][b + 2], S.c[a][b + 3], A[a], B[b], B[b + 1], B[b + 2], B[b + 3]);
            }
        }
        if constexpr (NB % 4 == 2)
            mac2v(S.m[a][NB - 2], S.m[a][NB - 1], S.c[a][NB - 2], S.c[a][NB - 1], A[a], B[NB - 2], B[NB - 1]);
    }
    if constexpr (C::PRIO == 7) {   // (measurements: the MAC rows first at 2, then row 0 at 1)
        __builtin_amdgcn_s_setprio(1);
        row0();
    }
}

// wave priority around an id's accumulation (Cfg PRIO; accumulate raises it
// further before the MAC rows for PRIO 3-6)
template <class C> __device__ __forceinline__ void prio_enter() {
    if constexpr (C::PRIO == 1 || C::PRIO == 4 || C::PRIO == 5) __builtin_amdgcn_s_setprio(1);
    if constexpr (C::PRIO == 6) __builtin_amdgcn_s_setprio(3);
    if constexpr (C::PRIO == 7) __builtin_amdgcn_s_setprio(2);
    if constexpr (C::PRIO == 2) __builtin_amdgcn_s_setprio(0);
}
template <class C> __device__ __forceinline__ void prio_exit() {
    if constexpr (C::PRIO == 1 || C::PRIO >= 3) __builtin_amdgcn_s_setprio(0);
    if constexpr (C::PRIO == 2) __builtin_amdgcn_s_setprio(1);
}

// xb / xnext: an offset pass's cached x^base and the next pass's (Cfg XC)
template <class C>
__device__ __forceinline__ void one(Acc<C::NB, C::NA, C::ROWS> &S, uint32_t id, uint32_t base = 0, uint32_t xb = 0,
                                    uint32_t *xnext = nullptr) {
    uint32_t B[C::NB], A[C::ROWS];
    const uint32_t w = powers<C>(id, B, A, base, xb, xnext);
    if (__builtin_expect(__any(w), 0)) {
        if (w) powers_exact<C>(B, A, base, xb, xnext);
    }
    prio_enter<C>();
    accumulate<C>(S, B, A);
    prio_exit<C>();
}

// two ids at once: their power chains are independent straight-line code, so
// the compiler interleaves them (ILP for the dependent modmul chains)
template <class C>
__device__ __forceinline__ void two(Acc<C::NB, C::NA, C::ROWS> &S, uint32_t id0, uint32_t id1) {
    static_assert(!C::OFF, "pairs: plain passes only");
    uint32_t B0[C::NB], A0[C::ROWS], B1[C::NB], A1[C::ROWS];
    const uint32_t w0 = powers<C>(id0, B0, A0);
    const uint32_t w1 = powers<C>(id1, B1, A1);
    if (__builtin_expect(__any(w0 | w1), 0)) {
        if (w0) powers_exact<C>(B0, A0);
        if (w1) powers_exact<C>(B1, A1);
    }
    prio_enter<C>();
    accumulate<C>(S, B0, A0);
    accumulate<C>(S, B1, A1);
    prio_exit<C>();
}

template <class C>
__device__ __forceinline__ void four(Acc<C::NB, C::NA, C::ROWS> &S, uint4 w, uint32_t base,
                                     uint4 xb = make_uint4(0, 0, 0, 0), uint4 *xn = nullptr) {
    if constexpr (C::PAIR) {
        two<C>(S, w.x, w.y);
        two<C>(S, w.z, w.w);
    } else {
        uint4 t = make_uint4(0, 0, 0, 0);
        one<C>(S, w.x, base, xb.x, &t.x);
        one<C>(S, w.y, base, xb.y, &t.y);
        one<C>(S, w.z, base, xb.z, &t.z);
        one<C>(S, w.w, base, xb.w, &t.w);
        if constexpr ((C::XC & 2) != 0) *xn = t;
    }
}

// Lane partials -> wave butterfly -> LDS -> one sum per power for the
// workgroup: out(m, s) receives power m + 1's sum (< 2^40) in thread m.
template <class C, class Out>
__device__ __forceinline__ void finish(const Acc<C::NB, C::NA, C::ROWS> &S, uint32_t T, Out out) {
    constexpr int NB = C::NB, NA = C::NA;
    __shared__ uint64_t sm[WAVES * NB * NA];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            // value = lo + c * W with W = 2^32 == 5 (a = 0) or 2^64 == 25 (a > 0);
            // a scalar-counted c is the wave's total, added once (by lane 0)
            const bool sc = scalar_group<C>(a, b);
            const uint32_t c = C::OFF ? S.c[a][b] : a == 0 ? S.c0[b] : S.c[a - C::ROW1][b];
            const uint32_t cl = sc ? (lane == 0 ? c : 0u) : c;
            uint64_t x;
            if (C::OFF) {
                x = (uint64_t)fold64_32(S.m[a][b]) + fold64_32((uint64_t)cl * 25u);
            } else if (a == 0) {
                if constexpr (C::ROW0 == 1) x = S.r0[b];
                else x = (uint64_t)S.lo0[b] + (uint64_t)cl * 5u;                      // < 6*2^32
            } else {
                x = (uint64_t)fold64_32(S.m[a - C::ROW1][b]) + fold64_32((uint64_t)cl * 25u);
            }
            x = fold64_32(x);                                                         // < 2^32
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) x += shfl_xor_u64(x, off);        // < 2^38
            if (lane == 0) sm[wave * (NB * NA) + a * NB + b] = x;
        }
    }
    __syncthreads();
    for (uint32_t m = threadIdx.x; m < T; m += BLOCK) {
        uint64_t s = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s += sm[w * (NB * NA) + m];
        out(m, s);
    }
}

// The kernel body: grid-stride over 16-byte groups of ids (+ unaligned head
// and tail), then lane partials -> wave butterfly -> LDS -> one partial per
// (power, block) stored [power][block].
//
// Every lane of a wave runs the wave's trip count (lane 0 has the largest):
// lanes past their range feed id 0, whose powers are all 0, so EXEC is full
// at every scalar-counted op.  The loop is split: while every lane of the
// wave still has a next group, the prefetch is unconditional; the last <= 2
// trips take the masked form.  Per-lane 32-bit trip counts (the host
// guarantees body / nthr < 2^32).
// body_gen: the ids are walked by `nthr` threads of which this is `gtid`
// (the whole grid for the headline kernel, one workgroup for a flow's work
// item); out(m, s) receives the workgroup's sum for power m + 1 (< 2^40) in
// thread m (an offset pass: power base + m + 1).
template <class C>
__device__ __forceinline__ void clear(Acc<C::NB, C::NA, C::ROWS> &S) {
#pragma unroll
    for (int b = 0; b < C::NB; ++b) {
        S.lo0[b] = 0;
        S.c0[b] = 0;
        S.r0[b] = 0;
#pragma unroll
        for (int a = 0; a < C::ROWS; ++a) { S.m[a][b] = 0; S.c[a][b] = 0; }
    }
}

// XC (offset passes): xin / xout are per-id arrays indexed like ids whose
// address is congruent to ids' modulo 16 (the same 16-byte groups).  The
// middle passes read and write the same cache (xin == xout): not restrict —
// each element is read one iteration before its own write, and the source
// order (next load, compute, this store) is the order kept.
template <class C, class Out>
__device__ __forceinline__ void body_gen(const uint32_t *__restrict__ ids, uint64_t n, uint32_t head, uint32_t T,
                                         uint64_t gtid, uint64_t nthr, Out out, uint32_t base = 0,
                                         const uint32_t *xin = nullptr,
                                         uint32_t *xout = nullptr) {
    constexpr bool XI = (C::XC & 1) != 0, XO = (C::XC & 2) != 0;
    Acc<C::NB, C::NA, C::ROWS> S;
    clear<C>(S);
    const uint64_t h = head < n ? head : n;
    const uint64_t nbody = (n - h) >> 2;
    const uint4 *__restrict__ v = reinterpret_cast<const uint4 *>(ids + h);
    const uint32_t iters = gtid < nbody ? (uint32_t)((nbody - gtid + nthr - 1) / nthr) : 0u;
    const uint32_t tmax = (uint32_t)__builtin_amdgcn_readfirstlane(iters);           // lane 0: most trips
    const uint32_t tmin = (uint32_t)__builtin_amdgcn_readlane((int)iters, 63);       // lane 63: fewest
    const uint4 *__restrict__ p = v + gtid;
    const uint4 *pc = XI ? reinterpret_cast<const uint4 *>(xin + h) + gtid : nullptr;
    uint4 *po = XO ? reinterpret_cast<uint4 *>(xout + h) + gtid : nullptr;
    uint4 nxt = make_uint4(0, 0, 0, 0), nxc = make_uint4(0, 0, 0, 0), xo = make_uint4(0, 0, 0, 0);
    if (iters) {
        nxt = *p;
        if constexpr (XI) nxc = *pc;
    }
    uint32_t it = 0;
    for (; it + 1 < tmin; ++it) {
        const uint4 w = nxt, c = nxc;
        p += nthr;
        nxt = *p;
        if constexpr (XI) {
            pc += nthr;
            nxc = *pc;
        }
        four<C>(S, w, base, c, &xo);
        if constexpr (XO) {
            *po = xo;
            po += nthr;
        }
    }
    for (; it < tmax; ++it) {
        const uint4 w = nxt, c = nxc;
        p += nthr;
        nxt = make_uint4(0, 0, 0, 0);
        if (it + 1 < iters) nxt = *p;
        if constexpr (XI) {
            pc += nthr;
            if (it + 1 < iters) nxc = *pc;
        }
        four<C>(S, w, base, c, &xo);
        if constexpr (XO) {
            if (it < iters) *po = xo;
            po += nthr;
        }
    }
    const uint64_t tail0 = h + (nbody << 2);
    {
        const bool in = gtid < h;
        uint32_t xn = 0;
        one<C>(S, in ? ids[gtid] : 0u, base, XI && in ? xin[gtid] : 0u, &xn);
        if (XO && in) xout[gtid] = xn;
    }
    {
        const bool in = gtid < n - tail0;
        uint32_t xn = 0;
        one<C>(S, in ? ids[tail0 + gtid] : 0u, base, XI && in ? xin[tail0 + gtid] : 0u, &xn);
        if (XO && in) xout[tail0 + gtid] = xn;
    }

    finish<C>(S, T, out);
}

// the headline kernel's form: grid-stride, one partial per (power, block)
// stored [power][block]
template <class C>
__device__ __forceinline__ void body(const uint32_t *__restrict__ ids, uint64_t n, uint32_t head, uint32_t T,
                                     uint64_t *__restrict__ partials, uint32_t base = 0,
                                     const uint32_t *xin = nullptr, uint32_t *xout = nullptr) {
    body_gen<C>(
        ids, n, head, T, (uint64_t)blockIdx.x * BLOCK + threadIdx.x, (uint64_t)gridDim.x * BLOCK,
        [=](uint32_t m, uint64_t s) { partials[(size_t)m * gridDim.x + blockIdx.x] = s; }, base, xin, xout);
}

} // namespace bsgs
} // namespace qk
