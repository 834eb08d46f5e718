// field.h — GF(p32) / GF(p64) arithmetic for the quACK engine, shared by the
// gfx950 kernels and the host scalar path (same code => bit-identical).
//
// p32 = 2^32 - 5 and p64 = 2^64 - 59 are pseudo-Mersenne: 2^32 == 5 (mod p32)
// and 2^64 == 59 (mod p64), so a double-width product H*2^w + L reduces by
// folding H*c + L twice, with no division and no data-dependent branch.
//
// "Lazy" values are congruent to the true residue but only bounded by 2^w
// (they may equal a value in [p, 2^w)); canon() maps them to [0, p).
// Every bound used below is proved in the comment next to it.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define QK_HD __host__ __device__ __forceinline__
#else
#define QK_HD static inline
#endif

namespace qk {

constexpr uint32_t P32 = 4294967291u;             // 2^32 - 5
constexpr uint64_t P64 = 18446744073709551557ull; // 2^64 - 59
constexpr uint32_t C32 = 5u;                      // 2^32 mod p32
constexpr uint64_t C64 = 59u;                     // 2^64 mod p64

// ---------------------------------------------------------------- GF(p32)
// x in [0, 2^32) -> x mod p32.  If x < p, x+5 does not wrap and min = x;
// if x >= p (only 2^32-5..2^32-1), x+5 wraps to x-p in [0,4] < x.
QK_HD uint32_t canon32(uint32_t x) {
    uint32_t a = x + C32;
    return a < x ? a : x;
}

// y, x < 2^32 (lazy) -> r < 2^32 with r == y*x (mod p32).
QK_HD uint32_t mul32_lazy(uint32_t y, uint32_t x) {
    uint64_t P = (uint64_t)y * x;                       // < 2^64
    uint64_t t = (P >> 32) * C32 + (uint32_t)P;         // < 5*2^32 + 2^32 = 6*2^32
    uint64_t u = (t >> 32) * C32 + (uint32_t)t;         // (t>>32) <= 5  ->  u < 2^32 + 25
    return (uint32_t)u + C32 * (uint32_t)(u >> 32);     // u>>32 == 1 => (uint32)u < 25: no wrap
}

// y*x + c for y, x, c < 2^32 (lazy) -> r < 2^32, r == y*x + c (mod p32).
// (2^32-1)^2 + (2^32-1) < 2^64, so the mad itself cannot overflow.
QK_HD uint32_t mad32_lazy(uint32_t y, uint32_t x, uint32_t c) {
    uint64_t P = (uint64_t)y * x + c;
    uint64_t t = (P >> 32) * C32 + (uint32_t)P;
    uint64_t u = (t >> 32) * C32 + (uint32_t)t;
    return (uint32_t)u + C32 * (uint32_t)(u >> 32);
}

// ---- "t-form": the chain representation used by the gfx950 kernels -------
// A residue is held as t = lo + hi*2^32 with hi <= 5 (t < 6*2^32).  With x and
// x5 = 5x mod p both canonical (<= p-1), one step t <- t*x + c (c <= p-1) is
//     P  = lo*x + (hi*x5 + c)      <= (2^32-1)(p-1) + 6(p-1) = (p-1)(2^32+5)
//                                   = 2^64 - 2^32 - 30 < 2^64   (no overflow)
//     t' = P_lo + 5*P_hi           P_hi <= 2^32-2  =>  t' < 6*2^32 (hi' <= 5)
// and t' == t*x + c (mod p) because hi*x5 == hi*5x == hi*2^32*x.  t' is
// formed as Q = P + 5*P_hi (mod 2^64) then Q_hi -= P_hi, i.e. P + 5P_hi -
// P_hi*2^32 = t' exactly (t' < 2^64): three v_mad_u64_u32 and one v_sub_u32,
// with no carry handling and no canonicalisation inside the chain.
QK_HD void tstep32(uint32_t &lo, uint32_t &hi, uint32_t x, uint32_t x5, uint32_t c) {
    const uint64_t P = (uint64_t)lo * x + ((uint64_t)hi * x5 + c);
    const uint32_t Ph = (uint32_t)(P >> 32);
    const uint64_t Q = P + (uint64_t)Ph * C32;
    lo = (uint32_t)Q;
    hi = (uint32_t)(Q >> 32) - Ph;
}
// Same step on a t-form value kept as one 64-bit register pair, so the
// accumulate that follows is a single 64-bit add of the pair.
QK_HD uint64_t tstep32p(uint64_t t, uint32_t x, uint32_t x5, uint32_t c) {
    const uint64_t P = (uint64_t)(uint32_t)t * x + ((uint64_t)(uint32_t)(t >> 32) * x5 + c);
    const uint32_t Ph = (uint32_t)(P >> 32);
    const uint64_t Q = P + (uint64_t)Ph * C32;
    return Q - ((uint64_t)Ph << 32);
}
// 32-bit lazy product for the baby-step/giant-step encode: y, x < 2^32 ->
// r < 2^32, r == y*x (mod p), except when t_lo + 5 t_hi wraps 2^32 (prob.
// <= 25/2^32 per call), which is reported through `wrapped` instead of being
// fixed inline; callers redo the (rare) id with mulfold32_exact.
QK_HD uint32_t mulfold32_fast(uint32_t y, uint32_t x, uint32_t &wrapped) {
    const uint64_t P = (uint64_t)y * x;
    const uint32_t Ph = (uint32_t)(P >> 32);
    const uint64_t Q = P + (uint64_t)Ph * C32;
    const uint32_t tl = (uint32_t)Q, th = (uint32_t)(Q >> 32) - Ph;  // t = tl + th*2^32, th <= 5
    const uint32_t m = th * C32;
    const uint32_t r = tl + m;
    wrapped |= (r < m);
    return r;
}
QK_HD uint32_t mulfold32_exact(uint32_t y, uint32_t x) {
    const uint64_t P = (uint64_t)y * x;
    const uint32_t Ph = (uint32_t)(P >> 32);
    const uint64_t Q = P + (uint64_t)Ph * C32;
    const uint32_t tl = (uint32_t)Q, th = (uint32_t)(Q >> 32) - Ph;
    const uint32_t m = th * C32;
    uint32_t r = tl + m;
    if (r < m) r += C32;  // wrapped past 2^32 == 5 (mod p); then r < 25, no second wrap
    return r;
}

// The BSGS kernels' lazy product (bsgs.h): the same t = tl + 5 th, then
// r = tl + 5 th mod 2^32 with no carry handling.  If that add wrapped, the
// true sum is r + 2^32 with r < 5 th <= 25, so the caller tracks mn = min(r)
// over an id's products and redoes the id exactly when mn < 25 (probability
// ~25 / 2^32 per product; a legitimately small r only costs a redo).
QK_HD uint32_t mulfold32_min(uint32_t y, uint32_t x, uint32_t &mn) {
    const uint64_t P = (uint64_t)y * x;
    const uint32_t Ph = (uint32_t)(P >> 32);
    const uint64_t Q = P + (uint64_t)Ph * C32;
    const uint32_t tl = (uint32_t)Q, th = (uint32_t)(Q >> 32) - Ph;
    const uint32_t r = tl + th * C32;
    mn = r < mn ? r : mn;
    return r;
}

// 5x mod p for canonical x (x5 in the step above)
QK_HD uint32_t times5_32(uint32_t x) {
    const uint64_t v = (uint64_t)x * C32;                   // < 5*2^32
    const uint64_t u = (v >> 32) * C32 + (uint32_t)v;        // < 2^32 + 20
    const uint32_t r = (uint32_t)u + C32 * (uint32_t)(u >> 32);
    const uint32_t a = r + C32;                              // canon
    return a < r ? a : r;
}

// Fold a 64-bit lazy accumulator (any value) to [0, 2^32), congruent.
QK_HD uint32_t fold64_32(uint64_t a) {
    uint64_t t = (a >> 32) * C32 + (uint32_t)a;         // < 6*2^32
    uint64_t u = (t >> 32) * C32 + (uint32_t)t;         // < 2^32 + 25
    return (uint32_t)u + C32 * (uint32_t)(u >> 32);
}

QK_HD uint32_t add32(uint32_t a, uint32_t b) {          // a, b canonical -> canonical
    uint64_t s = (uint64_t)a + b;                       // < 2p
    return (uint32_t)(s >= P32 ? s - P32 : s);
}
QK_HD uint32_t sub32(uint32_t a, uint32_t b) {          // a, b canonical -> canonical
    return a >= b ? a - b : (uint32_t)((uint64_t)a + P32 - b);
}
QK_HD uint32_t mul32(uint32_t a, uint32_t b) { return canon32(mul32_lazy(a, b)); }
QK_HD uint32_t neg32(uint32_t a) { return a == 0 ? 0 : P32 - a; }
QK_HD uint32_t pow32(uint32_t a, uint64_t e) {
    uint32_t r = 1;
    while (e) {
        if (e & 1) r = mul32(r, a);
        a = mul32(a, a);
        e >>= 1;
    }
    return r;
}
QK_HD uint32_t inv32(uint32_t a) { return pow32(a, P32 - 2); } // a != 0

// ---------------------------------------------------------------- GF(p64)
QK_HD uint64_t canon64(uint64_t x) {                    // same argument, +59
    uint64_t a = x + C64;
    return a < x ? a : x;
}

// 64x64 -> 128 product as (hi, lo).
QK_HD void mul64_wide(uint64_t a, uint64_t b, uint64_t &hi, uint64_t &lo) {
    unsigned __int128 P = (unsigned __int128)a * b;
    hi = (uint64_t)(P >> 64);
    lo = (uint64_t)P;
}

// a, b < 2^64 (lazy) -> r < 2^64, r == a*b (mod p64).
QK_HD uint64_t mul64_lazy(uint64_t a, uint64_t b) {
    uint64_t H, L;
    mul64_wide(a, b, H, L);
    // t = H*59 + L < 59*2^64 + 2^64 = 60*2^64: t = th*2^64 + tl, th <= 59
    unsigned __int128 t = (unsigned __int128)H * C64 + L;
    uint64_t th = (uint64_t)(t >> 64), tl = (uint64_t)t;
    // u = th*59 + tl < 3481 + 2^64: u_hi in {0,1}; u_hi == 1 => u_lo < 3481
    unsigned __int128 u = (unsigned __int128)th * C64 + tl;
    return (uint64_t)u + C64 * (uint64_t)(u >> 64);
}

// a*b + c for a, b, c < 2^64 (lazy): (2^64-1)^2 + 2^64-1 < 2^128.
QK_HD uint64_t mad64_lazy(uint64_t a, uint64_t b, uint64_t c) {
    unsigned __int128 P = (unsigned __int128)a * b + c;
    uint64_t H = (uint64_t)(P >> 64), L = (uint64_t)P;
    unsigned __int128 t = (unsigned __int128)H * C64 + L;
    uint64_t th = (uint64_t)(t >> 64), tl = (uint64_t)t;
    unsigned __int128 u = (unsigned __int128)th * C64 + tl;
    return (uint64_t)u + C64 * (uint64_t)(u >> 64);
}

// ---- u64 "t-form": v = t0 + t1*2^32 + th*2^64 with th <= 59 ---------------
// With x = (x1:x0) and x59 = 59x mod p = (y1:y0) canonical (<= p-1), one step
// v <- v*x is P = (t1:t0)*x + th*x59 <= (2^64-1)(p-1) + 59(p-1) = (p-1)(2^64+58)
// < 2^128, then v' = P_L + 59*P_H < 60*2^64 (th' <= 59), congruent because
// th*x59 == th*59x == th*2^64*x (mod p).  Eight v_mad_u64_u32 in 32-bit limbs;
// every intermediate bound is noted (no carry can be lost).
QK_HD void tstep64(uint32_t &t0, uint32_t &t1, uint32_t &th, uint32_t x0, uint32_t x1, uint32_t y0, uint32_t y1) {
    const uint64_t c0 = (uint64_t)t0 * x0;                                   // < 2^64
    const uint64_t c1 = (uint64_t)t1 * x0 + (c0 >> 32);                      // <= 2^64 - 2^32
    const uint64_t c2 = (uint64_t)t0 * x1 + (uint32_t)c1;                    // <= 2^64 - 2^32
    const uint64_t c3 = (uint64_t)t1 * x1 + (c1 >> 32) + (c2 >> 32);         // <= 2^64 - 1
    const uint64_t d0 = (uint64_t)th * y0 + (uint32_t)c0;                    // < 2^38
    const uint64_t d1 = (uint64_t)th * y1 + (uint32_t)c2 + (d0 >> 32);       // < 2^38
    const uint64_t PH = c3 + (d1 >> 32);                                      // P < 2^128 => no wrap
    const uint64_t e0 = (uint64_t)(uint32_t)PH * C64 + (uint32_t)d0;          // < 2^38
    const uint64_t e1 = (uint64_t)(uint32_t)(PH >> 32) * C64 + (uint32_t)d1 + (e0 >> 32); // < 60*2^32
    t0 = (uint32_t)e0;
    t1 = (uint32_t)e1;
    th = (uint32_t)(e1 >> 32);
}

// Fold a 96-bit lazy accumulator hi*2^64 + lo (hi < 2^32) to [0, 2^64).
QK_HD uint64_t fold96_64(uint32_t hi, uint64_t lo) {
    unsigned __int128 t = (unsigned __int128)hi * C64 + lo;   // < 2^38 + 2^64
    uint64_t th = (uint64_t)(t >> 64), tl = (uint64_t)t;      // th <= 59... in fact <= 1
    unsigned __int128 u = (unsigned __int128)th * C64 + tl;
    return (uint64_t)u + C64 * (uint64_t)(u >> 64);
}

QK_HD uint64_t add64(uint64_t a, uint64_t b) {          // canonical -> canonical
    uint64_t s = a + b;
    // true sum < 2p < 2^65. Wrapped (s < a) => true = s + 2^64 >= p, result s + 59 (< p).
    if (s < a) return s + C64;
    return s >= P64 ? s - P64 : s;
}
QK_HD uint64_t sub64(uint64_t a, uint64_t b) {
    return a >= b ? a - b : a + (P64 - b);              // a < b: a + p - b < p, no wrap
}
QK_HD uint64_t mul64(uint64_t a, uint64_t b) { return canon64(mul64_lazy(a, b)); }
QK_HD uint64_t neg64(uint64_t a) { return a == 0 ? 0 : P64 - a; }
QK_HD uint64_t pow64(uint64_t a, uint64_t e) {
    uint64_t r = 1;
    while (e) {
        if (e & 1) r = mul64(r, a);
        a = mul64(a, a);
        e >>= 1;
    }
    return r;
}
QK_HD uint64_t inv64(uint64_t a) { return pow64(a, P64 - 2); }

// ------------------------------------------------------------- splitmix64
constexpr uint64_t GAMMA = 0x9E3779B97F4A7C15ull;
QK_HD uint64_t splitmix_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

} // namespace qk
