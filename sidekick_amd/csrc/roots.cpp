// roots.cpp — host root finding for the decode-missing root test.
//
// The reference decode (media_client.rs:304-313) evaluates the monic
// polynomial P(z) = z^d + c_1 z^(d-1) + ... + c_d of diff.to_coeffs() at every
// entry x of the sender's log and keeps the entries with P(x) == 0.  Over
// GF(p), P(x) == 0  <=>  (x mod p) is one of P's roots in GF(p), so the same
// hit list follows from the (at most d) roots of P and a set-membership scan
// of the log (decode.hip k_root_scan_*): O(d^2 log p) host work once, then
// O(1) per candidate instead of d Horner steps.  Bit-exact by construction:
// the roots found here are exactly {r in GF(p) : P(r) == 0}.
//
// Root finding (p = p32 = 2^32 - 5 or p64 = 2^64 - 59):
//   1. factors z^k of P give the root 0; divide them out (then P(0) != 0)
//   2. g = gcd(P, z^(p-1) - 1): the product of (z - r) over P's distinct
//      nonzero roots r in GF(p).  z^(p-1) is not formed directly:
//      z^(2^w) mod P takes w squarings (w = 32 / 64), and 2^w = p + c
//      (c = 5 / 59), so z^(2^w) - z^(c+1) = z^(c+1) (z^(p-1) - 1) and, z being
//      prime to P, gcd(P, z^(2^w) - z^(c+1)) = g
//   3. Cantor-Zassenhaus equal-degree splitting of g into linear factors,
//      L ways at once: for a random a, w = (z + a)^((p-1)/L) mod g takes the
//      value chi_L(r + a) (an L-th root of unity) at each root r, and
//      gcd(g, w - zeta^j) collects the roots of class j — first by j mod 4
//      (or 2) through powers of w, then class by class; recurse on the
//      classes; quadratics by the root formula.
// In the decode case P is a product of linear factors (the missing ids), so
// step 3 runs on P itself first (the fast path, no z^(2^w) exponentiation);
// only a P that will not split that way (roots outside GF(p): a corrupt or
// mismatched difference) takes steps 2-3.
// Polynomial products accumulate lazily (u32: folded 32x32 products in
// 64-bit lanes; u64: 52-bit-limb column sums on IFMA) and reduce each
// coefficient once; the reduction mod the degree-m modulus adds the top
// coefficients times a precomputed table of z^k mod f (k = m .. 2m-2), so a
// squaring is ~1.5 m^2 multiply-adds with no sequential chain.
#include "quack_hip.h"
#include "field.h"
#include "simd64.h"

#include <string.h>

#include <immintrin.h>

#include <algorithm>
#include <new>
#include <vector>

namespace {

using namespace qk;


static bool cpu_has_avx512() {
    static const int ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
                          __builtin_cpu_supports("avx512dq");
    return ok;
}

// l + 5 h of each 64-bit lane (2^32 == 5): a product < 2^64 -> < 6 * 2^32
QK_AVX512 static inline __m512i fold512(__m512i m) {
    const __m512i h = _mm512_srli_epi64(m, 32);
    return _mm512_add_epi64(_mm512_and_si512(m, _mm512_set1_epi64(0xFFFFFFFFll)),
                            _mm512_add_epi64(h, _mm512_slli_epi64(h, 2)));
}

constexpr size_t IPAD32 = 8;
// a = acc mod f for lazy product sums acc[0 .. 2m-1) (2 mb + 16 slots,
// 64-byte aligned): the coefficients k = m .. 2m-2 reduced once, then
// sum_k s_k (z^k mod f) from the table (t64: one row of mb per k) added into
// register sums per output vector — no top-down chain
QK_AVX512 static void red32_tab(uint32_t *a, size_t m, const uint64_t *t64, uint64_t *acc) {
    const size_t mb = (m + 7) & ~(size_t)7;
    alignas(64) uint64_t sv[1024 + 8];   // (m <= 1024: ModRing)
    for (size_t k = m; k + 1 < 2 * m; ++k) sv[k - m] = canon32(fold64_32(acc[k]));
    for (size_t v0 = 0; 8 * v0 < m; v0 += 4) {   // four independent sums per table row
        const size_t nv = std::min<size_t>(4, (m - 8 * v0 + 7) / 8);
        __m512i S[4];
        for (size_t u = 0; u < 4; ++u) S[u] = _mm512_load_si512(acc + 8 * (v0 + (u < nv ? u : 0)));
        for (size_t r = 0; r + 1 < m; ++r) {
            if (!sv[r]) continue;
            const __m512i x = _mm512_set1_epi64((long long)sv[r]);
            const uint64_t *t = t64 + r * mb + 8 * v0;
            for (size_t u = 0; u < 4; ++u) {
                if (u >= nv) break;
                S[u] = _mm512_add_epi64(S[u], fold512(_mm512_mul_epu32(x, _mm512_load_si512(t + 8 * u))));
            }
        }
        for (size_t u = 0; u < nv; ++u) _mm512_store_si512(acc + 8 * (v0 + u), S[u]);
    }
    for (size_t i = 0; i < m; ++i) a[i] = canon32(fold64_32(acc[i]));
}

// GF(p32) squaring mod a monic f of degree m on AVX-512: lazy sums of
// folded products (< 6 * 2^32 each, at most 2m per coefficient), eight 32x32
// products per vpmuludq.  The products a_i a_j (i < j, through 2 a_i) go to
// the aligned coefficient vector q with a window of a (j = 8q + lane - i;
// a64: IPAD32 zeros, a, zeros), so every read-modify-write hits the same
// aligned 64-byte vectors; the reduction adds s_k (z^k mod f) for
// k = m .. 2m-2 from a precomputed table (t64: one row of mb per k) into
// register sums per output vector — no top-down chain.  acc: 2 mb + 16
// slots, 64-byte aligned.
QK_AVX512 static void sqr32_avx512(uint32_t *a, size_t m, const uint64_t *t64, uint64_t *a64, uint64_t *acc) {
    const size_t mb = (m + 7) & ~(size_t)7;
    for (size_t i = 0; i < m; ++i) a64[IPAD32 + i] = a[i];
    for (size_t i = 0; i < 2 * mb + 16; i += 8) _mm512_store_si512(acc + i, _mm512_setzero_si512());
    for (size_t i = 0; i + 1 < m; ++i) {
        const uint64_t ai = a[i];
        if (!ai) continue;
        const __m512i b = _mm512_set1_epi64((long long)add32((uint32_t)ai, (uint32_t)ai));
        for (size_t q = (2 * i + 1) / 8; 8 * q <= i + m - 1; ++q) {
            const long long lowest = (long long)(8 * q) - (long long)i;   // j of lane 0
            const int skip = (int)((long long)i - lowest + 1);          // lanes with j <= i
            const __mmask8 mk = skip <= 0 ? (__mmask8)0xFF : (__mmask8)(0xFFu << skip);
            const __m512i x = _mm512_maskz_loadu_epi64(mk, a64 + IPAD32 + lowest);
            __m512i *dst = reinterpret_cast<__m512i *>(acc + 8 * q);
            _mm512_store_si512(dst, _mm512_add_epi64(_mm512_load_si512(dst), fold512(_mm512_mul_epu32(b, x))));
        }
    }
    // the diagonal after the vector sums (a scalar store into a vector the
    // next load reads whole would not forward)
    for (size_t i = 0; i < m; ++i) {
        const uint64_t sq = (uint64_t)a[i] * a[i];
        acc[2 * i] += (sq >> 32) * C32 + (uint32_t)sq;
    }
    red32_tab(a, m, t64, acc);
}

// GF(p32) product a <- a b mod f on AVX-512, the same lazy sums with every
// a_i against a window of b (b64: IPAD32 zeros, b, zeros; j = 8q + lane - i,
// out-of-range lanes read zeros): m products per coefficient at most
QK_AVX512 static void mul32_avx512(uint32_t *a, const uint32_t *b, size_t m, const uint64_t *t64, uint64_t *b64,
                                   uint64_t *acc) {
    const size_t mb = (m + 7) & ~(size_t)7;
    for (size_t i = 0; i < m; ++i) b64[IPAD32 + i] = b[i];
    for (size_t i = 0; i < 2 * mb + 16; i += 8) _mm512_store_si512(acc + i, _mm512_setzero_si512());
    for (size_t i = 0; i < m; ++i) {
        if (!a[i]) continue;
        const __m512i x = _mm512_set1_epi64((long long)a[i]);
        for (size_t q = i / 8; 8 * q <= i + m - 1; ++q) {
            const __m512i y = _mm512_loadu_si512(b64 + IPAD32 + (long long)(8 * q) - (long long)i);
            __m512i *dst = reinterpret_cast<__m512i *>(acc + 8 * q);
            _mm512_store_si512(dst, _mm512_add_epi64(_mm512_load_si512(dst), fold512(_mm512_mul_epu32(x, y))));
        }
    }
    red32_tab(a, m, t64, acc);
}

// ---- row operations of the Euclid / division loops, u32 on AVX-512 -------
// canonical a * b over eight 64-bit lanes (a, b < p): two folds leave
// < 2^32 + 25, one conditional subtraction makes it canonical
QK_AVX512 static inline __m512i mulc512(__m512i a, __m512i b) {
    const __m512i P = _mm512_set1_epi64(P32);
    const __m512i r = fold512(fold512(_mm512_mul_epu32(a, b)));
    return _mm512_mask_sub_epi64(r, _mm512_cmpge_epu64_mask(r, P), r, P);
}
QK_AVX512 static inline __m512i subc512(__m512i a, __m512i b) {   // canonical a - b
    const __m512i d = _mm512_sub_epi64(a, b);
    return _mm512_mask_add_epi64(d, _mm512_cmplt_epu64_mask(a, b), d, _mm512_set1_epi64(P32));
}
QK_AVX512 static inline __m512i addc512(__m512i a, __m512i b) {   // canonical a + b
    const __m512i P = _mm512_set1_epi64(P32);
    const __m512i r = _mm512_add_epi64(a, b);
    return _mm512_mask_sub_epi64(r, _mm512_cmpge_epu64_mask(r, P), r, P);
}
QK_AVX512 static inline __m512i ld8(const uint32_t *p, size_t rem) {
    const __mmask8 m = rem >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << rem) - 1u);
    return _mm512_cvtepu32_epi64(_mm256_maskz_loadu_epi32(m, p));
}
QK_AVX512 static inline void st8(uint32_t *p, size_t rem, __m512i v) {
    const __mmask8 m = rem >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << rem) - 1u);
    _mm512_mask_cvtepi64_storeu_epi32(p, m, v);
}
// d[i] = alpha d[i] - beta s[i], i < m (alpha = 1: d[i] - beta s[i])
QK_AVX512 static void axmy32_avx512(uint32_t *d, const uint32_t *s, size_t m, uint32_t alpha, uint32_t beta) {
    const __m512i A = _mm512_set1_epi64(alpha), B = _mm512_set1_epi64(beta);
    for (size_t i = 0; i < m; i += 8) {
        const size_t r = m - i;
        __m512i x = ld8(d + i, r);
        if (alpha != 1) x = mulc512(x, A);
        st8(d + i, r, subc512(x, mulc512(ld8(s + i, r), B)));
    }
}
// a <- a (z + c) mod f: out[i] = a[i-1] + c a[i] + top nf[i]  (a[-1] = 0)
QK_AVX512 static void mullin32_avx512(uint32_t *a, size_t m, uint32_t c, const uint32_t *nf, uint32_t *tmp) {
    const uint32_t top = a[m - 1];
    tmp[0] = 0;
    for (size_t i = 1; i < m; ++i) tmp[i] = a[i - 1];
    const __m512i C = _mm512_set1_epi64(c), Tp = _mm512_set1_epi64(top);
    for (size_t i = 0; i < m; i += 8) {
        const size_t r = m - i;
        __m512i v = addc512(ld8(tmp + i, r), mulc512(ld8(a + i, r), C));
        if (top) v = addc512(v, mulc512(ld8(nf + i, r), Tp));
        st8(a + i, r, v);
    }
}

// ---- the u64 field (p64) on AVX-512: rows and the squaring --------------
// Lane products by simd64.h's mulmod64_512 (four vpmuludq, lazy < 2^64).
QK_AVX512 static inline __m512i ld8q(const uint64_t *p, size_t rem) {
    return rem >= 8 ? _mm512_loadu_si512(p) : _mm512_maskz_loadu_epi64((__mmask8)((1u << rem) - 1u), p);
}
QK_AVX512 static inline void st8q(uint64_t *p, size_t rem, __m512i v) {
    if (rem >= 8) _mm512_storeu_si512(p, v);
    else _mm512_mask_storeu_epi64(p, (__mmask8)((1u << rem) - 1u), v);
}
// d[i] = alpha d[i] - beta s[i], i < m (alpha = 1: d[i] - beta s[i])
QK_AVX512 static void axmy64_avx512(uint64_t *d, const uint64_t *s, size_t m, uint64_t alpha, uint64_t beta) {
    const __m512i A0 = simd::lo32x8(alpha), A1 = simd::hi32x8(alpha), B0 = simd::lo32x8(beta),
                  B1 = simd::hi32x8(beta);
    for (size_t i = 0; i < m; i += 8) {
        const size_t r = m - i;
        __m512i x = ld8q(d + i, r);
        if (alpha != 1) x = simd::canon64_512(simd::mulmod64_512(x, A0, A1));
        const __m512i y = simd::canon64_512(simd::mulmod64_512(ld8q(s + i, r), B0, B1));
        st8q(d + i, r, simd::sub64_512(x, y));
    }
}
// (lo, cnt) lanes += v: a lazy sum lo + cnt 2^64 (the carry restored by a compare)
QK_AVX512 static inline void addc64_512(uint64_t *lo, uint64_t *cnt, __m512i v) {
    const __m512i s = _mm512_add_epi64(_mm512_loadu_si512(lo), v);
    const __mmask8 c = _mm512_cmplt_epu64_mask(s, v);
    _mm512_storeu_si512(lo, s);
    const __m512i k = _mm512_loadu_si512(cnt);
    _mm512_storeu_si512(cnt, _mm512_mask_add_epi64(k, c, k, _mm512_set1_epi64(1)));
}
// lo + cnt 2^64 mod p, canonical (cnt small: 2^64 == 59)
static inline uint64_t red_lc(uint64_t lo, uint64_t cnt) {
    uint64_t s = lo + C64 * cnt;
    if (s < lo) s += C64;
    return canon64(s);
}
// GF(p64) squaring mod a monic f of degree m on AVX-512: products a_i a_j
// (i < j, doubled through 2 a_i) as lazy lane products summed into 64-bit
// lanes whose carries are counted, the top-down reduction by -f the same
// way, one canonical reduction per coefficient.  a64 / nf64 hold a and -f
// zero-padded to a multiple of 8 past m; lo / cnt have 2m + 16 slots.
QK_AVX512 static void sqr64_avx512(uint64_t *a, size_t m, const uint64_t *nf64, uint64_t *a64, uint64_t *lo,
                                   uint64_t *cnt) {
    const size_t mb = (m + 7) & ~(size_t)7;
    for (size_t i = 0; i < m; ++i) a64[i] = a[i];
    for (size_t i = m; i < mb + 8; ++i) a64[i] = 0;
    for (size_t i = 0; i < 2 * m + 16; ++i) lo[i] = cnt[i] = 0;
    for (size_t i = 0; i < m; ++i) {
        const uint64_t ai = a[i];
        if (!ai) continue;
        const uint64_t sq = mul64_lazy(ai, ai), o = lo[2 * i];
        lo[2 * i] = o + sq;
        cnt[2 * i] += lo[2 * i] < sq;
        const uint64_t a2 = add64(ai, ai);
        const __m512i A0 = simd::lo32x8(a2), A1 = simd::hi32x8(a2);
        for (size_t j = i + 1; j < m; j += 8)
            addc64_512(lo + i + j, cnt + i + j, simd::mulmod64_512(_mm512_loadu_si512(a64 + j), A0, A1));
    }
    for (size_t k = 2 * m - 1; k-- > m;) {
        const uint64_t q = red_lc(lo[k], cnt[k]);
        if (!q) continue;
        const __m512i Q0 = simd::lo32x8(q), Q1 = simd::hi32x8(q);
        for (size_t i = 0; i < m; i += 8)
            addc64_512(lo + k - m + i, cnt + k - m + i, simd::mulmod64_512(_mm512_loadu_si512(nf64 + i), Q0, Q1));
    }
    for (size_t i = 0; i < m; ++i) a[i] = red_lc(lo[i], cnt[i]);
}

// The same products on AVX-512 IFMA (52-bit limbs): a = l0 + l1 2^52
// (l1 < 2^12), and every product goes into three column sums of weights 1,
// 2^52 and 2^104 with seven vpmadd52{lo,hi}uq — no reduction per product;
// one reduction per eight coefficients (2^104 == 59 2^40).  A squaring sums
// the products a_i a_j (i < j) once and doubles the columns before the
// diagonal is added; the reduction mod f adds s_k (z^k mod f) from a table.
// Bounds: a column takes at most 2m products (m from the product, m - 1
// from the reduction, + the diagonal), i.e. 2m terms of < 2^52 in the
// low column, 6m in the middle one (< 2^64 needs m <= 682: IFMA_MAX) and 2m
// of < 2^25 in the top one (< 2^36; red_cols8 takes it as 64 bits).
#define QK_IFMA __attribute__((target("avx512f,avx512vl,avx512dq,avx512ifma")))
static bool cpu_has_ifma() {
    static const int ok = cpu_has_avx512() && __builtin_cpu_supports("avx512ifma");
    return ok;
}
constexpr uint64_t M52 = (1ull << 52) - 1;
constexpr size_t IFMA_MAX = 640;   // the largest modulus degree of the IFMA products
// the canonical values of column sums c0 + c1 2^52 + c2 2^104 on eight
// lanes: lo + hi 2^64 = c0 + c1 2^52 + c2 59 2^40 (2^104 == 59 2^40) with
// the carries restored by compares, then hi 2^64 == 59 hi (hi < 2^50)
QK_IFMA static inline __m512i red_cols8(__m512i c0, __m512i c1, __m512i c2) {
    const __m512i one = _mm512_set1_epi64(1), c59 = _mm512_set1_epi64(59);
    const __m512i lo1 = _mm512_add_epi64(c0, _mm512_slli_epi64(c1, 52));
    __m512i hi = _mm512_srli_epi64(c1, 12);
    hi = _mm512_mask_add_epi64(hi, _mm512_cmplt_epu64_mask(lo1, c0), hi, one);
    const __m512i w = _mm512_mullo_epi64(c2, c59);   // c2 < 2^58
    const __m512i lo = _mm512_add_epi64(lo1, _mm512_slli_epi64(w, 40));
    hi = _mm512_add_epi64(hi, _mm512_srli_epi64(w, 24));
    hi = _mm512_mask_add_epi64(hi, _mm512_cmplt_epu64_mask(lo, lo1), hi, one);
    const __m512i s = _mm512_add_epi64(lo, _mm512_mullo_epi64(hi, c59));
    __m512i r = _mm512_mask_add_epi64(s, _mm512_cmplt_epu64_mask(s, lo), s, c59);
    const __m512i P = _mm512_set1_epi64((long long)P64);
    return _mm512_mask_sub_epi64(r, _mm512_cmpge_epu64_mask(r, P), r, P);
}

// the aligned columns c[8q .. 8q+8) += x * y over eight lanes (x's limbs
// broadcast, y a window of limbs): every read-modify-write hits the same
// aligned 64-byte vectors, so a store forwards to the next load of it
QK_IFMA static inline void fma52x8(uint64_t *c0, uint64_t *c1, uint64_t *c2, __m512i x0, __m512i x1, __m512i y0,
                                   __m512i y1) {
    __m512i a = _mm512_load_si512(c0), b = _mm512_load_si512(c1), c = _mm512_load_si512(c2);
    a = _mm512_madd52lo_epu64(a, x0, y0);
    b = _mm512_madd52hi_epu64(b, x0, y0);
    b = _mm512_madd52lo_epu64(b, x0, y1);
    b = _mm512_madd52lo_epu64(b, x1, y0);
    c = _mm512_madd52hi_epu64(c, x0, y1);
    c = _mm512_madd52hi_epu64(c, x1, y0);
    c = _mm512_madd52lo_epu64(c, x1, y1);
    _mm512_store_si512(c0, a);
    _mm512_store_si512(c1, b);
    _mm512_store_si512(c2, c);
}
constexpr size_t IPAD = 8;   // zero limbs before index 0 of the limb arrays
// a = the columns mod f (c0 / c1 / c2: 2 mb + 16 column sums of the
// product, 64-byte aligned): z^k mod f for k = m .. 2m-2 is precomputed
// (tl0 / tl1: row k - m, mb limbs each), so the result is the low columns
// plus sum_k s_k (z^k mod f) — every s_k a canonical value of the product
// columns alone, the sums in registers per output vector
QK_IFMA static void red64_tab(uint64_t *a, size_t m, const uint64_t *tl0, const uint64_t *tl1, const uint64_t *c0,
                              const uint64_t *c1, const uint64_t *c2) {
    const size_t mb = (m + 7) & ~(size_t)7;
    alignas(64) uint64_t s0[1024 + 8], s1[1024 + 8];   // (m <= 1024: ModRing)
    const __m512i mk52 = _mm512_set1_epi64((long long)M52);
    for (size_t k = m; k + 1 < 2 * m; k += 8) {   // (lanes past 2m - 2 read zero columns)
        const __m512i v = red_cols8(_mm512_loadu_si512(c0 + k), _mm512_loadu_si512(c1 + k), _mm512_loadu_si512(c2 + k));
        _mm512_store_si512(s0 + (k - m), _mm512_and_si512(v, mk52));
        _mm512_store_si512(s1 + (k - m), _mm512_srli_epi64(v, 52));
    }
    // four output vectors at a time, and each weight's three IFMAs of a row
    // split over two accumulators (B / B2, C / C2, summed at the end): per
    // row a chain of at most two dependent IFMAs per accumulator instead of
    // three, below the unit's issue time for the row's 28
    for (size_t v0 = 0; 8 * v0 < m; v0 += 4) {
        const size_t nv = std::min<size_t>(4, (m - 8 * v0 + 7) / 8);
        __m512i A[4], B[4], C[4], B2[4], C2[4];
        for (size_t u = 0; u < 4; ++u) {
            const size_t o = 8 * (v0 + (u < nv ? u : 0));
            A[u] = _mm512_load_si512(c0 + o), B[u] = _mm512_load_si512(c1 + o), C[u] = _mm512_load_si512(c2 + o);
            B2[u] = C2[u] = _mm512_setzero_si512();
        }
        for (size_t r = 0; r + 1 < m; ++r) {
            const __m512i x0 = _mm512_set1_epi64((long long)s0[r]), x1 = _mm512_set1_epi64((long long)s1[r]);
            const uint64_t *t0 = tl0 + r * mb + 8 * v0, *t1 = tl1 + r * mb + 8 * v0;
            for (size_t u = 0; u < 4; ++u) {
                if (u >= nv) break;
                const __m512i y0 = _mm512_load_si512(t0 + 8 * u), y1 = _mm512_load_si512(t1 + 8 * u);
                A[u] = _mm512_madd52lo_epu64(A[u], x0, y0);
                B[u] = _mm512_madd52hi_epu64(B[u], x0, y0);
                C[u] = _mm512_madd52hi_epu64(C[u], x0, y1);
                B2[u] = _mm512_madd52lo_epu64(B2[u], x0, y1);
                C2[u] = _mm512_madd52hi_epu64(C2[u], x1, y0);
                B[u] = _mm512_madd52lo_epu64(B[u], x1, y0);
                C[u] = _mm512_madd52lo_epu64(C[u], x1, y1);
            }
        }
        for (size_t u = 0; u < nv; ++u) {
            B[u] = _mm512_add_epi64(B[u], B2[u]);
            C[u] = _mm512_add_epi64(C[u], C2[u]);
            const __m512i r = red_cols8(A[u], B[u], C[u]);
            const size_t v = v0 + u, rem = m - 8 * v;
            if (rem >= 8) _mm512_storeu_si512(a + 8 * v, r);
            else _mm512_mask_storeu_epi64(a + 8 * v, (__mmask8)((1u << rem) - 1u), r);
        }
    }
}

// l0 / l1: a's limbs (IPAD zeros, the m limbs, zeros to IPAD + mb + 16);
// tl0 / tl1: the limbs of z^k mod f, k = m .. 2m-2, one row of mb per k,
// 64-byte aligned; c0 / c1 / c2: 2 mb + 16 column sums, 64-byte aligned
QK_IFMA static void sqr64_ifma(uint64_t *a, size_t m, const uint64_t *tl0, const uint64_t *tl1, uint64_t *l0,
                               uint64_t *l1, uint64_t *c0, uint64_t *c1, uint64_t *c2) {
    const size_t mb = (m + 7) & ~(size_t)7;
    for (size_t i = 0; i < m; ++i) {
        l0[IPAD + i] = a[i] & M52;
        l1[IPAD + i] = a[i] >> 52;
    }
    for (size_t i = 0; i < 2 * mb + 16; ++i) c0[i] = c1[i] = c2[i] = 0;
    // off-diagonal products a_i a_j, i < j: column vector q gets j = 8q + lane - i
    for (size_t i = 0; i + 1 < m; ++i) {
        if (!a[i]) continue;
        const __m512i x0 = _mm512_set1_epi64((long long)(a[i] & M52)), x1 = _mm512_set1_epi64((long long)(a[i] >> 52));
        for (size_t q = (2 * i + 1) / 8; 8 * q <= i + m - 1; ++q) {
            const long long lowest = (long long)(8 * q) - (long long)i;   // j of lane 0
            // lanes with j <= i take no product
            const int skip = (int)((long long)i - lowest + 1);
            const __mmask8 mk = skip <= 0 ? (__mmask8)0xFF : (__mmask8)(0xFFu << skip);
            const uint64_t *w0 = l0 + IPAD + lowest, *w1 = l1 + IPAD + lowest;
            fma52x8(c0 + 8 * q, c1 + 8 * q, c2 + 8 * q, x0, x1, _mm512_maskz_loadu_epi64(mk, w0),
                    _mm512_maskz_loadu_epi64(mk, w1));
        }
    }
    for (size_t k = 0; k < 2 * mb; k += 8) {   // double the off-diagonal sums
        _mm512_store_si512(c0 + k, _mm512_slli_epi64(_mm512_load_si512(c0 + k), 1));
        _mm512_store_si512(c1 + k, _mm512_slli_epi64(_mm512_load_si512(c1 + k), 1));
        _mm512_store_si512(c2 + k, _mm512_slli_epi64(_mm512_load_si512(c2 + k), 1));
    }
    for (size_t i = 0; i < m; ++i) {   // the diagonal a_i^2 = l0^2 + 2 l0 l1 2^52 + l1^2 2^104
        const uint64_t u0 = a[i] & M52, u1 = a[i] >> 52;
        const unsigned __int128 p0 = (unsigned __int128)u0 * u0;
        const uint64_t v = u0 * u1;   // < 2^64
        c0[2 * i] += (uint64_t)p0 & M52;
        c1[2 * i] += (uint64_t)(p0 >> 52) + 2 * (v & M52);
        c2[2 * i] += 2 * (v >> 52) + u1 * u1;
    }
    red64_tab(a, m, tl0, tl1, c0, c1, c2);
}

// The same squaring with the product's column sums in registers (NQ = 2 mb /
// 8 <= 8 column vectors of each weight: 24 zmm at mb = 32): sqr64_ifma's
// per-(i, q) load-madd-store of the column vectors chains every row of a
// column through store-to-load forwarding; here the rows of one column are
// only a chain of register madds, and a column vector leaves (with its
// diagonal terms added) as soon as the last row reaching it is done, so at
// most ~5 column vectors are live.  The limbs and the diagonal are vector
// operations (scalar stores under vector loads do not forward).
template <int NQ>
QK_IFMA static void sqr64_ifma_reg(uint64_t *a, size_t m, const uint64_t *tl0, const uint64_t *tl1, uint64_t *l0,
                                   uint64_t *l1, uint64_t *c0, uint64_t *c1, uint64_t *c2) {
    const __m512i mk52 = _mm512_set1_epi64((long long)M52);
    for (size_t k = 0; k < m; k += 8) {   // the limbs, vector by vector
        const __mmask8 mk = m - k >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << (m - k)) - 1u);
        const __m512i v = _mm512_maskz_loadu_epi64(mk, a + k);
        _mm512_mask_storeu_epi64(l0 + IPAD + k, mk, _mm512_and_si512(v, mk52));
        _mm512_mask_storeu_epi64(l1 + IPAD + k, mk, _mm512_srli_epi64(v, 52));
    }
    __m512i A[NQ], B[NQ], C[NQ];
    for (int q = 0; q < NQ; ++q) A[q] = B[q] = C[q] = _mm512_setzero_si512();
    // rows i = 4s .. 4s+3 start at column vector s (their first product
    // a_i a_(i+1) lands in column 2i + 1): that vector takes a fixed lane
    // mask (j > i: lanes above 2t for i = 4s + t), the later ones full loads
#pragma GCC unroll 8
    for (int s = 0; s < NQ; ++s) {
#pragma GCC unroll 4
        for (int t = 0; t < 4; ++t) {
            const size_t i = 4 * (size_t)s + t;
            if (i + 1 >= m) break;
            if (!a[i]) continue;
            const __m512i x0 = _mm512_set1_epi64((long long)(a[i] & M52)),
                          x1 = _mm512_set1_epi64((long long)(a[i] >> 52));
            const int qhi = (int)((i + m - 1) / 8);
            const __mmask8 mk = (__mmask8)(0xFFu << (2 * t + 1));
            const uint64_t *w0 = l0 + IPAD + 8 * s - i, *w1 = l1 + IPAD + 8 * s - i;
            __m512i y0 = _mm512_maskz_loadu_epi64(mk, w0), y1 = _mm512_maskz_loadu_epi64(mk, w1);
#pragma GCC unroll 8
            for (int q = s; q < NQ; ++q) {
                if (q > qhi) break;
                if (q > s) {
                    y0 = _mm512_loadu_si512(w0 + 8 * (q - s));
                    y1 = _mm512_loadu_si512(w1 + 8 * (q - s));
                }
                A[q] = _mm512_madd52lo_epu64(A[q], x0, y0);
                B[q] = _mm512_madd52hi_epu64(B[q], x0, y0);
                C[q] = _mm512_madd52hi_epu64(C[q], x0, y1);
                B[q] = _mm512_madd52lo_epu64(B[q], x0, y1);
                C[q] = _mm512_madd52hi_epu64(C[q], x1, y0);
                B[q] = _mm512_madd52lo_epu64(B[q], x1, y0);
                C[q] = _mm512_madd52lo_epu64(C[q], x1, y1);
            }
        }
        // column vector s is complete (later rows start above it): its
        // doubled off-diagonal sums plus the diagonal a_i^2 (i = 4s .. 4s+3,
        // in the even lanes: u0^2 + 2 u0 u1 2^52 + u1^2 2^104 as lo / hi of
        // u0 u0, u0 (2 u1) and u1 u1) go out, and its registers are free
        const __m512i dix = _mm512_set_epi64(3, 3, 2, 2, 1, 1, 0, 0);
        const __m512i d0 = _mm512_maskz_permutexvar_epi64((__mmask8)0x55, dix, _mm512_loadu_si512(l0 + IPAD + 4 * s)),
                      d1 = _mm512_maskz_permutexvar_epi64((__mmask8)0x55, dix, _mm512_loadu_si512(l1 + IPAD + 4 * s)),
                      d1x2 = _mm512_add_epi64(d1, d1);
        _mm512_store_si512(c0 + 8 * s, _mm512_madd52lo_epu64(_mm512_slli_epi64(A[s], 1), d0, d0));
        _mm512_store_si512(c1 + 8 * s,
                           _mm512_madd52lo_epu64(_mm512_madd52hi_epu64(_mm512_slli_epi64(B[s], 1), d0, d0), d0, d1x2));
        _mm512_store_si512(c2 + 8 * s,
                           _mm512_madd52lo_epu64(_mm512_madd52hi_epu64(_mm512_slli_epi64(C[s], 1), d0, d1x2), d1, d1));
    }
    for (size_t k = 8 * NQ; k < 8 * NQ + 16; ++k) c0[k] = c1[k] = c2[k] = 0;
    red64_tab(a, m, tl0, tl1, c0, c1, c2);
}

// a <- a b mod f on IFMA: every a_i against a window of b's limbs (l0 /
// l1 hold b: IPAD zeros, b, zeros; out-of-range lanes read zeros), then
// red64_tab
QK_IFMA static void mul64_ifma(uint64_t *a, const uint64_t *b, size_t m, const uint64_t *tl0, const uint64_t *tl1,
                               uint64_t *l0, uint64_t *l1, uint64_t *c0, uint64_t *c1, uint64_t *c2) {
    const size_t mb = (m + 7) & ~(size_t)7;
    for (size_t i = 0; i < m; ++i) {
        l0[IPAD + i] = b[i] & M52;
        l1[IPAD + i] = b[i] >> 52;
    }
    for (size_t i = 0; i < 2 * mb + 16; ++i) c0[i] = c1[i] = c2[i] = 0;
    for (size_t i = 0; i < m; ++i) {
        if (!a[i]) continue;
        const __m512i x0 = _mm512_set1_epi64((long long)(a[i] & M52)), x1 = _mm512_set1_epi64((long long)(a[i] >> 52));
        for (size_t q = i / 8; 8 * q <= i + m - 1; ++q) {
            const long long lowest = (long long)(8 * q) - (long long)i;
            fma52x8(c0 + 8 * q, c1 + 8 * q, c2 + 8 * q, x0, x1, _mm512_loadu_si512(l0 + IPAD + lowest),
                    _mm512_loadu_si512(l1 + IPAD + lowest));
        }
    }
    red64_tab(a, m, tl0, tl1, c0, c1, c2);
}

// The product in registers, as sqr64_ifma_reg: rows i = 8s .. 8s+7 start
// at column vector s (windows below b's first limb read IPAD zeros), and a
// column vector leaves once the last row reaching it is done.
template <int NQ>
QK_IFMA static void mul64_ifma_reg(uint64_t *a, const uint64_t *b, size_t m, const uint64_t *tl0,
                                   const uint64_t *tl1, uint64_t *l0, uint64_t *l1, uint64_t *c0, uint64_t *c1,
                                   uint64_t *c2) {
    const __m512i mk52 = _mm512_set1_epi64((long long)M52);
    for (size_t k = 0; k < m; k += 8) {
        const __mmask8 mk = m - k >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << (m - k)) - 1u);
        const __m512i v = _mm512_maskz_loadu_epi64(mk, b + k);
        _mm512_mask_storeu_epi64(l0 + IPAD + k, mk, _mm512_and_si512(v, mk52));
        _mm512_mask_storeu_epi64(l1 + IPAD + k, mk, _mm512_srli_epi64(v, 52));
    }
    __m512i A[NQ], B[NQ], C[NQ];
    for (int q = 0; q < NQ; ++q) A[q] = B[q] = C[q] = _mm512_setzero_si512();
#pragma GCC unroll 8
    for (int s = 0; s < NQ; ++s) {
#pragma GCC unroll 8
        for (int t = 0; t < 8; ++t) {
            const size_t i = 8 * (size_t)s + t;
            if (i >= m) break;
            if (!a[i]) continue;
            const __m512i x0 = _mm512_set1_epi64((long long)(a[i] & M52)),
                          x1 = _mm512_set1_epi64((long long)(a[i] >> 52));
            const int qhi = (int)((i + m - 1) / 8);
            const uint64_t *w0 = l0 + IPAD + 8 * s - i, *w1 = l1 + IPAD + 8 * s - i;
#pragma GCC unroll 8
            for (int q = s; q < NQ; ++q) {
                if (q > qhi) break;
                const __m512i y0 = _mm512_loadu_si512(w0 + 8 * (q - s)), y1 = _mm512_loadu_si512(w1 + 8 * (q - s));
                A[q] = _mm512_madd52lo_epu64(A[q], x0, y0);
                B[q] = _mm512_madd52hi_epu64(B[q], x0, y0);
                C[q] = _mm512_madd52hi_epu64(C[q], x0, y1);
                B[q] = _mm512_madd52lo_epu64(B[q], x0, y1);
                C[q] = _mm512_madd52hi_epu64(C[q], x1, y0);
                B[q] = _mm512_madd52lo_epu64(B[q], x1, y0);
                C[q] = _mm512_madd52lo_epu64(C[q], x1, y1);
            }
        }
        _mm512_store_si512(c0 + 8 * s, A[s]);
        _mm512_store_si512(c1 + 8 * s, B[s]);
        _mm512_store_si512(c2 + 8 * s, C[s]);
    }
    for (size_t k = 8 * NQ; k < 8 * NQ + 16; ++k) c0[k] = c1[k] = c2[k] = 0;
    red64_tab(a, m, tl0, tl1, c0, c1, c2);
}

// axmy / scale for the u64 field on IFMA: alpha d + (p - beta) s as column
// sums of 52-bit limb products, one red_cols8 per eight coefficients
QK_IFMA static inline void split52(__m512i v, __m512i &l0, __m512i &l1) {
    l0 = _mm512_and_si512(v, _mm512_set1_epi64((long long)M52));
    l1 = _mm512_srli_epi64(v, 52);
}
QK_IFMA static inline void prod52(__m512i &A, __m512i &B, __m512i &C, __m512i x0, __m512i x1, __m512i y0,
                                  __m512i y1) {
    A = _mm512_madd52lo_epu64(A, x0, y0);
    B = _mm512_madd52hi_epu64(B, x0, y0);
    B = _mm512_madd52lo_epu64(B, x0, y1);
    B = _mm512_madd52lo_epu64(B, x1, y0);
    C = _mm512_madd52hi_epu64(C, x0, y1);
    C = _mm512_madd52hi_epu64(C, x1, y0);
    C = _mm512_madd52lo_epu64(C, x1, y1);
}
QK_IFMA static void axmy64_ifma(uint64_t *d, const uint64_t *s, size_t m, uint64_t alpha, uint64_t beta) {
    const uint64_t nb = beta ? P64 - beta : 0;
    const __m512i a0 = _mm512_set1_epi64((long long)(alpha & M52)), a1 = _mm512_set1_epi64((long long)(alpha >> 52)),
                  b0 = _mm512_set1_epi64((long long)(nb & M52)), b1 = _mm512_set1_epi64((long long)(nb >> 52));
    for (size_t i = 0; i < m; i += 8) {
        const size_t r = m - i;
        __m512i d0, d1, s0, s1;
        split52(ld8q(d + i, r), d0, d1);
        split52(ld8q(s + i, r), s0, s1);
        __m512i A = _mm512_setzero_si512(), B = A, C = A;
        prod52(A, B, C, a0, a1, d0, d1);
        prod52(A, B, C, b0, b1, s0, s1);
        st8q(d + i, r, red_cols8(A, B, C));
    }
}

// a <- a (z + c) mod f on IFMA: out[i] = a[i-1] + c a[i] + top nf[i] as
// column sums (a[i-1]'s limbs added to the low two columns)
// The shifted a (a[i-1]) is an unaligned load one slot down (the first
// vector: a's lanes moved up one by valignq); the vectors go from the top down, so each reads
// its window before the store of the vector below it overwrites a slot of
// it.  c = 0 (the reduction table's z z^k): no c a product.
QK_IFMA static void mullin64_ifma(uint64_t *a, size_t m, uint64_t c, const uint64_t *nf, uint64_t *tmp) {
    (void)tmp;
    const uint64_t top = a[m - 1];
    const __m512i c0 = _mm512_set1_epi64((long long)(c & M52)), c1 = _mm512_set1_epi64((long long)(c >> 52)),
                  t0 = _mm512_set1_epi64((long long)(top & M52)), t1 = _mm512_set1_epi64((long long)(top >> 52));
    for (size_t i = (m - 1) & ~(size_t)7;; i -= 8) {
        const size_t r = m - i;
        const __mmask8 mk = r >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << r) - 1u);
        __m512i a0, a1, n0, n1, A, B;
        const __m512i sh = i ? _mm512_maskz_loadu_epi64(mk, a + i - 1)   // (lane 0 of the first: a[-1] = 0)
                             : _mm512_alignr_epi64(_mm512_maskz_loadu_epi64(mk, a), _mm512_setzero_si512(), 7);
        split52(sh, A, B);
        split52(ld8q(nf + i, r), n0, n1);
        __m512i C = _mm512_setzero_si512();
        if (c) {
            split52(ld8q(a + i, r), a0, a1);
            prod52(A, B, C, c0, c1, a0, a1);
        }
        prod52(A, B, C, t0, t1, n0, n1);
        st8q(a + i, r, red_cols8(A, B, C));
        if (!i) break;
    }
}

template <class F> static inline bool vec32(size_t m) {
    if constexpr (F::W == 32) return m >= 8 && cpu_has_avx512();
    else return false;
}
template <class F> static inline bool vec64(size_t m) {
    if constexpr (F::W == 64) return m >= 8 && cpu_has_avx512();
    else return false;
}

// d[i] = alpha d[i] - beta s[i] mod p, i < m
template <class F>
static void axmy(typename F::T *d, const typename F::T *s, size_t m, typename F::T alpha, typename F::T beta) {
    if constexpr (F::W == 32) {
        if (vec32<F>(m)) return axmy32_avx512(d, s, m, alpha, beta);
    } else {
        if (vec64<F>(m)) return cpu_has_ifma() ? axmy64_ifma(d, s, m, alpha, beta) : axmy64_avx512(d, s, m, alpha, beta);
    }
    for (size_t i = 0; i < m; ++i) d[i] = F::sub(alpha == 1 ? d[i] : F::mul(d[i], alpha), F::mul(beta, s[i]));
}

// Field inverses by fixed addition chains on lazy products (every found
// factor is made monic, so the split pays ~one inverse per root):
// p32 - 2 = (2^29 - 1) 2^3 + 1: 31 squarings + 8 products (the binary
// ladder: 31 + 29); p64 - 2 = (2^58 - 1) 2^6 + 3: 63 + 9 (ladder: 63 + 60).
template <class U, U (*MUL)(U, U)> static inline U sqr_n(U x, int k) {
    while (k--) x = MUL(x, x);
    return x;
}
static uint32_t inv32_chain(uint32_t a) {
    constexpr auto S = sqr_n<uint32_t, mul32_lazy>;
    const uint32_t x2 = mul32_lazy(S(a, 1), a), x4 = mul32_lazy(S(x2, 2), x2), x8 = mul32_lazy(S(x4, 4), x4);
    const uint32_t x16 = mul32_lazy(S(x8, 8), x8), x24 = mul32_lazy(S(x16, 8), x8), x28 = mul32_lazy(S(x24, 4), x4);
    const uint32_t x29 = mul32_lazy(S(x28, 1), a);
    return canon32(mul32_lazy(S(x29, 3), a));
}
static uint64_t inv64_chain(uint64_t a) {
    constexpr auto S = sqr_n<uint64_t, mul64_lazy>;
    const uint64_t x2 = mul64_lazy(S(a, 1), a), x4 = mul64_lazy(S(x2, 2), x2), x8 = mul64_lazy(S(x4, 4), x4);
    const uint64_t x16 = mul64_lazy(S(x8, 8), x8), x32 = mul64_lazy(S(x16, 16), x16);
    const uint64_t x48 = mul64_lazy(S(x32, 16), x16), x56 = mul64_lazy(S(x48, 8), x8), x58 = mul64_lazy(S(x56, 2), x2);
    return canon64(mul64_lazy(S(x58, 6), x2));
}

// splitting arity per field (a divisor of p - 1; p32 - 1 = 2 5 19 ...,
// p64 - 1 = 4 11 137 ...).  With the power-of-two cuts first (Splitter),
// d = 32 on one Xeon core (tools/prof_roots.cpp): u32
// 10 / 19 / 38 / 190-way 67 / 76 / 56 / 144 us, u64 4 / 11 / 22 / 44 /
// 548-way 274 / 184 / 112 / 113 / 208 us (44 ahead at d = 64)
#ifndef SPLIT32
#define SPLIT32 38
#endif
#ifndef SPLIT64
#define SPLIT64 44
#endif

// Field policies: canonical elements T, lazy accumulator A (sums of folded
// products: < 2^35 (u32) / < 2^70 (u64) each, at most 2^11 of them).
struct F32 {
    using T = uint32_t;
    using A = uint64_t;
    static constexpr int W = 32;         // 2^W = p + C
    static constexpr uint64_t C = C32;
    static constexpr uint64_t PM1 = P32 - 1;       // = 2 * 5 * 19 * 22605091
    static constexpr uint32_t L = SPLIT32;         // splitting arity: L | p - 1
    static constexpr uint32_t E = L & (0u - L);    // its power-of-two part
    static constexpr uint32_t LO = L / E;          // and its odd part
    static T pow(T a, uint64_t e) { return pow32(a, e); }
    static T add(T a, T b) { return add32(a, b); }
    static T sub(T a, T b) { return sub32(a, b); }
    static T mul(T a, T b) { return mul32(a, b); }
    static T neg(T a) { return neg32(a); }
    static T inv(T a) { return inv32_chain(a); }
    static T canon_any(T a) { return canon32(a); }
    static void mac(A &acc, T a, T b) {
        const uint64_t p = (uint64_t)a * b;
        acc += (p >> 32) * C32 + (uint32_t)p;   // < 6 * 2^32
    }
    static T red(A acc) { return canon32(fold64_32(acc)); }
    // a square root of n, or false for a non-residue: p32 = 3 (mod 4), so
    // n^((p+1)/4) squares to n whenever n is a residue
    static bool sqrt(T n, T &r) {
        r = pow32(n, (uint64_t)(P32 + 1) / 4);
        return mul32(r, r) == n;
    }
    // the same in two halves around one exponentiation (sqrt_many)
    static constexpr uint64_t SQRT_E = (uint64_t)(P32 + 1) / 4;
    static T sqrt_base(T n) { return n; }
    static bool sqrt_fin(T n, T v, T &r) {
        r = v;
        return mul32(r, r) == n;
    }
};

// Small factors of a u32 split (degree <= small_split_deg, the factors of
// 3-4 roots a 38-way split leaves): split SPLIT32S = 5 ways — 5 class gcds
// instead of 38 for a handful of roots, the one exponentiation the same
// length (d = 32, 8 root sets on the EPYC: 19.4 us against 21.4; 10-way
// 19.8-20.2, 2-way 20.8, 19-way 21.1)
#ifndef SPLIT32S
#define SPLIT32S 5
#endif
struct F32s : F32 {
    static constexpr uint32_t L = SPLIT32S;
    static constexpr uint32_t E = L & (0u - L);
    static constexpr uint32_t LO = L / E;
};
template <class F> struct SmallSplit;
template <> struct SmallSplit<F32> { using type = F32s; };

struct F64 {
    using T = uint64_t;
    using A = unsigned __int128;
    static constexpr int W = 64;
    static constexpr uint64_t C = C64;
    static constexpr uint64_t PM1 = P64 - 1;       // = 4 * 11 * 137 * 547 * 5594472617641
    static constexpr uint32_t L = SPLIT64;
    static constexpr uint32_t E = L & (0u - L);
    static constexpr uint32_t LO = L / E;
    static T pow(T a, uint64_t e) { return pow64(a, e); }
    static T add(T a, T b) { return add64(a, b); }
    static T sub(T a, T b) { return sub64(a, b); }
    static T mul(T a, T b) { return mul64(a, b); }
    static T neg(T a) { return neg64(a); }
    static T inv(T a) { return inv64_chain(a); }
    static T canon_any(T a) { return canon64(a); }
    static void mac(A &acc, T a, T b) {
        const unsigned __int128 p = (unsigned __int128)a * b;
        acc += (unsigned __int128)(uint64_t)(p >> 64) * C64 + (uint64_t)p;   // < 60 * 2^64
    }
    static T red(A acc) {
        // acc < 2^81: acc = H 2^64 + L == 59 H + L  (< 2^64 + 2^23), twice
        unsigned __int128 t = (unsigned __int128)(uint64_t)(acc >> 64) * C64 + (uint64_t)acc;
        unsigned __int128 u = (unsigned __int128)(uint64_t)(t >> 64) * C64 + (uint64_t)t;
        return canon64((uint64_t)u + C64 * (uint64_t)(u >> 64));
    }
    // Atkin (p64 = 5 mod 8, where 2 is a non-residue): v = (2n)^((p-5)/8),
    // i = 2n v^2 (a square root of -1 when n is a residue), r = n v (i - 1);
    // one exponentiation, r^2 == n iff n is a residue
    static bool sqrt(T n, T &r) {
        const T n2 = add64(n, n), v = pow64(n2, (P64 - 5) / 8);
        const T i = mul64(n2, mul64(v, v));
        r = mul64(mul64(n, v), sub64(i, 1));
        return mul64(r, r) == n;
    }
    // the same in two halves around one exponentiation (sqrt_many)
    static constexpr uint64_t SQRT_E = (P64 - 5) / 8;
    static T sqrt_base(T n) { return add64(n, n); }
    static bool sqrt_fin(T n, T v, T &r) {
        const T n2 = add64(n, n), i = mul64(n2, mul64(v, v));
        r = mul64(mul64(n, v), sub64(i, 1));
        return mul64(r, r) == n;
    }
};
// and of a u64 split, where the factors of a group share one exponentiation
// mod their product (group_deg): SPLIT64S classes for a group of small
// factors — 44, the split's own (off): 2 / 4 / 11 / 22 measured within
// +-0.5 us of it at d = 32 (profiles/r06/s11_roots_small_split/)
#ifndef SPLIT64S
#define SPLIT64S 44
#endif
struct F64s : F64 {
    static constexpr uint32_t L = SPLIT64S;
    static constexpr uint32_t E = L & (0u - L);
    static constexpr uint32_t LO = L / E;
};
template <> struct SmallSplit<F64> { using type = F64s; };

// Square roots of several n at once (ok[j]: n_j is a residue): the
// exponentiations' square-and-multiply steps interleaved across the n_j, so
// their dependent product chains overlap
template <class F>
static void sqrt_many(const std::vector<typename F::T> &n, std::vector<typename F::T> &r, std::vector<char> &ok) {
    using T = typename F::T;
    const size_t cnt = n.size();
    std::vector<T> x(cnt), v(cnt, 1);
    for (size_t j = 0; j < cnt; ++j) x[j] = F::sqrt_base(n[j]);
    for (int b = 63 - __builtin_clzll(F::SQRT_E); b >= 0; --b) {
        for (size_t j = 0; j < cnt; ++j) v[j] = F::mul(v[j], v[j]);
        if ((F::SQRT_E >> b) & 1)
            for (size_t j = 0; j < cnt; ++j) v[j] = F::mul(v[j], x[j]);
    }
    r.resize(cnt);
    ok.resize(cnt);
    for (size_t j = 0; j < cnt; ++j) ok[j] = F::sqrt_fin(n[j], v[j], r[j]);
}

// Polynomials: coefficient vectors low degree first, canonical, no trailing
// zeros (the zero polynomial is empty).
template <class F> using Poly = std::vector<typename F::T>;

template <class F> void trim(Poly<F> &a) {
    while (!a.empty() && a.back() == 0) a.pop_back();
}

// a * inv(lead) (monic); a nonzero
template <class F> void make_monic(Poly<F> &a) {
    const typename F::T li = F::inv(a.back());
    for (auto &v : a) v = F::mul(v, li);
}

// a mod b (b monic, deg b >= 1), in place
template <class F> void rem_monic(Poly<F> &a, const Poly<F> &b) {
    const size_t m = b.size() - 1;
    for (size_t k = a.size(); k-- > m;) {
        const typename F::T q = a[k];
        if (q) axmy<F>(a.data() + k - m, b.data(), m, 1, q);
        a[k] = 0;
    }
    trim<F>(a);
}

// r_j = a mod b_j for several monic b_j at once: the same steps as
// rem_monic, one step of every remainder per sweep — each remainder is a
// chain of dependent steps (a step's quotient is the coefficient the
// previous step just wrote), the sweep lets the core overlap the chains
template <class F> std::vector<Poly<F>> rem_many(const Poly<F> &a, const std::vector<const Poly<F> *> &bs) {
    const size_t cnt = bs.size();
    std::vector<Poly<F>> r(cnt, a);
    std::vector<size_t> k(cnt, a.size());
    for (bool any = true; any;) {
        any = false;
        for (size_t j = 0; j < cnt; ++j) {
            const size_t m = bs[j]->size() - 1;
            if (k[j] <= m) continue;
            const size_t t = --k[j];
            const typename F::T q = r[j][t];
            if (q) axmy<F>(r[j].data() + t - m, bs[j]->data(), m, 1, q);
            r[j][t] = 0;
            any = true;
        }
    }
    for (auto &x : r) trim<F>(x);
    return r;
}

// a / b (b monic), exact division assumed
template <class F> Poly<F> div_monic(Poly<F> a, const Poly<F> &b) {
    const size_t m = b.size() - 1;
    if (a.size() <= m) return {};
    Poly<F> q(a.size() - m);
    for (size_t k = a.size(); k-- > m;) {
        const typename F::T c = a[k];
        q[k - m] = c;
        if (c) axmy<F>(a.data() + k - m, b.data(), m, 1, c);
    }
    return q;
}

// The same remainder sequence for operands of at most 8 NV coefficients on
// AVX-512, without a call or a tail mask per step: both operands sit in
// fixed 64-bit-lane buffers (8 NV zero lanes below each), every step is NV
// full-vector rows alpha a - beta (z^s b), and lanes above the degree stay 0
// (the top lane cancels exactly; z^s b is 0 above it).
QK_AVX512 static inline __m512i row_lanes32(__m512i d, __m512i s, uint64_t alpha, uint64_t beta) {
    return subc512(mulc512(d, _mm512_set1_epi64((long long)alpha)), mulc512(s, _mm512_set1_epi64((long long)beta)));
}
QK_AVX512 static inline __m512i row_lanes64(__m512i d, __m512i s, uint64_t alpha, uint64_t beta) {
    using namespace simd;
    return sub64_512(canon64_512(mulmod64_512(d, lo32x8(alpha), hi32x8(alpha))),
                     canon64_512(mulmod64_512(s, lo32x8(beta), hi32x8(beta))));
}
template <class F, int NV>
QK_AVX512 static size_t gcd_small(const typename F::T *a0, size_t na, const typename F::T *b0, size_t nb,
                                  typename F::T *out) {
    alignas(64) uint64_t buf[4 * 8 * NV] = {};
    uint64_t *pa = buf + 8 * NV, *pb = buf + 3 * 8 * NV;
    for (size_t i = 0; i < na; ++i) pa[i] = a0[i];
    for (size_t i = 0; i < nb; ++i) pb[i] = b0[i];
    while (nb) {
        const size_t m = nb - 1;
        const uint64_t lb = pb[m];
        while (na > m) {
            const uint64_t la = pa[na - 1];
            const size_t s = na - 1 - m;
            const size_t nv = (na + 7) / 8;
            for (int k = 0; k < NV; ++k) {
                if ((size_t)k >= nv) break;
                const __m512i d = _mm512_load_si512(pa + 8 * k), x = _mm512_loadu_si512(pb + 8 * k - s);
                _mm512_store_si512(pa + 8 * k, F::W == 32 ? row_lanes32(d, x, lb, la) : row_lanes64(d, x, lb, la));
            }
            --na;
            while (na && !pa[na - 1]) --na;
        }
        std::swap(pa, pb);
        std::swap(na, nb);
    }
    for (size_t i = 0; i < na; ++i) out[i] = (typename F::T)pa[i];
    return na;
}

// The p64 rows on IFMA (52-bit limb column sums, as axmy64_ifma): d' =
// alpha d - beta s in one pass of seven madd52 per product and one reduction.
QK_IFMA static inline __m512i row_lanes64_ifma(__m512i d, __m512i s, uint64_t alpha, uint64_t beta) {
    const uint64_t nb = beta ? P64 - beta : 0;
    __m512i d0, d1, s0, s1;
    split52(d, d0, d1);
    split52(s, s0, s1);
    __m512i A = _mm512_setzero_si512(), B = A, C = A;
    prod52(A, B, C, _mm512_set1_epi64((long long)(alpha & M52)), _mm512_set1_epi64((long long)(alpha >> 52)), d0, d1);
    prod52(A, B, C, _mm512_set1_epi64((long long)(nb & M52)), _mm512_set1_epi64((long long)(nb >> 52)), s0, s1);
    return red_cols8(A, B, C);
}
template <int NV>
QK_IFMA static size_t gcd_small64_ifma(const uint64_t *a0, size_t na, const uint64_t *b0, size_t nb, uint64_t *out) {
    alignas(64) uint64_t buf[4 * 8 * NV] = {};
    uint64_t *pa = buf + 8 * NV, *pb = buf + 3 * 8 * NV;
    for (size_t i = 0; i < na; ++i) pa[i] = a0[i];
    for (size_t i = 0; i < nb; ++i) pb[i] = b0[i];
    while (nb) {
        const size_t m = nb - 1;
        const uint64_t lb = pb[m];
        while (na > m) {
            const uint64_t la = pa[na - 1];
            const size_t s = na - 1 - m;
            const size_t nv = (na + 7) / 8;
            for (int k = 0; k < NV; ++k) {
                if ((size_t)k >= nv) break;
                const __m512i d = _mm512_load_si512(pa + 8 * k), x = _mm512_loadu_si512(pb + 8 * k - s);
                _mm512_store_si512(pa + 8 * k, row_lanes64_ifma(d, x, lb, la));
            }
            --na;
            while (na && !pa[na - 1]) --na;
        }
        std::swap(pa, pb);
        std::swap(na, nb);
    }
    for (size_t i = 0; i < na; ++i) out[i] = pa[i];
    return na;
}

// gcd(a, b_j) for cnt <= GB_MAX operands b_j at once (not monic), the same
// rows as gcd_small: one remainder step of every live gcd per sweep.  A
// single gcd is a chain of dependent rows (each row's leading coefficient is
// read back from the row just stored); the rows of different gcds are
// independent, so the core overlaps them — the class gcds of a part
// (Splitter::classes) run as one batch.
constexpr int GB_MAX = 24;
#define QK_GCD_BATCH_BODY(ROW)                                                                          \
    constexpr size_t SZ = 4 * 8 * NV;                                                                   \
    alignas(64) uint64_t buf[GB_MAX][SZ];                                                               \
    uint64_t *pa[GB_MAX], *pb[GB_MAX];                                                                  \
    size_t na[GB_MAX], nb[GB_MAX];                                                                      \
    bool live[GB_MAX];                                                                                  \
    int nlive = cnt;                                                                                    \
    for (int j = 0; j < cnt; ++j) {                                                                     \
        memset(buf[j], 0, sizeof(buf[j]));                                                              \
        pa[j] = buf[j] + 8 * NV;                                                                        \
        pb[j] = buf[j] + 3 * 8 * NV;                                                                    \
        for (size_t i = 0; i < na0[j]; ++i) pa[j][i] = a0[j][i];                                        \
        for (size_t i = 0; i < nb0[j]; ++i) pb[j][i] = b0[j][i];                                        \
        na[j] = na0[j];                                                                                 \
        nb[j] = nb0[j];                                                                                 \
        live[j] = true;                                                                                 \
    }                                                                                                   \
    while (nlive) {                                                                                     \
        for (int j = 0; j < cnt; ++j) {                                                                 \
            if (!live[j]) continue;                                                                     \
            if (!nb[j]) {                                                                               \
                for (size_t i = 0; i < na[j]; ++i) out[j * SO + i] = (T)pa[j][i];                       \
                nout[j] = na[j];                                                                        \
                live[j] = false;                                                                        \
                --nlive;                                                                                \
                continue;                                                                               \
            }                                                                                           \
            const size_t m = nb[j] - 1;                                                                 \
            if (na[j] <= m) {                                                                           \
                std::swap(pa[j], pb[j]);                                                                \
                std::swap(na[j], nb[j]);                                                                \
                continue;                                                                               \
            }                                                                                           \
            const uint64_t lb = pb[j][m], la = pa[j][na[j] - 1];                                        \
            const size_t s = na[j] - 1 - m, nv = (na[j] + 7) / 8;                                       \
            for (int k = 0; k < NV; ++k) {                                                              \
                if ((size_t)k >= nv) break;                                                             \
                const __m512i d = _mm512_load_si512(pa[j] + 8 * k), x = _mm512_loadu_si512(pb[j] + 8 * k - s); \
                _mm512_store_si512(pa[j] + 8 * k, ROW(d, x, lb, la));                                   \
            }                                                                                           \
            --na[j];                                                                                    \
            while (na[j] && !pa[j][na[j] - 1]) --na[j];                                                 \
        }                                                                                               \
    }
// out: cnt rows of SO = 8 NV coefficients; nout[j]: the gcd's coefficient count
template <class F, int NV>
QK_AVX512 static void gcd_batch(const typename F::T *const *a0, const size_t *na0, int cnt, const typename F::T *const *b0,
                                const size_t *nb0, typename F::T *out, size_t *nout) {
    using T = typename F::T;
    constexpr size_t SO = 8 * NV;
    if constexpr (F::W == 32) {
        QK_GCD_BATCH_BODY(row_lanes32)
    } else {
        QK_GCD_BATCH_BODY(row_lanes64)
    }
}
template <int NV>
QK_IFMA static void gcd_batch64_ifma(const uint64_t *const *a0, const size_t *na0, int cnt, const uint64_t *const *b0,
                                     const size_t *nb0, uint64_t *out, size_t *nout) {
    using T = uint64_t;
    constexpr size_t SO = 8 * NV;
    QK_GCD_BATCH_BODY(row_lanes64_ifma)
}
#undef QK_GCD_BATCH_BODY

// monic gcd(a, b), fraction-free: each step cancels a's leading term as
// lead(b) a - lead(a) z^s b (no inversion; a field inverse costs ~70
// multiplications, more than the extra row of products here), one pass per
// step over a's coefficients: a_i <- lb a_i - la b_(i-s) with b
// zero-extended below, so the scaling of the low part and the row operation
// are one vector row.  No vector per step: both operands live in one buffer
// each behind P zeros (P > either size), so b zero-extended below is b's own
// buffer read from s slots earlier, and the swap of a step swaps pointers.
// monic = false: the last nonzero remainder as the rows leave it (a scalar
// multiple of the gcd, no inversion), {1} when coprime
template <class F> Poly<F> gcd_rows(const Poly<F> &a0, const Poly<F> &b0, bool small, bool monic = true) {
    using T = typename F::T;
    size_t na = a0.size(), nb = b0.size();
    while (na && !a0[na - 1]) --na;
    while (nb && !b0[nb - 1]) --nb;
    const size_t n = std::max(na, nb);
    if (small && n <= 40 && cpu_has_avx512()) {
        T g[40];
        size_t ng;
        if constexpr (F::W == 64) {
            if (cpu_has_ifma()) {
                const uint64_t *a = (const uint64_t *)a0.data(), *b = (const uint64_t *)b0.data();
                uint64_t *o = (uint64_t *)g;
                ng = n <= 8    ? gcd_small64_ifma<1>(a, na, b, nb, o)
                     : n <= 16 ? gcd_small64_ifma<2>(a, na, b, nb, o)
                     : n <= 24 ? gcd_small64_ifma<3>(a, na, b, nb, o)
                     : n <= 32 ? gcd_small64_ifma<4>(a, na, b, nb, o)
                               : gcd_small64_ifma<5>(a, na, b, nb, o);
                goto have;
            }
        }
        ng = n <= 8    ? gcd_small<F, 1>(a0.data(), na, b0.data(), nb, g)
                          : n <= 16 ? gcd_small<F, 2>(a0.data(), na, b0.data(), nb, g)
                          : n <= 24 ? gcd_small<F, 3>(a0.data(), na, b0.data(), nb, g)
                          : n <= 32 ? gcd_small<F, 4>(a0.data(), na, b0.data(), nb, g)
                                    : gcd_small<F, 5>(a0.data(), na, b0.data(), nb, g);
    have:
        if (ng == 1) return Poly<F>{1};   // coprime: no inversion for the monic form
        Poly<F> r(g, g + ng);
        if (!r.empty() && monic) make_monic<F>(r);
        return r;
    }
    const size_t P = n + 1;
    std::vector<T> buf(4 * P, 0);
    T *pa = buf.data() + P, *pb = buf.data() + 3 * P;
    std::copy(a0.begin(), a0.begin() + na, pa);
    std::copy(b0.begin(), b0.begin() + nb, pb);
    while (nb) {
        const size_t m = nb - 1;
        const T lb = pb[m];
        while (na > m) {
            const T la = pa[na - 1];
            const size_t s = na - 1 - m;
            axmy<F>(pa, pb - s, na - 1, lb, la);   // the top term cancels
            --na;
            while (na && !pa[na - 1]) --na;
        }
        std::swap(pa, pb);
        std::swap(na, nb);
    }
    if (na == 1) return Poly<F>{1};
    Poly<F> g(pa, pa + na);
    if (!g.empty() && monic) make_monic<F>(g);
    return g;
}
template <class F> Poly<F> gcd(const Poly<F> &a, const Poly<F> &b) { return gcd_rows<F>(a, b, true); }

// gcd(a_j, b_j) for every j, as gcd_rows(a_j, b_j, true, false) would
// return them ({1} when coprime), the small cases as one gcd_batch
template <class F> std::vector<Poly<F>> gcd_pairs(const std::vector<const Poly<F> *> &as, const std::vector<Poly<F>> &bs) {
    using T = typename F::T;
    const int cnt = (int)bs.size();
    std::vector<Poly<F>> res(cnt);
    size_t n = 0;
    const T *ap[GB_MAX], *bp[GB_MAX];
    size_t na[GB_MAX], nb[GB_MAX];
    for (int j = 0; j < cnt && j < GB_MAX; ++j) {
        size_t ka = as[j]->size(), kb = bs[j].size();
        while (ka && !(*as[j])[ka - 1]) --ka;
        while (kb && !bs[j][kb - 1]) --kb;
        ap[j] = as[j]->data();
        na[j] = ka;
        bp[j] = bs[j].data();
        nb[j] = kb;
        n = std::max(n, std::max(ka, kb));
    }
    if (cnt <= GB_MAX && n <= 40 && cpu_has_avx512()) {
        alignas(64) T out[GB_MAX * 40];
        size_t nout[GB_MAX];
        const int nv = (int)((n + 7) / 8);
        if constexpr (F::W == 64) {
            if (cpu_has_ifma()) {
                uint64_t *o = (uint64_t *)out;
                const uint64_t *const *a = (const uint64_t *const *)ap, *const *b = (const uint64_t *const *)bp;
                switch (nv) {
                case 1: gcd_batch64_ifma<1>(a, na, cnt, b, nb, o, nout); break;
                case 2: gcd_batch64_ifma<2>(a, na, cnt, b, nb, o, nout); break;
                case 3: gcd_batch64_ifma<3>(a, na, cnt, b, nb, o, nout); break;
                case 4: gcd_batch64_ifma<4>(a, na, cnt, b, nb, o, nout); break;
                default: gcd_batch64_ifma<5>(a, na, cnt, b, nb, o, nout); break;
                }
                goto have;
            }
        }
        switch (nv) {
        case 1: gcd_batch<F, 1>(ap, na, cnt, bp, nb, out, nout); break;
        case 2: gcd_batch<F, 2>(ap, na, cnt, bp, nb, out, nout); break;
        case 3: gcd_batch<F, 3>(ap, na, cnt, bp, nb, out, nout); break;
        case 4: gcd_batch<F, 4>(ap, na, cnt, bp, nb, out, nout); break;
        default: gcd_batch<F, 5>(ap, na, cnt, bp, nb, out, nout); break;
        }
    have:
        // gcd_batch<NV> writes row j at j * 8 NV
        const size_t so = 8 * (size_t)nv;
        for (int j = 0; j < cnt; ++j) {
            if (nout[j] == 1) res[j] = Poly<F>{1};
            else res[j].assign(out + j * so, out + j * so + nout[j]);
        }
        return res;
    }
    for (int j = 0; j < cnt; ++j) res[j] = gcd_rows<F>(*as[j], bs[j], true, false);
    return res;
}
// gcd(a, b_j) for every j (one shared first operand)
template <class F> std::vector<Poly<F>> gcd_many(const Poly<F> &a, const std::vector<Poly<F>> &bs) {
    return gcd_pairs<F>(std::vector<const Poly<F> *>(bs.size(), &a), bs);
}

// the smallest modulus degree on the vector paths (a variable for
// tools/prof_roots.cpp's A/B: from degree 3 on, u64 roots at d = 32 took
// 44.6 against 43.4 us, u32 22.0 against 21.7 — below 8 coefficients the
// vector forms' fixed costs exceed the scalar loops)
static size_t ring_vec_min = 8;
static bool reg_sqr = true;   // sqr64_ifma_reg for moduli of <= 32 coefficients (prof_roots A/B)
static bool pair_cuts = true;  // Splitter::cut2 for the two second-level cuts (prof_roots A/B)
// Small moduli (degree 2 .. SMALL_MAX, the factors of a few roots that
// split() re-splits): the product's top coefficients reduced independently
// against a table of z^k mod f (k = M .. 2M-2, M coefficients each), fully
// unrolled per degree — no chain of dependent reductions down the product.
constexpr size_t SMALL_MAX = 7;
static bool small_rings = true;   // (tools/prof_roots.cpp's A/B)
template <class F, int M>
static void sqr_small(typename F::T *a, const typename F::T *tab) {
    using T = typename F::T;
    using A = typename F::A;
    A acc[2 * M - 1] = {};
    for (int i = 0; i < M; ++i) {
        F::mac(acc[2 * i], a[i], a[i]);
        const T a2 = F::add(a[i], a[i]);
        for (int j = i + 1; j < M; ++j) F::mac(acc[i + j], a2, a[j]);
    }
    T top[M - 1];
    for (int r = 0; r < M - 1; ++r) top[r] = F::red(acc[M + r]);
    for (int i = 0; i < M; ++i) {
        A t = acc[i];
        for (int r = 0; r < M - 1; ++r) F::mac(t, top[r], tab[r * M + i]);
        a[i] = F::red(t);
    }
}
template <class F, int M>
static void mul_small(typename F::T *a, const typename F::T *b, const typename F::T *tab) {
    using T = typename F::T;
    using A = typename F::A;
    A acc[2 * M - 1] = {};
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j) F::mac(acc[i + j], a[i], b[j]);
    T top[M - 1];
    for (int r = 0; r < M - 1; ++r) top[r] = F::red(acc[M + r]);
    for (int i = 0; i < M; ++i) {
        A t = acc[i];
        for (int r = 0; r < M - 1; ++r) F::mac(t, top[r], tab[r * M + i]);
        a[i] = F::red(t);
    }
}

// Arithmetic modulo a fixed monic f of degree m >= 1: residues are vectors of
// exactly m coefficients.
template <class F> struct ModRing {
    using T = typename F::T;
    using A = typename F::A;
    size_t m;
    std::vector<T> nf;       // -f_i, i < m
    std::vector<A> acc;      // 2m - 1 lazy accumulators
    // the AVX-512 form (m >= 8): -f (u32: widened) and a zero-padded; lazy
    // lane sums (u64 field: with carry counts)
    bool vec = false, ifma = false;
    std::vector<uint64_t> nf64, a64, acc64, cnt64;
    std::vector<uint64_t> tab, l0, l1, cols;   // the IFMA form (u64 field)
    const uint64_t *tl0 = nullptr, *tl1 = nullptr;
    std::vector<T> tmp;

    std::vector<T> stab;     // the small-modulus table (sqr_small)
    bool small = false;

    explicit ModRing(const Poly<F> &f) : m(f.size() - 1), nf(m), acc(2 * m) {
        for (size_t i = 0; i < m; ++i) nf[i] = F::neg(f[i]);
        vec = m >= ring_vec_min && m <= 1024 && cpu_has_avx512();
        small = !vec && small_rings && m >= 2 && m <= SMALL_MAX;
        if (small) {   // rows z^k mod f, k = m .. 2m-2, by z^(k+1) = z z^k
            stab.resize((m - 1) * m);
            std::vector<T> row(nf);
            for (size_t r = 0; r + 1 < m; ++r) {
                std::copy(row.begin(), row.end(), stab.begin() + r * m);
                if (r + 2 < m) mul_lin(row, 0);
            }
        }
        if (!vec) return;
        const size_t mb = (m + 7) & ~(size_t)7;
        nf64.assign(mb + 8, 0);
        for (size_t i = 0; i < m; ++i) nf64[i] = nf[i];
        a64.assign(mb + 8, 0);
        acc64.assign(2 * m + 16, 0);
        tmp.assign(m, 0);
        if constexpr (F::W == 32) {
            a64.assign(IPAD32 + mb + 16, 0);
            acc64.assign(2 * mb + 16 + 8, 0);
        } else {
            cnt64.assign(2 * m + 16, 0);
            ifma = cpu_has_ifma() && m <= IFMA_MAX;
            if (!ifma) return;
            l0.assign(IPAD + mb + 16, 0);
            l1.assign(IPAD + mb + 16, 0);
            cols.assign(3 * (2 * mb + 16) + 8, 0);   // + 8: room to align to 64 bytes
        }
        // the reduction table: z^k mod f for k = m .. 2m-2, one zero-padded
        // row of mb per k (u64: as 52-bit limb rows), from z^m = -f by
        // z^(k+1) = z z^k (mul_lin with c = 0, vectorised)
        const size_t rows = (m - 1) * mb;
        tab.assign((F::W == 32 ? 1 : 2) * rows + 8, 0);
        uint64_t *t0 = tab.data() + ((8 - ((uintptr_t)tab.data() / 8) % 8) % 8), *t1 = t0 + rows;
        std::vector<T> row(nf);
        for (size_t r = 0; r + 1 < m; ++r) {
            for (size_t i = 0; i < m; ++i) {
                if constexpr (F::W == 32) t0[r * mb + i] = row[i];
                else t0[r * mb + i] = (uint64_t)row[i] & M52, t1[r * mb + i] = (uint64_t)row[i] >> 52;
            }
            if (r + 2 < m) mul_lin(row, 0);
        }
        tl0 = t0;
        if constexpr (F::W == 64) tl1 = t1;
    }
    // acc[0 .. 2m-1) (degree <= 2m-2) -> r (m coefficients): top-down, each
    // top coefficient q adds q * (-f_i) below it
    void reduce_acc(std::vector<T> &r) {
        for (size_t k = 2 * m - 1; k-- > m;) {
            const T q = F::red(acc[k]);
            if (q)
                for (size_t i = 0; i < m; ++i) F::mac(acc[k - m + i], q, nf[i]);
        }
        for (size_t i = 0; i < m; ++i) r[i] = F::red(acc[i]);
    }
    void sqr(std::vector<T> &a) {
        if (small) {
            switch (m) {
            case 2: return sqr_small<F, 2>(a.data(), stab.data());
            case 3: return sqr_small<F, 3>(a.data(), stab.data());
            case 4: return sqr_small<F, 4>(a.data(), stab.data());
            case 5: return sqr_small<F, 5>(a.data(), stab.data());
            case 6: return sqr_small<F, 6>(a.data(), stab.data());
            default: return sqr_small<F, 7>(a.data(), stab.data());
            }
        }
        if (vec) {
            if constexpr (F::W == 32) {
                uint64_t *c = acc64.data() + ((8 - ((uintptr_t)acc64.data() / 8) % 8) % 8);   // 64-byte aligned
                sqr32_avx512(a.data(), m, tl0, a64.data(), c);
            } else if (ifma) {
                const size_t mb = (m + 7) & ~(size_t)7, cw = 2 * mb + 16;
                uint64_t *c = cols.data() + ((8 - ((uintptr_t)cols.data() / 8) % 8) % 8);   // 64-byte aligned
                uint64_t *x = (uint64_t *)a.data();
                if (reg_sqr) switch (mb) {
                    case 8: return sqr64_ifma_reg<2>(x, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
                    case 16: return sqr64_ifma_reg<4>(x, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
                    case 24: return sqr64_ifma_reg<6>(x, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
                    case 32: return sqr64_ifma_reg<8>(x, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
                    default: break;
                    }
                sqr64_ifma(x, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
            } else {
                sqr64_avx512((uint64_t *)a.data(), m, nf64.data(), a64.data(), acc64.data(), cnt64.data());
            }
            return;
        }
        std::fill(acc.begin(), acc.end(), A(0));
        for (size_t i = 0; i < m; ++i) {
            const T ai = a[i];
            if (!ai) continue;
            F::mac(acc[2 * i], ai, ai);
            const T a2 = F::add(ai, ai);
            for (size_t j = i + 1; j < m; ++j) F::mac(acc[i + j], a2, a[j]);
        }
        reduce_acc(a);
    }
    // a <- a b (both residues of m coefficients; b may alias a)
    void mul(std::vector<T> &a, const std::vector<T> &b) {
        if (&a == &b) return sqr(a);
        if (small) {
            switch (m) {
            case 2: return mul_small<F, 2>(a.data(), b.data(), stab.data());
            case 3: return mul_small<F, 3>(a.data(), b.data(), stab.data());
            case 4: return mul_small<F, 4>(a.data(), b.data(), stab.data());
            case 5: return mul_small<F, 5>(a.data(), b.data(), stab.data());
            case 6: return mul_small<F, 6>(a.data(), b.data(), stab.data());
            default: return mul_small<F, 7>(a.data(), b.data(), stab.data());
            }
        }
        if (vec) {
            if constexpr (F::W == 32) {
                uint64_t *c = acc64.data() + ((8 - ((uintptr_t)acc64.data() / 8) % 8) % 8);
                return mul32_avx512(a.data(), b.data(), m, tl0, a64.data(), c);
            } else if (ifma) {
                const size_t mb = (m + 7) & ~(size_t)7, cw = 2 * mb + 16;
                uint64_t *c = cols.data() + ((8 - ((uintptr_t)cols.data() / 8) % 8) % 8);
                uint64_t *x = (uint64_t *)a.data();
                const uint64_t *y = (const uint64_t *)b.data();
                if (reg_sqr) switch (mb) {
                    case 8: return mul64_ifma_reg<2>(x, y, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
                    case 16: return mul64_ifma_reg<4>(x, y, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
                    case 24: return mul64_ifma_reg<6>(x, y, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
                    case 32: return mul64_ifma_reg<8>(x, y, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
                    default: break;
                    }
                return mul64_ifma(x, y, m, tl0, tl1, l0.data(), l1.data(), c, c + cw, c + 2 * cw);
            }
        }
        std::fill(acc.begin(), acc.end(), A(0));
        for (size_t i = 0; i < m; ++i) {
            if (!a[i]) continue;
            for (size_t j = 0; j < m; ++j) F::mac(acc[i + j], a[i], b[j]);
        }
        reduce_acc(a);
    }
    // a^e (e >= 1)
    std::vector<T> pow(const std::vector<T> &a, uint64_t e) {
        std::vector<T> r = a;
        for (int b = 62 - __builtin_clzll(e); b >= 0; --b) {
            sqr(r);
            if ((e >> b) & 1) mul(r, a);
        }
        return r;
    }
    // a <- a * (z + c)
    void mul_lin(std::vector<T> &a, T c) {
        if constexpr (F::W == 32) {
            if (vec) return mullin32_avx512(a.data(), m, c, nf.data(), tmp.data());
        } else {
            if (ifma) return mullin64_ifma((uint64_t *)a.data(), m, c, (const uint64_t *)nf.data(), (uint64_t *)tmp.data());
        }
        const T top = a[m - 1];                       // coefficient of z^m after the shift
        for (size_t i = m; i-- > 0;) {
            const T lower = i ? a[i - 1] : 0;
            a[i] = F::add(lower, F::mul(c, a[i]));
        }
        if (top)
            for (size_t i = 0; i < m; ++i) a[i] = F::add(a[i], F::mul(top, nf[i]));
    }
    // (z + c)^e mod f
    std::vector<T> pow_lin(T c, uint64_t e) {
        std::vector<T> r(m, 0);
        r[0] = 1;
        bool started = false;
        for (int b = 63; b >= 0; --b) {
            if (started) sqr(r);
            if ((e >> b) & 1) {
                mul_lin(r, c);
                started = true;
            }
        }
        return r;
    }
};

template <class F> Poly<F> to_poly(std::vector<typename F::T> r) {
    Poly<F> p(std::move(r));
    trim<F>(p);
    return p;
}

// a b (plain product)
template <class F> Poly<F> mul_poly(const Poly<F> &a, const Poly<F> &b) {
    if (a.empty() || b.empty()) return {};
    std::vector<typename F::A> acc(a.size() + b.size() - 1, typename F::A(0));
    for (size_t i = 0; i < a.size(); ++i)
        for (size_t j = 0; j < b.size(); ++j) F::mac(acc[i + j], a[i], b[j]);
    Poly<F> r(acc.size());
    for (size_t i = 0; i < acc.size(); ++i) r[i] = F::red(acc[i]);
    return r;
}
// split(): the largest product of factors sharing one exponentiation (a
// variable for tools/prof_roots.cpp's A/B; 0: one exponentiation per factor).
// EPYC 9575F, d = 32, mean over 8 root sets (profiles/r05/roots/): u64 43.2-
// 45.0 us alone, 43.4-43.7 at 16, 43.3-43.4 at 24; u32 21.6 alone, 21.9 at
// 16 and 24 — grouped for u64 only
static size_t group_deg = 24;
static size_t small_split_deg = 6;   // SmallSplit factors up to this degree (0: none; tools/prof_roots.cpp A/B)

// a primitive L-th root of unity of GF(p) (L | p - 1)
template <class F> typename F::T root_of_unity() {
    using T = typename F::T;
    static const T z = [] {
        for (T c = 2;; ++c) {
            const T w = F::pow(c, F::PM1 / F::L);
            bool prim = w != 1;
            uint32_t l = F::L;
            for (uint32_t q = 2; q <= l && prim; ++q)
                if (l % q == 0) {
                    prim = F::pow(w, F::L / q) != 1;
                    while (l % q == 0) l /= q;
                }
            if (prim) return w;
        }
    }();
    return z;
}

// A factor of degree k >= 3 is split L ways at once (Cantor-Zassenhaus with
// the L-th power character): w = (z + a)^((p-1)/L) mod g takes at a root r
// the L-th root of unity chi(r + a) = zeta^j (0 for r = -a), and the roots
// of class j are gcd(g, w - zeta^j) — one exponentiation for ~log_L k levels
// instead of log_2 k (L = 38 for p32, 44 for p64).  The classes are not
// taken one gcd at a time over all of g: with L = E LO (E the power-of-two
// part), v = w^LO takes the E-th root of unity zeta^(LO j) at a class-j
// root, so gcds with v^(E/2) - 1, then v - zeta^(LO c) (E = 4) cut g into E
// parts by j mod E first (~k/E roots each), and the LO classes of each part
// run their gcds on that part only.
template <class F> class Splitter {
    using T = typename F::T;
    const T zeta = root_of_unity<F>();
    T zc[4];        // zeta^c, c < E: each part's first class
    T step;         // zeta^E: the next class of a part
    T i4;           // zeta^LO: a primitive E-th root of unity (E = 4)

  public:
    Splitter() {
        zc[0] = 1;
        for (uint32_t c = 1; c < 4; ++c) zc[c] = F::mul(zc[c - 1], zeta);
        step = F::pow(zeta, F::E);
        i4 = F::pow(zeta, F::LO);
    }
    // the roots of g (monic) of class j (j mod E == c) for each j, from w mod
    // g (p64, E = 4: 11 classes of ~k/4 roots each; p32, E = 2: 19 of ~k/2):
    // every class against the whole of g, the gcds as one gcd_many batch —
    // each gcd is a chain of dependent rows, the batch overlaps the chains
    // (EPYC 9575F, d = 32, profiles/r05/roots/: u64 roots 52.4 -> 46.2 us,
    // u32 24.3 -> 19.4 us against one gcd at a time, the u32 one on the rest
    // shrinking as factors were found).  The factors go to parts as they
    // leave the gcd rows (a scalar multiple of the monic factor: split()
    // makes the leaves' roots with one batched inversion).  A root -a (w = 0
    // there) is in no class; whatever else is missing lies outside GF(p) (the
    // fast path's failure case): then the found factors, made monic, and the
    // rest.
    void classes(const Poly<F> &g, const Poly<F> &w, uint32_t c, T a, std::vector<Poly<F>> &parts,
                 bool reduced = false) const {
        if (g.size() <= 1) return;
        if (g.size() == 2) {
            parts.push_back(g);
            return;
        }
        const size_t k = g.size() - 1;
        Poly<F> wg = w;   // w mod g (reduced: the caller's rem_many did it)
        if (!reduced) rem_monic<F>(wg, g);
        if (wg.empty()) wg.push_back(0);
        T zj = zc[c];
        std::vector<Poly<F>> hs, wrs;
        size_t found = 0;
        for (uint32_t j = c; j < F::L; j += F::E, zj = F::mul(zj, step)) {
            wrs.push_back(wg);
            wrs.back()[0] = F::sub(wrs.back()[0], zj);
        }
        for (auto &h : gcd_many<F>(g, wrs))
            if (h.size() > 1) {
                found += h.size() - 1;
                hs.push_back(std::move(h));
            }
        if (found < k) {   // the root -a?
            const T x = F::neg(a);
            T v = 1;
            for (size_t i = k; i-- > 0;) v = F::add(F::mul(v, x), g[i]);   // g monic: Horner from z^k
            if (v == 0) {
                hs.push_back(Poly<F>{a, 1});
                ++found;
            }
        }
        if (found == k) {
            for (auto &h : hs) parts.push_back(std::move(h));
            return;
        }
        Poly<F> rem = g;
        for (auto &h : hs) {
            make_monic<F>(h);
            rem = div_monic<F>(rem, h);
            parts.push_back(std::move(h));
        }
        if (rem.size() > 1) parts.push_back(std::move(rem));
    }
    // cut(g, u, c, ...) and cut(h, u, e, ...) at once: the two gcds as one
    // batch, their leading coefficients inverted together
    static void cut2(const Poly<F> &g, const Poly<F> &h, const Poly<F> &u, T c, T e, Poly<F> &gin, Poly<F> &gout,
                     Poly<F> &hin, Poly<F> &hout) {
        std::vector<Poly<F>> ur = rem_many<F>(u, {&g, &h});
        for (auto &r : ur)
            if (r.empty()) r.push_back(0);
        ur[0][0] = F::sub(ur[0][0], c);
        ur[1][0] = F::sub(ur[1][0], e);
        std::vector<Poly<F>> d = gcd_pairs<F>({&g, &h}, ur);
        const T lg = d[0].back(), lh = d[1].back();
        const T inv = F::inv(F::mul(lg, lh)), ig = F::mul(inv, lh), ih = F::mul(inv, lg);
        for (auto &v : d[0]) v = F::mul(v, ig);
        for (auto &v : d[1]) v = F::mul(v, ih);
        gin = std::move(d[0]);
        hin = std::move(d[1]);
        gout = gin.size() > 1 ? div_monic<F>(g, gin) : g;
        hout = hin.size() > 1 ? div_monic<F>(h, hin) : h;
        if (gin.size() <= 1) gin.clear();
        if (hin.size() <= 1) hin.clear();
    }
    // g = gcd(g, u - c) * (g / that): the roots where u == c, and the rest
    static void cut(const Poly<F> &g, const Poly<F> &u, T c, Poly<F> &in, Poly<F> &out) {
        Poly<F> ur = u;
        rem_monic<F>(ur, g);
        if (ur.empty()) ur.push_back(0);
        ur[0] = F::sub(ur[0], c);
        in = gcd<F>(g, ur);
        out = in.size() > 1 ? div_monic<F>(g, in) : g;
        if (in.size() <= 1) in.clear();
    }
    // The residues one L-way split needs, modulo the ring's f (g itself, or
    // the product of several parts split with the same a): w = (z + a)^((p -
    // 1)/L), v = w^LO (E > 1) and q = v^2 (E = 4)
    struct Pw {
        Poly<F> w, v, q;
    };
    static Pw powers(ModRing<F> &R, T a) {
        Pw r;
        const std::vector<T> wv = R.pow_lin(a, F::PM1 / F::L);
        r.w = to_poly<F>(wv);
        if constexpr (F::E > 1) {
            std::vector<T> vv = F::LO > 1 ? R.pow(wv, F::LO) : wv;
            r.v = to_poly<F>(vv);
            if constexpr (F::E == 4) {
                R.sqr(vv);
                r.q = to_poly<F>(std::move(vv));
            }
        }
        return r;
    }
    // every factor the split of g (monic, dividing the ring's f) by these
    // residues yields
    void split_with(const Poly<F> &g, const Pw &pw, T a, std::vector<Poly<F>> &parts) const {
        if constexpr (F::E == 1) {
            classes(g, pw.w, 0, a, parts);
        } else {
            Poly<F> A, B;
            if constexpr (F::E == 2) {
                cut(g, pw.v, 1, A, B);   // v = 1: even j; v = -1 (or r = -a): odd j
                classes(A, pw.w, 0, a, parts);
                classes(B, pw.w, 1, a, parts);
            } else {
                static_assert(F::E == 4, "p - 1 has at most 2^2");
                cut(g, pw.q, 1, A, B);   // v^2 = +-1: j even / odd
                Poly<F> A0, A2, B1, B3;
                if (A.size() > 2 && B.size() > 2 && pair_cuts) {
                    cut2(A, B, pw.v, 1, i4, A0, A2, B1, B3);   // both at once
                } else {
                    if (A.size() > 2) cut(A, pw.v, 1, A0, A2);   // j = 0 / 2 mod 4
                    else A2 = A;
                    if (B.size() > 2) cut(B, pw.v, i4, B1, B3);  // j = 1 / 3 mod 4
                    else B3 = B;
                }
                if (pair_cuts) {   // w mod the four parts as one rem_many
                    const Poly<F> one{1};
                    const Poly<F> *ps[4] = {&A0, &A2, &B1, &B3};
                    std::vector<const Poly<F> *> bs;
                    for (auto p : ps) bs.push_back(p->size() > 2 ? p : &one);
                    const std::vector<Poly<F>> wr = rem_many<F>(pw.w, bs);
                    const uint32_t cs[4] = {0, 2, 1, 3};
                    for (int i = 0; i < 4; ++i) classes(*ps[i], wr[i], cs[i], a, parts, true);
                } else {
                    classes(A0, pw.w, 0, a, parts);
                    classes(A2, pw.w, 2, a, parts);
                    classes(B1, pw.w, 1, a, parts);
                    classes(B3, pw.w, 3, a, parts);
                }
            }
        }
    }
    // every factor one L-way split of g (w = (z + a)^((p-1)/L) mod g) yields
    void run(ModRing<F> &R, const Poly<F> &g, T a, std::vector<Poly<F>> &parts) const {
        split_with(g, powers(R, a), a, parts);
    }
};

// Split g into linear factors, appending their roots.  exact: g is monic,
// squarefree, and all its roots lie in GF(p)*: always succeeds.  !exact
// (the fast path, any monic g with g(0) != 0): every leaf that is reached is a
// genuine linear factor of g (split products are exact divisions), so the
// roots appended are roots of g and, when it returns true, all of them; it
// returns false when a factor will not split into linear ones (an
// irreducible factor of degree >= 2, i.e. roots outside GF(p)), after a
// quadratic with a non-residue discriminant or 24 failed attempts on one
// factor.  The factors come out of the splitting as scalar multiples of
// their monic forms; a leaf's roots are fractions num / den whose
// denominators are inverted together at the end (Montgomery's trick: one
// inversion and 3 products per root instead of one inversion per factor).
template <class F> bool split(const Poly<F> &g0, std::vector<typename F::T> &out, bool exact) {
    using T = typename F::T;
    using Fs = typename SmallSplit<F>::type;
    constexpr bool HAS_SMALL = Fs::L != F::L;
    const Splitter<F> S{};
    const Splitter<Fs> Ss{};
    std::vector<T> num, den;
    std::vector<Poly<F>> todo{g0};
    std::vector<int> tries{0};
    std::vector<T> qdisc, qnb, qd2;   // the quadratic leaves, solved together at the end
    uint64_t s = 0x243F6A8885A308D3ull;   // fixed seed: a deterministic sequence of a's
    while (!todo.empty()) {
        // this generation: the leaves now, the factors of >= 3 roots (big)
        // split below
        std::vector<Poly<F>> big;
        std::vector<int> bt;
        for (size_t i = 0; i < todo.size(); ++i) {
            Poly<F> &g = todo[i];
            const size_t k = g.size() - 1;
            if (g.empty() || k == 0) continue;
            if (k == 1) {   // g1 z + g0
                num.push_back(F::neg(g[0]));
                den.push_back(g[1]);
                continue;
            }
            if (k == 2) {   // g2 z^2 + g1 z + g0: (-g1 +- sqrt(g1^2 - 4 g2 g0)) / (2 g2), below
                const T a2 = g[2], b = g[1], c = g[0];
                qdisc.push_back(F::sub(F::mul(b, b), F::mul(F::mul(4, a2), c)));
                qnb.push_back(F::neg(b));
                qd2.push_back(F::add(a2, a2));
                continue;
            }
            if (!exact && tries[i] >= 24) return false;
            big.push_back(std::move(g));
            bt.push_back(tries[i]);
        }
        todo.clear();
        tries.clear();
        if (big.empty()) break;
        // monic forms: the leading coefficients inverted together
        {
            std::vector<T> pre(big.size());
            T acc = 1;
            for (size_t i = 0; i < big.size(); ++i) pre[i] = acc = F::mul(acc, big[i].back());
            T inv = F::inv(acc);
            for (size_t i = big.size(); i-- > 0;) {
                const T li = i ? F::mul(inv, pre[i - 1]) : inv;
                inv = F::mul(inv, big[i].back());
                if (big[i].back() != 1)
                    for (auto &v : big[i]) v = F::mul(v, li);
            }
        }
        // groups of consecutive factors of <= group_deg total degree share one
        // exponentiation, taken mod their product (each factor then reduces
        // the residues mod itself in its cuts and classes): a small factor's
        // exponentiation is a chain of latency-bound squarings, so three of
        // degree 3-4 cost about what one of degree 10 does
        for (size_t i0 = 0; i0 < big.size();) {
            size_t i1 = i0 + 1, deg = big[i0].size() - 1;
            const size_t cap = F::W == 64 ? group_deg : 0;
            size_t dmax = deg;
            while (i1 < big.size() && deg + big[i1].size() - 1 <= cap) {
                dmax = std::max(dmax, big[i1].size() - 1);
                deg += big[i1++].size() - 1;
            }
            Poly<F> H = big[i0];
            for (size_t i = i0 + 1; i < i1; ++i) H = mul_poly<F>(H, big[i]);
            s += GAMMA;
            const T a = F::canon_any((T)splitmix_mix(s));
            const bool small = HAS_SMALL && dmax <= small_split_deg;   // every factor of the group small
            typename Splitter<F>::Pw pw;
            typename Splitter<Fs>::Pw pws;
            if (small) {
                ModRing<Fs> R(H);
                pws = Splitter<Fs>::powers(R, a);
            } else {
                ModRing<F> R(H);
                pw = Splitter<F>::powers(R, a);
            }
            for (size_t i = i0; i < i1; ++i) {
                std::vector<Poly<F>> parts;
                if (small) Ss.split_with(big[i], pws, a, parts);
                else S.split_with(big[i], pw, a, parts);
                if (parts.size() < 2) {   // no split with this a: again with the next one
                    todo.push_back(std::move(big[i]));
                    tries.push_back(bt[i] + 1);
                    continue;
                }
                for (auto &p : parts) {
                    todo.push_back(std::move(p));
                    tries.push_back(0);
                }
            }
            i0 = i1;
        }
    }
    // the quadratics: their square roots as one sqrt_many
    if (!qdisc.empty()) {
        std::vector<T> sq;
        std::vector<char> ok;
        sqrt_many<F>(qdisc, sq, ok);
        for (size_t j = 0; j < qdisc.size(); ++j) {
            if (!ok[j]) {
                if (!exact) return false;
                continue;   // (cannot happen for an exact-mode factor)
            }
            num.push_back(F::add(qnb[j], sq[j]));
            den.push_back(qd2[j]);
            num.push_back(F::sub(qnb[j], sq[j]));
            den.push_back(qd2[j]);
        }
    }
    // num_i / den_i: prefix products, one inversion, back substitution
    const size_t n = den.size();
    if (n) {
        std::vector<T> pre(n);
        pre[0] = den[0];
        for (size_t i = 1; i < n; ++i) pre[i] = F::mul(pre[i - 1], den[i]);
        T inv = F::inv(pre[n - 1]);
        for (size_t i = n; i-- > 0;) {
            const T di = i ? F::mul(inv, pre[i - 1]) : inv;   // 1 / den_i
            if (i) inv = F::mul(inv, den[i]);
            out.push_back(F::mul(num[i], di));
        }
    }
    return true;
}

// the distinct roots of z^d + c_1 z^(d-1) + ... + c_d in GF(p), ascending
template <class F> std::vector<typename F::T> roots(const typename F::T *c, uint32_t d) {
    using T = typename F::T;
    std::vector<T> out;
    if (d == 0) return out;
    Poly<F> f(d + 1);
    f[d] = 1;
    for (uint32_t i = 1; i <= d; ++i) f[d - i] = F::canon_any(c[i - 1]);
    // 1. the root 0
    size_t z = 0;
    while (z < f.size() && f[z] == 0) ++z;
    if (z) {
        out.push_back(0);
        f.erase(f.begin(), f.begin() + z);
    }
    if (f.size() > 1) {
        // fast path: the decode case (f a product of linear factors, the
        // missing ids) splits without step 2
        std::vector<T> r;
        if (!split<F>(f, r, false)) {
            // 2. g = gcd(f, z^(2^W) - z^(C+1)), then 3. split it
            r.clear();
            ModRing<F> R(f);
            std::vector<T> h(R.m, 0);
            if (R.m == 1) h[0] = F::neg(f[0]);          // z mod (z + f0)
            else h[1] = 1;
            for (int i = 0; i < F::W; ++i) R.sqr(h);    // z^(2^W)
            const std::vector<T> zc = R.pow_lin(0, F::C + 1);   // z^(C+1)
            for (size_t i = 0; i < R.m; ++i) h[i] = F::sub(h[i], zc[i]);
            Poly<F> g = gcd<F>(f, to_poly<F>(std::move(h)));
            if (g.size() > 1) split<F>(g, r, true);
        }
        out.insert(out.end(), r.begin(), r.end());
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

template <class F>
int roots_abi(const typename F::T *coeffs, uint32_t d, typename F::T *out, uint32_t cap, uint32_t *k) {
    if (!k || (d && !coeffs)) return QK_E_INVAL;
    *k = 0;
    std::vector<typename F::T> r;
    try {
        r = roots<F>(coeffs, d);
    } catch (const std::bad_alloc &) {
        return QK_E_NOMEM;
    }
    *k = (uint32_t)r.size();
    if (r.size() > cap || (!r.empty() && !out)) return QK_E_CAPACITY;
    std::copy(r.begin(), r.end(), out);
    return QK_OK;
}

} // namespace

extern "C" {

int qk_u32_roots(const uint32_t *coeffs, uint32_t d, uint32_t *roots, uint32_t cap, uint32_t *k) {
    return roots_abi<F32>(coeffs, d, roots, cap, k);
}

int qk_u64_roots(const uint64_t *coeffs, uint32_t d, uint64_t *roots, uint32_t cap, uint32_t *k) {
    return roots_abi<F64>(coeffs, d, roots, cap, k);
}

} // extern "C"
