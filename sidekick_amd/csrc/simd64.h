// simd64.h — GF(2^64 - 59) lane arithmetic on AVX-512 (host code only:
// host.cpp's sixteen-chain insert, roots.cpp's polynomial rows and squaring).
// Eight 64-bit lanes; products from four vpmuludq of the 32-bit halves.
#pragma once
#include <immintrin.h>
#include <stdint.h>

#include "field.h"

#define QK_AVX512 __attribute__((target("avx512f,avx512vl,avx512dq")))

namespace qk {
namespace simd {

// a b (lazy: < 2^64, == a b mod p) for any 64-bit a, with b's 32-bit halves
// b0 = b mod 2^32 and b1 = b >> 32 (broadcast): the 128-bit product from
// four vpmuludq with the carries of the middle and low sums restored by
// compares, then hi 2^64 == 59 hi twice as in mul64_lazy.
QK_AVX512 static inline __m512i mulmod64_512(__m512i a, __m512i b0, __m512i b1) {
    const __m512i a1 = _mm512_srli_epi64(a, 32);
    const __m512i p00 = _mm512_mul_epu32(a, b0), p01 = _mm512_mul_epu32(a, b1);
    const __m512i p10 = _mm512_mul_epu32(a1, b0), p11 = _mm512_mul_epu32(a1, b1);
    const __m512i mid = _mm512_add_epi64(p01, p10);
    const __mmask8 cm = _mm512_cmplt_epu64_mask(mid, p01);             // mid wrapped: + 2^96
    const __m512i lo = _mm512_add_epi64(p00, _mm512_slli_epi64(mid, 32));
    const __mmask8 cl = _mm512_cmplt_epu64_mask(lo, p00);              // lo wrapped: + 2^64
    __m512i hi = _mm512_add_epi64(p11, _mm512_srli_epi64(mid, 32));
    hi = _mm512_mask_add_epi64(hi, cm, hi, _mm512_set1_epi64(1ll << 32));
    hi = _mm512_mask_add_epi64(hi, cl, hi, _mm512_set1_epi64(1));      // a b = hi 2^64 + lo exactly
    // 59 hi + lo = c 2^64 + s2 with c <= 66, then s2 + 59 c (one more wrap at most)
    const __m512i c59 = _mm512_set1_epi64(59);
    const __m512i x = _mm512_mul_epu32(hi, c59), y = _mm512_mul_epu32(_mm512_srli_epi64(hi, 32), c59);
    const __m512i s1 = _mm512_add_epi64(x, _mm512_slli_epi64(y, 32));
    const __mmask8 c1 = _mm512_cmplt_epu64_mask(s1, x);
    const __m512i s2 = _mm512_add_epi64(s1, lo);
    const __mmask8 c2 = _mm512_cmplt_epu64_mask(s2, s1);
    __m512i c = _mm512_srli_epi64(y, 32);
    c = _mm512_mask_add_epi64(c, c1, c, _mm512_set1_epi64(1));
    c = _mm512_mask_add_epi64(c, c2, c, _mm512_set1_epi64(1));
    const __m512i r = _mm512_add_epi64(s2, _mm512_mul_epu32(c, c59));
    return _mm512_mask_add_epi64(r, _mm512_cmplt_epu64_mask(r, s2), r, c59);
}
// any 64-bit lane -> canonical
QK_AVX512 static inline __m512i canon64_512(__m512i r) {
    const __m512i P = _mm512_set1_epi64((long long)P64);
    return _mm512_mask_sub_epi64(r, _mm512_cmpge_epu64_mask(r, P), r, P);
}
// canonical a - b
QK_AVX512 static inline __m512i sub64_512(__m512i a, __m512i b) {
    const __m512i d = _mm512_sub_epi64(a, b);
    return _mm512_mask_add_epi64(d, _mm512_cmplt_epu64_mask(a, b), d, _mm512_set1_epi64((long long)P64));
}
// b broadcast as its 32-bit halves
QK_AVX512 static inline __m512i lo32x8(uint64_t b) { return _mm512_set1_epi64((long long)(b & 0xFFFFFFFFull)); }
QK_AVX512 static inline __m512i hi32x8(uint64_t b) { return _mm512_set1_epi64((long long)(b >> 32)); }

} // namespace simd
} // namespace qk
