// host.cpp — host-side (scalar) half of the quACK C ABI: sketch state,
// per-packet insert/remove, subtract/merge, Newton's identities, Horner
// evaluation and the bincode wire image.  These are the per-packet calls of
// the reference (sidekick.rs:42, media_client.rs:249,296,304,310,319); they
// stay on the host because one insert (~75 ns on CPU at t=20) is far below a
// kernel launch.  The batch paths live in encode.hip / decode.hip.
#include "quack_hip.h"
#include "field.h"
#include "simd64.h"

#include <string.h>

#include <immintrin.h>
#include <vector>

using namespace qk;

namespace {
static inline void put_le(uint8_t *p, uint64_t v, int nbytes) {
    for (int i = 0; i < nbytes; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
static inline uint64_t get_le(const uint8_t *p, int nbytes) {
    uint64_t v = 0;
    for (int i = 0; i < nbytes; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

template <typename Q, typename T>
int deser(const uint8_t *buf, size_t len, Q *q, uint32_t *t_out, T modulus) {
    if (!buf || len < 8) return QK_E_FORMAT;
    const uint64_t t = get_le(buf, 8);
    if (t > 0xFFFFFFFFull) return QK_E_FORMAT;
    if (t_out) *t_out = (uint32_t)t;
    const size_t body = 8 + sizeof(T) * (size_t)t;
    if (len < body + 1 + 4) return QK_E_FORMAT;
    const uint8_t tag = buf[body];
    if (tag > 1) return QK_E_FORMAT;
    const size_t need = body + 1 + (tag ? sizeof(T) : 0) + 4;
    if (len != need) return QK_E_FORMAT;
    if (!q) return QK_OK;
    // q must have been initialised for this threshold (qk_*_init(q, t) sizes
    // its power_sums): a smaller sketch would be overrun
    if (q->threshold != (uint32_t)t) return QK_E_MISMATCH;
    for (uint64_t k = 0; k < t; ++k) {
        const T v = (T)get_le(buf + 8 + sizeof(T) * k, sizeof(T));
        if (v >= modulus) return QK_E_FORMAT; // ModularInteger values are canonical
    }
    q->threshold = (uint32_t)t;
    for (uint64_t k = 0; k < t; ++k) q->power_sums[k] = (T)get_le(buf + 8 + sizeof(T) * k, sizeof(T));
    q->has_last = tag;
    q->last_value = tag ? (T)get_le(buf + body + 1, sizeof(T)) : 0;
    q->count = (uint32_t)get_le(buf + need - 4, 4);
    return QK_OK;
}
} // namespace

// ---------------------------------------------------------------- powers
// The per-packet path (sidekick.rs:42; one call per sniffed packet).  The
// reference walks x, x^2, .., x^t as one dependent chain of modmuls; here
// the powers run as four independent chains (x^(j+1) * (x^4)^i, j < 4) so the
// multiplier latency overlaps: ~3x fewer cycles per insert at t >= 16 on one
// core; on an AVX-512 CPU the powers run as sixteen chains in two zmm (u32
// t >= 8, u64 t >= 16) instead: on the GPU box's EPYC 9575F u32 t = 32 / 300
// 39 -> 16 / 320 -> 114 ns, u64 t = 80 / 300 118 -> 58 / 421 -> 215 ns.
// Chain values stay lazy (< 2^32 / < 2^64, any representative); every
// stored sum is canonical.
namespace {
struct F32 {
    using T = uint32_t;
    static T canon(T v) { return canon32(v); }
    static T mul(T a, T b) { return mul32_lazy(a, b); }
    static T add(T s, T y) { return add32(s, canon32(y)); }
    static T sub(T s, T y) { return sub32(s, canon32(y)); }
};
struct F64 {
    using T = uint64_t;
    static T canon(T v) { return canon64(v); }
    static T mul(T a, T b) { return mul64_lazy(a, b); }
    static T add(T s, T y) { return add64(s, canon64(y)); }
    static T sub(T s, T y) { return sub64(s, canon64(y)); }
};

// u32 on a CPU with AVX-512 (the GPU box hosts are Zen 5 EPYCs): sixteen
// chains in the 64-bit lanes of two zmm — lane j of v0 / v1 holds x^(j+1) /
// x^(j+9) times (x^16)^i — each step one vpmuludq per vector by x^16 and the
// same two pseudo-Mersenne folds as mul32_lazy (2^32 == 5), the two vectors'
// steps independent; the sums updated eight at a time (zero-extended loads,
// truncating stores, masked for the last < 8).  Lane values stay < 2^32
// (lazy), the stored sums canonical: the results are those of the scalar
// chains bit for bit (tests/test_host_abi.py, every t).
QK_AVX512 static inline __m512i fold512(__m512i m) {   // l + 5 h of each 64-bit lane
    const __m512i h = _mm512_srli_epi64(m, 32);
    return _mm512_add_epi64(_mm512_and_si512(m, _mm512_set1_epi64(0xFFFFFFFFll)),
                            _mm512_add_epi64(h, _mm512_slli_epi64(h, 2)));
}
QK_AVX512 static inline __m512i mulmod512(__m512i a, __m512i b) {   // a, b < 2^32 -> < 2^32, == a b
    const __m512i r = fold512(fold512(_mm512_mul_epu32(a, b)));     // < 2^32 + 25
    return _mm512_mask_sub_epi64(r, _mm512_cmpge_epu64_mask(r, _mm512_set1_epi64(1ll << 32)), r,
                                 _mm512_set1_epi64(P32));
}
// sums S[k..k+8) (masked past t) += or -= the canonical form of the lanes of v
QK_AVX512 static inline void acc32_512(uint32_t *S, uint32_t k, uint32_t t, __m512i v, bool add) {
    const __m512i P = _mm512_set1_epi64(P32);
    const uint32_t rem = t - k;
    // full chunks unmasked: the next insert's load of the same 32 bytes is
    // then forwarded from this store (masked stores do not forward)
    const __mmask8 m = rem >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << rem) - 1u);
    const __m256i sraw = rem >= 8 ? _mm256_loadu_si256(reinterpret_cast<const __m256i *>(S + k))
                                  : _mm256_maskz_loadu_epi32(m, S + k);
    const __m512i s = _mm512_cvtepu32_epi64(sraw);
    const __m512i y = _mm512_mask_sub_epi64(v, _mm512_cmpge_epu64_mask(v, P), v, P);   // canonical
    __m512i r;
    if (add) {
        r = _mm512_add_epi64(s, y);
        r = _mm512_mask_sub_epi64(r, _mm512_cmpge_epu64_mask(r, P), r, P);
    } else {
        r = _mm512_sub_epi64(s, y);
        r = _mm512_mask_add_epi64(r, _mm512_cmplt_epu64_mask(s, y), r, P);
    }
    if (rem >= 8) _mm256_storeu_si256(reinterpret_cast<__m256i *>(S + k), _mm512_cvtepi64_epi32(r));
    else _mm512_mask_cvtepi64_storeu_epi32(S + k, m, r);
}
// two chains of eight lanes (x^1..x^8 and x^9..x^16, step x^16): the two
// vector modmuls of a step are independent, so their latency overlaps
QK_AVX512 static void power_walk32_avx512(uint32_t *S, uint32_t t, uint32_t x, bool add) {
    uint32_t pw[8];
    pw[0] = x;
    for (int j = 1; j < 8; ++j) pw[j] = mul32_lazy(pw[(j - 1) / 2], pw[j / 2]);   // x^(j+1)
    __m512i v0 = _mm512_cvtepu32_epi64(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(pw)));
    __m512i v1 = t > 8 ? mulmod512(v0, _mm512_set1_epi64(pw[7])) : v0;           // x^9 .. x^16
    const __m512i step = _mm512_set1_epi64(t > 16 ? mul32_lazy(pw[7], pw[7]) : 0u);   // x^16
    for (uint32_t k = 0; k < t; k += 16) {
        acc32_512(S, k, t, v0, add);
        if (k + 8 < t) acc32_512(S, k + 8, t, v1, add);
        if (k + 16 < t) {
            v0 = mulmod512(v0, step);
            v1 = mulmod512(v1, step);
        }
    }
}

// u64 twin (p = 2^64 - 59): the lane product of simd64.h (four vpmuludq,
// carries restored by compares, 2^64 == 59 twice); b's halves are the chain
// step (hoisted).
using simd::mulmod64_512;
QK_AVX512 static inline void acc64_512(uint64_t *S, uint32_t k, uint32_t t, __m512i v, bool add) {
    const __m512i P = _mm512_set1_epi64((long long)P64), c59 = _mm512_set1_epi64(59);
    const uint32_t rem = t - k;
    const __mmask8 m = rem >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << rem) - 1u);
    const __m512i s = rem >= 8 ? _mm512_loadu_si512(S + k) : _mm512_maskz_loadu_epi64(m, S + k);
    const __m512i y = _mm512_mask_sub_epi64(v, _mm512_cmpge_epu64_mask(v, P), v, P);   // canonical
    __m512i r;
    if (add) {   // s + y < 2p: a wrap past 2^64 means s + y - p = r + 59
        r = _mm512_add_epi64(s, y);
        const __mmask8 w = _mm512_cmplt_epu64_mask(r, s);
        r = _mm512_mask_add_epi64(r, w, r, c59);
        r = _mm512_mask_sub_epi64(r, _mm512_cmpge_epu64_mask(r, P) & (__mmask8)~w, r, P);
    } else {     // s - y, + p when it borrowed
        r = _mm512_sub_epi64(s, y);
        r = _mm512_mask_add_epi64(r, _mm512_cmplt_epu64_mask(s, y), r, P);
    }
    if (rem >= 8) _mm512_storeu_si512(S + k, r);
    else _mm512_mask_storeu_epi64(S + k, m, r);
}
QK_AVX512 static void power_walk64_avx512(uint64_t *S, uint32_t t, uint64_t x, bool add) {
    uint64_t pw[8];
    pw[0] = x;
    for (int j = 1; j < 8; ++j) pw[j] = mul64_lazy(pw[(j - 1) / 2], pw[j / 2]);   // x^(j+1)
    const uint64_t x16 = t > 16 ? mul64_lazy(pw[7], pw[7]) : 0;
    __m512i v0 = _mm512_loadu_si512(pw);
    __m512i v1 = t > 8 ? mulmod64_512(v0, _mm512_set1_epi64((long long)(pw[7] & 0xFFFFFFFFull)),
                                      _mm512_set1_epi64((long long)(pw[7] >> 32)))
                       : v0;                                                          // x^9 .. x^16
    const __m512i b0 = _mm512_set1_epi64((long long)(x16 & 0xFFFFFFFFull)), b1 = _mm512_set1_epi64((long long)(x16 >> 32));
    for (uint32_t k = 0; k < t; k += 16) {
        acc64_512(S, k, t, v0, add);
        if (k + 8 < t) acc64_512(S, k + 8, t, v1, add);
        if (k + 16 < t) {
            v0 = mulmod64_512(v0, b0, b1);
            v1 = mulmod64_512(v1, b0, b1);
        }
    }
}

static bool cpu_has_avx512() {
    static const int ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
                          __builtin_cpu_supports("avx512dq");
    return ok;
}

template <class F, bool ADD>
inline void power_walk(typename F::T *S, uint32_t t, typename F::T x) {
    using T = typename F::T;
    if constexpr (sizeof(T) == 4) {
        if (t >= 8 && cpu_has_avx512()) {
            power_walk32_avx512(S, t, x, ADD);
            return;
        }
    } else {
        if (t >= 16 && cpu_has_avx512()) {   // below 16 the scalar chains win (measured)
            power_walk64_avx512(S, t, x, ADD);
            return;
        }
    }
    auto acc = [&](uint32_t k, T y) { S[k] = ADD ? F::add(S[k], y) : F::sub(S[k], y); };
    if (t < 8) {                         // short: the plain chain
        T y = x;
        for (uint32_t k = 0; k < t; ++k) {
            acc(k, y);
            y = F::mul(y, x);
        }
        return;
    }
    // C independent chains: p[j] = x^(j+1) * (x^C)^i
    constexpr int C = 4;
    T p[C];
    p[0] = x;
    for (int j = 1; j < C; ++j) p[j] = F::mul(p[(j - 1) / 2], p[j / 2]);   // x^(j+1) from two lower powers
    const T xc = p[C - 1];
    uint32_t k = 0;
    for (; k + C <= t; k += C) {
        for (int j = 0; j < C; ++j) acc(k + j, p[j]);
        for (int j = 0; j < C; ++j) p[j] = F::mul(p[j], xc);
    }
    for (int j = 0; k + j < t; ++j) acc(k + j, p[j]);
}
} // namespace

extern "C" {

const char *qk_strerror(int s) {
    switch (s) {
    case QK_OK: return "ok";
    case QK_E_INVAL: return "invalid argument";
    case QK_E_THRESHOLD: return "invalid threshold";
    case QK_E_MISMATCH: return "threshold mismatch";
    case QK_E_UNDECODABLE: return "undecodable: count exceeds threshold";
    case QK_E_CAPACITY: return "output buffer too small";
    case QK_E_HIP: return "HIP runtime error";
    case QK_E_NO_DEVICE: return "no usable gfx950 device";
    case QK_E_NOMEM: return "out of memory";
    case QK_E_FORMAT: return "malformed serialized quACK";
    case QK_E_COMM: return "collective failed (communicator aborted)";
    case QK_E_PEER: return "another rank of the communicator failed";
    default: return "unknown error";
    }
}

const char *qk_version(void) { return "quack-hip 0.1.0 (gfx950)"; }

size_t qk_u32_size(uint32_t t) { return sizeof(qk_u32) + (size_t)t * sizeof(uint32_t); }
size_t qk_u64_size(uint32_t t) { return sizeof(qk_u64) + (size_t)t * sizeof(uint64_t); }

int qk_u32_init(qk_u32 *q, uint32_t t) {
    if (!q) return QK_E_INVAL;
    memset(q, 0, qk_u32_size(t));
    q->threshold = t;
    return QK_OK;
}
int qk_u64_init(qk_u64 *q, uint32_t t) {
    if (!q) return QK_E_INVAL;
    memset(q, 0, qk_u64_size(t));
    q->threshold = t;
    return QK_OK;
}

// ---------------------------------------------------------------- insert

int qk_u32_insert(qk_u32 *q, uint32_t id) {
    if (!q) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    if (t == 0) return QK_E_THRESHOLD; // reference: index underflow panic
    power_walk<F32, true>(q->power_sums, t, canon32(id));
    q->count += 1u;
    q->has_last = 1;
    q->last_value = id;
    return QK_OK;
}

int qk_u64_insert(qk_u64 *q, uint64_t id) {
    if (!q) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    if (t == 0) return QK_E_THRESHOLD;
    power_walk<F64, true>(q->power_sums, t, canon64(id));
    q->count += 1u;
    q->has_last = 1;
    q->last_value = id;
    return QK_OK;
}

int qk_u32_remove(qk_u32 *q, uint32_t id) {
    if (!q) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    if (t == 0) return QK_E_THRESHOLD;
    power_walk<F32, false>(q->power_sums, t, canon32(id));
    q->count -= 1u;
    return QK_OK;
}

int qk_u64_remove(qk_u64 *q, uint64_t id) {
    if (!q) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    if (t == 0) return QK_E_THRESHOLD;
    power_walk<F64, false>(q->power_sums, t, canon64(id));
    q->count -= 1u;
    return QK_OK;
}

// ---------------------------------------------------------- sub / merge
int qk_u32_sub_assign(qk_u32 *q, const qk_u32 *r) {
    if (!q || !r) return QK_E_INVAL;
    if (q->threshold != r->threshold) return QK_E_MISMATCH;
    for (uint32_t k = 0; k < q->threshold; ++k) q->power_sums[k] = sub32(q->power_sums[k], r->power_sums[k]);
    q->count -= r->count;
    return QK_OK;
}
int qk_u64_sub_assign(qk_u64 *q, const qk_u64 *r) {
    if (!q || !r) return QK_E_INVAL;
    if (q->threshold != r->threshold) return QK_E_MISMATCH;
    for (uint32_t k = 0; k < q->threshold; ++k) q->power_sums[k] = sub64(q->power_sums[k], r->power_sums[k]);
    q->count -= r->count;
    return QK_OK;
}
int qk_u32_merge(qk_u32 *q, const qk_u32 *r) {
    if (!q || !r) return QK_E_INVAL;
    if (q->threshold != r->threshold) return QK_E_MISMATCH;
    for (uint32_t k = 0; k < q->threshold; ++k) q->power_sums[k] = add32(q->power_sums[k], r->power_sums[k]);
    q->count += r->count;
    if (r->has_last) { q->has_last = 1; q->last_value = r->last_value; }
    return QK_OK;
}
int qk_u64_merge(qk_u64 *q, const qk_u64 *r) {
    if (!q || !r) return QK_E_INVAL;
    if (q->threshold != r->threshold) return QK_E_MISMATCH;
    for (uint32_t k = 0; k < q->threshold; ++k) q->power_sums[k] = add64(q->power_sums[k], r->power_sums[k]);
    q->count += r->count;
    if (r->has_last) { q->has_last = 1; q->last_value = r->last_value; }
    return QK_OK;
}

// ------------------------------------------------------------ partials
size_t qk_u32_partial_words(uint32_t t) { return (size_t)t + 2; }
size_t qk_u64_partial_words(uint32_t t) { return 2 * (size_t)t + 2; }

int qk_u32_merge_partial(qk_u32 *q, const uint64_t *part, int has_last, uint32_t last) {
    if (!q || !part) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    for (uint32_t k = 0; k < t; ++k) q->power_sums[k] = add32(q->power_sums[k], canon32(fold64_32(part[k])));
    q->count += (uint32_t)part[t];
    if (has_last) { q->has_last = 1; q->last_value = last; }
    return QK_OK;
}
int qk_u64_merge_partial(qk_u64 *q, const uint64_t *part, int has_last, uint64_t last) {
    if (!q || !part) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    for (uint32_t k = 0; k < t; ++k) {
        // value = lo_sum + hi_sum * 2^32, each limb sum < 2^59
        const uint64_t lo = part[2 * k], hi = part[2 * k + 1];
        unsigned __int128 v = (unsigned __int128)hi * (1ull << 32) + lo; // < 2^92
        const uint64_t vhi = (uint64_t)(v >> 64), vlo = (uint64_t)v;    // vhi < 2^28
        q->power_sums[k] = add64(q->power_sums[k], canon64(fold96_64((uint32_t)vhi, vlo)));
    }
    q->count += (uint32_t)part[2 * t];
    if (has_last) { q->has_last = 1; q->last_value = last; }
    return QK_OK;
}

// ----------------------------------------------------------- to_coeffs
// Newton's identities, 0-indexed: c[i] = -(S[i] + sum_{j<i} S[j] c[i-j-1]) / (i+1).
// Inverses of 1..d by the linear recurrence inv[i] = -(p/i) * inv[p mod i].
} // extern "C"
namespace {
// sum_{j<i} S[j] c[i-j-1] on AVX-512: eight products per step (c read
// backwards by a lane reversal), each folded once to < 6 2^32 and summed in
// 64-bit lanes (< 2^29 terms cannot overflow), the lanes added at the end.
QK_AVX512 static uint64_t newton_dot_avx512(const uint32_t *S, const uint32_t *c, uint32_t i) {
    const __m512i rev = _mm512_set_epi64(0, 1, 2, 3, 4, 5, 6, 7);
    __m512i acc = _mm512_setzero_si512();
    uint32_t j = 0;
    for (; j + 8 <= i; j += 8) {
        const __m512i s = _mm512_cvtepu32_epi64(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(S + j)));
        // c[i-j-1] .. c[i-j-8]: load c[i-j-8 .. i-j-1] and reverse the lanes
        const __m512i cv = _mm512_permutexvar_epi64(
            rev, _mm512_cvtepu32_epi64(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(c + (i - j - 8)))));
        acc = _mm512_add_epi64(acc, fold512(_mm512_mul_epu32(s, cv)));
    }
    uint64_t r = _mm512_reduce_add_epi64(acc);   // < 2^29 * 6 * 2^32
    for (; j < i; ++j) r += mul32(S[j], c[i - j - 1]);
    return r;
}
} // namespace
extern "C" {

int qk_u32_to_coeffs(const qk_u32 *q, uint32_t *c, uint32_t cap, uint32_t *d_out) {
    if (!q || !d_out) return QK_E_INVAL;
    const uint32_t d = q->count;
    if (d > q->threshold) { *d_out = d; return QK_E_UNDECODABLE; }
    *d_out = d;
    if (cap < d || (d && !c)) return QK_E_CAPACITY;
    std::vector<uint32_t> inv(d + 2, 1);
    for (uint32_t i = 2; i <= d; ++i) inv[i] = mul32(P32 - P32 / i, inv[P32 % i]);
    const bool vec = d > 16 && cpu_has_avx512();
    for (uint32_t i = 0; i < d; ++i) {
        uint64_t acc = q->power_sums[i];            // lazy: < 2^32 + i * 6 * 2^32
        if (vec) {
            acc += newton_dot_avx512(q->power_sums, c, i);
        } else {
            for (uint32_t j = 0; j < i; ++j) acc += mul32(q->power_sums[j], c[i - j - 1]);
        }
        c[i] = mul32(neg32(canon32(fold64_32(acc))), inv[i + 1]);
    }
    return QK_OK;
}

} // extern "C"
namespace {
// u64 twin of newton_dot_avx512: lane products by mulmod64_512 (< 2^64, lazy)
// summed with the 2^64 == 59 wrap fix, the eight lanes folded canonically
QK_AVX512 static uint64_t newton_dot64_avx512(const uint64_t *S, const uint64_t *c, uint32_t i) {
    const __m512i rev = _mm512_set_epi64(0, 1, 2, 3, 4, 5, 6, 7), c59 = _mm512_set1_epi64(59);
    __m512i acc = _mm512_setzero_si512();
    uint32_t j = 0;
    for (; j + 8 <= i; j += 8) {
        const __m512i s = _mm512_loadu_si512(S + j);
        const __m512i cv = _mm512_permutexvar_epi64(rev, _mm512_loadu_si512(c + (i - j - 8)));
        const __m512i pr = mulmod64_512(s, cv, _mm512_srli_epi64(cv, 32));
        // acc, pr < 2^64 (lazy): a wrap adds 59, and that +59 can wrap once more
        // (sm > 2^64 - 60 only when both were near 2^64): then +59 again
        const __m512i sm = _mm512_add_epi64(acc, pr);
        const __mmask8 w1 = _mm512_cmplt_epu64_mask(sm, pr);
        const __m512i s1 = _mm512_mask_add_epi64(sm, w1, sm, c59);
        acc = _mm512_mask_add_epi64(s1, w1 & _mm512_cmplt_epu64_mask(s1, c59), s1, c59);
    }
    alignas(64) uint64_t lane[8];
    _mm512_store_si512(lane, acc);
    uint64_t r = 0;
    for (int k = 0; k < 8; ++k) r = add64(r, canon64(lane[k]));
    for (; j < i; ++j) r = add64(r, mul64(S[j], c[i - j - 1]));
    return r;
}
} // namespace
extern "C" {

int qk_u64_to_coeffs(const qk_u64 *q, uint64_t *c, uint32_t cap, uint32_t *d_out) {
    if (!q || !d_out) return QK_E_INVAL;
    const uint32_t d = q->count;
    if (d > q->threshold) { *d_out = d; return QK_E_UNDECODABLE; }
    *d_out = d;
    if (cap < d || (d && !c)) return QK_E_CAPACITY;
    std::vector<uint64_t> inv(d + 2, 1);
    for (uint32_t i = 2; i <= d; ++i) inv[i] = mul64(P64 - P64 / i, inv[P64 % i]);
    const bool vec = d > 16 && cpu_has_avx512();
    for (uint32_t i = 0; i < d; ++i) {
        uint64_t acc = q->power_sums[i];
        if (vec) acc = add64(acc, newton_dot64_avx512(q->power_sums, c, i));
        else
            for (uint32_t j = 0; j < i; ++j) acc = add64(acc, mul64(q->power_sums[j], c[i - j - 1]));
        c[i] = mul64(neg64(acc), inv[i + 1]);
    }
    return QK_OK;
}

// ---------------------------------------------------------------- eval
uint32_t qk_u32_eval(const uint32_t *c, uint32_t d, uint32_t id) {
    if (d == 0 || !c) return 1;
    const uint32_t x = canon32(id);
    uint32_t r = x;
    for (uint32_t i = 0; i + 1 < d; ++i) r = mul32(add32(r, c[i]), x);
    return add32(r, c[d - 1]);
}
uint64_t qk_u64_eval(const uint64_t *c, uint32_t d, uint64_t id) {
    if (d == 0 || !c) return 1;
    const uint64_t x = canon64(id);
    uint64_t r = x;
    for (uint32_t i = 0; i + 1 < d; ++i) r = mul64(add64(r, c[i]), x);
    return add64(r, c[d - 1]);
}

// ------------------------------------------------------------- host decode
// decode_with_log over a host-resident log (media_client.rs:304-313 for the
// short logs a receiver holds between quACKs: a kernel launch costs more
// than the whole test).  Same arithmetic forms as the device root test:
// t-form Horner r <- r*x + c_i for u32 (field.h tstep32), lazy 64-bit mads
// for u64; a root iff the canonical value is 0.
} // extern "C"
namespace {
// u32 candidate scan on an AVX-512 CPU: 32 candidates per iteration as four
// independent zmm Horner chains (lane value r < 2^32 lazy: r <- r x + c_i is
// < 2^64, then the two 2^32 == 5 folds); a root iff r == 0 or r == p.  Hits
// in log order.  Returns the number of hits (all counted, <= cap stored).
QK_AVX512 static size_t root_scan32_avx512(const uint32_t *c, uint32_t d, const uint32_t *log, size_t n,
                                           uint64_t *hits, size_t cap) {
    const __m512i P = _mm512_set1_epi64(P32), TWO32 = _mm512_set1_epi64(1ll << 32), ONE = _mm512_set1_epi64(1);
    size_t m = 0;
    for (size_t i = 0; i < n; i += 32) {
        __m512i x[4], r[4];
        __mmask8 valid[4];
        for (int u = 0; u < 4; ++u) {
            const size_t b = i + 8 * (size_t)u;
            const size_t rem = b < n ? n - b : 0;
            valid[u] = rem >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << rem) - 1u);
            const __m512i v = _mm512_cvtepu32_epi64(_mm256_maskz_loadu_epi32(valid[u], log + (b < n ? b : 0)));
            x[u] = _mm512_mask_sub_epi64(v, _mm512_cmpge_epu64_mask(v, P), v, P);   // canonical id
            r[u] = ONE;
        }
        for (uint32_t k = 0; k < d; ++k) {
            const __m512i ck = _mm512_set1_epi64(c[k]);
            for (int u = 0; u < 4; ++u) {
                const __m512i v = fold512(fold512(_mm512_add_epi64(_mm512_mul_epu32(r[u], x[u]), ck)));
                r[u] = _mm512_mask_sub_epi64(v, _mm512_cmpge_epu64_mask(v, TWO32), v, P);   // < 2^32
            }
        }
        for (int u = 0; u < 4; ++u) {
            __mmask8 h = (_mm512_cmpeq_epu64_mask(r[u], _mm512_setzero_si512()) |
                          _mm512_cmpeq_epu64_mask(r[u], P)) & valid[u];
            while (h) {
                const int j = __builtin_ctz(h);
                if (m < cap && hits) hits[m] = i + 8 * (size_t)u + j;
                ++m;
                h &= (__mmask8)(h - 1);
            }
        }
    }
    return m;
}

// u64 twin: r <- r x + c_i with the lane products of mulmod64_512 (x's
// halves per lane) and a lazy add (a wrap past 2^64 adds 59); a root iff
// r == 0 or r == p.  Same stop handling and hit order as the u32 scan.
QK_AVX512 static size_t root_scan64_avx512(const uint64_t *c, uint32_t d, const uint64_t *log, size_t n,
                                           uint64_t *hits, size_t cap) {
    const __m512i P = _mm512_set1_epi64((long long)P64), c59 = _mm512_set1_epi64(59), ONE = _mm512_set1_epi64(1);
    size_t m = 0;
    for (size_t i = 0; i < n; i += 32) {
        __m512i x0[4], x1[4], r[4];
        __mmask8 valid[4];
        for (int u = 0; u < 4; ++u) {
            const size_t b = i + 8 * (size_t)u;
            const size_t rem = b < n ? n - b : 0;
            valid[u] = rem >= 8 ? (__mmask8)0xFF : (__mmask8)((1u << rem) - 1u);
            const __m512i v = _mm512_maskz_loadu_epi64(valid[u], log + (b < n ? b : 0));
            x0[u] = v;                                  // vpmuludq reads the low halves
            x1[u] = _mm512_srli_epi64(v, 32);
            r[u] = ONE;
        }
        for (uint32_t k = 0; k < d; ++k) {
            const __m512i ck = _mm512_set1_epi64((long long)c[k]);
            for (int u = 0; u < 4; ++u) {
                const __m512i pr = mulmod64_512(r[u], x0[u], x1[u]);
                const __m512i sm = _mm512_add_epi64(pr, ck);
                r[u] = _mm512_mask_add_epi64(sm, _mm512_cmplt_epu64_mask(sm, pr), sm, c59);
            }
        }
        for (int u = 0; u < 4; ++u) {
            __mmask8 h = (_mm512_cmpeq_epu64_mask(r[u], _mm512_setzero_si512()) |
                          _mm512_cmpeq_epu64_mask(r[u], P)) & valid[u];
            while (h) {
                const int j = __builtin_ctz(h);
                if (m < cap && hits) hits[m] = i + 8 * (size_t)u + j;
                ++m;
                h &= (__mmask8)(h - 1);
            }
        }
    }
    return m;
}

template <typename Q, typename T, typename ToCoeffs, typename IsRoot>
int decode_host_impl(const Q *diff, const T *log, size_t n, int stop_at_last, uint64_t *hits, size_t cap,
                     size_t *n_hits, ToCoeffs to_coeffs, IsRoot is_root) {
    if (!diff || !n_hits || (n && !log)) return QK_E_INVAL;
    *n_hits = 0;
    if (diff->count == 0) return QK_OK;
    std::vector<T> c(diff->threshold ? diff->threshold : 1);
    uint32_t d = 0;
    if (int rc = to_coeffs(diff, c.data(), (uint32_t)c.size(), &d)) return rc;
    const bool stop = stop_at_last && diff->has_last;
    size_t m = 0;
    if (cpu_has_avx512() && d > 0) {
        size_t ne = n;   // the scan ends at the first entry equal to last_value (media_client.rs:307-309)
        if (stop)
            for (size_t i = 0; i < n; ++i)
                if (log[i] == (T)diff->last_value) { ne = i; break; }
        if constexpr (sizeof(T) == 4) m = root_scan32_avx512(c.data(), d, log, ne, hits, cap);
        else m = root_scan64_avx512(c.data(), d, log, ne, hits, cap);
        *n_hits = m;
        return m > cap || (m && !hits) ? QK_E_CAPACITY : QK_OK;
    }
    for (size_t i = 0; i < n; ++i) {
        if (stop && log[i] == (T)diff->last_value) break;   // media_client.rs:307-309
        if (is_root(c.data(), d, log[i])) {
            if (m < cap && hits) hits[m] = i;
            ++m;
        }
    }
    *n_hits = m;
    return m > cap || (m && !hits) ? QK_E_CAPACITY : QK_OK;
}

bool root32(const uint32_t *c, uint32_t d, uint32_t id) {
    const uint32_t x = canon32(id), x5 = times5_32(x);
    uint32_t lo = 1, hi = 0;
    for (uint32_t i = 0; i < d; ++i) tstep32(lo, hi, x, x5, c[i]);
    return canon32(fold64_32(((uint64_t)hi << 32) | lo)) == 0;
}
bool root64(const uint64_t *c, uint32_t d, uint64_t id) {
    uint64_t r = 1;
    for (uint32_t i = 0; i < d; ++i) r = mad64_lazy(r, id, c[i]);
    return canon64(r) == 0;
}
} // namespace
extern "C" {

int qk_u32_decode_host(const qk_u32 *diff, const uint32_t *log, size_t n, int stop_at_last, uint64_t *hits,
                       size_t cap, size_t *n_hits) {
    return decode_host_impl(diff, log, n, stop_at_last, hits, cap, n_hits, qk_u32_to_coeffs, root32);
}
int qk_u64_decode_host(const qk_u64 *diff, const uint64_t *log, size_t n, int stop_at_last, uint64_t *hits,
                       size_t cap, size_t *n_hits) {
    return decode_host_impl(diff, log, n, stop_at_last, hits, cap, n_hits, qk_u64_to_coeffs, root64);
}

// ------------------------------------------------------------- bincode
// bincode 1.3 default options: little-endian fixed-width ints, u64 length
// prefix for Vec, u8 tag for Option.  Field order as declared in the
// crate's struct: power_sums, last_value, count  ([RECALL]).
size_t qk_u32_serialized_size(const qk_u32 *q) {
    return q ? 8 + 4 * (size_t)q->threshold + 1 + (q->has_last ? 4 : 0) + 4 : 0;
}
size_t qk_u64_serialized_size(const qk_u64 *q) {
    return q ? 8 + 8 * (size_t)q->threshold + 1 + (q->has_last ? 8 : 0) + 4 : 0;
}

int qk_u32_serialize(const qk_u32 *q, uint8_t *buf, size_t cap, size_t *len) {
    if (!q || !len) return QK_E_INVAL;
    const size_t need = qk_u32_serialized_size(q);
    *len = need;
    if (cap < need || !buf) return QK_E_CAPACITY;
    uint8_t *p = buf;
    put_le(p, q->threshold, 8); p += 8;
    for (uint32_t k = 0; k < q->threshold; ++k) { put_le(p, q->power_sums[k], 4); p += 4; }
    *p++ = q->has_last ? 1 : 0;
    if (q->has_last) { put_le(p, q->last_value, 4); p += 4; }
    put_le(p, q->count, 4);
    return QK_OK;
}
int qk_u64_serialize(const qk_u64 *q, uint8_t *buf, size_t cap, size_t *len) {
    if (!q || !len) return QK_E_INVAL;
    const size_t need = qk_u64_serialized_size(q);
    *len = need;
    if (cap < need || !buf) return QK_E_CAPACITY;
    uint8_t *p = buf;
    put_le(p, q->threshold, 8); p += 8;
    for (uint32_t k = 0; k < q->threshold; ++k) { put_le(p, q->power_sums[k], 8); p += 8; }
    *p++ = q->has_last ? 1 : 0;
    if (q->has_last) { put_le(p, q->last_value, 8); p += 8; }
    put_le(p, q->count, 4);
    return QK_OK;
}

int qk_u32_deserialize(const uint8_t *buf, size_t len, qk_u32 *q, uint32_t *t_out) {
    return deser<qk_u32, uint32_t>(buf, len, q, t_out, P32);
}
int qk_u64_deserialize(const uint8_t *buf, size_t len, qk_u64 *q, uint32_t *t_out) {
    return deser<qk_u64, uint64_t>(buf, len, q, t_out, P64);
}

} // extern "C"
