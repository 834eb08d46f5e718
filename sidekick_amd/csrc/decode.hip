// decode.hip — decode-missing root test on gfx950.
//
// Replaces the candidate scan of media_client.rs:306-313
//     for (seqno, id) in log { if Some(id) == diff.last_value() { break }
//                              if arithmetic::eval(&coeffs, id).value() == 0 { missing.push } }
// for a candidate log resident in HBM.  Each lane tests 4 (u32) or 2 (u64)
// candidates per 16-byte load; the d coefficients are wave-uniform and come
// from the scalar cache.  The polynomial is evaluated in the fused form
// r <- r*x + c_i (one lazy mad per coefficient), which is the same
// polynomial z^d + c_1 z^(d-1) + ... + c_d as the reference's
// r <- (r + c_i)*x form, so the canonical value (and the ==0 test) is
// identical.  Hits are rare (d roots among n candidates): appended with an
// atomic ticket; the host sorts them into log order.  The `break` at the
// first log entry equal to diff.last_value() becomes an atomicMin of that
// position; the host drops hits at or after it.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "bsgs64.h"
#include "ctx.h"
#include "field.h"

namespace qk {

QK_WARM_KERNEL(decode)

constexpr int RT_BLOCK = 256;

// hout (optional, k_root_scan): the hit / stop also into pinned host memory.
// hbase / sbase: the values the hit / stop tickets (counters[0], [3]) start
// from in this launch (0 after the host reset them; the kernel-argument form
// of the scan keeps them running across calls instead of resetting them)
__device__ __forceinline__ void rt_record(uint64_t pos, bool hit, bool stop, uint64_t *hits, uint64_t cap,
                                          uint64_t *counters, uint64_t *hout = nullptr, uint32_t nhpf = 0,
                                          uint64_t hbase = 0, uint64_t sbase = 0) {
    // the slots in pinned host memory by system-scope stores (written
    // through the L2: no write-back needed before the host reads them)
    auto put = [&](size_t i, uint64_t v) { __hip_atomic_store(&hout[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    if (hit) {
        const uint64_t slot = atomicAdd((unsigned long long *)&counters[0], 1ull) - hbase;
        if (slot < cap) hits[slot] = pos;
        if (hout) {
            if (slot < nhpf) put(4 + slot, pos);
            else put(2, 1);
        }
    }
    if (stop) {
        atomicMin((unsigned long long *)&counters[1], (unsigned long long)pos);
        if (hout) {
            const uint64_t k = atomicAdd((unsigned long long *)&counters[3], 1ull) - sbase;
            if (k < RT_NSTOP) put(RT_STOP0 + k, pos);
            else put(2, 1);
        }
    }
}

// ------------------------------------------------------------------ u32
// Horner in t-form (field.h tstep32): r <- r*x + c_i is three mads + one sub.
__device__ __forceinline__ bool t_is_zero32(uint32_t lo, uint32_t hi) {
    return canon32(fold64_32(((uint64_t)hi << 32) | lo)) == 0;
}

__device__ __forceinline__ bool is_root32(uint32_t id, const uint32_t *__restrict__ c, uint32_t d) {
    const uint32_t x = canon32(id), x5 = times5_32(x);
    uint32_t lo = 1, hi = 0;
    for (uint32_t i = 0; i < d; ++i) tstep32(lo, hi, x, x5, c[i]);
    return t_is_zero32(lo, hi);
}

template <int D> // D > 0: compile-time degree (fully unrolled); D == 0: runtime d
__device__ __forceinline__ void horner32x4(uint4 w, const uint32_t *__restrict__ c, uint32_t d, bool (&hit)[4]) {
    const uint32_t x0 = canon32(w.x), x1 = canon32(w.y), x2 = canon32(w.z), x3 = canon32(w.w);
    const uint32_t f0 = times5_32(x0), f1 = times5_32(x1), f2 = times5_32(x2), f3 = times5_32(x3);
    uint32_t l0 = 1, l1 = 1, l2 = 1, l3 = 1, h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    if constexpr (D > 0) {
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const uint32_t ci = c[i];
            tstep32(l0, h0, x0, f0, ci);
            tstep32(l1, h1, x1, f1, ci);
            tstep32(l2, h2, x2, f2, ci);
            tstep32(l3, h3, x3, f3, ci);
        }
    } else {
#pragma unroll 4
        for (uint32_t i = 0; i < d; ++i) {
            const uint32_t ci = c[i];
            tstep32(l0, h0, x0, f0, ci);
            tstep32(l1, h1, x1, f1, ci);
            tstep32(l2, h2, x2, f2, ci);
            tstep32(l3, h3, x3, f3, ci);
        }
    }
    hit[0] = t_is_zero32(l0, h0);
    hit[1] = t_is_zero32(l1, h1);
    hit[2] = t_is_zero32(l2, h2);
    hit[3] = t_is_zero32(l3, h3);
}

template <int D>
__global__ __launch_bounds__(RT_BLOCK) void k_root_test_u32(const uint32_t *__restrict__ log, uint64_t n,
                                                            uint32_t head, const uint32_t *__restrict__ c,
                                                            uint32_t d, int use_stop, uint32_t stop_value,
                                                            uint64_t *__restrict__ hits, uint64_t cap,
                                                            uint64_t *__restrict__ counters) {
    const uint64_t gtid = (uint64_t)blockIdx.x * RT_BLOCK + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * RT_BLOCK;
    const uint64_t h = head < n ? head : n;
    const uint64_t body = (n - h) >> 2;
    const uint4 *__restrict__ v = reinterpret_cast<const uint4 *>(log + h);
    for (uint64_t i = gtid; i < body; i += nthr) {
        const uint4 w = v[i];
        bool hit[4];
        horner32x4<D>(w, c, d, hit);
        const uint64_t pos = h + 4 * i;
        const bool s0 = use_stop && w.x == stop_value, s1 = use_stop && w.y == stop_value;
        const bool s2 = use_stop && w.z == stop_value, s3 = use_stop && w.w == stop_value;
        if (hit[0] | hit[1] | hit[2] | hit[3] | s0 | s1 | s2 | s3) {
            rt_record(pos + 0, hit[0], s0, hits, cap, counters);
            rt_record(pos + 1, hit[1], s1, hits, cap, counters);
            rt_record(pos + 2, hit[2], s2, hits, cap, counters);
            rt_record(pos + 3, hit[3], s3, hits, cap, counters);
        }
    }
    const uint64_t tail0 = h + (body << 2);
    if (gtid < h) {
        const uint32_t x = log[gtid];
        rt_record(gtid, is_root32(x, c, d), use_stop && x == stop_value, hits, cap, counters);
    }
    if (gtid < n - tail0) {
        const uint64_t pos = tail0 + gtid;
        const uint32_t x = log[pos];
        rt_record(pos, is_root32(x, c, d), use_stop && x == stop_value, hits, cap, counters);
    }
}

// ------------------------------------------------------------------ u64
// Horner r <- r*x + c_i with the hand-scheduled p64 step (bsgs64.h: 7
// mads, exact, result < 2^64) followed by a 64-bit add of c_i: a wrap past
// 2^64 leaves < c_i < p - 59, so the +59 cannot wrap again.  r pinned in
// v[2:3] like the step; c_i in VGPRs (gfx950 VALU reads at most one SGPR).
__device__ __forceinline__ void horner64_step(uint64_t &V, uint32_t x0, uint32_t x1, uint64_t c) {
    uint64_t cw, cx, cc, ce, cy;
    uint32_t tmp;
    asm volatile(QK_U64_MULV_ASM
                 "v_add_co_u32_e64 v2, %[cy], v2, %[c0]\n\t"
                 "s_nop 1\n\t"
                 "v_addc_co_u32_e64 v3, %[cy], v3, %[c1], %[cy]\n\t"
                 "s_nop 1\n\t"
                 "v_cndmask_b32_e64 v11, 0, 1, %[cy]\n\t"
                 "v_mad_u64_u32 v[2:3], %[cx], v11, 59, v[2:3]"
                 : "+{v[2:3]}"(V), [cw] "=&s"(cw), [cx] "=&s"(cx), [cc] "=&s"(cc), [ce] "=&s"(ce), [cy] "=&s"(cy),
                   [tmp] "=&v"(tmp)
                 : [x0] "v"(x0), [x1] "v"(x1), [c0] "v"((uint32_t)c), [c1] "v"((uint32_t)(c >> 32))
                 : "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11");
}

__device__ __forceinline__ bool is_root64(uint64_t x, const uint64_t *__restrict__ c, uint32_t d) {
    const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32);
    uint64_t r = 1;
    for (uint32_t i = 0; i < d; ++i) horner64_step(r, x0, x1, c[i]);
    return canon64(r) == 0;
}

__global__ __launch_bounds__(RT_BLOCK) void k_root_test_u64(const uint64_t *__restrict__ log, uint64_t n,
                                                            uint32_t head, const uint64_t *__restrict__ c,
                                                            uint32_t d, int use_stop, uint64_t stop_value,
                                                            uint64_t *__restrict__ hits, uint64_t cap,
                                                            uint64_t *__restrict__ counters) {
    const uint64_t gtid = (uint64_t)blockIdx.x * RT_BLOCK + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * RT_BLOCK;
    const uint64_t h = head < n ? head : n;
    const uint64_t body = (n - h) >> 1;
    const ulonglong2 *__restrict__ v = reinterpret_cast<const ulonglong2 *>(log + h);
    for (uint64_t i = gtid; i < body; i += nthr) {
        const ulonglong2 w = v[i];
        const bool h0 = is_root64(w.x, c, d), h1 = is_root64(w.y, c, d);
        const bool s0 = use_stop && w.x == stop_value, s1 = use_stop && w.y == stop_value;
        if (h0 | h1 | s0 | s1) {
            rt_record(h + 2 * i, h0, s0, hits, cap, counters);
            rt_record(h + 2 * i + 1, h1, s1, hits, cap, counters);
        }
    }
    const uint64_t tail0 = h + (body << 1);
    if (gtid < h) {
        const uint64_t x = log[gtid];
        rt_record(gtid, is_root64(x, c, d), use_stop && x == stop_value, hits, cap, counters);
    }
    if (gtid < n - tail0) {
        const uint64_t pos = tail0 + gtid;
        const uint64_t x = log[pos];
        rt_record(pos, is_root64(x, c, d), use_stop && x == stop_value, hits, cap, counters);
    }
}

// u64, baby-step / giant-step evaluation for 16 <= d <= RT64_BSGS_MAXD:
//   P(x) = x^d + sum_{k<d} p_k x^k = sum_a x^(8a) Q_a(x),  Q_a = sum_{b<8} p_(8a+b) x^b
// (the top block holds x^r, r = d mod 8, as a coefficient 1; d = 8A: R starts
// at 1), then Horner in x^8 over the blocks.  The inner sums are carry-free:
// the babies x^1..x^7 are split into 22-bit limbs l_j (B = l0 + l1 2^22 +
// l2 2^44), and the host pre-shifts every coefficient by 2^(22j) mod p, so
//   p * B == sum_j l_j * (p 2^(22j) mod p)
// is six 22x32-bit mads into two 64-bit sums (weights 1 and 2^32) per term:
// 21 products < 2^54 per sum stay below 2^59, no carry is ever counted.
// Per candidate at d = 32: 7 + 4 p64 multiplies and 168 mads, against 32
// Horner steps of 7 multiplies each.  Table: tab[(8a + b) * 3 + j] =
// p_(8a+b) * 2^(22j) mod p (u64), blocks a = 0 .. nblk - 1 (the last one the
// top block when d % 8 != 0).
constexpr uint32_t RT64_BSGS_MIND = 16;
constexpr uint32_t RT64_BSGS_MAXD = 1000;   // (ceil((d+1)/8) * 24 words <= SMALL_NHITS - RT_C)

__device__ __forceinline__ uint64_t rt_limb_sum(uint64_t lo, uint64_t hi, uint64_t c) {
    // lo + hi * 2^32 + c  (lo, hi < 2^59) reduced below 2^64 (not canonical)
    const uint64_t h1 = hi >> 32, h0 = hi & 0xFFFFFFFFull;
    unsigned __int128 v = (unsigned __int128)lo + (h0 << 32) + (unsigned __int128)h1 * C64 + c;
    uint64_t r = (uint64_t)v;
    const uint64_t top = (uint64_t)(v >> 64);           // <= 2
    const uint64_t add = top * C64;
    uint64_t q = r + add;
    if (q < r) q += C64;                                 // wrapped past 2^64 once: < 2*59 + 59, no second wrap
    return q;
}

// Q_a of W candidates at once: the block's coefficients are loaded once (scalar
// loads) and feed the MACs of every candidate
template <int W>
__device__ __forceinline__ void rt_block(const uint64_t *__restrict__ tab, uint32_t a,
                                         const uint32_t (&l)[W][7][3], uint64_t (&q)[W]) {
    uint64_t slo[W], shi[W];
#pragma unroll
    for (int w = 0; w < W; ++w) { slo[w] = 0; shi[w] = 0; }
#pragma unroll
    for (int b = 1; b < 8; ++b)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const uint64_t c = tab[((size_t)a * 8 + b) * 3 + j];
#pragma unroll
            for (int w = 0; w < W; ++w) {
                slo[w] += (uint64_t)l[w][b - 1][j] * (uint32_t)c;
                shi[w] += (uint64_t)l[w][b - 1][j] * (uint32_t)(c >> 32);
            }
        }
    const uint64_t c0 = tab[(size_t)a * 8 * 3];
#pragma unroll
    for (int w = 0; w < W; ++w) q[w] = rt_limb_sum(slo[w], shi[w], c0);
}

// V + c (c < 2^64), reduced below 2^64
__device__ __forceinline__ uint64_t rt_add64(uint64_t V, uint64_t c) {
    uint64_t r = V + c;
    if (r < V) r += C64;   // 2^64 == 59; r < c here, so no second wrap
    return r;
}

// W candidates; NF > 0: the number of full blocks at compile time (unrolled)
template <int W, int NF>
__device__ __forceinline__ void is_root64_bsgs(const uint64_t (&x)[W], const uint64_t *__restrict__ tab,
                                               uint32_t nfull, bool top, bool (&hit)[W]) {
    uint32_t l[W][7][3], g0[W], g1[W];
    uint64_t R[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const uint32_t x0 = (uint32_t)x[w], x1 = (uint32_t)(x[w] >> 32);
        uint64_t V = x[w];
#pragma unroll
        for (int b = 1; b <= 7; ++b) {
            if (b > 1) bsgs64::mulv(V, x0, x1);
            l[w][b - 1][0] = (uint32_t)V & 0x3FFFFFu;
            l[w][b - 1][1] = (uint32_t)(V >> 22) & 0x3FFFFFu;
            l[w][b - 1][2] = (uint32_t)(V >> 44);
        }
        bsgs64::mulv(V, x0, x1);                        // x^8
        g0[w] = (uint32_t)V;
        g1[w] = (uint32_t)(V >> 32);
    }
    const uint32_t nf = NF > 0 ? (uint32_t)NF : nfull;
    if (top) {
        rt_block<W>(tab, nf, l, R);                     // x^r + lower terms of the top block
    } else {
#pragma unroll
        for (int w = 0; w < W; ++w) R[w] = 1;
    }
    uint64_t q[W];
    if constexpr (NF > 0) {
#pragma unroll
        for (int a = NF - 1; a >= 0; --a) {
            rt_block<W>(tab, (uint32_t)a, l, q);
#pragma unroll
            for (int w = 0; w < W; ++w) {
                bsgs64::mulv(R[w], g0[w], g1[w]);
                R[w] = rt_add64(R[w], q[w]);
            }
        }
    } else {
        for (uint32_t a = nf; a-- > 0;) {
            rt_block<W>(tab, a, l, q);
#pragma unroll
            for (int w = 0; w < W; ++w) {
                bsgs64::mulv(R[w], g0[w], g1[w]);
                R[w] = rt_add64(R[w], q[w]);
            }
        }
    }
#pragma unroll
    for (int w = 0; w < W; ++w) hit[w] = canon64(R[w]) == 0;
}

// candidates interleaved per evaluation (2 would share the coefficient loads,
// but the pinned-register p64 step then forces hundreds of register copies)
constexpr int RT64_W = 1;

template <int NF>
__global__ __launch_bounds__(RT_BLOCK) void k_root_test_u64_bsgs(const uint64_t *__restrict__ log, uint64_t n,
                                                                 uint32_t head, const uint64_t *__restrict__ tab,
                                                                 uint32_t nfull, int top, int use_stop,
                                                                 uint64_t stop_value, uint64_t *__restrict__ hits,
                                                                 uint64_t cap, uint64_t *__restrict__ counters) {
    const uint64_t gtid = (uint64_t)blockIdx.x * RT_BLOCK + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * RT_BLOCK;
    const uint64_t h = head < n ? head : n;
    const uint64_t body = (n - h) >> 1;
    const ulonglong2 *__restrict__ v = reinterpret_cast<const ulonglong2 *>(log + h);
    for (uint64_t i = gtid; i < body; i += nthr) {
        const ulonglong2 wv = v[i];
        bool hit[2];
        if constexpr (RT64_W == 2) {
            const uint64_t x[2] = {wv.x, wv.y};
            is_root64_bsgs<2, NF>(x, tab, nfull, top, hit);
        } else {
            const uint64_t x0[1] = {wv.x}, x1[1] = {wv.y};
            bool h0[1], h1[1];
            is_root64_bsgs<1, NF>(x0, tab, nfull, top, h0);
            is_root64_bsgs<1, NF>(x1, tab, nfull, top, h1);
            hit[0] = h0[0];
            hit[1] = h1[0];
        }
        const bool s0 = use_stop && wv.x == stop_value, s1 = use_stop && wv.y == stop_value;
        if (hit[0] | hit[1] | s0 | s1) {
            rt_record(h + 2 * i, hit[0], s0, hits, cap, counters);
            rt_record(h + 2 * i + 1, hit[1], s1, hits, cap, counters);
        }
    }
    const uint64_t tail0 = h + (body << 1);
    if (gtid < h) {
        const uint64_t x[1] = {log[gtid]};
        bool hit[1];
        is_root64_bsgs<1, NF>(x, tab, nfull, top, hit);
        rt_record(gtid, hit[0], use_stop && x[0] == stop_value, hits, cap, counters);
    }
    if (gtid < n - tail0) {
        const uint64_t pos = tail0 + gtid;
        const uint64_t x[1] = {log[pos]};
        bool hit[1];
        is_root64_bsgs<1, NF>(x, tab, nfull, top, hit);
        rt_record(pos, hit[0], use_stop && x[0] == stop_value, hits, cap, counters);
    }
}

bool rt64_use_bsgs(const qk_ctx *ctx, uint32_t d) {
    (void)ctx;
    return d >= RT64_BSGS_MIND && d <= RT64_BSGS_MAXD;
}

// host: the limb-shifted coefficient table of the BSGS kernel into out[]
// (canonical c_1..c_d of the monic polynomial); returns the words written
size_t rt64_bsgs_table(const uint64_t *coeffs, uint32_t d, uint64_t *out) {
    const uint32_t nfull = d / 8, r = d % 8, nblk = nfull + (r ? 1 : 0);
    const size_t words = (size_t)nblk * 24;
    for (size_t i = 0; i < words; ++i) out[i] = 0;
    for (uint32_t k = 0; k < 8 * nblk; ++k) {
        uint64_t pk;   // coefficient of x^k: p_d = 1, p_(d-i) = c_i
        if (k > d) pk = 0;
        else if (k == d) pk = 1;
        else pk = coeffs[d - k - 1];
        unsigned __int128 v = pk;
        for (int j = 0; j < 3; ++j) {
            out[(size_t)k * 3 + j] = (uint64_t)(v % P64);
            v = (v % P64) << 22;
        }
    }
    return words;
}

template <typename KernelT>
static uint32_t rs_grid(qk_ctx *ctx, KernelT kern, uint64_t units, size_t lds) {
    if (ctx->grid_override) return ctx->grid_override;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, RT_BLOCK, lds) != hipSuccess || occ < 1) occ = 1;
    const uint64_t full = (uint64_t)ctx->num_cus * occ;
    uint64_t need = (units + RT_BLOCK - 1) / RT_BLOCK;
    if (need < 1) need = 1;
    return (uint32_t)(need < full ? need : full);
}

// ------------------------------------------------------- root-set scan
// The same hit list from the roots of P (roots.cpp): P(x) == 0 exactly when
// x mod p is a root, so each candidate is reduced mod p and looked up in a
// hash set of the k <= d roots held in LDS — O(1) per candidate, the scan is
// bound by the HBM read of the log instead of d Horner steps.
// Set layout (built on the host, rt_scan_table): nb = 2^b buckets of S
// slots; root r sits in bucket h(r) = (lo(r) m1 + hi(r) m2 mod 2^32) >> (32 - b)
// (hi = 0 for u32), the multipliers chosen so that no bucket overflows; free
// slots hold all-ones (>= p, never equal to a reduced candidate).
template <typename T> __device__ __forceinline__ T rs_reduce(T x);
template <> __device__ __forceinline__ uint32_t rs_reduce<uint32_t>(uint32_t x) {
    const uint32_t y = x + C32;   // wraps exactly when x >= p (to x - p)
    return y < x ? y : x;
}
template <> __device__ __forceinline__ uint64_t rs_reduce<uint64_t>(uint64_t x) {
    const uint64_t y = x + C64;
    return y < x ? y : x;
}

template <typename T, int S>
__device__ __forceinline__ bool rs_member(T x, const T *__restrict__ set, uint32_t m1, uint32_t m2, uint32_t shift) {
    const T xr = rs_reduce<T>(x);
    uint32_t hh = (uint32_t)xr * m1;
    if constexpr (sizeof(T) == 8) hh += (uint32_t)(xr >> 32) * m2;
    const T *b = set + (size_t)(hh >> shift) * S;
    bool hit = false;
#pragma unroll
    for (int j = 0; j < S; ++j) hit |= b[j] == xr;
    return hit;
}

// hout (pinned host memory, the context's h_small from SMALL_NHITS): every
// recorded hit also goes straight to the host — hit slot k < nhpf to
// hout[4 + k], a stop to one of the RT_NSTOP stop slots (device counter
// counters[3]) — and a slot past either sets the overflow flag hout[2], so
// the host reads the result after the kernel with no copy behind it (the
// slots are pre-filled with ~0 by the host; a decode finds ~d hits).
// One 16-byte load per lane per iteration (2 / 4 in flight measured slower,
// DESIGN.md §3.4), nontemporal (the log is read once).  tab: the set in
// device memory (k_root_scan: copied with the counters, multipliers from
// counters[2]) or in the kernel arguments (k_root_scan_k).
template <typename T, int S>
__device__ __forceinline__ void root_scan_body(const T *__restrict__ log, uint64_t n, uint32_t head, const T *tab,
                                               uint32_t words, uint32_t m1, uint32_t m2, uint32_t shift, int use_stop,
                                               T stop_value, uint64_t *__restrict__ hits, uint64_t cap,
                                               uint64_t *__restrict__ counters, uint64_t *hout, uint32_t nhpf,
                                               uint64_t hbase, uint64_t sbase) {
    extern __shared__ __align__(16) unsigned char rs_lds[];
    T *set = reinterpret_cast<T *>(rs_lds);
    for (uint32_t i = threadIdx.x; i < words; i += RT_BLOCK) set[i] = tab[i];
    __syncthreads();
    constexpr int V = 16 / sizeof(T);   // candidates per 16-byte load
    using Vec = typename std::conditional<sizeof(T) == 4, uint4, ulonglong2>::type;
    const uint64_t gtid = (uint64_t)blockIdx.x * RT_BLOCK + threadIdx.x;
    const uint64_t nthr = (uint64_t)gridDim.x * RT_BLOCK;
    const uint64_t h = head < n ? head : n;
    const uint64_t body = (n - h) / V;
    const Vec *__restrict__ v = reinterpret_cast<const Vec *>(log + h);
    for (uint64_t i = gtid; i < body; i += nthr) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(&v[i]));
        Vec w;
        __builtin_memcpy(&w, &x, 16);
        const T *e = reinterpret_cast<const T *>(&w);
        bool any = false, hit[V], st[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
            hit[j] = rs_member<T, S>(e[j], set, m1, m2, shift);
            st[j] = use_stop && e[j] == stop_value;
            any |= hit[j] | st[j];
        }
        if (any) {
#pragma unroll
            for (int j = 0; j < V; ++j)
                rt_record(h + (uint64_t)V * i + j, hit[j], st[j], hits, cap, counters, hout, nhpf, hbase, sbase);
        }
    }
    const uint64_t tail0 = h + body * V;
    if (gtid < h) {
        const T x = log[gtid];
        rt_record(gtid, rs_member<T, S>(x, set, m1, m2, shift), use_stop && x == stop_value, hits, cap, counters,
                  hout, nhpf, hbase, sbase);
    }
    if (gtid < n - tail0) {
        const uint64_t pos = tail0 + gtid;
        const T x = log[pos];
        rt_record(pos, rs_member<T, S>(x, set, m1, m2, shift), use_stop && x == stop_value, hits, cap, counters,
                  hout, nhpf, hbase, sbase);
    }
}

template <typename T, int S>
__global__ __launch_bounds__(RT_BLOCK) void k_root_scan(const T *__restrict__ log, uint64_t n, uint32_t head,
                                                        const T *__restrict__ tab, uint32_t words, uint32_t shift,
                                                        int use_stop, T stop_value, uint64_t *__restrict__ hits,
                                                        uint64_t cap, uint64_t *__restrict__ counters, uint64_t *hout,
                                                        uint32_t nhpf) {
    const uint64_t mm = counters[2];   // m1 | m2 << 32, copied with the set
    root_scan_body<T, S>(log, n, head, tab, words, (uint32_t)mm, (uint32_t)(mm >> 32), shift, use_stop, stop_value,
                         hits, cap, counters, hout, nhpf, 0, 0);
}

// The set in the kernel arguments (a table of at most RT_KTAB_BYTES): no
// copy in front of the scan — at configs[4] (d = 32) the H2D copy's API call
// and blit kernel were ~8 of the call's ~100 µs.  The tickets run on from
// hbase / sbase (no counter reset either).  Completion: each workgroup,
// its hits and stops written, takes a ticket of its group (workgroup index
// mod G, G = min(grid, RT_DONE_GROUPS), done[16 g]); the last of a group
// takes a ticket of the groups (done[16 G_max]), and the last of those
// writes gen to hout[SMALL_DONE - SMALL_NHITS], the word the host polls — it
// sees the result without waiting for the end-of-kernel signal.  Each last
// taker resets its ticket for the next launch.
template <typename T, int S>
__global__ __launch_bounds__(RT_BLOCK) void k_root_scan_k(const T *__restrict__ log, uint64_t n, uint32_t head,
                                                          RtKTab tab, uint32_t words, uint32_t m1, uint32_t m2,
                                                          uint32_t shift, int use_stop, T stop_value,
                                                          uint64_t *__restrict__ hits, uint64_t cap,
                                                          uint64_t *__restrict__ counters, uint64_t *hout,
                                                          uint32_t nhpf, uint64_t hbase, uint64_t sbase,
                                                          uint64_t *__restrict__ done, uint64_t gen) {
    root_scan_body<T, S>(log, n, head, reinterpret_cast<const T *>(tab.w), words, m1, m2, shift, use_stop, stop_value,
                         hits, cap, counters, hout, nhpf, hbase, sbase);
    // every wave's stores performed — the hits and stops went to the pinned
    // slots through the L2 (rt_record) — before the workgroup's ticket (the
    // barrier itself waits for LDS only).  No system-scope fence: an L2
    // write-back per workgroup costs +75 µs over the grid, and one in each
    // of the ~d workgroups that recorded something +20 µs of the u32 scan
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t G = gridDim.x < RT_DONE_GROUPS ? gridDim.x : RT_DONE_GROUPS;
        const uint32_t g = blockIdx.x % G;
        unsigned long long *cg = reinterpret_cast<unsigned long long *>(done) + 16 * g;
        unsigned long long *ct = reinterpret_cast<unsigned long long *>(done) + 16 * RT_DONE_GROUPS;
        if (__hip_atomic_fetch_add(cg, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (gridDim.x - g + G - 1) / G - 1) {
            __hip_atomic_store(cg, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__hip_atomic_fetch_add(ct, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1) {
                __hip_atomic_store(ct, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&hout[SMALL_DONE - SMALL_NHITS], gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// host: the hash set of the roots (see k_root_scan).  S = 1 for up to 32
// roots (2^b >= 2 k^2 buckets: a multiplier pair without collisions is found
// in ~1.3 tries on average), else S = 4 with 2^b >= 2k buckets (mean load
// 1/2).  compact: S = 1 with 2^b >= k^2 / 6 — a table small enough for the
// kernel arguments (k = 32: 256 words; a collision-free multiplier pair is
// then found in ~e^(k^2 / 2^(b+1)) = 7 tries, a few hundred host hashes).
// (S = 4 with 2^b >= 2k, the other small layout, costs the u32 scan 84
// against 65 µs at configs[4]: four compares per candidate.)  Returns false
// when no multipliers fit within the attempt limit.
template <typename T>
bool rt_scan_table(const T *roots, uint32_t k, RtScanSet &set, std::vector<T> &out, bool compact) {
    set.S = k <= 32 || compact ? 1 : 4;
    uint32_t b = 4;
    const uint64_t want = compact ? ((uint64_t)k * k + 5) / 6 : set.S == 1 ? 2ull * k * k : 2ull * k;
    while ((1ull << b) < want) ++b;
    set.shift = 32 - b;
    const uint32_t nb = 1u << b;
    set.words = nb * set.S;
    out.assign(set.words, (T)~(T)0);
    std::vector<uint32_t> fill(nb);
    uint64_t st = 0x9E3779B97F4A7C15ull ^ k;
    for (int attempt = 0; attempt < 1000; ++attempt) {
        st = splitmix_mix(st + GAMMA);
        set.m1 = (uint32_t)st | 1u;
        set.m2 = (uint32_t)(st >> 32) | 1u;
        std::fill(fill.begin(), fill.end(), 0u);
        std::fill(out.begin(), out.end(), (T)~(T)0);
        bool ok = true;
        for (uint32_t r = 0; r < k && ok; ++r) {
            const T x = roots[r];
            uint32_t hh = (uint32_t)x * set.m1;
            if constexpr (sizeof(T) == 8) hh += (uint32_t)((uint64_t)x >> 32) * set.m2;
            const uint32_t bi = hh >> set.shift;
            if (fill[bi] == set.S) ok = false;
            else out[(size_t)bi * set.S + fill[bi]++] = x;
        }
        if (ok) return true;
    }
    return false;
}
template bool rt_scan_table<uint32_t>(const uint32_t *, uint32_t, RtScanSet &, std::vector<uint32_t> &, bool);
template bool rt_scan_table<uint64_t>(const uint64_t *, uint32_t, RtScanSet &, std::vector<uint64_t> &, bool);

template <typename T>
int launch_root_scan(qk_ctx *ctx, const T *d_tab, const RtScanSet &set, const T *log, size_t n, int use_stop,
                     T stop_value, uint64_t *hits, uint64_t cap, uint64_t *counters, uint64_t *hout,
                     hipStream_t s) {
    const uintptr_t a = (uintptr_t)log;
    if (a & (sizeof(T) - 1)) return QK_E_INVAL;
    const uint32_t head = (uint32_t)(((16 - (a & 15)) & 15) / sizeof(T));
    const size_t lds = (size_t)set.words * sizeof(T);
    // one nontemporal 16-byte load per lane per iteration: u32 kernel 70 us
    // against 84 / 78 us with 2 / 4 in flight (profiles/r04/decode_scan_u/);
    // nontemporal 72 -> 66 us, u64 135 -> 125 us (profiles/r05/decode_nt/)
    const uint64_t units = (n + (16 / sizeof(T)) - 1) / (16 / sizeof(T));
    hipEvent_t e0 = prof_begin(ctx, s);
#define QK_RS(SS)                                                                                             \
    hipLaunchKernelGGL((k_root_scan<T, SS>), dim3(rs_grid(ctx, k_root_scan<T, SS>, units, lds)), dim3(RT_BLOCK), \
                       lds, s, log, (uint64_t)n, head, d_tab, set.words, set.shift, use_stop, stop_value, hits, cap, \
                       counters, hout, (uint32_t)SMALL_HITPF_N)
    if (set.S == 1) QK_RS(1);
    else QK_RS(4);
#undef QK_RS
    prof_end(ctx, s, e0);
    QK_HIP_TRY(hipGetLastError());
    return QK_OK;
}

// ---------------------------------------------------------- launchers
template <typename KernelT>
static uint32_t rt_grid(qk_ctx *ctx, KernelT kern, uint64_t units) {
    if (ctx->grid_override) return ctx->grid_override;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, RT_BLOCK, 0) != hipSuccess || occ < 1) occ = 1;
    const uint64_t full = (uint64_t)ctx->num_cus * occ;
    uint64_t need = (units + RT_BLOCK - 1) / RT_BLOCK;
    if (need < 1) need = 1;
    return (uint32_t)(need < full ? need : full);
}

int launch_root_test_u32(qk_ctx *ctx, const uint32_t *d_c, uint32_t d, const uint32_t *log, size_t n,
                         int use_stop, uint32_t stop_value, uint64_t *hits, uint64_t cap, uint64_t *counters,
                         hipStream_t s) {
    const uintptr_t a = (uintptr_t)log;
    if (a & 3) return QK_E_INVAL;
    const uint32_t head = (uint32_t)(((16 - (a & 15)) & 15) / 4);
    const uint64_t units = (n + 3) / 4;
    hipEvent_t e0 = prof_begin(ctx, s);
#define QK_RT32(DD)                                                                                \
    hipLaunchKernelGGL(k_root_test_u32<DD>, dim3(rt_grid(ctx, k_root_test_u32<DD>, units)),        \
                       dim3(RT_BLOCK), 0, s, log, (uint64_t)n, head, d_c, d, use_stop, stop_value, \
                       hits, cap, counters)
    switch (d) {
    case 8: QK_RT32(8); break;
    case 16: QK_RT32(16); break;
    case 20: QK_RT32(20); break;
    case 32: QK_RT32(32); break;
    default: QK_RT32(0); break;
    }
#undef QK_RT32
    prof_end(ctx, s, e0);
    QK_HIP_TRY(hipGetLastError());
    return QK_OK;
}

int launch_root_test_u64(qk_ctx *ctx, const uint64_t *d_c, uint32_t d, const uint64_t *log, size_t n,
                         int use_stop, uint64_t stop_value, uint64_t *hits, uint64_t cap, uint64_t *counters,
                         hipStream_t s) {
    const uintptr_t a = (uintptr_t)log;
    if (a & 7) return QK_E_INVAL;
    const uint32_t head = (uint32_t)(((16 - (a & 15)) & 15) / 8);
    const uint64_t units = (n + 1) / 2;
    hipEvent_t e0 = prof_begin(ctx, s);
    if (rt64_use_bsgs(ctx, d)) {
        // d_c holds the limb-shifted table (root_test_begin, rt64_bsgs_table)
        // one runtime loop over the blocks: an unrolled loop (d / 8 fixed) or
        // two interleaved candidates made the compiler shuttle every value
        // around the pinned registers of the p64 step (1300 copies per
        // evaluation); measured slower
        hipLaunchKernelGGL(k_root_test_u64_bsgs<0>, dim3(rt_grid(ctx, k_root_test_u64_bsgs<0>, units)),
                           dim3(RT_BLOCK), 0, s, log, (uint64_t)n, head, d_c, d / 8, (int)(d % 8 != 0), use_stop,
                           stop_value, hits, cap, counters);
    } else {
        hipLaunchKernelGGL(k_root_test_u64, dim3(rt_grid(ctx, k_root_test_u64, units)), dim3(RT_BLOCK), 0, s, log,
                           (uint64_t)n, head, d_c, d, use_stop, stop_value, hits, cap, counters);
    }
    prof_end(ctx, s, e0);
    QK_HIP_TRY(hipGetLastError());
    return QK_OK;
}

template <typename T>
int launch_root_scan_k(qk_ctx *ctx, const std::vector<T> &tabv, const RtScanSet &set, const T *log, size_t n,
                       int use_stop, T stop_value, uint64_t *hits, uint64_t cap, uint64_t *counters, uint64_t *hout,
                       uint64_t hbase, uint64_t sbase, uint64_t *done, uint64_t gen, hipStream_t s) {
    const uintptr_t a = (uintptr_t)log;
    if (a & (sizeof(T) - 1)) return QK_E_INVAL;
    if (set.words * sizeof(T) > RT_KTAB_BYTES || set.S != 1) return QK_E_INVAL;
    RtKTab tab;
    memcpy(tab.w, tabv.data(), (size_t)set.words * sizeof(T));
    const uint32_t head = (uint32_t)(((16 - (a & 15)) & 15) / sizeof(T));
    const size_t lds = (size_t)set.words * sizeof(T);
    const uint64_t units = (n + (16 / sizeof(T)) - 1) / (16 / sizeof(T));
    hipEvent_t e0 = prof_begin(ctx, s);
    // workgroups per CU asked once per context (the runtime's occupancy
    // query costs microseconds of a ~100 µs call), at the largest table
    int &occ = ctx->rt_occ_k[sizeof(T) == 8];
    if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_root_scan_k<T, 1>, RT_BLOCK, RT_KTAB_BYTES) !=
                     hipSuccess || occ < 1))
        occ = 1;
    const uint64_t need = std::max<uint64_t>(1, (units + RT_BLOCK - 1) / RT_BLOCK);
    const uint32_t grid =
        ctx->grid_override ? ctx->grid_override : (uint32_t)std::min<uint64_t>(need, (uint64_t)ctx->num_cus * occ);
    hipLaunchKernelGGL((k_root_scan_k<T, 1>), dim3(grid), dim3(RT_BLOCK), lds,
                       s, log, (uint64_t)n, head, tab, set.words, set.m1, set.m2, set.shift, use_stop, stop_value,
                       hits, cap, counters, hout, (uint32_t)SMALL_HITPF_N, hbase, sbase, done, gen);
    prof_end(ctx, s, e0);
    QK_HIP_TRY(hipGetLastError());
    return QK_OK;
}
template int launch_root_scan_k<uint32_t>(qk_ctx *, const std::vector<uint32_t> &, const RtScanSet &,
                                          const uint32_t *, size_t, int, uint32_t, uint64_t *, uint64_t, uint64_t *,
                                          uint64_t *, uint64_t, uint64_t, uint64_t *, uint64_t, hipStream_t);
template int launch_root_scan_k<uint64_t>(qk_ctx *, const std::vector<uint64_t> &, const RtScanSet &,
                                          const uint64_t *, size_t, int, uint64_t, uint64_t *, uint64_t, uint64_t *,
                                          uint64_t *, uint64_t, uint64_t, uint64_t *, uint64_t, hipStream_t);

template int launch_root_scan<uint32_t>(qk_ctx *, const uint32_t *, const RtScanSet &, const uint32_t *, size_t, int,
                                        uint32_t, uint64_t *, uint64_t, uint64_t *, uint64_t *, hipStream_t);
template int launch_root_scan<uint64_t>(qk_ctx *, const uint64_t *, const RtScanSet &, const uint64_t *, size_t, int,
                                        uint64_t, uint64_t *, uint64_t, uint64_t *, uint64_t *, hipStream_t);

} // namespace qk
