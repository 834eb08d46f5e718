// segments.hip — the segmented encode: one quACK per
// segment of a grouped id array.  Used by the per-flow batch (flows.hip, the
// grouped ids of a SidekickMulti batch, sidekick_multi.rs:65-90) and exposed
// as the CSR primitive qk_u32_encode_segments_device (caller-grouped ids).
//   k_seg_small<Cfg>   one lane per flow of <= SMALL_SEG ids: the headline
//                      kernel's baby-step/giant-step body (bsgs.h) with per-
//                      lane wrap counters, the flow's record written in place
//   k_seg_bsgs / k_seg_encode<G,K>   one workgroup per work item of <=
//                      SEG_CHUNK ids (5 <= T <= 80: the headline body; else
//                      power chains), one integer atomicAdd per (flow, power)
//                      per item — order-independent, exact
#include <string.h>

#include <algorithm>
#include <vector>

#include "bsgs.h"
#include "ctx.h"
#include "field.h"
#include "segments.h"

namespace qk {

QK_WARM_KERNEL(segments)

static_assert(sizeof(qk_u32) == 16, "qk_u32 header is 4 words (k_seg_small writes it)");

constexpr int SG_BLOCK = 256;
constexpr int SG_WAVES = SG_BLOCK / 64;

__device__ __forceinline__ uint64_t sg_shfl_xor_u64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((int)(uint32_t)v, m, 64);
    const uint32_t hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// lane j of a G-group: start = x^(j+1), step = x^G (canonical)
template <int G>
__device__ __forceinline__ void sg_group_powers(uint32_t x, int j, uint32_t &start, uint32_t &step) {
    uint32_t b = x, r = 1;
    const uint32_t e = (uint32_t)j + 1;
#pragma unroll
    for (int bit = 0; (1 << bit) <= G; ++bit) {
        const uint32_t rb = mul32_lazy(r, b);
        r = ((e >> bit) & 1) ? rb : r;
        if ((1 << bit) < G) b = mul32_lazy(b, b);
    }
    start = r;
    step = canon32(b);
}

template <int G, int K>
__global__ __launch_bounds__(SG_BLOCK) void k_seg_encode(const uint32_t *__restrict__ ids,
                                                         const SegItem *__restrict__ items, uint32_t T,
                                                         unsigned long long *__restrict__ acc_out) {
    __shared__ uint64_t sm[SG_WAVES * G * K];
    const SegItem it = items[blockIdx.x];
    uint64_t acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0;
    const int j = threadIdx.x % G;
    for (uint64_t i = it.lo + threadIdx.x / G; i < it.hi; i += SG_BLOCK / G) {
        const uint32_t x = canon32(ids[i]);
        uint32_t start, step;
        if constexpr (G == 1) { start = x; step = x; }
        else sg_group_powers<G>(x, j, start, step);
        const uint32_t step5 = times5_32(step);
        uint64_t t = start;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc[k] += t;
            if (k + 1 < K) t = tstep32p(t, step, step5, 0u);
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint64_t v = fold64_32(acc[k]);
#pragma unroll
        for (int off = 32; off >= G; off >>= 1) v += sg_shfl_xor_u64(v, off);
        if (lane < G) sm[wave * (G * K) + lane + k * G] = v;
    }
    __syncthreads();
    for (uint32_t m = threadIdx.x; m < T; m += SG_BLOCK) {
        uint64_t s = 0;
#pragma unroll
        for (int w = 0; w < SG_WAVES; ++w) s += sm[w * (G * K) + m];   // < 2^40
        atomicAdd(&acc_out[(size_t)it.seg * T + m], (unsigned long long)fold64_32(s));
    }
}

// Work items of 5 <= T <= 80: one workgroup walks its item [lo, hi) with the
// headline kernel's baby-step/giant-step body (bsgs.h).  All lanes of the
// workgroup belong to one flow, so the wave-level scalar wrap counts stay
// valid; the workgroup's sums go to the flow's accumulator row by atomicAdd.
// (no s_setprio around the MACs: with it 1e6 flows took 7.57 vs 6.80 ms,
// profiles/r04/prio/ab_flows_prio.jsonl)
template <int NB, int NA, int SG>
__global__ __launch_bounds__(bsgs::BLOCK, (NB * NA == 32 ? 5 : NB * NA > 64 ? 2 : NB * NA > 40 ? 3 : 4)) void k_seg_bsgs(
    const uint32_t *__restrict__ ids, const SegItem *__restrict__ items, uint32_t T,
    unsigned long long *__restrict__ acc_out) {
    const SegItem it = items[blockIdx.x];
    const uint32_t *p = ids + it.lo;
    const uint32_t head = (uint32_t)(((16u - ((uint32_t)(uintptr_t)p & 15u)) & 15u) >> 2);   // ids to 16-B alignment
    unsigned long long *row = acc_out + (size_t)it.seg * T;
    bsgs::body_gen<bsgs::Cfg<NB, NA, SG, 1, 1, false, false, 0, false, 0>>(p, it.hi - it.lo, head, T, threadIdx.x,
                                                                             (uint64_t)bsgs::BLOCK,
                                          [=](uint32_t m, uint64_t s) {
                                              atomicAdd(&row[m], (unsigned long long)fold64_32(s));
                                          });
}

// ---- small flows (the many-flow case) ---------------------------------------
// A flow of <= SMALL_SEG ids is encoded by ONE lane: the whole flow stays in
// that lane's registers, so there is no cross-lane reduction and no atomic
// (the lane owns its flow's accumulator row).  Per id it runs the headline
// kernel's baby-step/giant-step work (bsgs.h) with per-lane wrap counters —
// the lanes of a wave belong to different flows, so the wave-level scalar
// count of the headline kernel would mix them.  Flows above SMALL_SEG keep
// the work-item kernel above (a long flow in one lane would stall its wave).

// Output: acc_out rows [nseg][T] of folded sums (the CSR primitive), or —
// rec != null, the per-flow batch — each flow's finished qk_u32 record
// (header + T canonical sums) at its output rank (rseg[g], or g itself): no
// accumulator round trip and no finalize pass for the small flows.  The last
// id is the segment's last (packet order kept by the grouping sort) or, after
// the histogram grouping (any order inside a flow), lastid[g].
template <class C>
__global__ __launch_bounds__(SG_BLOCK, 4) void k_seg_small(const uint32_t *__restrict__ ids,
                                                        const uint64_t *__restrict__ offs, uint32_t nseg,
                                                        uint32_t T, unsigned long long *__restrict__ acc_out,
                                                        uint32_t *__restrict__ rec, const uint32_t *__restrict__ rseg,
                                                        const uint32_t *__restrict__ lastid) {
    const uint32_t g = blockIdx.x * SG_BLOCK + threadIdx.x;
    if (g >= nseg) return;
    const uint64_t b = offs[g], e = offs[g + 1];
    if (e - b > SMALL_SEG) return;   // a work-item flow
    bsgs::Acc<C::NB, C::NA> S;
#pragma unroll
    for (int j = 0; j < C::NB; ++j) {
        S.lo0[j] = 0;
        S.c0[j] = 0;
        S.r0[j] = 0;
#pragma unroll
        for (int a = 0; a < C::NA - 1; ++a) { S.m[a][j] = 0; S.c[a][j] = 0; }
    }
    // The lane walks its flow in the 16-byte blocks that hold it (4 ids per
    // load; components outside [b, e) of the first and last block read as id
    // 0, which adds nothing): the 64 lanes of a wave read 64 different lines,
    // so 4-byte loads moved a whole cache line from L2 per id.  A 16-byte
    // block never straddles a page, so the partial end blocks are safe reads.
    // The next block's load is issued before this block's four ids are
    // encoded (one block ahead: the load's latency under the arithmetic).
    const uintptr_t lo = (uintptr_t)(ids + b), hi = (uintptr_t)(ids + e);
    uintptr_t blk = lo & ~(uintptr_t)15;
    uint4 nxt = make_uint4(0, 0, 0, 0);
    if (blk < hi) nxt = *reinterpret_cast<const uint4 *>(blk);
    for (; blk < hi; blk += 16) {
        uint4 w = nxt;
        if (blk + 16 < hi) nxt = *reinterpret_cast<const uint4 *>(blk + 16);
        if (blk < lo || blk + 16 > hi) {
            w.x = blk + 0 >= lo && blk + 0 < hi ? w.x : 0u;
            w.y = blk + 4 >= lo && blk + 4 < hi ? w.y : 0u;
            w.z = blk + 8 >= lo && blk + 8 < hi ? w.z : 0u;
            w.w = blk + 12 >= lo && blk + 12 < hi ? w.w : 0u;
        }
        bsgs::four<C>(S, w, 0);
    }
    // power a*NB + j + 1: a = 0 row is a 64-bit sum; a >= 1 is m + c * 2^64,
    // 2^64 == 25 (mod p)
    uint32_t *o = nullptr;
    if (rec) {
        o = rec + (size_t)(rseg ? rseg[g] : g) * (4 + T);
        o[0] = T;
        o[1] = (uint32_t)(e - b);   // count
        o[2] = 1u;                  // has_last (a flow has >= 1 id)
        o[3] = lastid ? lastid[g] : ids[e - 1];
    }
#pragma unroll
    for (int a = 0; a < C::NA; ++a) {
#pragma unroll
        for (int j = 0; j < C::NB; ++j) {
            const uint32_t m = (uint32_t)(a * C::NB + j);
            if (m < T) {
                const uint64_t v = a == 0 ? (uint64_t)fold64_32(S.r0[j])
                                          : (uint64_t)fold64_32(S.m[a - 1][j]) +
                                                fold64_32((uint64_t)S.c[a - 1][j] * 25u);
                if (o) o[4 + m] = canon32(fold64_32(v));
                else acc_out[(size_t)g * T + m] = fold64_32(v);
            }
        }
    }
}

int seg_small_launch(uint32_t T, const uint32_t *ids, const uint64_t *d_offs, uint32_t nseg,
                            unsigned long long *acc, const SmallOut &so, hipStream_t s) {
    const dim3 grid((nseg + SG_BLOCK - 1) / SG_BLOCK), block(SG_BLOCK);
#define QK_SMALL(NB_, NA_)                                                                                         \
    hipLaunchKernelGGL((k_seg_small<bsgs::Cfg<NB_, NA_, 0, 1, 1, false, false, 0, false, 0>>), grid, block, 0, s, ids, \
                       d_offs, nseg, T, acc, so.rec, so.rseg, so.lastid)
    if (T <= 8) QK_SMALL(4, 2);
    else if (T <= 12) QK_SMALL(4, 3);
    else if (T <= 16) QK_SMALL(4, 4);
    else if (T <= 24) QK_SMALL(6, 4);
    else QK_SMALL(8, 4);
#undef QK_SMALL
    return hipGetLastError() == hipSuccess ? QK_OK : QK_E_HIP;
}

// (G, K) for a threshold: smallest G with ceil(T/G) <= 32, K = ceil(T/G) rounded to a supported size
static void seg_choose(uint32_t T, int &G, int &K) {
    G = 1;
    while ((T + G - 1) / G > 32u) G *= 2;
    const uint32_t kneed = (T + G - 1) / G;
    static const int ks[] = {4, 8, 16, 20, 24, 32};
    K = 32;
    for (int k : ks)
        if ((uint32_t)k >= kneed) { K = k; break; }
}

template <int G, int K>
static int seg_launch_gk(const uint32_t *ids, const SegItem *items, uint32_t nitems, uint32_t T,
                         unsigned long long *acc, hipStream_t s) {
    hipLaunchKernelGGL((k_seg_encode<G, K>), dim3(nitems), dim3(SG_BLOCK), 0, s, ids, items, T, acc);
    return hipGetLastError() == hipSuccess ? QK_OK : QK_E_HIP;
}

template <int G>
static int seg_launch_g(int K, const uint32_t *ids, const SegItem *items, uint32_t nitems, uint32_t T,
                        unsigned long long *acc, hipStream_t s) {
    switch (K) {
    case 4: return seg_launch_gk<G, 4>(ids, items, nitems, T, acc, s);
    case 8: return seg_launch_gk<G, 8>(ids, items, nitems, T, acc, s);
    case 16: return seg_launch_gk<G, 16>(ids, items, nitems, T, acc, s);
    case 20: return seg_launch_gk<G, 20>(ids, items, nitems, T, acc, s);
    case 24: return seg_launch_gk<G, 24>(ids, items, nitems, T, acc, s);
    default: return seg_launch_gk<G, 32>(ids, items, nitems, T, acc, s);
    }
}

// last id of each non-empty segment
__global__ void k_seg_last(const uint32_t *__restrict__ ids, const uint64_t *__restrict__ offs, uint64_t nseg,
                           uint32_t *__restrict__ last) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nseg) last[i] = offs[i + 1] > offs[i] ? ids[offs[i + 1] - 1] : 0u;
}

// (the work items of flow j of the list accumulate into row j)
std::vector<SegItem> seg_items_from_big(const std::vector<SegItem> &big) {
    std::vector<SegItem> items;
    for (size_t j = 0; j < big.size(); ++j)
        for (uint64_t lo = big[j].lo; lo < big[j].hi; lo += SEG_CHUNK)
            items.push_back({(uint32_t)j, 0u, lo, std::min<uint64_t>(lo + SEG_CHUNK, big[j].hi)});
    return items;
}
static std::vector<SegItem> seg_items(const std::vector<uint64_t> &offs, uint32_t T) {
    std::vector<SegItem> items;
    for (size_t g = 0; g + 1 < offs.size(); ++g) {
        if (small_ok(T) && offs[g + 1] - offs[g] <= SMALL_SEG) continue;
        for (uint64_t lo = offs[g]; lo < offs[g + 1]; lo += SEG_CHUNK)
            items.push_back({(uint32_t)g, 0u, lo, std::min<uint64_t>(lo + SEG_CHUNK, offs[g + 1])});
    }
    return items;
}

// Segmented encode of a grouped id array: the small flows by k_seg_small
// (d_offs: the nseg + 1 offsets on the device) into accumulator rows or
// records (so), the rest by the work items from seg_items into the
// accumulator rows item.seg of d_acc (u64, acc_rows rows, zeroed here).  The
// items go to the kernels through the context's pinned item buffer, read in
// place over the bus (one 24-byte item per workgroup), not by an H2D copy.
// small_done: the caller already launched k_seg_small (before it waited
// for the work-item list)
int seg_encode(qk_ctx *ctx, const uint32_t *d_ids, const uint64_t *d_offs, const std::vector<SegItem> &items,
               size_t nseg, uint32_t T, unsigned long long *d_acc, size_t acc_rows, const SmallOut &so, hipStream_t s,
               bool small_done) {
    if (acc_rows) QK_HIP_TRY(hipMemsetAsync(d_acc, 0, acc_rows * T * sizeof(uint64_t), s));
    if (small_ok(T) && nseg && !small_done) {
        hipEvent_t e0 = prof_begin(ctx, s);
        const int rs = seg_small_launch(T, d_ids, d_offs, (uint32_t)nseg, d_acc, so, s);
        prof_end(ctx, s, e0);
        if (rs) return rs;
    }
    // the caller's host offsets vector must outlive its async copy
    if (items.empty()) return hipStreamSynchronize(s) == hipSuccess ? QK_OK : QK_E_HIP;
    int rc = ensure_items(ctx, items.size() * sizeof(SegItem));
    const SegItem *d_items = (const SegItem *)ctx->h_items_dev;
    if (!rc) memcpy(ctx->h_items, items.data(), items.size() * sizeof(SegItem));
    if (!rc) {
        int G, K;
        seg_choose(T, G, K);
        const uint32_t ni = (uint32_t)items.size();
        hipEvent_t e0 = prof_begin(ctx, s);
        const dim3 grid(ni), block(bsgs::BLOCK);
        if (T >= 5 && T <= 80) {   // same configurations as the headline encode
#define QK_SEGB(NB_, NA_, SG_)                                                                                     \
    hipLaunchKernelGGL((k_seg_bsgs<NB_, NA_, SG_>), grid, block, 0, s, d_ids, d_items, T, d_acc)
            if (T <= 8) QK_SEGB(4, 2, 1);
            else if (T <= 12) QK_SEGB(4, 3, 3);
            else if (T <= 16) QK_SEGB(4, 4, 4);
            else if (T <= 24) QK_SEGB(6, 4, 4);
            else if (T <= 32) QK_SEGB(8, 4, 8);
            else if (T <= 40) QK_SEGB(8, 5, 10);
            else if (T <= 48) QK_SEGB(8, 6, 12);
            else if (T <= 56) QK_SEGB(8, 7, 14);
            else if (T <= 64) QK_SEGB(8, 8, 16);
            else QK_SEGB(8, 10, 16);
#undef QK_SEGB
            rc = hipGetLastError() == hipSuccess ? QK_OK : QK_E_HIP;
            G = 0;
        }
        switch (G) {
        case 0: break;
        case 1: rc = seg_launch_g<1>(K, d_ids, d_items, ni, T, d_acc, s); break;
        case 2: rc = seg_launch_g<2>(K, d_ids, d_items, ni, T, d_acc, s); break;
        case 4: rc = seg_launch_g<4>(K, d_ids, d_items, ni, T, d_acc, s); break;
        case 8: rc = seg_launch_g<8>(K, d_ids, d_items, ni, T, d_acc, s); break;
        case 16: rc = seg_launch_g<16>(K, d_ids, d_items, ni, T, d_acc, s); break;
        case 32: rc = seg_launch_g<32>(K, d_ids, d_items, ni, T, d_acc, s); break;
        default: rc = QK_E_THRESHOLD;
        }
        prof_end(ctx, s, e0);
    }
    // the pinned items must outlive the kernels
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = QK_E_HIP;
    return rc;
}

} // namespace qk

using namespace qk;

extern "C" int qk_u32_encode_segments_device(qk_ctx *ctx, const uint32_t *d_ids, const uint64_t *offsets,
                                             size_t nseg, uint32_t threshold, uint8_t *sketches, void *stream) {
    if (!ctx || !offsets || (nseg && !sketches)) return QK_E_INVAL;
    if (threshold == 0 || threshold > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if (nseg == 0) return QK_OK;
    std::vector<uint64_t> offs(offsets, offsets + nseg + 1);
    for (size_t g = 0; g < nseg; ++g)
        if (offs[g + 1] < offs[g]) return QK_E_INVAL;
    const uint64_t n = offs[nseg] - offs[0];
    if (n && (!d_ids || !is_device_ptr(d_ids))) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = pick_stream(ctx, stream);
    const uint32_t T = threshold;
    const std::vector<SegItem> items = seg_items(offs, T);
    Carve probe{nullptr};
    probe.take<unsigned long long>(nseg * T);
    probe.take<uint32_t>(nseg);
    probe.take<uint64_t>(nseg + 1);
    if (int e = ensure_flow(ctx, 1, probe.off, s)) return e;
    Carve cv{(char *)ctx->d_flow[1]};
    unsigned long long *d_acc = cv.take<unsigned long long>(nseg * T);
    uint32_t *d_last = cv.take<uint32_t>(nseg);
    uint64_t *d_offs = cv.take<uint64_t>(nseg + 1);
    int rc = QK_OK;
    if (hipMemcpyAsync(d_offs, offs.data(), (nseg + 1) * 8, hipMemcpyHostToDevice, s) != hipSuccess) rc = QK_E_HIP;
    if (!rc) rc = seg_encode(ctx, d_ids, d_offs, items, nseg, T, d_acc, nseg, SmallOut{}, s);
    std::vector<uint64_t> acc(nseg * T);
    std::vector<uint32_t> last(nseg, 0);
    if (!rc && hipMemcpyAsync(acc.data(), d_acc, acc.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = QK_E_HIP;
    if (!rc) {
        hipLaunchKernelGGL(k_seg_last, dim3((uint32_t)((nseg + 255) / 256)), dim3(256), 0, s, d_ids, d_offs,
                           (uint64_t)nseg, d_last);
        if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
    }
    if (!rc && hipMemcpyAsync(last.data(), d_last, nseg * 4, hipMemcpyDeviceToHost, s) != hipSuccess) rc = QK_E_HIP;
    if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = QK_E_HIP;
    if (rc) return rc;
    const size_t rec = qk_u32_size(T);
    for (size_t i = 0; i < nseg; ++i) {
        qk_u32 *q = (qk_u32 *)(sketches + i * rec);
        qk_u32_init(q, T);
        for (uint32_t m = 0; m < T; ++m) q->power_sums[m] = canon32(fold64_32(acc[i * T + m]));
        q->count = (uint32_t)(offs[i + 1] - offs[i]);
        if (offs[i + 1] > offs[i]) { q->has_last = 1; q->last_value = last[i]; }
    }
    return QK_OK;
}

