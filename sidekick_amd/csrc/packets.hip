// packets.hip — packet-batch identifier extraction fused in front of the
// encode.
//
// Replaces, for a batch of captured packets, the per-packet sniff loop of
// sidekick/src/sidekick.rs:76-124:
//     if Direction::Incoming != addr.sll_pkttype.into() { continue }      (:78-80)
//     if addr.sll_protocol != ETH_P_IP.to_be()          { continue }      (:81-84)
//     if !UdpParser::is_udp(&buf)  /* buf[23] == 17 */  { continue }      (:85-88)
//     if parse_dst_ip(&buf) == my_ipv4_addr { sc.reset(); continue }      (:92-96)
//     if n != BUFFER_SIZE                               { continue }      (:99-102)
//     sc.insert_packet(parse_identifier(&buf))  /* BE u32 at byte 63 */   (:103-115)
// (buffer.rs:6-7,80-83,88-90,99-106).
//
// Fused (5 <= t <= 32, batches without a reset): k_pkt_kernel<Cfg> (t <= 12)
// classifies the staged records and feeds the ids straight into the headline
// kernel's baby-step/giant-step accumulators, k_pkt_kernel<Shared<NA>>
// (13 <= t <= 32) the same sums split across the workgroup's waves through
// LDS — one pass over the records, no id array.
//
// Pass 1 (k_pkt_kernel<NoEncode>): each workgroup owns a contiguous chunk of packets
// and walks it in tiles of 256 records staged into LDS with coalesced 16-byte
// loads (records are `stride` bytes, 67 in the reference, so a lane's fields
// are unaligned).  Each lane classifies one record and writes its id (0 for a
// skipped packet: x = 0 adds nothing to any power sum) to a compact u32
// array, so pass 2 is the ordinary encode over that array from the last reset
// on.  Per-chunk bookkeeping (last reset, inserts after it, last insert) is
// combined on the host in chunk order.  The pass reads every record byte once:
// it is HBM-bound (~67 B per packet), not VALU-bound.
#include <string.h>

#include <algorithm>
#include <type_traits>
#include <vector>

#include "bsgs.h"
#include "ctx.h"
#include "field.h"
#include "records.h"

namespace qk {

QK_WARM_KERNEL(packets)

constexpr int PK_BLOCK = REC_TILE;
constexpr uint64_t PK_WGPC = 4;   // workgroups per CU

struct ChunkStat {       // per workgroup chunk, written by lane 0
    int64_t last_reset;  // absolute packet index of the last reset in the chunk, -1 if none
    int64_t last_insert; // absolute index of the last insert (after last_reset), -1 if none
    uint64_t inserts;    // inserts after last_reset (all inserts if no reset)
    uint64_t resets;     // resets in the chunk
    uint64_t all_inserts; // inserts in the chunk, before or after resets
    uint64_t last_insert_id; // id of last_insert (fused kernel)
};

// C == void: extract (ids to ids_out, for the separate encode).  Otherwise
// the fused form: every lane feeds its record's id (0 if not an insert)
// straight into the baby-step/giant-step accumulators of the headline kernel
// (bsgs.h, the same body) and the workgroup writes one partial per power,
// [power][block] into partials; no id array.  The fused sums cover the whole
// chunk, resets included: the host uses them only when the batch has no
// reset (otherwise it reruns the exact extract + encode-from-last-reset).
struct NoEncode {};
// Shared<NA> (13 <= t <= 32, t <= 8 NA): the (8, NA) baby-step/giant-step
// sums with the work of a tile split across the workgroup's waves through
// LDS, as the u64 kernel does (bsgs64.h): every lane computes its record's
// babies x^1..x^8 and giants x^16 .. x^(8 (NA-1)) (7 + NA - 2 lazy modmuls)
// into LDS, then wave w runs, over the tile's 256 ids (4 per lane), the
// a = 0 row and the NA - 1 MAC rows of babies 2w+1 and 2w+2 — 4 NA
// accumulator VGPRs per lane instead of the lane-private form's (182 VGPRs
// at t = 32, 2 waves/SIMD: slower than the two passes, below).  Wraps
// counted per lane (v_addc): the record stream, not the arithmetic, bounds
// the kernel.
template <int NA_> struct Shared {
    static constexpr int NA = NA_;
    using Pw = bsgs::Cfg<8, NA_, 0, 1, 1>;   // the powers (min-tracked lazy folds)
};
template <class C> struct IsShared : std::false_type {};
template <int NA> struct IsShared<Shared<NA>> : std::true_type {};
template <class C, bool SH = IsShared<C>::value> struct AccOf { using type = bsgs::Acc<C::NB, C::NA, C::ROWS>; };
template <class C> struct AccOf<C, true> { using type = int; };
template <> struct AccOf<NoEncode, false> { using type = int; };
template <class C, bool SH = IsShared<C>::value> struct ShNA { static constexpr int value = 1; };
template <class C> struct ShNA<C, true> { static constexpr int value = C::NA; };
// NT (knob pkt_nt): the records read nontemporal
template <class C, bool NT = false>
__global__ __launch_bounds__(PK_BLOCK) void k_pkt_kernel(const uint8_t *__restrict__ bufs, uint64_t n,
                                                         uint32_t stride, const qk_pkt_meta *__restrict__ meta,
                                                         uint32_t my_ip_le, int check_reset, uint64_t chunk,
                                                         uint32_t *__restrict__ ids_out, ChunkStat *stats,
                                                         uint32_t T, uint64_t *__restrict__ partials) {
    constexpr bool SH = IsShared<C>::value;
    constexpr bool FUSED = !std::is_same<C, NoEncode>::value && !SH;
    constexpr int SNA = ShNA<C>::value;   // Shared: giant rows (a = 0 .. SNA-1)
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
    // Shared: the tile's babies x^1..x^8 (rows 0-7) and giants x^16 ..
    // (rows 8 ..), [value][record]; this wave's accumulators: rows a of
    // babies 2w+1, 2w+2, and the MAC rows' per-lane wrap counts
    __shared__ uint32_t sh_v[SH ? 8 + SNA - 2 : 1][SH ? PK_BLOCK : 1];
    [[maybe_unused]] uint64_t sh_acc[SNA][2];
    [[maybe_unused]] uint32_t sh_c[SNA][2];
    if constexpr (SH) {
#pragma unroll
        for (int a = 0; a < SNA; ++a) sh_acc[a][0] = sh_acc[a][1] = 0, sh_c[a][0] = sh_c[a][1] = 0;
    }
    __shared__ int64_t s_reset[PK_BLOCK / 64], s_insert[PK_BLOCK / 64];
    __shared__ uint64_t s_cnt[PK_BLOCK / 64], s_nres[PK_BLOCK / 64], s_nins[PK_BLOCK / 64], s_iid[PK_BLOCK / 64];
    [[maybe_unused]] typename AccOf<C>::type S;
    if constexpr (FUSED) bsgs::clear<C>(S);
    uint64_t blk_iid = 0;     // id of blk_insert (thread 0)
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t c1 = c0 + chunk < n ? c0 + chunk : n;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

    // chunk-level state, kept by thread 0 while walking the tiles in order
    int64_t blk_reset = -1;   // last reset seen so far
    uint64_t blk_cnt = 0;     // inserts after blk_reset so far
    int64_t blk_insert = -1;  // last insert after blk_reset
    uint64_t blk_nres = 0, blk_nins = 0;

    const bool pipe = stage_pipelined(stride, PK_BLOCK);
    TileStage st;
    if (pipe && c0 < c1) stage_issue<NT>(bufs, n, stride, c0, c1 - c0 < PK_BLOCK ? c1 - c0 : PK_BLOCK, st);
    for (uint64_t p0 = c0; p0 < c1; p0 += PK_BLOCK) {
        const uint64_t np = (c1 - p0) < PK_BLOCK ? (c1 - p0) : PK_BLOCK;
        __syncthreads(); // previous tile fully consumed
        const uint32_t r0 = pipe ? stage_commit(bufs, n, stride, st, tile) : stage_records<NT>(bufs, n, stride, p0, np, tile);
        __syncthreads();
        if (pipe && p0 + PK_BLOCK < c1)   // next tile's loads fly while this one is classified
            stage_issue<NT>(bufs, n, stride, p0 + PK_BLOCK, c1 - p0 - PK_BLOCK < PK_BLOCK ? c1 - p0 - PK_BLOCK : PK_BLOCK, st);
        // classify one record per lane
        uint32_t cls = 0, id = 0; // 0 skip, 1 insert, 2 reset
        const uint64_t pi = p0 + threadIdx.x;
        if (threadIdx.x < np) {
            const uint8_t *rec = tile + r0 + threadIdx.x * stride;
            const qk_pkt_meta m = record_meta<NT>(meta, pi);
            if (record_is_incoming_udp(m, rec)) {
                const uint32_t dst = (uint32_t)rec[30] | ((uint32_t)rec[31] << 8) | ((uint32_t)rec[32] << 16) |
                                     ((uint32_t)rec[33] << 24);
                if (check_reset && dst == my_ip_le) cls = 2;
                else if (m.len == (uint32_t)QK_BUFFER_SIZE) {
                    cls = 1;
                    id = record_identifier(rec);
                }
            }
            if constexpr (std::is_same<C, NoEncode>::value) ids_out[pi] = cls == 1 ? id : 0u;   // the extract pass only
        }
        if constexpr (FUSED) bsgs::one<C>(S, cls == 1 ? id : 0u);   // every lane: EXEC full
        if constexpr (SH) {   // this record's powers into LDS (read after the barrier below)
            using Pw = typename C::Pw;
            uint32_t B[8], A[Pw::ROWS];   // A[r] = x^(8 (r + 1))
            const uint32_t w = bsgs::powers<Pw>(cls == 1 ? id : 0u, B, A);
            if (__builtin_expect(__any(w), 0)) {
                if (w) bsgs::powers_exact<Pw>(B, A);
            }
#pragma unroll
            for (int b = 0; b < 8; ++b) sh_v[b][threadIdx.x] = B[b];
#pragma unroll
            for (int r = 1; r < Pw::ROWS; ++r) sh_v[7 + r][threadIdx.x] = A[r];
        }
        // tile bookkeeping: last reset in tile, inserts after it, last insert
        const unsigned long long rmask = __ballot(cls == 2);
        const unsigned long long imask = __ballot(cls == 1);
        const uint32_t last_id = (uint32_t)__shfl((int)id, imask ? 63 - __clzll(imask) : 0, 64);
        if (lane == 0) {
            int64_t wr = -1, wi = -1;
            uint64_t wc;
            if (rmask) {
                const int hb = 63 - __clzll(rmask);
                wr = (int64_t)(p0 + wave * 64 + hb);
                const unsigned long long after = hb == 63 ? 0ull : (imask & (~0ull << (hb + 1)));
                wc = __popcll(after);
            } else {
                wc = __popcll(imask);
            }
            if (imask) wi = (int64_t)(p0 + wave * 64 + 63 - __clzll(imask));
            s_reset[wave] = wr;
            s_iid[wave] = 0;
            s_insert[wave] = wi;
            s_cnt[wave] = wc;
            s_nres[wave] = __popcll(rmask);
            s_nins[wave] = __popcll(imask);
            s_iid[wave] = last_id;
        }
        __syncthreads();
        if constexpr (SH) {   // this wave's rows over the tile's 256 records (wave-uniform)
            const int b0 = 2 * wave;
#pragma unroll
            for (int q = 0; q < PK_BLOCK / 64; ++q) {
                const int j = q * 64 + lane;
                const uint32_t B0 = sh_v[b0][j], B1 = sh_v[b0 + 1][j];
                bsgs::row2m(sh_acc[0][0], sh_acc[0][1], B0, B1);
#pragma unroll
                for (int a = 1; a < SNA; ++a)   // giant x^(8a): baby 8 (row 7), then rows 8 ..
                    bsgs::mac2v(sh_acc[a][0], sh_acc[a][1], sh_c[a][0], sh_c[a][1], sh_v[6 + a][j], B0, B1);
            }
        }
        if (threadIdx.x == 0) {
            for (int w = 0; w < PK_BLOCK / 64; ++w) { // waves in packet order
                blk_nres += s_nres[w];
                blk_nins += s_nins[w];
                if (s_reset[w] >= 0) { blk_reset = s_reset[w]; blk_cnt = s_cnt[w]; blk_insert = -1; }
                else blk_cnt += s_cnt[w];
                if (s_insert[w] > blk_reset && s_insert[w] > blk_insert) {
                    blk_insert = s_insert[w];
                    blk_iid = s_iid[w];
                }
            }
        }
    }
    if (threadIdx.x == 0) {
        ChunkStat st;
        st.last_reset = blk_reset;
        st.last_insert = blk_insert;
        st.inserts = blk_cnt;
        st.resets = blk_nres;
        st.all_inserts = blk_nins;
        st.last_insert_id = blk_iid;
        stats[blockIdx.x] = st;
    }
    if constexpr (FUSED)
        bsgs::finish<C>(S, T, [=](uint32_t m, uint64_t v) { partials[(size_t)m * gridDim.x + blockIdx.x] = v; });
    if constexpr (SH) {   // power 8a + b + 1 is owned by the wave of baby b: lane sums, written by lane 0
#pragma unroll
        for (int a = 0; a < SNA; ++a) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t m = 8 * a + 2 * wave + k;
                // value = acc + c 2^64 with 2^64 == 25 (mod p) for the MAC rows
                uint64_t x = a == 0 ? fold64_32(sh_acc[0][k])
                                    : (uint64_t)fold64_32(sh_acc[a][k]) + fold64_32((uint64_t)sh_c[a][k] * 25u);
                x = fold64_32(x);
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) x += bsgs::shfl_xor_u64(x, off);   // < 2^38
                if (lane == 0 && m < T) partials[(size_t)m * gridDim.x + blockIdx.x] = x;
            }
        }
    }
}

} // namespace qk

using namespace qk;

extern "C" int qk_u32_encode_packets_device(qk_ctx *ctx, const uint8_t *d_bufs, size_t n, size_t stride,
                                            const qk_pkt_meta *d_meta, const uint8_t my_ipv4[4], qk_u32 *q,
                                            qk_pkt_stats *out_stats, void *stream) {
    if (!ctx || !q || (n && !d_bufs)) return QK_E_INVAL;
    if (stride < QK_BUFFER_SIZE || stride > 512) return QK_E_INVAL; // one LDS tile = 256 records
    const uint32_t t = q->threshold;
    if (t == 0 || t > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    qk_pkt_stats st = {0, 0, 0, 0, -1};
    if (n == 0) {
        if (out_stats) *out_stats = st;
        return QK_OK;
    }
    if (!is_device_ptr(d_bufs) || (d_meta && !is_device_ptr(d_meta))) return QK_E_INVAL;
    const uint32_t my_ip_le = my_ipv4 ? ((uint32_t)my_ipv4[0] | ((uint32_t)my_ipv4[1] << 8) |
                                         ((uint32_t)my_ipv4[2] << 16) | ((uint32_t)my_ipv4[3] << 24))
                                      : 0u;
    const int check_reset = my_ipv4 != nullptr; // no own address given: nothing resets
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = pick_stream(ctx, stream);

    // chunking: >= 4 tiles per workgroup, PK_WGPC workgroups per CU (each
    // keeps one staged tile of loads in flight)
    const uint64_t tiles = (n + PK_BLOCK - 1) / PK_BLOCK;
    const uint64_t wgs = (uint64_t)ctx->num_cus * PK_WGPC;
    uint64_t tiles_per_chunk = std::max<uint64_t>(4, (tiles + wgs - 1) / wgs);
    const uint64_t chunk = tiles_per_chunk * PK_BLOCK;
    const uint32_t nchunks = (uint32_t)((n + chunk - 1) / chunk);

    // device scratch in the context's per-packet arena (grow-only, shared with
    // the flow batches under ctx->mu): compact ids (n u32) + chunk stats
    const size_t ids_bytes = ((size_t)n * sizeof(uint32_t) + 255) & ~(size_t)255;
    if (int e = ensure_flow(ctx, 0, ids_bytes + (size_t)nchunks * sizeof(ChunkStat), s)) return e;
    uint32_t *d_ids = (uint32_t *)ctx->d_flow[0];
    ChunkStat *d_stats = (ChunkStat *)((char *)ctx->d_flow[0] + ids_bytes);
    const size_t lds = (size_t)PK_BLOCK * stride + 32;
    int rc = QK_OK;
    std::vector<ChunkStat> hs(nchunks);
    // Fused fast path (5 <= t <= 32): records -> baby-step/giant-step sums in
    // one kernel, no id array.  Used when the batch holds no reset (the
    // common case); a batch with a reset takes the exact two-pass path below.
    // Lane-private accumulators up to t = 12; above, they cut the kernel's
    // occupancy (182 VGPRs at t = 32, 2 waves/SIMD) below what the record
    // stream needs (per 1e8 records, lane-private fused vs two-pass: t = 12
    // 1.40 vs 1.68 ms, 16 1.89 vs 1.69, 24 1.95 vs 1.75, 32 2.06 vs 1.81), so
    // 13 <= t <= 32 splits the sums across the waves (Shared<NA>): t = 16 /
    // 24 / 32 1.37 / 1.44 / 1.45-1.56 ms (profiles/r06/s8_packets_shared/).
    if (t >= 5 && t <= 32) {
        int frc = QK_OK;
        if (int e = ensure_scratch(ctx, (size_t)nchunks * 32 * sizeof(uint64_t), s)) return e;
        if (int e = scratch_acquire(ctx, s)) return e;
        uint64_t *partials = (uint64_t *)ctx->d_scratch;
#define QK_PKT_FUSED(NB_, NA_, SG_)                                                                          \
    hipLaunchKernelGGL((k_pkt_kernel<bsgs::Cfg<NB_, NA_, SG_>, true>), dim3(nchunks), dim3(PK_BLOCK), lds, s, d_bufs,                                                \
                       (uint64_t)n, (uint32_t)stride, d_meta, my_ip_le, check_reset, chunk, (uint32_t *)nullptr,   \
                       d_stats, t, partials)
        hipEvent_t e0 = prof_begin(ctx, s);
        // per-lane (VALU) wrap counts (SG = 0): the record stream, not the
        // arithmetic, bounds this kernel, and the scalar form's SGPR
        // accumulators cannot live across the tile loop's divergent
        // bookkeeping (the compiler rejects it)
        if (t <= 8) QK_PKT_FUSED(4, 2, 0);
        else if (t <= 12) QK_PKT_FUSED(4, 3, 0);
#undef QK_PKT_FUSED
#define QK_PKT_SHARED(NA_)                                                                                       \
    hipLaunchKernelGGL((k_pkt_kernel<Shared<NA_>, true>), dim3(nchunks), dim3(PK_BLOCK), lds, s, d_bufs, (uint64_t)n, \
                       (uint32_t)stride, d_meta, my_ip_le, check_reset, chunk, (uint32_t *)nullptr, d_stats, t,         \
                       partials)
        else if (t <= 16) QK_PKT_SHARED(2);
        else if (t <= 24) QK_PKT_SHARED(3);
        else QK_PKT_SHARED(4);
#undef QK_PKT_SHARED
        prof_end(ctx, s, e0);
        if (hipGetLastError() != hipSuccess) frc = QK_E_HIP;
        if (!frc) frc = launch_finalize_powers_u32(partials, nchunks, t, ctx->d_small, s);
        if (int e = scratch_release(ctx, s); e && !frc) frc = e;
        if (!frc && (hipMemcpyAsync(hs.data(), d_stats, nchunks * sizeof(ChunkStat), hipMemcpyDeviceToHost, s) !=
                         hipSuccess ||
                     hipMemcpyAsync(ctx->h_small, ctx->d_small, (size_t)t * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
                     hipStreamSynchronize(s) != hipSuccess))
            frc = QK_E_HIP;
        if (frc) return frc;
        uint64_t resets = 0, inserts = 0;
        int64_t last_insert = -1;
        uint32_t last_id = 0;
        for (const ChunkStat &c : hs) {
            resets += c.resets;
            inserts += c.inserts;
            if (c.last_insert > last_insert) { last_insert = c.last_insert; last_id = (uint32_t)c.last_insert_id; }
        }
        if (resets == 0) {
            st.inserted = inserts;
            st.filtered = n - inserts;
            qk_u32 *tmp = (qk_u32 *)malloc(qk_u32_size(t));
            if (!tmp) return QK_E_NOMEM;
            qk_u32_init(tmp, t);
            ctx->h_small[t] = inserts;   // count = inserts
            rc = qk_u32_merge_partial(tmp, ctx->h_small, last_insert >= 0, last_id);
            if (!rc) rc = qk_u32_merge(q, tmp);
            free(tmp);
            if (out_stats) *out_stats = st;
            return rc;
        }
        // a reset in the batch: the exact path
    }
    // records read nontemporal (t = 32, 1e8 records: 1.83-1.84 -> 1.74-1.76
    // ms, profiles/r05/packets_nt/)
    auto kx = k_pkt_kernel<NoEncode, true>;
    hipLaunchKernelGGL(kx, dim3(nchunks), dim3(PK_BLOCK), lds, s, d_bufs, (uint64_t)n,
                       (uint32_t)stride, d_meta, my_ip_le, check_reset, chunk, d_ids, d_stats, 0u,
                       (uint64_t *)nullptr);
    if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
    if (!rc && hipMemcpyAsync(hs.data(), d_stats, nchunks * sizeof(ChunkStat), hipMemcpyDeviceToHost, s) != hipSuccess)
        rc = QK_E_HIP;
    if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = QK_E_HIP;
    if (!rc) {
        // combine chunks in packet order: the state after the last reset wins
        int64_t last_reset = -1, last_insert = -1;
        uint64_t inserts = 0, resets = 0, all_inserts = 0;
        for (const ChunkStat &c : hs) {
            resets += c.resets;
            all_inserts += c.all_inserts;
            if (c.last_reset >= 0) { last_reset = c.last_reset; inserts = c.inserts; last_insert = -1; }
            else inserts += c.inserts;
            if (c.last_insert > last_reset && c.last_insert > last_insert) last_insert = c.last_insert;
        }
        st.resets = resets;
        st.last_reset_index = last_reset;
        st.inserted = inserts;
        st.discarded = all_inserts - inserts;
        // encode ids after the last reset (skipped packets are 0 and add nothing)
        const uint64_t from = (uint64_t)(last_reset + 1);
        qk_u32 *tmp = (qk_u32 *)malloc(qk_u32_size(t));
        if (!tmp) rc = QK_E_NOMEM;
        else {
            qk_u32_init(tmp, t);
            if (from < n) rc = launch_encode_u32(ctx, d_ids + from, n - from, t, ctx->d_small, s);
            if (!rc && from < n) {
                const size_t w = qk_u32_partial_words(t);
                uint32_t last_id = 0;   // fetched with the partial: one synchronisation
                if (hipMemcpyAsync(ctx->h_small, ctx->d_small, w * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
                    (last_insert >= 0 &&
                     hipMemcpyAsync(&last_id, d_ids + last_insert, 4, hipMemcpyDeviceToHost, s) != hipSuccess) ||
                    hipStreamSynchronize(s) != hipSuccess)
                    rc = QK_E_HIP;
                else {
                    ctx->h_small[t] = inserts; // count = inserts, not array length
                    rc = qk_u32_merge_partial(tmp, ctx->h_small, last_insert >= 0, last_id);
                }
            }
            if (!rc) {
                if (last_reset >= 0) qk_u32_init(q, t); // Sidekick::reset (sidekick.rs:47-50)
                rc = qk_u32_merge(q, tmp);
            }
            free(tmp);
        }
    }
    (void)hipStreamSynchronize(s); // the arena is reused by the next call
    st.filtered = n - st.inserted - st.discarded - st.resets;
    if (out_stats) *out_stats = st;
    return rc;
}
