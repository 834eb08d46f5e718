// flows.hip — segmented multi-flow encode.
//
// Replaces, for a batch, SidekickMulti's per-packet flow table
// (sidekick/src/sidekick_multi.rs:36,65-90,101-143):
//     match process_one_packet(n, &buf, &addr, my_addr) {
//         Insert { addr_key, id } => senders.entry(addr_key).or_insert(new(t)).insert(id),
//         Reset  { .. }           => senders = HashMap::new(),          (:205, :265)
//         Skip => {} }
// with AddrKey = [src ip(4), src port(2), dst ip(4), dst port(2)] = buf[26..30],
// buf[34..36], buf[30..34], buf[36..38] (buffer.rs:91-95).  A Reset (a packet
// whose dst ip:port IS the proxy's own address) wipes EVERY flow — the sniff
// loops replace the whole map, they do not call SidekickMulti::reset — so the
// batch's table is the inserts after its last reset, and the caller clears
// its own table before merging when stats.resets > 0.  The caller merges the
// batch table into its own with qk_u32_merge, flow by flow.
//
// Device pipeline:
//   1. k_flow_extract   LDS-staged records -> per packet the filters and, for
//                       an Insert, its flow's slot in a device hash table
//                       (packets of a tile that share a flow elect one leader
//                       in LDS, which probes / inserts once); writes slot + id
//                       and the batch's last reset position.  A batch with a
//                       reset reruns the pass over the packets after it with
//                       an empty table (resets are rare: one per receiver
//                       request, media_client.rs:272).
//   2. the occupied slots (DeviceSelect) sorted by AddrKey (two stable 48-bit
//      radix sorts of the flows only) -> rank of each flow = output order.
//   3. per packet slot -> rank; one stable radix sort of (rank, id) pairs over
//      bit_width(flows) bits (1 pass for <= 256 flows) groups the ids by flow
//      with packet order preserved (last_value = last id); offsets from the
//      rank changes.  Flows of > SMALL_SEG ids (or any flow when T > 32) ->
//      work items of <= 64 Ki ids per workgroup.
//   4. k_seg_small<Cfg>   one lane per small flow: baby-step/giant-step per id
//      (bsgs.h) with the whole flow in that lane's registers, one plain store
//      per (flow, power); k_seg_encode<G,K> for the work items: power chains
//      per id, block reduction, one integer atomicAdd per (flow, power) per
//      work item (order-independent, exact).
// The CSR primitive qk_u32_encode_segments_device runs step 4 directly on
// caller-grouped ids.
#include <string.h>

#include <algorithm>
#include <hipcub/hipcub.hpp>
#include <vector>

#include "bsgs.h"
#include "ctx.h"
#include "field.h"
#include "radix.h"
#include "records.h"

namespace qk {

static_assert(sizeof(qk_flow_key) == 12, "qk_flow_key is 12 packed bytes");
static_assert(sizeof(qk_u32) == 16, "qk_u32 header is 4 words (k_flow_finalize writes it)");

constexpr int SG_BLOCK = 256;
constexpr int SG_WAVES = SG_BLOCK / 64;
constexpr uint32_t SEG_CHUNK = 1u << 16;     // ids per work item

struct SegItem {
    uint32_t seg;
    uint32_t pad;
    uint64_t lo, hi; // [lo, hi) in the grouped id array
};

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
template <int NB, int NA, int SG, int PRIO>
__global__ __launch_bounds__(bsgs::BLOCK, (NB * NA == 32 ? 5 : NB * NA > 64 ? 2 : NB * NA > 40 ? 3 : 4)) void k_seg_bsgs(
    const uint32_t *__restrict__ ids, const SegItem *__restrict__ items, uint32_t T,
    unsigned long long *__restrict__ acc_out) {
    const SegItem it = items[blockIdx.x];
    const uint32_t *p = ids + it.lo;
    const uint32_t head = (uint32_t)(((16u - ((uint32_t)(uintptr_t)p & 15u)) & 15u) >> 2);   // ids to 16-B alignment
    unsigned long long *row = acc_out + (size_t)it.seg * T;
    bsgs::body_gen<bsgs::Cfg<NB, NA, SG, 1, 1, false, false, 0, false, PRIO>>(p, it.hi - it.lo, head, T, threadIdx.x,
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
constexpr uint64_t SMALL_SEG = 4096;

template <class C>
__global__ __launch_bounds__(SG_BLOCK, 4) void k_seg_small(const uint32_t *__restrict__ ids,
                                                        const uint64_t *__restrict__ offs, uint32_t nseg,
                                                        uint32_t T, unsigned long long *__restrict__ acc_out) {
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
    const uintptr_t lo = (uintptr_t)(ids + b), hi = (uintptr_t)(ids + e);
    for (uintptr_t blk = lo & ~(uintptr_t)15; blk < hi; blk += 16) {
        uint4 w = *reinterpret_cast<const uint4 *>(blk);
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
#pragma unroll
    for (int a = 0; a < C::NA; ++a) {
#pragma unroll
        for (int j = 0; j < C::NB; ++j) {
            const uint32_t m = (uint32_t)(a * C::NB + j);
            if (m < T) {
                const uint64_t v = a == 0 ? (uint64_t)fold64_32(S.r0[j])
                                          : (uint64_t)fold64_32(S.m[a - 1][j]) +
                                                fold64_32((uint64_t)S.c[a - 1][j] * 25u);
                acc_out[(size_t)g * T + m] = fold64_32(v);
            }
        }
    }
}

// per-lane (VALU) wrap counters: SG = 0; P: s_setprio around the MACs
template <int P>
static void seg_small_launch_p(uint32_t T, const uint32_t *ids, const uint64_t *d_offs, uint32_t nseg,
                               unsigned long long *acc, hipStream_t s) {
    const dim3 grid((nseg + SG_BLOCK - 1) / SG_BLOCK), block(SG_BLOCK);
#define QK_SMALL(NB_, NA_)                                                                                         \
    hipLaunchKernelGGL((k_seg_small<bsgs::Cfg<NB_, NA_, 0, 1, 1, false, false, 0, false, P>>), grid, block, 0, s, ids, \
                       d_offs, nseg, T, acc)
    if (T <= 8) QK_SMALL(4, 2);
    else if (T <= 12) QK_SMALL(4, 3);
    else if (T <= 16) QK_SMALL(4, 4);
    else if (T <= 24) QK_SMALL(6, 4);
    else QK_SMALL(8, 4);
#undef QK_SMALL
}
static int seg_small_launch(int prio, uint32_t T, const uint32_t *ids, const uint64_t *d_offs, uint32_t nseg,
                            unsigned long long *acc, hipStream_t s) {
    if (prio) seg_small_launch_p<1>(T, ids, d_offs, nseg, acc, s);
    else seg_small_launch_p<0>(T, ids, d_offs, nseg, acc, s);
    return hipGetLastError() == hipSuccess ? QK_OK : QK_E_HIP;
}

// ---- flow table --------------------------------------------------------------
// Open addressing with linear probing over C = 2^k slots of two words:
//   w0 = (src + 1) | (dst >> 33) << 49   0 = empty
//   w1 = (dst & (2^33 - 1)) | 1 << 40     0 = not yet set
// (src, dst = the 48-bit big-endian ip:port halves of the AddrKey).  Each word
// goes 0 -> final value exactly once, by CAS, so any nonzero value read (cached
// or not) is final and a 0 is resolved by the CAS itself.  A lane whose key
// matches w0 sets w1 itself if it is still 0, so no lane ever waits for
// another (no intra-wave spin hazard): the slot belongs to the key whose w1
// lands first, and every lane decides on final values only, so all lanes of
// one key stop at the same slot.
struct alignas(16) FlowSlot {
    uint64_t w0, w1;
};
constexpr uint32_t SLOT_NONE = 0xFFFFFFFFu;
constexpr uint64_t FT_OVERFLOW = 1;   // counters[3] flag

__device__ __forceinline__ uint64_t ft_w0(uint64_t src, uint64_t dst) { return (src + 1) | ((dst >> 33) << 49); }
__device__ __forceinline__ uint64_t ft_w1(uint64_t dst) { return (dst & ((1ull << 33) - 1)) | (1ull << 40); }
__device__ __forceinline__ uint64_t ft_src(const FlowSlot &e) { return (e.w0 & ((1ull << 49) - 1)) - 1; }
__device__ __forceinline__ uint64_t ft_dst(const FlowSlot &e) { return ((e.w0 >> 49) << 33) | (e.w1 & ((1ull << 33) - 1)); }
__device__ __forceinline__ uint32_t ft_hash(uint64_t src, uint64_t dst) {
    uint64_t z = src * 0x9E3779B97F4A7C15ull ^ (dst + 0x632BE59BD9B4E019ull) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 31;
    z *= 0x94D049BB133111EBull;
    return (uint32_t)(z >> 32);
}
// value of a write-once word, setting it to `want` if still 0
__device__ __forceinline__ uint64_t ft_settle(uint64_t *w, uint64_t want) {
    const uint64_t v = *w;
    if (v != 0) return v;
    const uint64_t o = atomicCAS((unsigned long long *)w, 0ull, (unsigned long long)want);
    return o == 0 ? want : o;
}

// slot of (src, dst), inserting it if absent (++created when this call made
// the flow); SLOT_NONE (and a flag) when the probe limit is reached
__device__ uint32_t ft_find_or_insert(FlowSlot *tab, uint32_t mask, uint32_t probe_limit, uint64_t src,
                                      uint64_t dst, unsigned long long *counters, uint32_t &created) {
    const uint64_t a0 = ft_w0(src, dst), a1 = ft_w1(dst);
    // slot `mask` (all ones) is never used: SLOT_NONE then sorts after every
    // slot on the low log2(C) bits (the by-slot grouping sort)
    uint32_t slot = ft_hash(src, dst) & mask;
    if (slot == mask) slot = 0;
    for (uint32_t probe = 0; probe < probe_limit; ++probe, slot = slot + 1 == mask ? 0 : slot + 1) {
        const FlowSlot e = tab[slot];                  // one 16-byte read: the common cases
        if (e.w0 == a0 && e.w1 == a1) return slot;
        if (e.w0 != 0 && (e.w0 != a0 || e.w1 != 0)) continue;
        if (ft_settle(&tab[slot].w0, a0) != a0) continue;
        const uint64_t v = tab[slot].w1;
        if (v == a1) return slot;
        if (v != 0) continue;
        const uint64_t o = atomicCAS((unsigned long long *)&tab[slot].w1, 0ull, (unsigned long long)a1);
        if (o == 0) {
            ++created;   // this key owns the slot (summed per workgroup by the caller)
            return slot;
        }
        if (o == a1) return slot;
    }
    atomicOr(&counters[3], (unsigned long long)FT_OVERFLOW);
    return SLOT_NONE;
}

// Per packet: the SidekickMulti filters (records.h) and, for an Insert, its
// flow's table slot.  Packets of one tile that share a flow elect a leader in
// LDS first (one table probe per flow per tile: with few flows the table
// lines are not hammered by every packet).  Writes slot (SLOT_NONE if not an
// Insert) and id per packet; counters: [0] inserts, [1] resets, [2] distinct
// flows, [3] flags, [4] 1 + the position of the last reset (0: none).
__global__ __launch_bounds__(REC_TILE) void k_flow_extract(const uint8_t *__restrict__ bufs, uint64_t n,
                                                           uint32_t stride, const qk_pkt_meta *__restrict__ meta,
                                                           uint64_t my_key_lo, uint64_t chunk,
                                                           FlowSlot *__restrict__ tab, uint32_t mask,
                                                           uint32_t probe_limit, uint32_t *__restrict__ slots,
                                                           uint32_t *__restrict__ ids,
                                                           unsigned long long *__restrict__ counters) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
    constexpr uint32_t LH = 2 * REC_TILE;                // LDS election table
    __shared__ uint64_t l_src[REC_TILE], l_dst[REC_TILE];
    __shared__ uint32_t l_lead[LH];
    __shared__ uint32_t l_slot[REC_TILE];
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t c1 = c0 + chunk < n ? c0 + chunk : n;
    uint64_t n_ins = 0, n_rst = 0;   // thread 0's running totals
    uint64_t my_rst = 0;             // 1 + this thread's last reset position (0: none)
    __shared__ unsigned long long l_rst;
    if (threadIdx.x == 0) l_rst = 0;
    // flows this thread created; summed in LDS and added with one atomic per
    // workgroup (a per-flow atomic on one counter serialises at 1e6 flows)
    __shared__ uint32_t l_new;
    uint32_t n_new = 0;
    if (threadIdx.x == 0) l_new = 0;
    const bool pipe = stage_pipelined(stride, REC_TILE);
    TileStage st;
    if (pipe && c0 < c1) stage_issue(bufs, n, stride, c0, c1 - c0 < (uint64_t)REC_TILE ? c1 - c0 : REC_TILE, st);
    for (uint64_t p0 = c0; p0 < c1; p0 += REC_TILE) {
        const uint64_t np = c1 - p0 < (uint64_t)REC_TILE ? c1 - p0 : (uint64_t)REC_TILE;
        __syncthreads();   // previous tile fully consumed
        const uint32_t r0 = pipe ? stage_commit(bufs, n, stride, st, tile) : stage_records(bufs, n, stride, p0, np, tile);
        for (uint32_t h = threadIdx.x; h < LH; h += REC_TILE) l_lead[h] = SLOT_NONE;
        __syncthreads();
        if (pipe && p0 + REC_TILE < c1)   // next tile's loads fly while this one is classified
            stage_issue(bufs, n, stride, p0 + REC_TILE,
                        c1 - p0 - REC_TILE < (uint64_t)REC_TILE ? c1 - p0 - REC_TILE : REC_TILE, st);
        const bool valid = threadIdx.x < np;
        const uint64_t i = p0 + threadIdx.x;
        const uint8_t *rec = tile + r0 + threadIdx.x * stride;
        uint64_t src = 0, dst = 0;
        uint32_t id = 0;
        int cls = 0; // 0 skip, 1 insert, 2 reset
        const qk_pkt_meta m = valid ? record_meta(meta, i) : qk_pkt_meta{};
        if (valid && record_is_incoming_udp(m, rec)) {
            // AddrKey halves, big-endian so numeric order == byte order
            src = ((uint64_t)rec[26] << 40) | ((uint64_t)rec[27] << 32) | ((uint64_t)rec[28] << 24) |
                  ((uint64_t)rec[29] << 16) | ((uint64_t)rec[34] << 8) | (uint64_t)rec[35];
            dst = ((uint64_t)rec[30] << 40) | ((uint64_t)rec[31] << 32) | ((uint64_t)rec[32] << 24) |
                  ((uint64_t)rec[33] << 16) | ((uint64_t)rec[36] << 8) | (uint64_t)rec[37];
            if (dst == my_key_lo) {
                cls = 2;
                my_rst = i + 1;
            } else if (m.len == QK_BUFFER_SIZE) {
                cls = 1;
                id = record_identifier(rec);
            }
        }
        l_src[threadIdx.x] = src;
        l_dst[threadIdx.x] = dst;
        __syncthreads();
        // packets of this tile that share a flow elect one leader
        uint32_t lead = SLOT_NONE;
        if (cls == 1) {
            uint32_t h = ft_hash(src, dst) & (LH - 1);
            for (;;) {   // at most REC_TILE claims in LH slots: terminates
                const uint32_t o = atomicCAS(&l_lead[h], SLOT_NONE, threadIdx.x);
                if (o == SLOT_NONE) { lead = threadIdx.x; break; }
                if (l_src[o] == src && l_dst[o] == dst) { lead = o; break; }
                h = (h + 1) & (LH - 1);
            }
            if (lead == threadIdx.x)
                l_slot[threadIdx.x] = ft_find_or_insert(tab, mask, probe_limit, src, dst, counters, n_new);
        }
        __syncthreads();
        if (valid) {
            slots[i] = cls == 1 ? l_slot[lead] : SLOT_NONE;
            ids[i] = id;
        }
        const int ins = __syncthreads_count(cls == 1), rst = __syncthreads_count(cls == 2);
        n_ins += (uint64_t)ins;
        n_rst += (uint64_t)rst;
    }
    if (n_new) atomicAdd(&l_new, n_new);
    if (my_rst) atomicMax(&l_rst, (unsigned long long)my_rst);
    __syncthreads();
    // one atomic per workgroup (a per-packet atomic on one address
    // serialises: 1.2 s per 1e8 packets)
    if (threadIdx.x == 0) {
        if (n_ins) atomicAdd(&counters[0], (unsigned long long)n_ins);
        if (n_rst) atomicAdd(&counters[1], (unsigned long long)n_rst);
        if (l_new) atomicAdd(&counters[2], (unsigned long long)l_new);
        if (l_rst) atomicMax(&counters[4], l_rst);
    }
}

struct SlotUsed {
    const FlowSlot *tab;
    __device__ bool operator()(uint32_t s) const { return tab[s].w0 != 0; }
};

// the AddrKey halves of listed slots (either output may be null)
__global__ void k_slot_keys(const FlowSlot *__restrict__ tab, const uint32_t *__restrict__ slot, uint32_t nf,
                            uint64_t *__restrict__ dst_key, uint64_t *__restrict__ src_key) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nf) return;
    const FlowSlot e = tab[slot[r]];
    if (dst_key) dst_key[r] = ft_dst(e);
    if (src_key) src_key[r] = ft_src(e);
}

// flows in ascending AddrKey order: rank r <-> slot; info[4r] = src, [4r+1] = dst
__global__ void k_slot_rank(const FlowSlot *__restrict__ tab, const uint32_t *__restrict__ slot_of_rank, uint32_t nf,
                            uint32_t *__restrict__ rank_of_slot, uint64_t *__restrict__ info) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nf) return;
    const uint32_t s = slot_of_rank[r];
    const FlowSlot e = tab[s];
    rank_of_slot[s] = r;
    info[4 * (uint64_t)r + 0] = ft_src(e);
    info[4 * (uint64_t)r + 1] = ft_dst(e);
}

// by-slot grouping: pos_of_slot[used[p]] = p (segments are in slot order)
__global__ void k_slot_pos(const uint32_t *__restrict__ used, uint32_t nf, uint32_t *__restrict__ pos_of_slot) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < nf) pos_of_slot[used[p]] = p;
}

// by-slot grouping: output rank r -> segment perm[r]; info[4r] = src, [4r+1] = dst
__global__ void k_rank_perm(const FlowSlot *__restrict__ tab, const uint32_t *__restrict__ slot_of_rank, uint32_t nf,
                            const uint32_t *__restrict__ pos_of_slot, uint32_t *__restrict__ perm,
                            uint64_t *__restrict__ info) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nf) return;
    const uint32_t s = slot_of_rank[r];
    const FlowSlot e = tab[s];
    perm[r] = pos_of_slot[s];
    info[4 * (uint64_t)r + 0] = ft_src(e);
    info[4 * (uint64_t)r + 1] = ft_dst(e);
}

// ---- histogram grouping (few flows: a table of <= HIST_MAX slots) ----------
// Instead of radix-sorting the packets, workgroup w takes the contiguous
// packets [w chunk, (w + 1) chunk): k_hist_count counts its packets per slot
// in LDS and writes the nonzero counts to hist[slot * nwg + w] (zeroed
// before) and the slot's last packet index (+1) with one atomicMax per
// (workgroup, slot); an exclusive sum of hist in that slot-major order gives
// every (slot, workgroup) its place, and k_hist_scatter sends each id there
// (+ its rank within the workgroup's run of that slot, from an LDS counter).
// Segments come out in slot order; the order inside a segment is arbitrary
// (power sums are order-independent) and last_value comes from the last
// packet index, so nothing depends on it.
constexpr uint32_t HIST_MAX = 8192;   // slots (LDS counters per workgroup: 32 KB)

__global__ __launch_bounds__(256) void k_hist_count(const uint32_t *__restrict__ slots, uint64_t n, uint64_t chunk,
                                                    uint32_t C, uint32_t nwg, uint32_t *__restrict__ hist,
                                                    uint32_t *__restrict__ last) {
    extern __shared__ uint32_t lh[];   // C counts, C last indices (+1)
    uint32_t *lc = lh, *ll = lh + C;
    for (uint32_t j = threadIdx.x; j < C; j += blockDim.x) { lc[j] = 0; ll[j] = 0; }
    __syncthreads();
    // four packets per thread and step (chunk is a multiple of 4, the arrays
    // are arena buffers: 16-byte aligned): independent loads in flight
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
    auto one = [&](uint32_t sl, uint64_t i) {
        if (sl != SLOT_NONE) {
            atomicAdd(&lc[sl], 1u);
            atomicMax(&ll[sl], (uint32_t)i + 1u);   // n < 2^32
        }
    };
    const uint64_t v1 = c0 + ((c1 - c0) & ~(uint64_t)3);
    for (uint64_t i = c0 + 4 * threadIdx.x; i < v1; i += 4 * blockDim.x) {
        const uint4 sv = *reinterpret_cast<const uint4 *>(slots + i);
        one(sv.x, i); one(sv.y, i + 1); one(sv.z, i + 2); one(sv.w, i + 3);
    }
    for (uint64_t i = v1 + threadIdx.x; i < c1; i += blockDim.x) one(slots[i], i);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < C; j += blockDim.x) {
        if (lc[j]) {
            hist[(size_t)j * nwg + blockIdx.x] = lc[j];
            atomicMax(&last[j], ll[j]);
        }
    }
}

__global__ __launch_bounds__(256) void k_hist_scatter(const uint32_t *__restrict__ slots,
                                                      const uint32_t *__restrict__ ids, uint64_t n, uint64_t chunk,
                                                      uint32_t C, uint32_t nwg, const uint32_t *__restrict__ base,
                                                      uint32_t *__restrict__ grouped) {
    extern __shared__ uint32_t lc[];   // C running counts
    for (uint32_t j = threadIdx.x; j < C; j += blockDim.x) lc[j] = 0;
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
    auto one = [&](uint32_t sl, uint32_t id) {
        if (sl != SLOT_NONE) {
            const uint32_t r = atomicAdd(&lc[sl], 1u);
            grouped[base[(size_t)sl * nwg + blockIdx.x] + r] = id;
        }
    };
    const uint64_t v1 = c0 + ((c1 - c0) & ~(uint64_t)3);
    for (uint64_t i = c0 + 4 * threadIdx.x; i < v1; i += 4 * blockDim.x) {
        const uint4 sv = *reinterpret_cast<const uint4 *>(slots + i);
        const uint4 iv = *reinterpret_cast<const uint4 *>(ids + i);
        one(sv.x, iv.x); one(sv.y, iv.y); one(sv.z, iv.z); one(sv.w, iv.w);
    }
    for (uint64_t i = v1 + threadIdx.x; i < c1; i += blockDim.x) one(slots[i], ids[i]);
}

// histogram grouping: segment p = the p-th occupied slot (ascending), its
// start = the place of (slot, workgroup 0)
__global__ void k_hist_offsets(const uint32_t *__restrict__ used, uint32_t nf, const uint32_t *__restrict__ base,
                               uint32_t nwg, uint64_t inserted, uint64_t *__restrict__ offs) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < nf) offs[p] = base[(size_t)used[p] * nwg];
    if (p == 0) offs[nf] = inserted;
}

// histogram grouping: info[4r+2] = count, [4r+3] = the id of the flow's last packet
__global__ void k_hist_info(const uint32_t *__restrict__ perm, const uint64_t *__restrict__ offs, uint32_t nf,
                            const uint32_t *__restrict__ used, const uint32_t *__restrict__ last,
                            const uint32_t *__restrict__ ids, uint64_t *__restrict__ info) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nf) return;
    const uint32_t g = perm[r];   // rank -> segment (slot order)
    info[4 * (uint64_t)r + 2] = offs[g + 1] - offs[g];
    info[4 * (uint64_t)r + 3] = ids[last[used[g]] - 1];
}

// by-slot grouping: segment starts of the slot-sorted packets
// Segment starts of the sorted keys: position i starts a segment when
// key[i] != key[i-1].  Each thread compares 4 keys of one 16-byte load (key
// is an arena buffer, 256-byte aligned) with the last key of the previous
// block; segment `seg(k)` gets offs[seg(k)] = i.
template <class Seg>
__device__ __forceinline__ void segment_starts(const uint32_t *__restrict__ key, uint64_t ninserted, uint32_t nf,
                                               uint64_t *__restrict__ offs, Seg seg) {
    const uint64_t nv = ninserted >> 2;
    const uint4 *__restrict__ kv = reinterpret_cast<const uint4 *>(key);
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 k = kv[v];
        const uint64_t i = v << 2;
        if (v == 0 || k.x != key[i - 1]) offs[seg(k.x)] = i;
        if (k.y != k.x) offs[seg(k.y)] = i + 1;
        if (k.z != k.y) offs[seg(k.z)] = i + 2;
        if (k.w != k.z) offs[seg(k.w)] = i + 3;
    }
    const uint64_t t = (nv << 2) + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;   // < 4 tail keys
    if (t < ninserted && (t == 0 || key[t] != key[t - 1])) offs[seg(key[t])] = t;
    if (blockIdx.x == 0 && threadIdx.x == 0) offs[nf] = ninserted;
}

__global__ void k_slot_offsets(const uint32_t *__restrict__ key, uint64_t ninserted,
                               const uint32_t *__restrict__ pos_of_slot, uint32_t nf, uint64_t *__restrict__ offs) {
    segment_starts(key, ninserted, nf, offs, [=](uint32_t k) { return pos_of_slot[k]; });
}

// per packet, in place: slot -> flow rank (non-inserts -> nf, sorting last)
__global__ void k_slot_to_rank(uint32_t *__restrict__ key, const uint32_t *__restrict__ rank_of_slot, uint64_t n,
                               uint32_t nf) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = key[i];
        key[i] = s == SLOT_NONE ? nf : rank_of_slot[s];
    }
}

// segment starts of the rank-sorted packets (every rank 0..nf-1 occurs)
__global__ void k_rank_offsets(const uint32_t *__restrict__ key, uint64_t ninserted, uint32_t nf,
                               uint64_t *__restrict__ offs) {
    segment_starts(key, ninserted, nf, offs, [](uint32_t k) { return k; });
}

// info[4r+2] = count, [4r+3] = last id of flow r (segment perm[r], or r)
__global__ void k_flow_counts(const uint64_t *__restrict__ offs, const uint32_t *__restrict__ ids, uint32_t nf,
                              const uint32_t *__restrict__ perm, uint64_t *__restrict__ info) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nf) return;
    const uint32_t g = perm ? perm[r] : r;
    info[4 * (uint64_t)r + 2] = offs[g + 1] - offs[g];
    info[4 * (uint64_t)r + 3] = ids[offs[g + 1] - 1];
}

// the flows the lane-per-flow kernel does not take (all of them when !small,
// else those of more than SMALL_SEG ids), as (segment, [lo, hi)) work-item
// seeds in any order: the host cuts them into SEG_CHUNK items.  With many
// small flows the list is empty and the host never sees the offsets.
__global__ void k_list_big(const uint64_t *__restrict__ offs, uint32_t nseg, int small,
                           unsigned int *__restrict__ nbig, SegItem *__restrict__ big) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg) return;
    const uint64_t lo = offs[g], hi = offs[g + 1];
    if (hi == lo || (small && hi - lo <= SMALL_SEG)) return;
    const unsigned int k = atomicAdd(nbig, 1u);
    big[k] = SegItem{g, 0u, lo, hi};
}

template <typename Idx>
__device__ __forceinline__ void flow_finalize_body(const unsigned long long *__restrict__ acc,
                                                   const uint64_t *__restrict__ info, const uint32_t *__restrict__ perm,
                                                   Idx nseg, uint32_t T, uint32_t *__restrict__ rec,
                                                   uint8_t *__restrict__ keys) {
    const Idx words = (Idx)4 + T, stride = (Idx)gridDim.x * blockDim.x, tid = (Idx)blockIdx.x * blockDim.x + threadIdx.x;
    for (Idx j = tid; j < nseg * words; j += stride) {
        const Idx i = j / words;
        const uint32_t w = (uint32_t)(j - i * words);
        uint32_t v;
        if (w == 0) v = T;
        else if (w == 1) v = (uint32_t)info[4 * (uint64_t)i + 2];  // count
        else if (w == 2) v = 1u;                                    // has_last
        else if (w == 3) v = (uint32_t)info[4 * (uint64_t)i + 3];  // last_value
        else v = canon32(fold64_32(acc[(perm ? (uint64_t)perm[i] : (uint64_t)i) * T + (w - 4)]));
        rec[j] = v;
    }
    if (((uintptr_t)keys & 3) == 0) {
        // 12 key bytes = 3 words per flow: the two 48-bit halves, big-endian
        uint32_t *kw = reinterpret_cast<uint32_t *>(keys);
        for (Idx j = tid; j < nseg * 3; j += stride) {
            const Idx i = j / 3;
            const uint32_t q = (uint32_t)(j - i * 3);
            const uint64_t a = info[4 * (uint64_t)i], b = info[4 * (uint64_t)i + 1];
            // byte 4q + r of the key is byte 4q + r of (a[47..0], b[47..0]) in big-endian order
            uint32_t v = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t bi = 4 * q + r;
                const uint64_t k = bi < 6 ? a : b;
                v |= (uint32_t)(uint8_t)(k >> (40 - 8 * (bi % 6))) << (8 * r);
            }
            kw[j] = v;
        }
    } else {
        for (Idx j = tid; j < nseg * 12; j += stride) {
            const Idx i = j / 12;
            const uint32_t bi = (uint32_t)(j - i * 12);
            const uint64_t k = bi < 6 ? info[4 * (uint64_t)i] : info[4 * (uint64_t)i + 1];
            keys[j] = (uint8_t)(k >> (40 - 8 * (bi % 6)));
        }
    }
}

// qk_u32 records (header + T canonical sums) and AddrKey bytes of every flow,
// written on the device so the host receives exactly its output in two copies
// (32-bit index arithmetic whenever the record words fit: a 64-bit division
// per word made this kernel 4x slower than its stores)
__global__ void k_flow_finalize(const unsigned long long *__restrict__ acc, const uint64_t *__restrict__ info,
                                const uint32_t *__restrict__ perm, uint64_t nseg, uint32_t T,
                                uint32_t *__restrict__ rec, uint8_t *__restrict__ keys) {
    if (nseg * (4ull + T) < (1ull << 31) && nseg * 12 < (1ull << 31))
        flow_finalize_body<uint32_t>(acc, info, perm, (uint32_t)nseg, T, rec, keys);
    else
        flow_finalize_body<uint64_t>(acc, info, perm, nseg, T, rec, keys);
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

// Bump allocator over a ctx flow arena (256-byte aligned sub-buffers); with
// base == nullptr it only measures.
struct Carve {
    char *base;
    size_t off = 0;
    template <typename T> T *take(size_t count) {
        off = (off + 255) & ~(size_t)255;
        T *p = base ? reinterpret_cast<T *>(base + off) : nullptr;
        off += std::max<size_t>(count * sizeof(T), 8);
        return p;
    }
};

// last id of each non-empty segment
__global__ void k_seg_last(const uint32_t *__restrict__ ids, const uint64_t *__restrict__ offs, uint64_t nseg,
                           uint32_t *__restrict__ last) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nseg) last[i] = offs[i + 1] > offs[i] ? ids[offs[i + 1] - 1] : 0u;
}

// work items of the flows k_seg_small does not take: every flow when T > 32,
// else the flows of more than SMALL_SEG ids
static bool small_ok(uint32_t T) { return T <= 32; }
static std::vector<SegItem> seg_items_from_big(const std::vector<SegItem> &big) {
    std::vector<SegItem> items;
    for (const SegItem &b : big)
        for (uint64_t lo = b.lo; lo < b.hi; lo += SEG_CHUNK)
            items.push_back({b.seg, 0u, lo, std::min<uint64_t>(lo + SEG_CHUNK, b.hi)});
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

// Segmented encode of a grouped id array into a device accumulator [nseg][T]
// (u64, zeroed here): the small flows by k_seg_small (d_offs: the nseg + 1
// offsets on the device), the rest by the work items from seg_items (d_items
// holds items.size() entries).
static int seg_encode(qk_ctx *ctx, const uint32_t *d_ids, const uint64_t *d_offs,
                      const std::vector<SegItem> &items, size_t nseg, uint32_t T, unsigned long long *d_acc,
                      SegItem *d_items, hipStream_t s) {
    QK_HIP_TRY(hipMemsetAsync(d_acc, 0, nseg * T * sizeof(uint64_t), s));
    if (small_ok(T) && nseg) {
        hipEvent_t e0 = prof_begin(ctx, s);
        const int rs = seg_small_launch(ctx->knobs.flow_prio, T, d_ids, d_offs, (uint32_t)nseg, d_acc, s);
        prof_end(ctx, s, e0);
        if (rs) return rs;
    }
    // the caller's host offsets / items vectors must outlive their async copies
    if (items.empty()) return hipStreamSynchronize(s) == hipSuccess ? QK_OK : QK_E_HIP;
    int rc = QK_OK;
    if (hipMemcpyAsync(d_items, items.data(), items.size() * sizeof(SegItem), hipMemcpyHostToDevice, s) != hipSuccess)
        rc = QK_E_HIP;
    if (!rc) {
        int G, K;
        seg_choose(T, G, K);
        const uint32_t ni = (uint32_t)items.size();
        hipEvent_t e0 = prof_begin(ctx, s);
        const dim3 grid(ni), block(bsgs::BLOCK);
        if (T >= 5 && T <= 80) {   // same configurations as the headline encode
            const bool fp = ctx->knobs.flow_prio;   // s_setprio around the MACs (knob flow_prio)
#define QK_SEGB(NB_, NA_, SG_)                                                                                     \
    hipLaunchKernelGGL((fp ? k_seg_bsgs<NB_, NA_, SG_, 1> : k_seg_bsgs<NB_, NA_, SG_, 0>), grid, block, 0, s, d_ids, \
                       d_items, T, d_acc)
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
    // the host vector `items` must outlive the async copy
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = QK_E_HIP;
    return rc;
}

static uint64_t next_pow2(uint64_t v) {
    uint64_t c = 1;
    while (c < v) c <<= 1;
    return c;
}
static int bit_width32(uint32_t v) { return v ? 32 - __builtin_clz(v) : 0; }

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
    probe.take<SegItem>(items.size());
    probe.take<uint32_t>(nseg);
    probe.take<uint64_t>(nseg + 1);
    if (int e = ensure_flow(ctx, 1, probe.off, s)) return e;
    Carve cv{(char *)ctx->d_flow[1]};
    unsigned long long *d_acc = cv.take<unsigned long long>(nseg * T);
    SegItem *d_items = cv.take<SegItem>(items.size());
    uint32_t *d_last = cv.take<uint32_t>(nseg);
    uint64_t *d_offs = cv.take<uint64_t>(nseg + 1);
    int rc = QK_OK;
    if (hipMemcpyAsync(d_offs, offs.data(), (nseg + 1) * 8, hipMemcpyHostToDevice, s) != hipSuccess) rc = QK_E_HIP;
    if (!rc) rc = seg_encode(ctx, d_ids, d_offs, items, nseg, T, d_acc, d_items, s);
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

// The grouping sort (radix.h): chunks of the packets, one per workgroup
struct RsPlan {
    uint32_t nwg;
    uint64_t chunk;   // a multiple of 4
};
// wgpc workgroups per CU (at most: one per 4096 packets)
static RsPlan rs_plan(const qk_ctx *ctx, uint64_t n, uint32_t wgpc) {
    const uint32_t nwg = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>((uint64_t)ctx->num_cus * wgpc, (n + 4095) / 4096));
    return {nwg, (((n + nwg - 1) / nwg) + 3) & ~(uint64_t)3};
}
constexpr uint32_t RS_WGPC_MAX = 4;
// Stable sort of (key, val) by the low `bits` bits of key, 8 bits per pass,
// ping-ponging between region X = (k0, v0) and region Y = (k1, v1); each
// region must also hold n (key, value) pairs from k0 / k1 (arena layout: the
// value array follows the key array).  The first pass reads two arrays, the
// last writes two, the passes between use pair arrays (knob flow_sort 2, 3;
// 1: two arrays throughout).  Returns in `where` the region holding the
// result: 1 = Y, 0 = X (an even number of passes).
template <int D, int BLK, int K, bool PAIRS, uint32_t WGPC, bool DIRECT = false>
static int rs_sort_k(const qk_ctx *ctx, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, uint64_t n, int bits,
                     uint32_t *cnt, uint32_t *base, void *temp, size_t temp_bytes, hipStream_t s, int &where) {
    static_assert(WGPC <= RS_WGPC_MAX, "scratch is sized for RS_WGPC_MAX");
    where = 0;
    if (n == 0 || bits <= 0) return QK_OK;
    const RsPlan pl = rs_plan(ctx, n, WGPC);
    const int passes = (bits + D - 1) / D;
    const int dd = (bits + passes - 1) / passes;   // the digit width actually used (<= D): balanced passes
    uint32_t *ki = k0, *vi = v0, *ko = k1, *vo = v1;
    for (int q = 0; q < passes; ++q) {
        const uint32_t shift = (uint32_t)(q * dd);
        const int left = bits - q * dd;
        const uint32_t mask = left >= dd ? (1u << dd) - 1 : (1u << left) - 1;
        const bool ip = PAIRS && q > 0, op = PAIRS && q + 1 < passes;
        auto count = ip ? rsort::k_rs_count<D, true> : rsort::k_rs_count<D, false>;
        hipLaunchKernelGGL(count, dim3(pl.nwg), dim3(256), 0, s, ki, n, pl.chunk, shift, mask, pl.nwg, cnt);
        if (hipGetLastError() != hipSuccess) return QK_E_HIP;
        size_t tb = temp_bytes;
        if (hipcub::DeviceScan::ExclusiveSum(temp, tb, cnt, base, (int)((1u << D) * pl.nwg), s) != hipSuccess)
            return QK_E_HIP;
        auto kern = ip ? (op ? rsort::k_rs_scatter<D, BLK, K, true, true, DIRECT>
                             : rsort::k_rs_scatter<D, BLK, K, true, false, DIRECT>)
                       : (op ? rsort::k_rs_scatter<D, BLK, K, false, true, DIRECT>
                             : rsort::k_rs_scatter<D, BLK, K, false, false, DIRECT>);
        hipLaunchKernelGGL(kern, dim3(pl.nwg), dim3(BLK), 0, s, ki, vi, n, pl.chunk, shift, mask, pl.nwg, base, ko, vo);
        if (hipGetLastError() != hipSuccess) return QK_E_HIP;
        std::swap(ki, ko);
        std::swap(vi, vo);
    }
    where = passes % 2;
    return QK_OK;
}
static int rs_sort(const qk_ctx *ctx, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, uint64_t n, int bits,
                   uint32_t *cnt, uint32_t *base, void *temp, size_t temp_bytes, hipStream_t s, int &where) {
#define QK_RS(D, BLK, K, PAIRS, WGPC, ...)                                                              \
    return rs_sort_k<D, BLK, K, PAIRS, WGPC, ##__VA_ARGS__>(ctx, k0, v0, k1, v1, n, bits, cnt, base, temp,         \
                                                           temp_bytes, s, where)
    switch (ctx->knobs.flow_sort) {
    case 1: QK_RS(8, 256, 16, false, 4);
    case 2: QK_RS(8, 256, 16, true, 4);
    case 3: QK_RS(8, 512, 16, true, 2);
    case 4: QK_RS(8, 1024, 16, true, 1);
    case 5: QK_RS(11, 512, 16, true, 1);
    case 6: QK_RS(11, 1024, 8, true, 1);
    case 7: QK_RS(8, 256, 16, true, 4, true);
    case 8: QK_RS(11, 512, 16, true, 1, true);
    default: QK_RS(11, 1024, 8, true, 1, true);
    }
#undef QK_RS
}

extern "C" int qk_u32_encode_flows_device(qk_ctx *ctx, const uint8_t *d_bufs, size_t n, size_t stride,
                                          const qk_pkt_meta *d_meta, const uint8_t my_addr[6], uint32_t threshold,
                                          qk_flow_key *keys, uint8_t *sketches, size_t cap, size_t *n_flows,
                                          qk_pkt_stats *stats, void *stream) {
    if (!ctx || !n_flows || (n && !d_bufs)) return QK_E_INVAL;
    if (stride < QK_BUFFER_SIZE || stride > 512) return QK_E_INVAL;
    if (threshold == 0 || threshold > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if (n >= (1ull << 32)) return QK_E_INVAL; // packet indices are u32
    *n_flows = 0;
    qk_pkt_stats st = {0, 0, 0, 0, -1};
    if (n == 0) {
        if (stats) *stats = st;
        return QK_OK;
    }
    if (!is_device_ptr(d_bufs) || (d_meta && !is_device_ptr(d_meta))) return QK_E_INVAL;
    uint64_t my_key = ~0ull; // no own address: no packet is a reset
    if (my_addr)
        my_key = ((uint64_t)my_addr[0] << 40) | ((uint64_t)my_addr[1] << 32) | ((uint64_t)my_addr[2] << 24) |
                 ((uint64_t)my_addr[3] << 16) | ((uint64_t)my_addr[4] << 8) | (uint64_t)my_addr[5];
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = pick_stream(ctx, stream);
    const uint32_t T = threshold;

    // device scratch.  Arena 0, per packet: slot/rank key, id, their sorted
    // copies (16 B per packet), counters, hipCUB temp storage.  Arena 2: the
    // flow table (C slots) and slot -> rank.  Arena 1, per flow: see below.
    const uint64_t cmax = std::min<uint64_t>(next_pow2(2 * (uint64_t)n + 2), 1ull << 31);
    // table slots per expected flow (knob flow_load, [2, 64], for measurements)
    const uint64_t spf = (uint64_t)ctx->knobs.flow_load;
    uint64_t C = std::min<uint64_t>(cmax, next_pow2(std::max<uint64_t>(4096, spf * (uint64_t)ctx->flow_hint)));
    size_t tb = 0;
    {
        uint32_t *u = nullptr;
        uint64_t *k = nullptr;
        size_t b = 0;
        for (int bits = 1; bits <= 32; ++bits) {   // the per-packet sort runs over bit_width(flows) bits
            if (hipcub::DeviceRadixSort::SortPairs(nullptr, b, u, u, u, u, (uint32_t)n, 0, bits, s) != hipSuccess)
                return QK_E_HIP;
            tb = std::max(tb, b);
        }
        if (hipcub::DeviceRadixSort::SortPairs(nullptr, b, k, k, u, u, (uint32_t)n, 0, 48, s) != hipSuccess)
            return QK_E_HIP;
        tb = std::max(tb, b);
        if (hipcub::DeviceSelect::If(nullptr, b, hipcub::CountingInputIterator<uint32_t>(0), u, u, (int64_t)cmax,
                                     SlotUsed{nullptr}, s) != hipSuccess)
            return QK_E_HIP;
        tb = std::max(tb, b);
        if (hipcub::DeviceScan::ExclusiveSum(nullptr, b, u, u, (int)(rsort::RMAX * rs_plan(ctx, n, RS_WGPC_MAX).nwg), s) != hipSuccess)
            return QK_E_HIP;
        tb = std::max(tb, b);
    }
    const uint32_t rs_nwg = rs_plan(ctx, n, RS_WGPC_MAX).nwg;
    uint32_t *slots = nullptr, *ids = nullptr, *key_s = nullptr, *id_s = nullptr, *rs_cnt = nullptr, *rs_base = nullptr;
    unsigned long long *counters = nullptr, *acc = nullptr;
    void *temp = nullptr;
    auto layout0 = [&](Carve &c) {
        slots = c.take<uint32_t>(n); ids = c.take<uint32_t>(n); key_s = c.take<uint32_t>(n); id_s = c.take<uint32_t>(n);
        counters = c.take<unsigned long long>(5);
        temp = c.take<char>(tb);
        rs_cnt = c.take<uint32_t>((size_t)rsort::RMAX * rs_nwg);
        rs_base = c.take<uint32_t>((size_t)rsort::RMAX * rs_nwg);
    };
    {
        Carve probe{nullptr};
        layout0(probe);
        if (int e = ensure_flow(ctx, 0, probe.off, s)) return e;
        Carve cv{(char *)ctx->d_flow[0]};
        layout0(cv);
    }
    // pass 1: filters + flow table over packets [p_from, n); a table that
    // overflows its probe limit is regrown and the pass rerun (the next batch
    // starts from this size).  When the batch holds a reset, every flow made
    // before it is wiped (sidekick_multi.rs:205,265): the pass reruns over the
    // packets after the last reset with an empty table.
    int rc = QK_OK;
    FlowSlot *tab = nullptr;
    uint32_t *rank_of_slot = nullptr;
    uint64_t hc[5] = {0, 0, 0, 0, 0};
    auto pass1 = [&](uint64_t p_from) -> int {
        const uint64_t pn = n - p_from;
        const uint8_t *pb = d_bufs + p_from * stride;
        const qk_pkt_meta *pm = d_meta ? d_meta + p_from : nullptr;
        // >= 4 tiles per workgroup, enough workgroups to cover the chip
        const uint64_t ntiles = (pn + REC_TILE - 1) / REC_TILE;
        // knob flow_wgpc: workgroups per CU (measurements; default 12: 4, 6, 8, 12 measured, 12 best at 1e4 and 1e6 flows)
        const uint64_t wgpc = (uint64_t)ctx->knobs.flow_wgpc;
        const uint64_t tiles_per_chunk =
            std::max<uint64_t>(4, (ntiles + (uint64_t)ctx->num_cus * wgpc - 1) / ((uint64_t)ctx->num_cus * wgpc));
        const uint64_t chunk = tiles_per_chunk * REC_TILE;
        const uint32_t nchunks = (uint32_t)std::max<uint64_t>(1, (pn + chunk - 1) / chunk);
        for (;;) {
            {
                Carve probe{nullptr};
                probe.take<FlowSlot>(C);
                probe.take<uint32_t>(C);
                if (int e = ensure_flow(ctx, 2, probe.off, s)) return e;
                Carve cv{(char *)ctx->d_flow[2]};
                tab = cv.take<FlowSlot>(C);
                rank_of_slot = cv.take<uint32_t>(C);
            }
            if (hipMemsetAsync(tab, 0, C * sizeof(FlowSlot), s) != hipSuccess ||
                hipMemsetAsync(counters, 0, 5 * 8, s) != hipSuccess)
                return QK_E_HIP;
            const uint32_t probe_limit = C == cmax ? (uint32_t)C - 1 : 64u;   // load <= 1/4 when sized from the hint
            if (pn)
                hipLaunchKernelGGL(k_flow_extract, dim3(nchunks), dim3(REC_TILE), (size_t)REC_TILE * stride + 32, s,
                                   pb, pn, (uint32_t)stride, pm, my_key, chunk, tab, (uint32_t)(C - 1), probe_limit,
                                   slots, ids, counters);
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(hc, counters, 40, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return QK_E_HIP;
            if (!(hc[3] & FT_OVERFLOW)) return QK_OK;
            if (C == cmax) return QK_E_NOMEM;   // > 2^31 flows: no table size left
            C = std::min<uint64_t>(cmax, next_pow2(std::max<uint64_t>(16 * C, 4 * hc[2])));
        }
    };
    rc = pass1(0);
    const uint64_t all_inserts = hc[0], resets = hc[1];
    if (!rc && hc[4]) {
        st.last_reset_index = (int64_t)hc[4] - 1;
        rc = pass1(hc[4]);   // the packets after the last reset (no reset among them)
    }
    const uint64_t n_eff = n - (uint64_t)(st.last_reset_index + 1);
    const uint64_t inserted = hc[0];
    const uint32_t nf = (uint32_t)hc[2];
    if (!rc) {
        ctx->flow_hint = nf;
        st.inserted = inserted;
        st.discarded = all_inserts - inserted;
        st.resets = resets;
        st.filtered = n - all_inserts - resets;
        *n_flows = nf;
        if (nf > cap || (nf && (!keys || !sketches))) rc = QK_E_CAPACITY;
    }
    // output in device memory (both arrays): k_flow_finalize writes it in
    // place and nothing crosses PCIe; host memory gets two copies
    const bool dev_out = keys && sketches && is_device_ptr(keys);
    if (!rc && keys && sketches && dev_out != is_device_ptr(sketches)) rc = QK_E_INVAL;
    if (!rc && nf) {
        // per-flow arena 1: info, acc, work items (at most one per flow plus
        // one per SEG_CHUNK ids), output records and keys, offsets, and the
        // flow-key sort buffers
        const size_t items_max = (size_t)nf + inserted / SEG_CHUNK + 1;
        const size_t rec = qk_u32_size(T);
        uint64_t *info = nullptr, *d_offs = nullptr, *kd = nullptr, *kd2 = nullptr, *ks = nullptr, *ks2 = nullptr;
        SegItem *d_items = nullptr;
        uint32_t *d_rec = nullptr, *used = nullptr, *sl2 = nullptr, *sl3 = nullptr, *nsel = nullptr, *perm = nullptr;
        SegItem *big = nullptr;
        uint8_t *d_keys = nullptr;
        void *temp2 = nullptr;   // hipCUB temp of the flow-key branch (runs beside the packet sort)
        size_t tb2 = 0;
        {
            size_t b = 0;
            uint64_t *k = nullptr;
            uint32_t *u = nullptr;
            if (hipcub::DeviceRadixSort::SortPairs(nullptr, b, k, k, u, u, nf, 0, 48, s) != hipSuccess) rc = QK_E_HIP;
            tb2 = std::max(tb2, b);
            if (hipcub::DeviceSelect::If(nullptr, b, hipcub::CountingInputIterator<uint32_t>(0), u, u, (int64_t)C,
                                         SlotUsed{nullptr}, s) != hipSuccess)
                rc = QK_E_HIP;
            tb2 = std::max(tb2, b);
        }
        // histogram grouping: few flows (a table of <= HIST_MAX slots)
        const bool hist = C <= HIST_MAX && ctx->knobs.flow_hist;
        const uint32_t hnwg = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)ctx->num_cus * 4,
                                                                                  (n_eff + 4095) / 4096));
        const uint64_t hchunk = ((n_eff + hnwg - 1) / hnwg + 3) & ~(uint64_t)3;   // a multiple of 4 (16-byte reads)
        uint32_t *hcnt = nullptr, *hlast = nullptr, *hbase = nullptr;
        void *temp3 = nullptr;
        size_t tb3 = 0;
        if (hist) {
            uint32_t *u = nullptr;
            if (hipcub::DeviceScan::ExclusiveSum(nullptr, tb3, u, u, (int)(C * hnwg), s) != hipSuccess) rc = QK_E_HIP;
        }
        auto layout1 = [&](Carve &c) {
            if (hist) {
                hcnt = c.take<uint32_t>((size_t)C * hnwg);
                hbase = c.take<uint32_t>((size_t)C * hnwg);
                hlast = c.take<uint32_t>(C);
                temp3 = c.take<char>(tb3);
            }
            info = c.take<uint64_t>((size_t)nf * 4);
            acc = c.take<unsigned long long>((size_t)nf * T);
            d_items = c.take<SegItem>(items_max);
            d_rec = dev_out ? (uint32_t *)sketches : (uint32_t *)c.take<uint8_t>((size_t)nf * rec);
            d_keys = dev_out ? (uint8_t *)keys : c.take<uint8_t>((size_t)nf * 12);
            d_offs = c.take<uint64_t>((size_t)nf + 1);
            kd = c.take<uint64_t>(nf); kd2 = c.take<uint64_t>(nf); ks = c.take<uint64_t>(nf); ks2 = c.take<uint64_t>(nf);
            used = c.take<uint32_t>(nf); sl2 = c.take<uint32_t>(nf); sl3 = c.take<uint32_t>(nf);
            perm = c.take<uint32_t>(nf);
            nsel = c.take<uint32_t>(2);   // [0] selected slots, [1] flows needing work items
            big = c.take<SegItem>(nf);
            temp2 = c.take<char>(tb2);
        };
        {
            Carve probe{nullptr};
            layout1(probe);
            rc = ensure_flow(ctx, 1, probe.off, s);
        }
        if (!rc) {
            Carve cv{(char *)ctx->d_flow[1]};
            layout1(cv);
        }
        const uint32_t fblocks = (nf + 255) / 256;
        const uint32_t gb = (uint32_t)std::min<uint64_t>((n_eff + 255) / 256, (uint64_t)ctx->num_cus * 8);
        // Two branches (sidekick_multi.rs:265's map iteration order, and the
        // per-packet grouping) that meet at the offsets:
        //   side stream s2: flows in ascending AddrKey order — stable LSD sort
        //     of the occupied slots by dst, then by src (48-bit halves) —
        //     then slot -> segment / rank maps (nf-sized, launch-bound passes);
        //   stream s: one stable radix sort of the packets (key, id), which
        //     groups the ids by flow with packet order kept (last_value = the
        //     flow's last packet).  By slot (no remap: segments come out in
        //     slot order and perm maps rank -> segment) when the table's
        //     log2(C) bits need no more 8-bit passes than the flow count's;
        //     then the sort overlaps the whole s2 branch.  Otherwise by rank
        //     (slot -> rank remap per packet, bit_width(flows) bits), which
        //     waits for s2 first.
        const int fbits = bit_width32(nf), cbits = bit_width32((uint32_t)(C - 1));
        const bool by_slot = (cbits + 7) / 8 <= (fbits + 7) / 8;
        const uint32_t ob = (uint32_t)std::min<uint64_t>((inserted + 255) / 256, (uint64_t)ctx->num_cus * 8);
        hipStream_t s2 = s == ctx->copy_stream ? ctx->stream : ctx->copy_stream;
        if (!rc && (hipEventRecord(ctx->flow_ev[0], s) != hipSuccess || hipStreamWaitEvent(s2, ctx->flow_ev[0], 0) != hipSuccess))
            rc = QK_E_HIP;
        if (!rc && hipcub::DeviceSelect::If(temp2, tb2, hipcub::CountingInputIterator<uint32_t>(0), used, nsel,
                                            (int64_t)C, SlotUsed{tab}, s2) != hipSuccess)
            rc = QK_E_HIP;
        if (!rc) hipLaunchKernelGGL(k_slot_keys, dim3(fblocks), dim3(256), 0, s2, tab, used, nf, kd, (uint64_t *)nullptr);
        if (!rc && hipcub::DeviceRadixSort::SortPairs(temp2, tb2, kd, kd2, used, sl2, nf, 0, 48, s2) != hipSuccess)
            rc = QK_E_HIP;
        if (!rc) hipLaunchKernelGGL(k_slot_keys, dim3(fblocks), dim3(256), 0, s2, tab, sl2, nf, (uint64_t *)nullptr, ks);
        if (!rc && hipcub::DeviceRadixSort::SortPairs(temp2, tb2, ks, ks2, sl2, sl3, nf, 0, 48, s2) != hipSuccess)
            rc = QK_E_HIP;
        if (!rc) {
            if (by_slot || hist) {
                hipLaunchKernelGGL(k_slot_pos, dim3(fblocks), dim3(256), 0, s2, used, nf, rank_of_slot);
                hipLaunchKernelGGL(k_rank_perm, dim3(fblocks), dim3(256), 0, s2, tab, sl3, nf, rank_of_slot, perm, info);
            } else {
                hipLaunchKernelGGL(k_slot_rank, dim3(fblocks), dim3(256), 0, s2, tab, sl3, nf, rank_of_slot, info);
            }
            if (hipGetLastError() != hipSuccess || hipEventRecord(ctx->flow_ev[1], s2) != hipSuccess) rc = QK_E_HIP;
        }
        if (!rc && hist) {
            if (hipMemsetAsync(hcnt, 0, (size_t)C * hnwg * 4, s) != hipSuccess ||
                hipMemsetAsync(hlast, 0, (size_t)C * 4, s) != hipSuccess)
                rc = QK_E_HIP;
            if (!rc) {
                hipLaunchKernelGGL(k_hist_count, dim3(hnwg), dim3(256), (size_t)C * 8, s, slots, n_eff, hchunk, (uint32_t)C,
                                   hnwg, hcnt, hlast);
                if (hipGetLastError() != hipSuccess ||
                    hipcub::DeviceScan::ExclusiveSum(temp3, tb3, hcnt, hbase, (int)(C * hnwg), s) != hipSuccess)
                    rc = QK_E_HIP;
            }
            if (!rc) {
                hipLaunchKernelGGL(k_hist_scatter, dim3(hnwg), dim3(256), (size_t)C * 4, s, slots, ids, n_eff, hchunk,
                                   (uint32_t)C, hnwg, hbase, id_s);
                if (hipGetLastError() != hipSuccess || hipStreamWaitEvent(s, ctx->flow_ev[1], 0) != hipSuccess)
                    rc = QK_E_HIP;
            }
            if (!rc) {
                hipLaunchKernelGGL(k_hist_offsets, dim3(fblocks), dim3(256), 0, s, used, nf, hbase, hnwg, inserted,
                                   d_offs);
                hipLaunchKernelGGL(k_hist_info, dim3(fblocks), dim3(256), 0, s, perm, d_offs, nf, used, hlast, ids, info);
                if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
            }
        } else if (!rc && by_slot) {
            // the grouping sort: radix.h (knob flow_sort = 0: hipCUB's onesweep)
            if (ctx->knobs.flow_sort) {
                int where = 0;
                rc = rs_sort(ctx, slots, ids, key_s, id_s, n_eff, cbits, rs_cnt, rs_base, temp, tb, s, where);
                if (!rc && where == 0) {   // even number of passes: the result is in (slots, ids)
                    std::swap(slots, key_s);
                    std::swap(ids, id_s);
                }
            } else if (hipcub::DeviceRadixSort::SortPairs(temp, tb, slots, key_s, ids, id_s, (uint32_t)n_eff, 0, cbits,
                                                          s) != hipSuccess) {
                rc = QK_E_HIP;
            }
            if (!rc && hipStreamWaitEvent(s, ctx->flow_ev[1], 0) != hipSuccess) rc = QK_E_HIP;
            if (!rc) {
                hipLaunchKernelGGL(k_slot_offsets, dim3(std::max(ob, 1u)), dim3(256), 0, s, key_s, inserted,
                                   rank_of_slot, nf, d_offs);
                hipLaunchKernelGGL(k_flow_counts, dim3(fblocks), dim3(256), 0, s, d_offs, id_s, nf, perm, info);
                if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
            }
        } else if (!rc) {
            if (hipStreamWaitEvent(s, ctx->flow_ev[1], 0) != hipSuccess) rc = QK_E_HIP;
            if (!rc) hipLaunchKernelGGL(k_slot_to_rank, dim3(gb), dim3(256), 0, s, slots, rank_of_slot, n_eff, nf);
            if (!rc && hipGetLastError() != hipSuccess) rc = QK_E_HIP;
            if (!rc && ctx->knobs.flow_sort) {
                int where = 0;
                rc = rs_sort(ctx, slots, ids, key_s, id_s, n_eff, fbits, rs_cnt, rs_base, temp, tb, s, where);
                if (!rc && where == 0) {
                    std::swap(slots, key_s);
                    std::swap(ids, id_s);
                }
            } else if (!rc && hipcub::DeviceRadixSort::SortPairs(temp, tb, slots, key_s, ids, id_s, (uint32_t)n_eff, 0,
                                                                 fbits, s) != hipSuccess) {
                rc = QK_E_HIP;
            }
            if (!rc) {
                hipLaunchKernelGGL(k_rank_offsets, dim3(std::max(ob, 1u)), dim3(256), 0, s, key_s, inserted, nf,
                                   d_offs);
                hipLaunchKernelGGL(k_flow_counts, dim3(fblocks), dim3(256), 0, s, d_offs, id_s, nf,
                                   (const uint32_t *)nullptr, info);
                if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
            }
        }
        // only the flows that need work items come back to the host (none
        // in the many-small-flows case): 8 bytes of counts, then their seeds
        uint32_t hsel[2] = {0, 0};
        std::vector<SegItem> bigs;
        if (!rc) {
            if (hipMemsetAsync(nsel + 1, 0, 4, s) != hipSuccess) rc = QK_E_HIP;
            if (!rc) hipLaunchKernelGGL(k_list_big, dim3(fblocks), dim3(256), 0, s, d_offs, nf, (int)small_ok(T),
                                        nsel + 1, big);
            if (!rc && (hipGetLastError() != hipSuccess ||
                        hipMemcpyAsync(hsel, nsel, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
                        hipStreamSynchronize(s) != hipSuccess))
                rc = QK_E_HIP;
        }
        if (!rc && hsel[0] != nf) rc = QK_E_HIP;   // every occupied slot holds exactly one flow
        if (!rc && hsel[1]) {
            bigs.resize(hsel[1]);
            if (hipMemcpyAsync(bigs.data(), big, bigs.size() * sizeof(SegItem), hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                rc = QK_E_HIP;
        }
        if (!rc) rc = seg_encode(ctx, id_s, d_offs, seg_items_from_big(bigs), nf, T, acc, d_items, s);
        if (!rc) {
            const uint32_t fb = (uint32_t)std::min<uint64_t>(((uint64_t)nf * (4 + T) + 255) / 256,
                                                             (uint64_t)ctx->num_cus * 16);
            hipLaunchKernelGGL(k_flow_finalize, dim3(fb), dim3(256), 0, s, acc, info,
                               by_slot || hist ? (const uint32_t *)perm : nullptr, (uint64_t)nf, T, d_rec, d_keys);
            if (hipGetLastError() != hipSuccess)
                rc = QK_E_HIP;
            else if (!dev_out && (hipMemcpyAsync(sketches, d_rec, (size_t)nf * rec, hipMemcpyDeviceToHost, s) != hipSuccess ||
                                  hipMemcpyAsync(keys, d_keys, (size_t)nf * 12, hipMemcpyDeviceToHost, s) != hipSuccess))
                rc = QK_E_HIP;
        }
    }
    (void)hipStreamSynchronize(s); // the arenas are reused by the next call
    (void)hipStreamSynchronize(s == ctx->copy_stream ? ctx->stream : ctx->copy_stream);   // the flow-key branch
    if (stats) *stats = st;
    return rc;
}
