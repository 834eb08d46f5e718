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
//   2. the occupied slots listed in slot order (k_used_count / k_used_write)
//      and sorted by AddrKey (radix.h over the three 32-bit words of the
//      96-bit key, or one workgroup's rank sort for few flows) -> rank of each
//      flow = output order.
//   3. one stable radix sort of (key, id) pairs (radix.h) groups the ids by
//      flow with packet order preserved (last_value = last id): keyed by the
//      table slot when its bits need no more 8-bit passes than the flow
//      count's (the first pass's chunk histograms come fused from step 1),
//      else by flow rank (a per-packet slot -> rank remap first); few flows
//      (a table of <= 8192 slots) are grouped by per-chunk slot histograms
//      instead.  Offsets from the key changes.  Flows of > SMALL_SEG ids (or
//      any flow when T > 32) -> work items of <= 64 Ki ids per workgroup.
//   4. k_seg_small<Cfg>   one lane per small flow: baby-step/giant-step per id
//      (bsgs.h) with the whole flow in that lane's registers, writing the
//      flow's finished qk_u32 record at its output rank; k_seg_bsgs /
//      k_seg_encode<G,K> for the work items (one workgroup per item, one
//      integer atomicAdd per (flow, power) per item: order-independent,
//      exact), then k_flow_finalize_big writes those flows' records.  The
//      key bytes come from step 2.
// Step 4's kernels and the CSR primitive qk_u32_encode_segments_device (step
// 4 directly on caller-grouped ids) are in segments.hip.
#include <string.h>

#include <algorithm>
#include <vector>

#include "bsgs.h"
#include "ctx.h"
#include "field.h"
#include "radix.h"
#include "records.h"
#include "segments.h"

namespace qk {

QK_WARM_KERNEL(flows)

static_assert(sizeof(qk_flow_key) == 12, "qk_flow_key is 12 packed bytes");
static_assert(sizeof(qk_u32) == 16, "qk_u32 header is 4 words (k_flow_finalize_big writes it)");

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

// home slot of (src, dst): slot `mask` (all ones) is never used, so
// SLOT_NONE then sorts after every slot on the low log2(C) bits (the by-slot
// grouping sort)
__device__ __forceinline__ uint32_t ft_home(uint64_t src, uint64_t dst, uint32_t mask) {
    const uint32_t slot = ft_hash(src, dst) & mask;
    return slot == mask ? 0 : slot;
}

// slot of (src, dst), inserting it if absent (++created when this call made
// the flow); SLOT_NONE (and a flag) when the probe limit is reached.
__device__ uint32_t ft_find_or_insert(FlowSlot *tab, uint32_t mask, uint32_t probe_limit, uint64_t src,
                                      uint64_t dst, unsigned long long *counters, uint32_t &created) {
    const uint64_t a0 = ft_w0(src, dst), a1 = ft_w1(dst);
    uint32_t slot = ft_home(src, dst, mask);
    for (uint32_t probe = 0; probe < probe_limit; ++probe, slot = slot + 1 == mask ? 0 : slot + 1) {
        const FlowSlot e = tab[slot];   // one 16-byte read: the common cases
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
// hcnt != null: also the chunk's histogram of the grouping sort's first
// digit (slot & hmask, SLOT_NONE included), digit-major as k_rs_count writes
// it, added into the sort's chunk (hgroup consecutive extract chunks; hcnt
// zeroed first): the sort's first pass then reads no keys.
// The records are read and the (slot, id) written nontemporal (1e6 flows
// 6.04 -> 5.93 ms, 16 flows 2.88 -> 2.81 ms, profiles/r05/flows_nt/): the
// table's lines stay cached instead of being pushed out by the records.
// Bail: an overflowing pass stops early (it is rerun on a regrown table and
// its outputs dropped) — a workgroup whose own probe overflowed leaves at its
// next tile, and every FLOW_BAIL-th tile thread 0 reads the global overflow
// flag (a load per tile measured 5 % slower; a fresh context's 1e6-flow
// batch 64.5 -> 7.3 ms, profiles/r05/flows_bail/).
constexpr uint32_t FLOW_BAIL = 64;
__global__ __launch_bounds__(REC_TILE) void k_flow_extract(const uint8_t *__restrict__ bufs, uint64_t n,
                                                           uint32_t stride, const qk_pkt_meta *__restrict__ meta,
                                                           uint64_t my_key_lo, uint64_t chunk,
                                                           FlowSlot *__restrict__ tab, uint32_t mask,
                                                           uint32_t probe_limit, uint32_t *__restrict__ slots,
                                                           uint32_t *__restrict__ ids,
                                                           unsigned long long *__restrict__ counters,
                                                           uint32_t hmask, uint32_t *__restrict__ hcnt,
                                                           uint32_t hgroup) {
    constexpr bool NT = true;
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];
    __shared__ uint32_t l_stop;
    uint32_t since = 0;   // tiles since the last overflow check
    if (threadIdx.x == 0) l_stop = 0;   // (read only after the loop's first barrier)
    __shared__ uint32_t l_hist[rsort::R];
    if (hcnt)
        for (uint32_t j = threadIdx.x; j < rsort::R; j += REC_TILE) l_hist[j] = 0;
    constexpr uint32_t LH = 2 * REC_TILE;                // LDS election table
    __shared__ uint64_t l_src[REC_TILE], l_dst[REC_TILE];
    __shared__ uint32_t l_lead[LH];
    __shared__ uint32_t l_slot[REC_TILE];
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t c1 = c0 + chunk < n ? c0 + chunk : n;
    uint32_t n_ins = 0, n_rst = 0;   // this thread's inserts and resets (< 2^32 packets)
    __shared__ unsigned long long l_ins, l_rsts;
    if (threadIdx.x == 0) l_ins = l_rsts = 0;
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
    if (pipe && c0 < c1) stage_issue<NT>(bufs, n, stride, c0, c1 - c0 < (uint64_t)REC_TILE ? c1 - c0 : REC_TILE, st);
    for (uint64_t p0 = c0; p0 < c1; p0 += REC_TILE) {
        const uint64_t np = c1 - p0 < (uint64_t)REC_TILE ? c1 - p0 : (uint64_t)REC_TILE;
        __syncthreads();   // previous tile fully consumed
        // bail: stop once this workgroup's own probes overflowed, or (flag
        // read every FLOW_BAIL-th tile) any other's
        const bool chk = ++since >= FLOW_BAIL;
        if (chk) since = 0;
        const uint64_t fl = chk && threadIdx.x == 0
                                ? __hip_atomic_load(&counters[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : 0ull;
        const uint32_t r0 = pipe ? stage_commit(bufs, n, stride, st, tile) : stage_records<NT>(bufs, n, stride, p0, np, tile);
        for (uint32_t h = threadIdx.x; h < LH; h += REC_TILE) l_lead[h] = SLOT_NONE;
        if (fl & FT_OVERFLOW) l_stop = 1;
        __syncthreads();
        if (l_stop) break;   // uniform: set only before the barrier above (0 -> 1 once)
        // (since: same count in every thread, so chk is uniform too)
        if (pipe && p0 + REC_TILE < c1)   // next tile's loads fly while this one is classified
            stage_issue<NT>(bufs, n, stride, p0 + REC_TILE,
                        c1 - p0 - REC_TILE < (uint64_t)REC_TILE ? c1 - p0 - REC_TILE : REC_TILE, st);
        const bool valid = threadIdx.x < np;
        const uint64_t i = p0 + threadIdx.x;
        const uint8_t *rec = tile + r0 + threadIdx.x * stride;
        uint64_t src = 0, dst = 0;
        uint32_t id = 0;
        int cls = 0; // 0 skip, 1 insert, 2 reset
        const qk_pkt_meta m = valid ? record_meta<NT>(meta, i) : qk_pkt_meta{};
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
            if (lead == threadIdx.x) {
                const uint32_t sl = ft_find_or_insert(tab, mask, probe_limit, src, dst, counters, n_new);
                l_slot[threadIdx.x] = sl;
                if (sl == SLOT_NONE) l_stop = 1;   // this workgroup overflowed: it leaves at the next tile
            }
        }
        __syncthreads();
        if (valid) {
            const uint32_t sl = cls == 1 ? l_slot[lead] : SLOT_NONE;
            __builtin_nontemporal_store(sl, &slots[i]);
            __builtin_nontemporal_store(id, &ids[i]);
            if (hcnt) atomicAdd(&l_hist[sl & hmask], 1u);
        }
        n_ins += cls == 1;   // summed once per workgroup below (no per-tile barrier count)
        n_rst += cls == 2;
    }
    if (n_new) atomicAdd(&l_new, n_new);
    if (my_rst) atomicMax(&l_rst, (unsigned long long)my_rst);
    if (n_ins) atomicAdd(&l_ins, (unsigned long long)n_ins);
    if (n_rst) atomicAdd(&l_rsts, (unsigned long long)n_rst);
    __syncthreads();
    if (hcnt)
        for (uint32_t j = threadIdx.x; j < rsort::R; j += REC_TILE)
            if (l_hist[j]) atomicAdd(&hcnt[(size_t)j * ((gridDim.x + hgroup - 1) / hgroup) + blockIdx.x / hgroup], l_hist[j]);
    // one atomic per workgroup (a per-packet atomic on one address
    // serialises: 1.2 s per 1e8 packets)
    if (threadIdx.x == 0) {
        if (l_ins) atomicAdd(&counters[0], l_ins);
        if (l_rsts) atomicAdd(&counters[1], l_rsts);
        if (l_new) atomicAdd(&counters[2], (unsigned long long)l_new);
        if (l_rst) atomicMax(&counters[4], l_rst);
    }
}

// ---- the occupied slots in slot order (an ordered compaction) -------------
// nb workgroups, workgroup w takes slots [w chunk, (w + 1) chunk) (chunk a
// multiple of 256): k_used_count counts its occupied slots, k_used_write
// finds its place (the counts of the workgroups before it) and writes them in
// order, one 256-slot round at a time (ballot ranks within a wave, the wave
// offsets in LDS); the last workgroup writes the total to *nsel.
__global__ __launch_bounds__(256) void k_used_count(const FlowSlot *__restrict__ tab, uint64_t C, uint64_t chunk,
                                                    uint32_t *__restrict__ wcnt) {
    __shared__ uint32_t ws[4];
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < C ? c0 + chunk : C;
    uint32_t k = 0;
    for (uint64_t i = c0 + threadIdx.x; i < c1; i += 256) k += tab[i].w0 != 0;
    uint32_t all;
    (void)rsort::block_excl<4>(k, ws, &all);
    if (threadIdx.x == 0) wcnt[blockIdx.x] = all;
}

__global__ __launch_bounds__(256) void k_used_write(const FlowSlot *__restrict__ tab, uint64_t C, uint64_t chunk,
                                                    const uint32_t *__restrict__ wcnt, uint32_t *__restrict__ used,
                                                    uint32_t *__restrict__ nsel) {
    __shared__ uint32_t ws[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // this workgroup's place: the counts of the workgroups before it
    uint32_t before = 0;
    for (uint32_t w = threadIdx.x; w < blockIdx.x; w += 256) before += wcnt[w];
    uint32_t pos;
    (void)rsort::block_excl<4>(before, ws, &pos);
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < C ? c0 + chunk : C;
    for (uint64_t b = c0; b < c1; b += 256) {
        const uint64_t i = b + threadIdx.x;
        const bool u = i < c1 && tab[i].w0 != 0;
        const uint64_t m = __ballot(u);
        if (lane == 0) ws[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t off = 0, round = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            off += w < wave ? ws[w] : 0u;
            round += ws[w];
        }
        if (u) used[pos + off + rsort::lanes_below(m)] = (uint32_t)i;
        pos += round;
        __syncthreads();
    }
    if (blockIdx.x + 1 == gridDim.x && threadIdx.x == 0) *nsel = pos;
}

// ---- flows in ascending AddrKey order ---------------------------------------
// The 96-bit key src48 2^48 + dst48 as three 32-bit words, least significant
// first (an LSD sort takes them in that order)
__device__ __forceinline__ uint32_t ft_word(const FlowSlot &e, int q) {
    const uint64_t src = ft_src(e), dst = ft_dst(e);
    return q == 0 ? (uint32_t)dst : q == 1 ? (uint32_t)(dst >> 32) | (uint32_t)(src & 0xFFFF) << 16
                                           : (uint32_t)(src >> 16);
}

// key[i] = word q of slot val[i]'s key (val == slots: also copied to vals)
__global__ void k_slot_word(const FlowSlot *__restrict__ tab, const uint32_t *__restrict__ slots, uint32_t nf, int q,
                            uint32_t *__restrict__ key, uint32_t *__restrict__ vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    const uint32_t sl = slots[i];
    key[i] = ft_word(tab[sl], q);
    if (vals) vals[i] = sl;
}

// few flows (nf <= KR_MAX): one workgroup ranks every key against all the
// others in LDS (keys are distinct: one flow per occupied slot)
constexpr uint32_t KR_MAX = 2048;
__global__ __launch_bounds__(1024) void k_key_rank_small(const FlowSlot *__restrict__ tab,
                                                         const uint32_t *__restrict__ used, uint32_t nf,
                                                         uint32_t *__restrict__ sorted) {
    __shared__ uint32_t kw[3][KR_MAX];
    for (uint32_t i = threadIdx.x; i < nf; i += blockDim.x) {
        const FlowSlot e = tab[used[i]];
        kw[0][i] = ft_word(e, 0);
        kw[1][i] = ft_word(e, 1);
        kw[2][i] = ft_word(e, 2);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nf; i += blockDim.x) {
        const uint32_t a2 = kw[2][i], a1 = kw[1][i], a0 = kw[0][i];
        uint32_t rank = 0;
        for (uint32_t j = 0; j < nf; ++j) {
            const uint32_t b2 = kw[2][j], b1 = kw[1][j], b0 = kw[0][j];
            rank += b2 < a2 || (b2 == a2 && (b1 < a1 || (b1 == a1 && b0 < a0)));
        }
        sorted[rank] = used[i];
    }
}

// the AddrKey halves of listed slots (either output may be null)
__global__ void k_slot_keys(const FlowSlot *__restrict__ tab, const uint32_t *__restrict__ slot, uint32_t nf,
                            uint64_t *__restrict__ dst_key, uint64_t *__restrict__ src_key) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nf) return;
    const FlowSlot e = tab[slot[r]];
    if (dst_key) dst_key[r] = ft_dst(e);
    if (src_key) src_key[r] = ft_src(e);
}

// the 12 AddrKey bytes of output rank r: src48 then dst48, big-endian
// (3 words when the array is 4-byte aligned)
__device__ __forceinline__ void put_key(uint8_t *__restrict__ keys, uint32_t r, uint64_t a, uint64_t b) {
    auto byte = [&](uint32_t bi) { return (uint8_t)((bi < 6 ? a : b) >> (40 - 8 * (bi % 6))); };
    if (((uintptr_t)keys & 3) == 0) {
        uint32_t *kw = reinterpret_cast<uint32_t *>(keys) + 3 * (size_t)r;
#pragma unroll
        for (uint32_t q = 0; q < 3; ++q)
            kw[q] = (uint32_t)byte(4 * q) | (uint32_t)byte(4 * q + 1) << 8 | (uint32_t)byte(4 * q + 2) << 16 |
                    (uint32_t)byte(4 * q + 3) << 24;
    } else {
        for (uint32_t bi = 0; bi < 12; ++bi) keys[12 * (size_t)r + bi] = byte(bi);
    }
}

// flows in ascending AddrKey order: rank r <-> slot; the key bytes of rank r
__global__ void k_slot_rank(const FlowSlot *__restrict__ tab, const uint32_t *__restrict__ slot_of_rank, uint32_t nf,
                            uint32_t *__restrict__ rank_of_slot, uint8_t *__restrict__ keys) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nf) return;
    const uint32_t s = slot_of_rank[r];
    const FlowSlot e = tab[s];
    rank_of_slot[s] = r;
    put_key(keys, r, ft_src(e), ft_dst(e));
}

// by-slot grouping: pos_of_slot[used[p]] = p (segments are in slot order)
__global__ void k_slot_pos(const uint32_t *__restrict__ used, uint32_t nf, uint32_t *__restrict__ pos_of_slot) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < nf) pos_of_slot[used[p]] = p;
}

// by-slot grouping: segment (occupied-slot position) -> output rank; the key
// bytes of rank r
__global__ void k_rank_perm(const FlowSlot *__restrict__ tab, const uint32_t *__restrict__ slot_of_rank, uint32_t nf,
                            const uint32_t *__restrict__ pos_of_slot, uint32_t *__restrict__ rseg,
                            uint8_t *__restrict__ keys) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nf) return;
    const uint32_t s = slot_of_rank[r];
    const FlowSlot e = tab[s];
    rseg[pos_of_slot[s]] = r;
    put_key(keys, r, ft_src(e), ft_dst(e));
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

// the per-packet arrays read nontemporal (read once, as the grouping sort's
// scatters read theirs)
__device__ __forceinline__ uint4 ld_u4(const uint32_t *p) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
}
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
    const int lane = threadIdx.x & 63;
    for (uint64_t i = c0 + 4 * threadIdx.x; i < v1; i += 4 * blockDim.x) {
        const uint4 sv = ld_u4(slots + i);
        // a wave whose packets all hold one slot (one flow, or a skewed
        // batch) adds them with one LDS atomic instead of 256 on one counter
        const uint32_t s0 = __builtin_amdgcn_readfirstlane(sv.x);
        if (__all(sv.x == s0 && sv.y == s0 && sv.z == s0 && sv.w == s0) && s0 != SLOT_NONE) {
            const uint64_t act = __ballot(1);
            const int first = __ffsll((unsigned long long)act) - 1, last = 63 - __clzll((long long)act);
            const uint64_t ilast = (uint64_t)__shfl((unsigned long long)i, last);
            if (lane == first) {
                atomicAdd(&lc[s0], 4u * (uint32_t)__popcll(act));
                atomicMax(&ll[s0], (uint32_t)ilast + 4u);   // the wave's last packet + 1
            }
        } else {
            one(sv.x, i); one(sv.y, i + 1); one(sv.z, i + 2); one(sv.w, i + 3);
        }
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
                                                      const uint32_t *__restrict__ spre,
                                                      uint32_t *__restrict__ grouped) {
    extern __shared__ uint32_t lc[];   // C running counts
    for (uint32_t j = threadIdx.x; j < C; j += blockDim.x) lc[j] = 0;
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
    auto one = [&](uint32_t sl, uint32_t id) {
        if (sl != SLOT_NONE) {
            const uint32_t r = atomicAdd(&lc[sl], 1u);
            grouped[spre[sl] + base[(size_t)sl * nwg + blockIdx.x] + r] = id;   // k_row_scan's two levels
        }
    };
    const uint64_t v1 = c0 + ((c1 - c0) & ~(uint64_t)3);
    const int lane = threadIdx.x & 63;
    for (uint64_t i = c0 + 4 * threadIdx.x; i < v1; i += 4 * blockDim.x) {
        const uint4 sv = ld_u4(slots + i);
        const uint4 iv = ld_u4(ids + i);
        // one slot across the wave (as k_hist_count): one LDS atomic reserves
        // the wave's places, each lane takes four in lane order
        const uint32_t s0 = __builtin_amdgcn_readfirstlane(sv.x);
        if (__all(sv.x == s0 && sv.y == s0 && sv.z == s0 && sv.w == s0) && s0 != SLOT_NONE) {
            const uint64_t act = __ballot(1);
            const int first = __ffsll((unsigned long long)act) - 1;
            uint32_t r = 0;
            if (lane == first) r = atomicAdd(&lc[s0], 4u * (uint32_t)__popcll(act));
            r = (uint32_t)__shfl((int)r, first) + 4u * rsort::lanes_below(act);
            uint32_t *g = grouped + spre[s0] + base[(size_t)s0 * nwg + blockIdx.x] + r;
            g[0] = iv.x;
            g[1] = iv.y;
            g[2] = iv.z;
            g[3] = iv.w;
        } else {
            one(sv.x, iv.x); one(sv.y, iv.y); one(sv.z, iv.z); one(sv.w, iv.w);
        }
    }
    for (uint64_t i = v1 + threadIdx.x; i < c1; i += blockDim.x) one(slots[i], ids[i]);
}

// histogram grouping: segment p = the p-th occupied slot (ascending), its
// start = the place of (slot, workgroup 0): the slot's prefix
__global__ void k_hist_offsets(const uint32_t *__restrict__ used, uint32_t nf, const uint32_t *__restrict__ spre,
                               uint64_t inserted, uint64_t *__restrict__ offs) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < nf) offs[p] = spre[used[p]];
    if (p == 0) offs[nf] = inserted;
}

// histogram grouping: lastid[p] = the id of segment p's last packet (the
// order inside a segment is arbitrary; last[] holds the slot's last index + 1)
__global__ void k_hist_last(const uint32_t *__restrict__ used, uint32_t nf, const uint32_t *__restrict__ last,
                            const uint32_t *__restrict__ ids, uint32_t *__restrict__ lastid) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < nf) lastid[p] = ids[last[used[p]] - 1];
}

// by-slot grouping: segment starts of the slot-sorted packets
// Segment starts of the sorted keys: position i starts a segment when
// key[i] != key[i-1].  Each thread compares 4 keys of one 16-byte load (key
// is an arena buffer, 256-byte aligned) with the last key of the previous
// block — the previous lane's, by a shuffle (lane 0 loads it); segment
// `seg(k)` gets offs[seg(k)] = i.  SS_U blocks per thread per trip, their
// loads issued together (nontemporal: the keys are read once): one load in
// flight per thread left the kernel at 48 dependent round trips per thread
// at 10^6 flows (138 µs for 4e8 bytes).
constexpr int SS_U = 4;
template <class Seg>
__device__ __forceinline__ void segment_starts(const uint32_t *__restrict__ key, uint64_t ninserted, uint32_t nf,
                                               uint64_t *__restrict__ offs, Seg seg) {
    const uint64_t nv = ninserted >> 2;
    const uint4 *__restrict__ kv = reinterpret_cast<const uint4 *>(key);
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    const int lane = threadIdx.x & 63;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    for (uint64_t v0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v0 < nv; v0 += SS_U * nthr) {
        uint4 k[SS_U];
#pragma unroll
        for (int u = 0; u < SS_U; ++u) {   // the trip's loads first
            const uint64_t v = v0 + u * nthr;
            u32x4 x = {0u, 0u, 0u, 0u};
            if (v < nv) x = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(&kv[v]));
            k[u] = make_uint4(x[0], x[1], x[2], x[3]);
        }
#pragma unroll
        for (int u = 0; u < SS_U; ++u) {
            const uint64_t v = v0 + u * nthr;
            // lanes of a wave hold consecutive blocks (v - 1 is the lane below,
            // active whenever this lane is)
            uint32_t prev = (uint32_t)__shfl_up((int)k[u].w, 1, 64);
            if (lane == 0) prev = v > 0 && v < nv ? key[(v << 2) - 1] : ~k[u].x;
            if (v >= nv) break;
            const uint64_t i = v << 2;
            if (v == 0 || k[u].x != prev) offs[seg(k[u].x)] = i;
            if (k[u].y != k[u].x) offs[seg(k[u].y)] = i + 1;
            if (k[u].z != k[u].y) offs[seg(k[u].z)] = i + 2;
            if (k[u].w != k[u].z) offs[seg(k[u].w)] = i + 3;
        }
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

// The records (header + T canonical sums) of the flows that went through work
// items — big[j] = (segment g, its ids [lo, hi)), accumulator row j — at
// their output ranks; k_seg_small wrote every other flow's record itself.
// (32-bit index arithmetic whenever the words fit: a 64-bit division per word
// made the all-flows form of this kernel 4x slower than its stores)
template <typename Idx>
__device__ __forceinline__ void finalize_big_body(const unsigned long long *__restrict__ acc,
                                                  const SegItem *__restrict__ big, Idx nbig,
                                                  const uint32_t *__restrict__ rseg,
                                                  const uint32_t *__restrict__ lastid,
                                                  const uint32_t *__restrict__ ids, uint32_t T,
                                                  uint32_t *__restrict__ rec) {
    const Idx words = (Idx)4 + T, stride = (Idx)gridDim.x * blockDim.x, tid = (Idx)blockIdx.x * blockDim.x + threadIdx.x;
    for (Idx i = tid; i < nbig * words; i += stride) {
        const Idx j = i / words;
        const uint32_t w = (uint32_t)(i - j * words);
        const SegItem it = big[j];
        uint32_t v;
        if (w == 0) v = T;
        else if (w == 1) v = (uint32_t)(it.hi - it.lo);                   // count
        else if (w == 2) v = 1u;                                          // has_last
        else if (w == 3) v = lastid ? lastid[it.seg] : ids[it.hi - 1];    // last_value
        else v = canon32(fold64_32(acc[(uint64_t)j * T + (w - 4)]));
        rec[(uint64_t)(rseg ? rseg[it.seg] : it.seg) * words + w] = v;
    }
}

__global__ void k_flow_finalize_big(const unsigned long long *__restrict__ acc, const SegItem *__restrict__ big,
                                    uint64_t nbig, const uint32_t *__restrict__ rseg,
                                    const uint32_t *__restrict__ lastid, const uint32_t *__restrict__ ids, uint32_t T,
                                    uint32_t *__restrict__ rec) {
    if (nbig * (4ull + T) < (1ull << 31)) finalize_big_body<uint32_t>(acc, big, (uint32_t)nbig, rseg, lastid, ids, T, rec);
    else finalize_big_body<uint64_t>(acc, big, nbig, rseg, lastid, ids, T, rec);
}

static uint64_t next_pow2(uint64_t v) {
    uint64_t c = 1;
    while (c < v) c <<= 1;
    return c;
}
static int bit_width32(uint32_t v) { return v ? 32 - __builtin_clz(v) : 0; }

} // namespace qk

using namespace qk;

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
// per-digit chunk counts, their prefixes within each digit and the digit
// totals (k_row_scan) for one sort at a time; dig: one byte per item, the
// next pass's 8-bit digit written by the scatter
struct RsScratch {
    uint32_t *cnt, *base, *tot;
    uint8_t *dig;
    template <class Carver> void take(Carver &c, uint32_t nwg, uint64_t n) {
        cnt = c.template take<uint32_t>((size_t)rsort::R * nwg);
        base = c.template take<uint32_t>((size_t)rsort::R * nwg);
        tot = c.template take<uint32_t>(rsort::R);
        dig = c.template take<uint8_t>(n + 16);
    }
};
// Stable sort of (key, val) by the low `bits` bits of key, 8 bits per pass,
// ping-ponging between region X = (k0, v0) and region Y = (k1, v1); each
// region must also hold n (key, value) pairs from k0 / k1 (arena layout: the
// value array follows the key array).  The first pass reads two arrays, the
// last writes two, the passes between use pair arrays.  Every scatter writes
// the next pass's digit as a byte beside each item, so the later passes
// count 1 byte per item (k_rs_count8) instead of 8.  Returns in `where` the
// region holding the result: 1 = Y, 0 = X (an even number of passes).
// plan: the chunking to use instead of rs_plan's (pre0: sc.cnt already holds
// the first pass's counts for it — k_flow_extract's fused histogram; the
// scratch must hold R x plan->nwg counts)
template <int BLK, int K, uint32_t WGPC>
static int rs_sort_k(const qk_ctx *ctx, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, uint64_t n, int bits,
                     const RsScratch &sc, hipStream_t s, int &where, const RsPlan *plan = nullptr, bool pre0 = false) {
    static_assert(WGPC <= RS_WGPC_MAX, "scratch is sized for RS_WGPC_MAX");
    constexpr int D = rsort::DBITS;
    where = 0;
    if (n == 0 || bits <= 0) return QK_OK;
    const RsPlan pl0 = plan ? *plan : rs_plan(ctx, n, WGPC);
    // the digit byte stream needs 16-item chunks (k_rs_count8's loads)
    const RsPlan pl = RsPlan{pl0.nwg, (pl0.chunk + 15) & ~(uint64_t)15};
    const int passes = (bits + D - 1) / D;
    const int dd = (bits + passes - 1) / passes;   // the digit width actually used (<= D): balanced passes
    uint32_t *ki = k0, *vi = v0, *ko = k1, *vo = v1;
    for (int q = 0; q < passes; ++q) {
        const uint32_t shift = (uint32_t)(q * dd);
        const int left = bits - q * dd;
        const uint32_t mask = left >= dd ? (1u << dd) - 1 : (1u << left) - 1;
        const bool ip = q > 0, op = q + 1 < passes;
        if (q > 0)   // the previous scatter wrote this pass's digits as bytes
            hipLaunchKernelGGL(rsort::k_rs_count8, dim3(pl.nwg), dim3(256), 0, s, sc.dig, n, pl.chunk, pl.nwg, sc.cnt);
        else if (!pre0)
            hipLaunchKernelGGL(rsort::k_rs_count, dim3(pl.nwg), dim3(256), 0, s, ki, n, pl.chunk, shift, mask, pl.nwg,
                               sc.cnt);
        if (hipGetLastError() != hipSuccess) return QK_E_HIP;
        // digit-major counts -> each digit's chunk prefixes + the digit totals
        // (the scatter scans the totals itself)
        hipLaunchKernelGGL(rsort::k_row_scan<256>, dim3(1u << D), dim3(256), 0, s, sc.cnt, pl.nwg, sc.base, sc.tot);
        if (hipGetLastError() != hipSuccess) return QK_E_HIP;
        auto kern = ip ? (op ? rsort::k_rs_scatter<D, BLK, K, true, true> : rsort::k_rs_scatter<D, BLK, K, true, false>)
                       : (op ? rsort::k_rs_scatter<D, BLK, K, false, true> : rsort::k_rs_scatter<D, BLK, K, false, false>);
        // the next pass's digit as a byte beside each item
        const uint32_t nshift = (uint32_t)((q + 1) * dd);
        const int nleft = bits - (q + 1) * dd;
        const uint32_t nmask = nleft >= dd ? (1u << dd) - 1 : (1u << (nleft > 0 ? nleft : 0)) - 1;
        hipLaunchKernelGGL(kern, dim3(pl.nwg), dim3(BLK), 0, s, ki, vi, n, pl.chunk, shift, mask, pl.nwg, sc.base,
                           sc.tot, ko, vo, op ? sc.dig : (uint8_t *)nullptr, nshift, nmask);
        if (hipGetLastError() != hipSuccess) return QK_E_HIP;
        std::swap(ki, ko);
        std::swap(vi, vo);
    }
    where = passes % 2;
    return QK_OK;
}
// the grouping sort: 256 threads x 16 items per sub-tile, 4 workgroups per CU
static int rs_sort(const qk_ctx *ctx, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, uint64_t n, int bits,
                   const RsScratch &sc, hipStream_t s, int &where, const RsPlan *plan = nullptr, bool pre0 = false) {
    return rs_sort_k<256, 16, 4>(ctx, k0, v0, k1, v1, n, bits, sc, s, where, plan, pre0);
}

// k_flow_extract's chunking of pn packets: >= 4 tiles per workgroup, enough
// workgroups to cover the chip (FLOW_WGPC workgroups per CU; 4, 6, 8, 12
// measured, 12 best at 1e4 and 1e6 flows).  With the fused first-digit
// histogram the grouping sort keeps this chunking (RsPlan).
constexpr uint32_t FLOW_WGPC = 12;
static RsPlan extract_plan(const qk_ctx *ctx, uint64_t pn) {
    const uint64_t ntiles = (pn + REC_TILE - 1) / REC_TILE;
    const uint64_t wg = (uint64_t)ctx->num_cus * FLOW_WGPC;
    const uint64_t chunk = std::max<uint64_t>(4, (ntiles + wg - 1) / wg) * REC_TILE;
    return {(uint32_t)std::max<uint64_t>(1, (pn + chunk - 1) / chunk), chunk};
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
    // copies (16 B per packet), counters, the grouping sort's scan scratch.
    // Arena 2: the flow table (C slots) and slot -> rank.  Arena 1, per flow:
    // see below.
    const uint64_t cmax = std::min<uint64_t>(next_pow2(2 * (uint64_t)n + 2), 1ull << 31);
    // table slots per expected flow (2 / 8 measured slower at 1e6 / 1e4 flows,
    // profiles/r02/s3/flows_load/, profiles/r05/flows_nd/)
    const uint64_t spf = 4;
    uint64_t C = std::min<uint64_t>(cmax, next_pow2(std::max<uint64_t>(4096, spf * (uint64_t)ctx->flow_hint)));
    // the grouping sort's chunk counts: its own plan's, or the extract's
    const uint32_t rs_nwg = std::max(rs_plan(ctx, n, RS_WGPC_MAX).nwg, extract_plan(ctx, n).nwg);
    uint32_t *slots = nullptr, *ids = nullptr, *key_s = nullptr, *id_s = nullptr;
    unsigned long long *counters = nullptr, *acc = nullptr;
    RsScratch rs{};
    auto layout0 = [&](Carve &c) {
        slots = c.take<uint32_t>(n); ids = c.take<uint32_t>(n); key_s = c.take<uint32_t>(n); id_s = c.take<uint32_t>(n);
        counters = c.take<unsigned long long>(5);
        rs.take(c, rs_nwg, n);
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
    RsPlan xpl{1, 4};   // the extract's chunking of the last pass 1
    // the grouping sort's chunks when the extract counts its first digit: hg
    // consecutive extract chunks each (~RS_WGPC_MAX workgroups per CU: the
    // scatter's LDS allows 4; the extract's 12 per CU measured slower)
    const uint32_t hg = (FLOW_WGPC + RS_WGPC_MAX - 1) / RS_WGPC_MAX;
    auto sort_plan = [&]() { return RsPlan{(xpl.nwg + hg - 1) / hg, xpl.chunk * hg}; };
    // the extract writes the by-slot sort's first-digit counts (1e6 flows
    // 6.71 -> 6.61 ms, profiles/r05/check4/ab_fuse0.log)
    auto pass1 = [&](uint64_t p_from) -> int {
        const uint64_t pn = n - p_from;
        const uint8_t *pb = d_bufs + p_from * stride;
        const qk_pkt_meta *pm = d_meta ? d_meta + p_from : nullptr;
        xpl = extract_plan(ctx, pn);
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
                hipMemsetAsync(counters, 0, 5 * 8, s) != hipSuccess ||
                hipMemsetAsync(rs.cnt, 0, (size_t)rsort::R * sort_plan().nwg * 4, s) != hipSuccess)
                return QK_E_HIP;
            const uint32_t probe_limit = C == cmax ? (uint32_t)C - 1 : 64u;   // load <= 1/4 when sized from the hint
            // the by-slot sort's first digit (8-bit variants): its passes and
            // width as rs_sort_k cuts bits(C - 1)
            const int cb = bit_width32((uint32_t)(C - 1)), np = (cb + 7) / 8, dd = (cb + np - 1) / np;
            if (pn)
                hipLaunchKernelGGL(k_flow_extract, dim3(xpl.nwg), dim3(REC_TILE), (size_t)REC_TILE * stride + 32, s,
                                   pb, pn, (uint32_t)stride, pm, my_key, xpl.chunk, tab, (uint32_t)(C - 1), probe_limit,
                                   slots, ids, counters, (1u << dd) - 1, rs.cnt, hg);
            // the counters into pinned memory (an async copy to pageable memory
            // would hold the host until the extract ends); flow_ev[0]: the
            // table is complete (the key-ranking branch waits for it)
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(ctx->h_flow, counters, 40, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipEventRecord(ctx->flow_ev[2], s) != hipSuccess || hipEventRecord(ctx->flow_ev[0], s) != hipSuccess)
                return QK_E_HIP;
            if (hipEventSynchronize(ctx->flow_ev[2]) != hipSuccess) return QK_E_HIP;
            std::copy(ctx->h_flow, ctx->h_flow + 5, hc);
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
        // per-flow arena 1: the work-item accumulator rows, output records
        // and keys, offsets, and the flow-key sort buffers
        const size_t rec = qk_u32_size(T);
        uint64_t *d_offs = nullptr;
        uint32_t *d_rec = nullptr, *used = nullptr, *sl3 = nullptr, *nsel = nullptr, *rseg = nullptr;
        uint32_t *kA = nullptr, *vA = nullptr, *kB = nullptr, *vB = nullptr, *wcnt = nullptr, *lastid = nullptr;
        SegItem *big = nullptr;
        uint8_t *d_keys = nullptr;
        // histogram grouping: few flows (a table of <= HIST_MAX slots and at
        // most knob flow_hist flows: above a few dozen flows every workgroup
        // scatters into that many runs and the radix sort is faster,
        // profiles/r05/flows_hist/)
        const bool hist = C <= HIST_MAX && nf <= (uint32_t)ctx->knobs.flow_hist;
        const uint32_t hnwg = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)ctx->num_cus * 4,
                                                                                  (n_eff + 4095) / 4096));
        const uint64_t hchunk = ((n_eff + hnwg - 1) / hnwg + 3) & ~(uint64_t)3;   // a multiple of 4 (16-byte reads)
        uint32_t *hcnt = nullptr, *hpre = nullptr, *htot = nullptr, *hspre = nullptr, *hlast = nullptr;
        // the occupied-slot compaction (unb workgroups of uchunk slots) and
        // the flow-key sort's scan scratch (the side stream's own)
        const uint32_t unb = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1024, (C + 4095) / 4096));
        const uint64_t uchunk = ((C + unb - 1) / unb + 255) & ~(uint64_t)255;
        const uint32_t ks_nwg = rs_plan(ctx, nf, RS_WGPC_MAX).nwg;
        RsScratch krs{};
        auto layout1 = [&](Carve &c) {
            if (hist) {
                hcnt = c.take<uint32_t>((size_t)C * hnwg);
                hpre = c.take<uint32_t>((size_t)C * hnwg);
                htot = c.take<uint32_t>(C);
                hspre = c.take<uint32_t>(C);
                hlast = c.take<uint32_t>(C);
                lastid = c.take<uint32_t>(nf);
            }
            // accumulator rows of the work-item flows (< 4096 ids: none of
            // them for t <= 32; every flow for t > 32), row j = list entry j
            acc = c.take<unsigned long long>((size_t)(small_ok(T) ? std::min<uint64_t>(nf, inserted / (SMALL_SEG + 1))
                                                                   : nf) * T);
            d_rec = dev_out ? (uint32_t *)sketches : (uint32_t *)c.take<uint8_t>((size_t)nf * rec);
            d_keys = dev_out ? (uint8_t *)keys : c.take<uint8_t>((size_t)nf * 12);
            d_offs = c.take<uint64_t>((size_t)nf + 1);
            // (key word, slot) arrays of the flow-key sort, taken in this order:
            // each key array followed by its value array holds nf pairs (radix.h)
            kA = c.take<uint32_t>(nf); vA = c.take<uint32_t>(nf); kB = c.take<uint32_t>(nf); vB = c.take<uint32_t>(nf);
            used = c.take<uint32_t>(nf); sl3 = c.take<uint32_t>(nf);
            rseg = c.take<uint32_t>(nf);
            nsel = c.take<uint32_t>(2);   // [0] selected slots, [1] flows needing work items
            big = c.take<SegItem>(nf);
            wcnt = c.take<uint32_t>(unb);
            krs.take(c, ks_nwg, nf);
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
        //   side stream s2: the occupied slots in slot order, then in
        //     ascending AddrKey order (a rank sort in one workgroup for
        //     <= KR_MAX flows, else LSD radix passes over the 96-bit key's
        //     three words), then the key bytes of every output rank and the
        //     segment -> rank map (nf-sized, launch-bound passes);
        //   stream s: one stable radix sort of the packets (key, id), which
        //     groups the ids by flow with packet order kept (last_value = the
        //     flow's last packet).  By slot (no remap: segments come out in
        //     slot order and rseg maps a segment to its output rank) when the
        //     table's log2(C) bits need no more 8-bit passes than the flow
        //     count's; then the sort is enqueued first and overlaps the whole
        //     s2 branch (its ~40 launches would otherwise delay the sort's by
        //     their host launch time).  Otherwise by rank (slot -> rank remap
        //     per packet, bit_width(flows) bits), which waits for s2 first.
        const int fbits = bit_width32(nf), cbits = bit_width32((uint32_t)(C - 1));
        // By rank costs a remap pass over the packets (k_slot_to_rank) and the
        // wait for s2 before the sort, ~one sort pass and more: it is taken
        // when it saves two passes, or leaves one (knob flow_byslot: 0 this
        // rule, 1 by slot, 2 by rank; profiles/r05/flows_byslot/)
        const int sp = (cbits + 7) / 8, rp = (fbits + 7) / 8;
        const bool by_slot = ctx->knobs.flow_byslot == 0 ? !(sp >= rp + 2 || (rp <= 1 && sp > 1))
                                                         : ctx->knobs.flow_byslot == 1;
        const uint32_t ob = (uint32_t)std::min<uint64_t>((inserted + 255) / 256, (uint64_t)ctx->num_cus * 8);
        hipStream_t s2 = s == ctx->copy_stream ? ctx->stream : ctx->copy_stream;
        if (!rc && hipStreamWaitEvent(s2, ctx->flow_ev[0], 0) != hipSuccess)   // (recorded behind the last extract)
            rc = QK_E_HIP;
        auto side = [&]() -> int {
            // the occupied slots in slot order
            hipLaunchKernelGGL(k_used_count, dim3(unb), dim3(256), 0, s2, tab, C, uchunk, wcnt);
            hipLaunchKernelGGL(k_used_write, dim3(unb), dim3(256), 0, s2, tab, C, uchunk, wcnt, used, nsel);
            if (hipGetLastError() != hipSuccess) return QK_E_HIP;
            // ... in AddrKey order: one workgroup's rank sort for few flows,
            // else an LSD radix sort of (key word, slot) pairs over the key's
            // three 32-bit words (the next word gathered through the slots)
            const uint32_t *sorted = sl3;
            if (nf <= KR_MAX) {
                hipLaunchKernelGGL(k_key_rank_small, dim3(1), dim3(1024), 0, s2, tab, used, nf, sl3);
                if (hipGetLastError() != hipSuccess) return QK_E_HIP;
            } else {
                for (int q = 0; q < 3; ++q) {
                    hipLaunchKernelGGL(k_slot_word, dim3(fblocks), dim3(256), 0, s2, tab, q ? vA : used, nf, q, kA,
                                       q ? (uint32_t *)nullptr : vA);
                    if (hipGetLastError() != hipSuccess) return QK_E_HIP;
                    int where = 1;
                    if (int e = rs_sort_k<256, 16, RS_WGPC_MAX>(ctx, kA, vA, kB, vB, nf, 32, krs, s2, where))
                        return e;
                    if (where != 0) return QK_E_HIP;   // four passes: the result is back in (kA, vA)
                }
                sorted = vA;
            }
            if (by_slot || hist) {
                hipLaunchKernelGGL(k_slot_pos, dim3(fblocks), dim3(256), 0, s2, used, nf, rank_of_slot);
                hipLaunchKernelGGL(k_rank_perm, dim3(fblocks), dim3(256), 0, s2, tab, sorted, nf, rank_of_slot, rseg,
                                   d_keys);
            } else {
                hipLaunchKernelGGL(k_slot_rank, dim3(fblocks), dim3(256), 0, s2, tab, sorted, nf, rank_of_slot, d_keys);
            }
            if (hipGetLastError() != hipSuccess || hipEventRecord(ctx->flow_ev[1], s2) != hipSuccess) return QK_E_HIP;
            return QK_OK;
        };
        if (!rc && hist) {
            if (hipMemsetAsync(hcnt, 0, (size_t)C * hnwg * 4, s) != hipSuccess ||
                hipMemsetAsync(hlast, 0, (size_t)C * 4, s) != hipSuccess)
                rc = QK_E_HIP;
            if (!rc) {
                hipLaunchKernelGGL(k_hist_count, dim3(hnwg), dim3(256), (size_t)C * 8, s, slots, n_eff, hchunk, (uint32_t)C,
                                   hnwg, hcnt, hlast);
                // slot-major counts -> each slot's workgroup prefixes, then the slots' prefix
                hipLaunchKernelGGL(rsort::k_row_scan<256>, dim3((uint32_t)C), dim3(256), 0, s, hcnt, hnwg, hpre, htot);
                hipLaunchKernelGGL(rsort::k_tot_scan<1024>, dim3(1), dim3(1024), 0, s, htot, (uint32_t)C, hspre);
                hipLaunchKernelGGL(k_hist_scatter, dim3(hnwg), dim3(256), (size_t)C * 4, s, slots, ids, n_eff, hchunk,
                                   (uint32_t)C, hnwg, hpre, hspre, id_s);
                if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
            }
            if (!rc) rc = side();
            if (!rc && hipStreamWaitEvent(s, ctx->flow_ev[1], 0) != hipSuccess) rc = QK_E_HIP;
            if (!rc) {
                hipLaunchKernelGGL(k_hist_offsets, dim3(fblocks), dim3(256), 0, s, used, nf, hspre, inserted, d_offs);
                hipLaunchKernelGGL(k_hist_last, dim3(fblocks), dim3(256), 0, s, used, nf, hlast, ids, lastid);
                if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
            }
        } else if (!rc && by_slot) {
            // the grouping sort (radix.h); with the extract's fused histogram
            // its first pass reads no keys and every pass keeps the extract's
            // chunking
            int where = 0;
            const RsPlan spl = sort_plan();
            rc = rs_sort(ctx, slots, ids, key_s, id_s, n_eff, cbits, rs, s, where, &spl, true);
            if (!rc && where == 0) {   // even number of passes: the result is in (slots, ids)
                std::swap(slots, key_s);
                std::swap(ids, id_s);
            }
            if (!rc) rc = side();
            if (!rc && hipStreamWaitEvent(s, ctx->flow_ev[1], 0) != hipSuccess) rc = QK_E_HIP;
            if (!rc) {
                hipLaunchKernelGGL(k_slot_offsets, dim3(std::max(ob, 1u)), dim3(256), 0, s, key_s, inserted,
                                   rank_of_slot, nf, d_offs);
                if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
            }
        } else if (!rc) {
            rc = side();
            if (!rc && hipStreamWaitEvent(s, ctx->flow_ev[1], 0) != hipSuccess) rc = QK_E_HIP;
            if (!rc) hipLaunchKernelGGL(k_slot_to_rank, dim3(gb), dim3(256), 0, s, slots, rank_of_slot, n_eff, nf);
            if (!rc && hipGetLastError() != hipSuccess) rc = QK_E_HIP;
            if (!rc) {
                int where = 0;
                rc = rs_sort(ctx, slots, ids, key_s, id_s, n_eff, fbits, rs, s, where);
                if (!rc && where == 0) {
                    std::swap(slots, key_s);
                    std::swap(ids, id_s);
                }
            }
            if (!rc) {
                hipLaunchKernelGGL(k_rank_offsets, dim3(std::max(ob, 1u)), dim3(256), 0, s, key_s, inserted, nf,
                                   d_offs);
                if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
            }
        }
        // by slot / histogram: segment g is output rank rseg[g]; by rank: g
        const uint32_t *seg_rank = by_slot || hist ? rseg : nullptr;
        // the small flows' records straight from k_seg_small, the work-item
        // flows' through their accumulator rows and k_flow_finalize_big
        SmallOut so;
        so.rec = d_rec;
        so.rseg = seg_rank;
        so.lastid = hist ? lastid : nullptr;
        // k_seg_small needs no host decision: it goes first, and the host's
        // wait for the work-item list below overlaps it
        const bool small_first = small_ok(T) && nf;
        if (!rc && small_first) {
            hipEvent_t e0 = prof_begin(ctx, s);
            rc = seg_small_launch(T, id_s, d_offs, nf, acc, so, s);
            prof_end(ctx, s, e0);
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
        if (!rc)
            rc = seg_encode(ctx, id_s, d_offs, seg_items_from_big(bigs), nf, T, acc, hsel[1], so, s, small_first);
        if (!rc && hsel[1]) {
            const uint32_t fb = (uint32_t)std::min<uint64_t>(((uint64_t)hsel[1] * (4 + T) + 255) / 256,
                                                             (uint64_t)ctx->num_cus * 16);
            hipLaunchKernelGGL(k_flow_finalize_big, dim3(fb), dim3(256), 0, s, acc, big, (uint64_t)hsel[1], seg_rank,
                               so.lastid, id_s, T, d_rec);
            if (hipGetLastError() != hipSuccess) rc = QK_E_HIP;
        }
        if (!rc && !dev_out &&
            (hipMemcpyAsync(sketches, d_rec, (size_t)nf * rec, hipMemcpyDeviceToHost, s) != hipSuccess ||
             hipMemcpyAsync(keys, d_keys, (size_t)nf * 12, hipMemcpyDeviceToHost, s) != hipSuccess))
            rc = QK_E_HIP;
    }
    (void)hipStreamSynchronize(s); // the arenas are reused by the next call
    (void)hipStreamSynchronize(s == ctx->copy_stream ? ctx->stream : ctx->copy_stream);   // the flow-key branch
    if (stats) *stats = st;
    return rc;
}
