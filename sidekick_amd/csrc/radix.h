// radix.h — the per-flow batch's grouping sort (flows.hip):
// a stable LSD radix sort of (u32 key, u32 value) pairs over the low `bits`
// bits of the key, 8-bit digits, one chunked counting scatter per digit.
//
// It replaces sidekick_multi.rs:65-90's per-packet HashMap update for a batch
// of 1e8 packets: grouping the ids by flow slot, packet order kept inside a
// flow (the last id of a flow is its last_value, sidekick_multi.rs:82 inserts
// in packet order).
//
// Per digit (pass), with the packets cut into nwg contiguous chunks, one per
// workgroup (no decoupled look-back: a chunk's place in every digit's run is
// known before its scatter starts):
//   k_rs_count    chunk w's digit histogram in LDS -> cnt[d * nwg + w]
//   (scan)        exclusive sum of cnt in that digit-major order -> base: the
//                 output position of chunk w's first item of digit d
//   k_rs_scatter  chunk w in sub-tiles of 256 x K items, in order.  Each wave
//                 takes 64 K consecutive items in K rounds of 64; a round ranks
//                 its lanes among the lanes of the same digit by ballots on the
//                 digit's bits (stable: lower lanes first) on top of the
//                 wave's running per-digit count in LDS.  Then per digit: the
//                 waves' exclusive prefix, the sub-tile's digit runs (block
//                 scan), and every item is staged in LDS at its place in the
//                 digit-sorted sub-tile; the staged items go out in order, so
//                 consecutive lanes write consecutive positions of one digit's
//                 run (~16 items per run at 8-bit digits and 4096-item
//                 sub-tiles: coalesced, where a direct scatter would write 64
//                 lines per wave store).
// Traffic per pass: 4 B read (count; 8 B from a pair array) + 8 B read + 8 B
// written (scatter).  The passes between the first and the last keep the
// items as (key, value) pairs in one array.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace qk {
namespace rsort {

constexpr int DBITS = 8;                  // the digit width
constexpr uint32_t R = 1u << DBITS;

// The first pass's chunk histograms from the key array (the later passes
// count from the digit bytes, k_rs_count8; the per-flow batch's by-slot sort
// has its first pass counted by k_flow_extract).  chunk is a multiple of 4
// and keys is 16-byte aligned (arena buffers).
__global__ __launch_bounds__(256) void k_rs_count(const uint32_t *__restrict__ keys, uint64_t n, uint64_t chunk,
                                                  uint32_t shift, uint32_t mask, uint32_t nwg,
                                                  uint32_t *__restrict__ cnt) {
    __shared__ uint32_t h[R];
    for (uint32_t j = threadIdx.x; j < R; j += blockDim.x) h[j] = 0;
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
    const uint64_t v1 = c0 < c1 ? c0 + ((c1 - c0) & ~(uint64_t)3) : c0;
    for (uint64_t i = c0 + 4 * threadIdx.x; i < v1; i += 4 * blockDim.x) {
        const uint4 k = *reinterpret_cast<const uint4 *>(keys + i);
        atomicAdd(&h[(k.x >> shift) & mask], 1u);
        atomicAdd(&h[(k.y >> shift) & mask], 1u);
        atomicAdd(&h[(k.z >> shift) & mask], 1u);
        atomicAdd(&h[(k.w >> shift) & mask], 1u);
    }
    for (uint64_t i = v1 + threadIdx.x; i < c1; i += blockDim.x) atomicAdd(&h[(keys[i] >> shift) & mask], 1u);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < R; j += blockDim.x) cnt[(size_t)j * nwg + blockIdx.x] = h[j];
}

// the same histogram from a byte per item: the digit the previous pass's
// scatter wrote beside each item (k_rs_scatter nd_out), 16 per load — the
// pass reads 1 byte per item instead of the 8 of a (key, value) pair
__global__ __launch_bounds__(256) void k_rs_count8(const uint8_t *__restrict__ dig, uint64_t n, uint64_t chunk,
                                                   uint32_t nwg, uint32_t *__restrict__ cnt) {
    __shared__ uint32_t h[R];
    for (uint32_t j = threadIdx.x; j < R; j += blockDim.x) h[j] = 0;
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
    // chunk is a multiple of 16 here (rs_sort_k), dig 16-byte aligned
    const uint64_t v1 = c0 < c1 ? c0 + ((c1 - c0) & ~(uint64_t)15) : c0;
    for (uint64_t i = c0 + 16 * threadIdx.x; i < v1; i += 16 * blockDim.x) {
        const uint4 w = *reinterpret_cast<const uint4 *>(dig + i);
        const uint32_t q[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int b = 0; b < 4; ++b) atomicAdd(&h[(q[k] >> (8 * b)) & 0xFFu], 1u);
    }
    for (uint64_t i = v1 + threadIdx.x; i < c1; i += blockDim.x) atomicAdd(&h[dig[i]], 1u);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < R; j += blockDim.x) cnt[(size_t)j * nwg + blockIdx.x] = h[j];
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// exclusive scan over the block (NW waves) of one value per thread; returns
// the prefix, *total = the block's sum.  Uses ws[NW].
template <int NW>
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t *ws, uint32_t *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) ws[wave] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint32_t s = ws[w];
        if (w < wave) before += s;
        all += s;
    }
    *total = all;
    return before + x - v;
}

// Exclusive scan of a row-major rows x cols array of counts (the radix
// pass's digit-major cnt[d * nwg + w]; the few-flow histogram's
// hist[slot * nwg + w]) in two levels: k_row_scan (workgroup r) scans row r
// into pre[r * cols + c], the prefix within the row, and writes the row's
// total; the prefix of the row totals comes from k_tot_scan (one workgroup)
// or, for the radix pass's 2^D digits, from the scatter kernel itself.  The
// full exclusive prefix of (r, c) is rpre[r] + pre[r * cols + c].  (A
// last-workgroup ticket instead of the second step serialised 4096
// workgroups on one atomic: 0.19 ms for the histogram's 4096 x 1024.)
template <int BLK>
__device__ __forceinline__ uint32_t block_scan_run(const uint32_t *__restrict__ src, uint32_t len,
                                                   uint32_t *__restrict__ dst, uint32_t *ws) {
    constexpr int NW = BLK / 64;
    // thread t takes the ipt consecutive entries [t ipt, (t + 1) ipt); four
    // per thread (a row of 4 BLK): one 16-byte load and store
    uint32_t all;
    if (len == 4u * BLK && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0) {
        const uint4 v = reinterpret_cast<const uint4 *>(src)[threadIdx.x];
        const uint32_t run = block_excl<NW>(v.x + v.y + v.z + v.w, ws, &all);
        reinterpret_cast<uint4 *>(dst)[threadIdx.x] = make_uint4(run, run + v.x, run + v.x + v.y, run + v.x + v.y + v.z);
        return all;
    }
    const uint32_t ipt = (len + BLK - 1) / BLK;
    const uint32_t b = threadIdx.x * ipt, e = b + ipt < len ? b + ipt : len;
    uint32_t s = 0;
    for (uint32_t i = b; i < e; ++i) s += src[i];
    uint32_t run = block_excl<NW>(s, ws, &all);
    for (uint32_t i = b; i < e; ++i) {
        const uint32_t v = src[i];
        dst[i] = run;
        run += v;
    }
    return all;
}

template <int BLK>
__global__ __launch_bounds__(BLK) void k_row_scan(const uint32_t *__restrict__ cnt, uint32_t cols,
                                                  uint32_t *__restrict__ pre, uint32_t *__restrict__ tot) {
    __shared__ uint32_t ws[BLK / 64];
    const uint32_t r = blockIdx.x;
    const uint32_t all = block_scan_run<BLK>(cnt + (size_t)r * cols, cols, pre + (size_t)r * cols, ws);
    if (threadIdx.x == 0) tot[r] = all;
}

// rpre = exclusive prefix of tot[0 .. rows), one workgroup
template <int BLK>
__global__ __launch_bounds__(BLK) void k_tot_scan(const uint32_t *__restrict__ tot, uint32_t rows,
                                                  uint32_t *__restrict__ rpre) {
    __shared__ uint32_t ws[BLK / 64];
    (void)block_scan_run<BLK>(tot, rows, rpre, ws);
}

// D: digit bits; BLK threads; K items per thread and sub-tile.  IP / OP:
// input / output as one array of (key, value) pairs (keys / keys_out then
// point at it; vals / vals_out are unused) instead of two arrays — the passes
// between the first and the last: one 8-byte store per item.  The input is
// read nontemporal (read once; the scattered output runs keep L2 for write
// combining: 1e6 flows 6.16 -> 6.02 ms, nontemporal stores +15 %,
// profiles/r05/flows_nt/ab_rsnt.jsonl).  (Round 4-5 variants measured and
// removed: a direct scatter without LDS staging, 11-bit digits with 512 /
// 1024 threads, two arrays throughout, 8 and 24 items per thread; DESIGN
// §3.6.)  nd_out != null: also the item's next digit ((key >> nshift) &
// nmask, < 256) as a byte at its output position, for the next pass's
// k_rs_count8.
template <int D, int BLK, int K, bool IP, bool OP>
__global__ __launch_bounds__(BLK) void k_rs_scatter(const uint32_t *__restrict__ keys,
                                                    const uint32_t *__restrict__ vals, uint64_t n, uint64_t chunk,
                                                    uint32_t shift, uint32_t mask, uint32_t nwg,
                                                    const uint32_t *__restrict__ base,
                                                    const uint32_t *__restrict__ dtot,
                                                    uint32_t *__restrict__ keys_out, uint32_t *__restrict__ vals_out,
                                                    uint8_t *__restrict__ nd_out, uint32_t nshift, uint32_t nmask) {
    constexpr uint32_t RD = 1u << D, TILE = BLK * K;
    constexpr int NW = BLK / 64;
    constexpr int DPT = RD >= (uint32_t)BLK ? RD / BLK : 1;   // digits per thread in the per-digit steps
    constexpr uint32_t NOD = 0xFFFFFFFFu;                      // an item past the chunk
    static_assert(RD % BLK == 0 || BLK % RD == 0, "digits over threads");
    // counts and staged places stay below TILE <= 2^16: 16-bit when the
    // 32-bit table would not fit beside the staging area
    using WT = std::conditional_t<(NW * RD * 4 > 65536), uint16_t, uint32_t>;
    static_assert(TILE <= 65536 || sizeof(WT) == 4, "16-bit wave counters");
    __shared__ WT wc[NW][RD];         // per wave: running digit counts, then the staged place of its first item
    __shared__ uint32_t dl[RD];       // output position of the sub-tile's run start of the digit, minus its
                                      // staged start (dst = dl[d] + staged index)
    __shared__ uint32_t ws[NW];
    __shared__ uint2 stage[TILE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk, c1 = c0 + chunk < n ? c0 + chunk : n;
    // this thread's digits: tid * DPT .. + DPT (when RD < BLK: digit tid, threads past RD idle)
    const bool dth = DPT > 1 || (uint32_t)tid < RD;
    uint32_t gp[DPT];   // output position of the chunk's next item of each of this thread's digits
    // the digits' prefix from their totals (k_row_scan): block scan of this
    // thread's digits' sum, then a running add
    uint32_t dsum = 0;
#pragma unroll
    for (int j = 0; j < DPT; ++j) dsum += dth ? dtot[(uint32_t)tid * DPT + j] : 0u;
    uint32_t dall;
    uint32_t drun = block_excl<NW>(dsum, ws, &dall);
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
        const uint32_t d = (uint32_t)tid * DPT + j;
        gp[j] = dth ? base[(size_t)d * nwg + blockIdx.x] + drun : 0u;   // the two levels of the scan
        drun += dth ? dtot[d] : 0u;
        if (dth)
#pragma unroll
            for (int w = 0; w < NW; ++w) wc[w][d] = 0;
    }
    __syncthreads();
    for (uint64_t sub = c0; sub < c1; sub += TILE) {
        uint32_t dg[K], pw[K];
        uint2 it[K];
        const uint64_t wbase = sub + (uint64_t)wave * 64 * K;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t p = wbase + (uint64_t)k * 64 + lane;
            if constexpr (IP) {
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 x = p < c1 ? __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(keys) + p)
                                       : u32x2{0u, 0u};
                it[k] = make_uint2(x.x, x.y);
            } else {
                it[k] = p < c1 ? make_uint2(__builtin_nontemporal_load(keys + p), __builtin_nontemporal_load(vals + p))
                               : make_uint2(0u, 0u);
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t p = wbase + (uint64_t)k * 64 + lane;
            const bool valid = p < c1;
            const uint32_t d = (it[k].x >> shift) & mask;
            uint64_t m = __ballot(valid);
#pragma unroll
            for (int b = 0; b < D; ++b) {
                const uint64_t bb = __ballot(valid && ((d >> b) & 1u));
                m &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t below = lanes_below(m);
            const uint32_t before = wc[wave][d];
            pw[k] = before + below;
            if (valid && below == 0) wc[wave][d] = (WT)(before + (uint32_t)__popcll(m));
            dg[k] = valid ? d : NOD;
        }
        __syncthreads();
        // per digit: its count in every wave (registers), the digit's total,
        // the sub-tile's runs (block scan over the digits in order), then
        // wc[w][d] = the staged place of wave w's first item of digit d
        uint32_t cw[DPT][NW], tot[DPT], tsum = 0;
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const uint32_t d = (uint32_t)tid * DPT + j;
            uint32_t a = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                cw[j][w] = dth ? wc[w][d] : 0u;
                a += cw[j][w];
            }
            tot[j] = a;
            tsum += a;
        }
        uint32_t nsub;
        uint32_t ls = block_excl<NW>(tsum, ws, &nsub);   // staged start of this thread's first digit
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const uint32_t d = (uint32_t)tid * DPT + j;
            if (dth) {
                dl[d] = gp[j] - ls;
                uint32_t a = ls;
#pragma unroll
                for (int w = 0; w < NW; ++w) {
                    wc[w][d] = (WT)a;
                    a += cw[j][w];
                }
            }
            ls += tot[j];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (dg[k] != NOD) stage[wc[wave][dg[k]] + pw[k]] = it[k];
        __syncthreads();
        // out in staged order: consecutive lanes write consecutive positions
        // of a digit's run
        for (uint32_t i = tid; i < nsub; i += BLK) {
            const uint2 v = stage[i];
            const uint32_t dst = dl[(v.x >> shift) & mask] + i;
            if constexpr (OP) {
                reinterpret_cast<uint2 *>(keys_out)[dst] = v;
            } else {
                keys_out[dst] = v.x;
                vals_out[dst] = v.y;
            }
            if (nd_out) nd_out[dst] = (uint8_t)((v.x >> nshift) & nmask);
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const uint32_t d = (uint32_t)tid * DPT + j;
            gp[j] += tot[j];
            if (dth)
#pragma unroll
                for (int w = 0; w < NW; ++w) wc[w][d] = 0;
        }
        __syncthreads();
    }
}

} // namespace rsort
} // namespace qk
