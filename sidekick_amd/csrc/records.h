// records.h — internal: staging fixed-stride packet records into LDS and the
// per-packet filters of the reference sniff loops (sidekick.rs:76-103,
// sidekick_multi.rs:101-143, buffer.rs:6-7,80-106).  Shared by packets.hip
// (single quACK) and flows.hip (one quACK per AddrKey).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "quack_hip.h"

namespace qk {

constexpr int REC_TILE = 256;      // records per LDS tile (one per thread)
constexpr uint32_t REC_UDP = 17;   // IPPROTO_UDP

// A 16-byte load of the record stream, nontemporal when NT (the stream is
// read once: kept out of the way of data that is reused, e.g. a flow table)
template <bool NT>
__device__ __forceinline__ uint4 rec_ld16(const uint8_t *p) {
    if constexpr (NT) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
        return make_uint4(x.x, x.y, x.z, x.w);
    } else {
        return *reinterpret_cast<const uint4 *>(p);
    }
}

// Copy records [p0, p0+np) of `bufs` (stride bytes each, n records in all)
// into `tile` with 16-byte loads aligned on the absolute address; returns the
// byte offset of record p0 inside `tile`.  Bytes outside [0, n*stride) are
// never read.  Caller brackets with __syncthreads().
template <bool NT = false>
__device__ __forceinline__ uint32_t stage_records(const uint8_t *__restrict__ bufs, uint64_t n, uint32_t stride,
                                                  uint64_t p0, uint64_t np, uint8_t *tile) {
    const uintptr_t base = (uintptr_t)bufs;
    const uint64_t total = n * (uint64_t)stride;
    const uint64_t b_lo = p0 * stride, b_hi = (p0 + np) * stride;
    const uint64_t a_lo = ((base + b_lo) & ~(uintptr_t)15) - base;  // may wrap below 0 (mod 2^64)
    const uint64_t a_hi = ((base + b_hi + 15) & ~(uintptr_t)15) - base;
    const uint32_t nvec = (uint32_t)((a_hi - a_lo) / 16);
    // STAGE_V loads in flight per lane before any LDS write (a load -> wait ->
    // write loop would pay one HBM round trip per 16 bytes); 5 covers a
    // 256 x 67 B tile in one round
    // (loads are unconditional, from an aligned in-range fallback address when
    // a vector is partial or past the tile, so none waits inside a branch;
    // total >= 67 bytes, so the first aligned vector is in range)
    constexpr int STAGE_V = 5;
    const uint64_t safe = ((base + 15) & ~(uintptr_t)15) - base;
    for (uint32_t v0 = 0; v0 < nvec; v0 += STAGE_V * blockDim.x) {
        uint4 r[STAGE_V];
        bool ok[STAGE_V];
#pragma unroll
        for (int k = 0; k < STAGE_V; ++k) {
            const uint32_t v = v0 + k * blockDim.x + threadIdx.x;
            const uint64_t off = a_lo + 16ull * v; // relative to bufs, mod 2^64
            ok[k] = v < nvec && off < total && off + 16 <= total;
            r[k] = rec_ld16<NT>(bufs + (ok[k] ? off : safe));
        }
        // pin the loads here (otherwise each is sunk into its store's branch
        // and waited for alone)
#pragma unroll
        for (int k = 0; k < STAGE_V; ++k) asm volatile("" : "+v"(r[k].x), "+v"(r[k].y), "+v"(r[k].z), "+v"(r[k].w));
#pragma unroll
        for (int k = 0; k < STAGE_V; ++k) {
            const uint32_t v = v0 + k * blockDim.x + threadIdx.x;
            if (v >= nvec) continue;
            if (ok[k]) {
                *reinterpret_cast<uint4 *>(tile + 16 * v) = r[k];
            } else {
                const uint64_t off = a_lo + 16ull * v;
#pragma unroll
                for (int b = 0; b < 16; ++b) {
                    const uint64_t o = off + b; // a wrapped head offset comes back into range exactly
                    tile[16 * v + b] = o < total ? bufs[o] : 0;
                }
            }
        }
    }
    return (uint32_t)(b_lo - a_lo);
}

// Software-pipelined form for tiles of at most STAGE_V 16-byte vectors per
// lane (stride <= 79 at 256 records): stage_issue() starts a tile's loads into
// registers, stage_commit() writes them to LDS.  A kernel issues tile k+1
// right after committing tile k and classifies tile k meanwhile, so each
// tile's HBM latency hides behind the previous tile's work.
constexpr int STAGE_VEC = 5;
struct TileStage {
    uint4 r[STAGE_VEC];
    uint32_t ok;     // bit k: vector k is fully in range (else the byte path)
    uint32_t nvec;
    uint64_t a_lo;
    uint32_t r0;
};

__device__ __forceinline__ bool stage_pipelined(uint32_t stride, uint32_t threads) {
    return ((uint64_t)REC_TILE * stride + 15) / 16 + 1 <= (uint64_t)STAGE_VEC * threads;
}

template <bool NT = false>
__device__ __forceinline__ void stage_issue(const uint8_t *__restrict__ bufs, uint64_t n, uint32_t stride,
                                            uint64_t p0, uint64_t np, TileStage &st) {
    const uintptr_t base = (uintptr_t)bufs;
    const uint64_t total = n * (uint64_t)stride;
    const uint64_t b_lo = p0 * stride, b_hi = (p0 + np) * stride;
    st.a_lo = ((base + b_lo) & ~(uintptr_t)15) - base;
    const uint64_t a_hi = ((base + b_hi + 15) & ~(uintptr_t)15) - base;
    st.nvec = (uint32_t)((a_hi - st.a_lo) / 16);
    st.r0 = (uint32_t)(b_lo - st.a_lo);
    const uint64_t safe = ((base + 15) & ~(uintptr_t)15) - base;   // in range: total >= 67
    st.ok = 0;
#pragma unroll
    for (int k = 0; k < STAGE_VEC; ++k) {
        const uint32_t v = k * blockDim.x + threadIdx.x;
        const uint64_t off = st.a_lo + 16ull * v;
        const bool ok = v < st.nvec && off < total && off + 16 <= total;
        st.ok |= (uint32_t)ok << k;
        st.r[k] = rec_ld16<NT>(bufs + (ok ? off : safe));
    }
}

__device__ __forceinline__ uint32_t stage_commit(const uint8_t *__restrict__ bufs, uint64_t n, uint32_t stride,
                                                 TileStage &st, uint8_t *tile) {
    const uint64_t total = n * (uint64_t)stride;
#pragma unroll
    for (int k = 0; k < STAGE_VEC; ++k)   // the loads complete here, not inside a branch below
        asm volatile("" : "+v"(st.r[k].x), "+v"(st.r[k].y), "+v"(st.r[k].z), "+v"(st.r[k].w));
#pragma unroll
    for (int k = 0; k < STAGE_VEC; ++k) {
        const uint32_t v = k * blockDim.x + threadIdx.x;
        if (v >= st.nvec) continue;
        if ((st.ok >> k) & 1) {
            *reinterpret_cast<uint4 *>(tile + 16 * v) = st.r[k];
        } else {
            const uint64_t off = st.a_lo + 16ull * v;
#pragma unroll
            for (int b = 0; b < 16; ++b) {
                const uint64_t o = off + b;
                tile[16 * v + b] = o < total ? bufs[o] : 0;
            }
        }
    }
    return st.r0;
}

template <bool NT = false>
__device__ __forceinline__ qk_pkt_meta record_meta(const qk_pkt_meta *__restrict__ meta, uint64_t i) {
    static_assert(sizeof(qk_pkt_meta) == 8, "qk_pkt_meta is one 8-byte word");
    qk_pkt_meta m;
    if (meta) {
        if constexpr (NT) {   // read once, like the records (rec_ld16)
            const uint64_t v = __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(meta) + i);
            __builtin_memcpy(&m, &v, 8);
        } else {
            m = meta[i];
        }
    } else {
        m.pkttype = 0;          // PACKET_HOST
        m.reserved = 0;
        m.protocol_be = 0x0008; // htons(ETH_P_IP) as stored
        m.len = QK_BUFFER_SIZE;
    }
    return m;
}

// Direction::Incoming && sll_protocol == ETH_P_IP && buf[23] == IPPROTO_UDP
__device__ __forceinline__ bool record_is_incoming_udp(const qk_pkt_meta &m, const uint8_t *rec) {
    const bool incoming = m.pkttype == 0 || m.pkttype == 3; // PACKET_HOST | PACKET_OTHERHOST
    return incoming && m.protocol_be == 0x0008 && rec[23] == REC_UDP;
}

// big-endian u32 at QK_ID_OFFSET (UdpParser::parse_identifier)
__device__ __forceinline__ uint32_t record_identifier(const uint8_t *rec) {
    return ((uint32_t)rec[QK_ID_OFFSET] << 24) | ((uint32_t)rec[QK_ID_OFFSET + 1] << 16) |
           ((uint32_t)rec[QK_ID_OFFSET + 2] << 8) | (uint32_t)rec[QK_ID_OFFSET + 3];
}

} // namespace qk
