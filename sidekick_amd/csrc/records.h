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

// Copy records [p0, p0+np) of `bufs` (stride bytes each, n records in all)
// into `tile` with 16-byte loads aligned on the absolute address; returns the
// byte offset of record p0 inside `tile`.  Bytes outside [0, n*stride) are
// never read.  Caller brackets with __syncthreads().
__device__ __forceinline__ uint32_t stage_records(const uint8_t *__restrict__ bufs, uint64_t n, uint32_t stride,
                                                  uint64_t p0, uint64_t np, uint8_t *tile) {
    const uintptr_t base = (uintptr_t)bufs;
    const uint64_t total = n * (uint64_t)stride;
    const uint64_t b_lo = p0 * stride, b_hi = (p0 + np) * stride;
    const uint64_t a_lo = ((base + b_lo) & ~(uintptr_t)15) - base;  // may wrap below 0 (mod 2^64)
    const uint64_t a_hi = ((base + b_hi + 15) & ~(uintptr_t)15) - base;
    const uint32_t nvec = (uint32_t)((a_hi - a_lo) / 16);
    for (uint32_t v = threadIdx.x; v < nvec; v += blockDim.x) {
        const uint64_t off = a_lo + 16ull * v; // relative to bufs, mod 2^64
        if (off < total && off + 16 <= total) {
            *reinterpret_cast<uint4 *>(tile + 16 * v) = *reinterpret_cast<const uint4 *>(bufs + off);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint64_t o = off + k; // a wrapped head offset comes back into range exactly
                tile[16 * v + k] = o < total ? bufs[o] : 0;
            }
        }
    }
    return (uint32_t)(b_lo - a_lo);
}

__device__ __forceinline__ qk_pkt_meta record_meta(const qk_pkt_meta *__restrict__ meta, uint64_t i) {
    qk_pkt_meta m;
    if (meta) m = meta[i];
    else {
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
