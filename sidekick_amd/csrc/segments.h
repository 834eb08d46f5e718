// segments.h — internal: the segmented encode shared by the per-flow batch
// (flows.hip) and the CSR primitive qk_u32_encode_segments_device
// (segments.hip): flows of <= SMALL_SEG ids one per lane (k_seg_small), the
// others cut into work items of <= SEG_CHUNK ids, one workgroup each
// (k_seg_bsgs / k_seg_encode).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "ctx.h"

namespace qk {

constexpr uint32_t SEG_CHUNK = 1u << 16;   // ids per work item
// A flow of <= SMALL_SEG ids is encoded by ONE lane (k_seg_small).
constexpr uint64_t SMALL_SEG = 4096;

struct SegItem {
    uint32_t seg;
    uint32_t pad;
    uint64_t lo, hi; // [lo, hi) in the grouped id array
};

// per-lane (VALU) wrap counters: SG = 0; no s_setprio
// where k_seg_small writes (SmallOut: acc rows, or records by rank)
struct SmallOut {
    uint32_t *rec = nullptr;
    const uint32_t *rseg = nullptr, *lastid = nullptr;
};

// work items of the flows k_seg_small does not take: every flow when T > 32,
// else the flows of more than SMALL_SEG ids
inline bool small_ok(uint32_t T) { return T <= 32; }

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

// the small flows' lane-per-flow kernel for threshold T (segments.hip)
int seg_small_launch(uint32_t T, const uint32_t *ids, const uint64_t *d_offs, uint32_t nseg, unsigned long long *acc,
                     const SmallOut &so, hipStream_t s);
// the work items of the listed big flows (flow j of the list accumulates into row j)
std::vector<SegItem> seg_items_from_big(const std::vector<SegItem> &big);
// Segmented encode of a grouped id array (segments.hip; see there)
int seg_encode(qk_ctx *ctx, const uint32_t *d_ids, const uint64_t *d_offs, const std::vector<SegItem> &items,
               size_t nseg, uint32_t T, unsigned long long *d_acc, size_t acc_rows, const SmallOut &so, hipStream_t s,
               bool small_done = false);

} // namespace qk
