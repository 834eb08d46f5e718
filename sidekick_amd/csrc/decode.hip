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
#include "bsgs64.h"
#include "ctx.h"
#include "field.h"

namespace qk {

constexpr int RT_BLOCK = 256;

__device__ __forceinline__ void rt_record(uint64_t pos, bool hit, bool stop, uint64_t *hits, uint64_t cap,
                                          uint64_t *counters) {
    if (hit) {
        const uint64_t slot = atomicAdd((unsigned long long *)&counters[0], 1ull);
        if (slot < cap) hits[slot] = pos;
    }
    if (stop) atomicMin((unsigned long long *)&counters[1], (unsigned long long)pos);
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
    hipLaunchKernelGGL(k_root_test_u64, dim3(rt_grid(ctx, k_root_test_u64, units)), dim3(RT_BLOCK), 0, s, log,
                       (uint64_t)n, head, d_c, d, use_stop, stop_value, hits, cap, counters);
    prof_end(ctx, s, e0);
    QK_HIP_TRY(hipGetLastError());
    return QK_OK;
}

} // namespace qk
