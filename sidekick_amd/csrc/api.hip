// api.hip — device half of the quACK C ABI: context, scratch management,
// profiling events, batch encode entry points (device- and host-resident
// ids), the decode root test, and the synthetic id generators.
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

#include "ctx.h"
#include "field.h"

using namespace qk;

// teardown paths ignore the status of hipFree/hipEventDestroy/... by design
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"

namespace qk {

QK_WARM_KERNEL(api)

// NULL is the HIP null (legacy default) stream, as in every HIP API: work
// enqueued there is ordered with the caller's default-stream work (torch's
// default stream has handle 0).
hipStream_t pick_stream(qk_ctx *ctx, void *stream) {
    (void)ctx;
    return (hipStream_t)stream;
}

int scratch_acquire(qk_ctx *ctx, hipStream_t s) {
    if (ctx->scratch_ev_valid) QK_HIP_TRY(hipStreamWaitEvent(s, ctx->scratch_ev, 0));
    return QK_OK;
}

int scratch_release(qk_ctx *ctx, hipStream_t s) {
    QK_HIP_TRY(hipEventRecord(ctx->scratch_ev, s));
    ctx->scratch_ev_valid = true;
    return QK_OK;
}

// Grow-only device buffers.  hipFree performs an implicit
// hipDeviceSynchronize, which would stall every stream of the device (the
// caller's unrelated work included) whenever a buffer grows, so a grown-out
// buffer is retired instead: it stays allocated until qk_ctx_trim or
// qk_ctx_destroy.  Growth is geometric (at least 2x), so the retired
// buffers together stay smaller than the live one.  A retired buffer may
// still be read by queued work (the encode scratch is handed between
// streams by ctx->scratch_ev; the flow arenas and the hit buffer are used
// only inside synchronous calls): nothing waits for that here.
static int regrow(qk_ctx *ctx, void **buf, size_t *have, size_t sz) {
    if (*buf) {
        ctx->retired.push_back(*buf);
        sz = std::max(sz, 2 * *have);
        *buf = nullptr;
        *have = 0;
    }
    if (hipMalloc(buf, sz) != hipSuccess) {
        (void)hipGetLastError();
        *buf = nullptr;
        return QK_E_NOMEM;
    }
    *have = sz;
    return QK_OK;
}

int ensure_scratch(qk_ctx *ctx, size_t bytes, hipStream_t s) {
    (void)s;
    if (bytes <= ctx->scratch_bytes) return QK_OK;
    return regrow(ctx, &ctx->d_scratch, &ctx->scratch_bytes, std::max(bytes, (size_t)1 << 20));
}

int ensure_flow(qk_ctx *ctx, int which, size_t bytes, hipStream_t s) {
    (void)s;
    if (bytes <= ctx->flow_bytes[which]) return QK_OK;
    // headroom for growing batches
    return regrow(ctx, &ctx->d_flow[which], &ctx->flow_bytes[which], std::max(bytes + bytes / 8, (size_t)1 << 20));
}

int ensure_hits(qk_ctx *ctx, size_t cap, hipStream_t s) {
    (void)s;
    if (cap <= ctx->hits_cap) return QK_OK;
    size_t bytes = ctx->hits_cap * sizeof(uint64_t);
    const int rc = regrow(ctx, (void **)&ctx->d_hits, &bytes, std::max(cap, (size_t)1 << 16) * sizeof(uint64_t));
    ctx->hits_cap = rc ? 0 : bytes / sizeof(uint64_t);
    return rc;
}

int ensure_stage(qk_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->stage_bytes) return QK_OK;
    for (int i = 0; i < 2; ++i) {
        if (ctx->h_stage[i]) hipHostFree(ctx->h_stage[i]);
        if (ctx->d_stage[i]) hipFree(ctx->d_stage[i]);
        ctx->h_stage[i] = ctx->d_stage[i] = nullptr;
    }
    ctx->stage_bytes = 0;
    for (int i = 0; i < 2; ++i) {
        if (hipHostMalloc(&ctx->h_stage[i], bytes, hipHostMallocDefault) != hipSuccess) return QK_E_NOMEM;
        if (hipMalloc(&ctx->d_stage[i], bytes) != hipSuccess) return QK_E_NOMEM;
    }
    ctx->stage_bytes = bytes;
    return QK_OK;
}

int ensure_items(qk_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->h_items_bytes) return QK_OK;
    // the previous buffer is idle: every user synchronises before returning
    if (ctx->h_items) hipHostFree(ctx->h_items);
    ctx->h_items = ctx->h_items_dev = nullptr;
    ctx->h_items_bytes = 0;
    bytes = std::max(bytes, (size_t)1 << 20);
    if (hipHostMalloc(&ctx->h_items, bytes, hipHostMallocDefault) != hipSuccess ||
        hipHostGetDevicePointer(&ctx->h_items_dev, ctx->h_items, 0) != hipSuccess) {
        (void)hipGetLastError();
        if (ctx->h_items) hipHostFree(ctx->h_items);
        ctx->h_items = ctx->h_items_dev = nullptr;
        return QK_E_NOMEM;
    }
    ctx->h_items_bytes = bytes;
    return QK_OK;
}

bool is_device_ptr(const void *p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

static bool is_pinned_host_ptr(const void *p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

hipEvent_t prof_begin(qk_ctx *ctx, hipStream_t s) {
    if (!ctx->profiling) return nullptr;
    hipEvent_t e;
    if (!ctx->ev_pool.empty()) {
        e = ctx->ev_pool.back();
        ctx->ev_pool.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
        return nullptr;
    }
    (void)hipEventRecord(e, s);
    return e;
}

void prof_end(qk_ctx *ctx, hipStream_t s, hipEvent_t begin) {
    if (!ctx->profiling || !begin) return;
    hipEvent_t e;
    if (!ctx->ev_pool.empty()) {
        e = ctx->ev_pool.back();
        ctx->ev_pool.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
        ctx->ev_pool.push_back(begin);
        return;
    }
    (void)hipEventRecord(e, s);
    ctx->prof_pending.emplace_back(begin, e);
}

// ------------------------------------------------------------ fill kernels
__global__ void k_fill_u32(uint32_t *out, uint64_t n, uint64_t seed, uint64_t start) {
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr)
        out[i] = (uint32_t)(splitmix_mix(seed + (start + i + 1) * GAMMA) >> 32);
}
__global__ void k_fill_u64(uint64_t *out, uint64_t n, uint64_t seed, uint64_t start) {
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthr)
        out[i] = splitmix_mix(seed + (start + i + 1) * GAMMA);
}


// Pageable -> pinned staging copy, split over a few host threads: one core's
// memcpy (~24 GB/s) is under half of the PCIe Gen5 rate the DMA can take.
static void staging_copy(void *dst, const void *src, size_t bytes) {
    static const unsigned nthr = [] {
        const unsigned hc = std::thread::hardware_concurrency();
        return hc >= 4 ? std::min(8u, hc / 2) : 1u;
    }();
    if (nthr <= 1 || bytes < ((size_t)8 << 20)) {
        memcpy(dst, src, bytes);
        return;
    }
    const size_t part = (bytes / nthr + 4095) & ~(size_t)4095;
    std::vector<std::thread> pool;
    pool.reserve(nthr - 1);
    size_t done = part;   // pieces below `done` are handed out (piece 0 to this thread)
    try {
        for (unsigned i = 1; i < nthr && done < bytes; ++i) {
            const size_t b = done, e = std::min(bytes, done + part);
            pool.emplace_back([=] { memcpy((char *)dst + b, (const char *)src + b, e - b); });
            done = e;
        }
    } catch (...) {   // no thread to spare: this thread copies the rest (no exception crosses the C ABI)
    }
    memcpy(dst, src, std::min(bytes, part));
    if (done < bytes) memcpy((char *)dst + done, (const char *)src + done, bytes - done);
    for (auto &th : pool) th.join();
}

// Host-resident ids: chunked H2D on copy_stream overlapped with the encode
// kernel on ctx->stream; two device slots.  Pinned input is DMA'd directly,
// pageable input is first copied into pinned staging (staging_copy).
template <typename IdT, typename Launch>
static int encode_host_impl(qk_ctx *ctx, const IdT *h_ids, size_t n, uint32_t t, size_t words, Launch launch,
                            uint64_t *partial_out) {
    const size_t chunk_ids = (size_t)64 << 20 >> (sizeof(IdT) == 4 ? 2 : 3); // 64 MiB chunks
    const size_t chunk_bytes = chunk_ids * sizeof(IdT);
    int rc = ensure_stage(ctx, chunk_bytes);
    if (rc) return rc;
    const bool pinned = is_pinned_host_ptr(h_ids);
    hipStream_t cs = ctx->copy_stream, ks = ctx->stream;
    // destroyed on every exit; the streams are drained first so that no
    // queued wait or record still refers to them
    struct Events {
        hipEvent_t copied[2] = {nullptr, nullptr}, consumed[2] = {nullptr, nullptr};
        hipStream_t cs, ks;
        ~Events() {
            (void)hipStreamSynchronize(ks);
            (void)hipStreamSynchronize(cs);
            for (int i = 0; i < 2; ++i) {
                if (copied[i]) (void)hipEventDestroy(copied[i]);
                if (consumed[i]) (void)hipEventDestroy(consumed[i]);
            }
        }
    } ev;
    ev.cs = cs;
    ev.ks = ks;
    hipEvent_t *copied = ev.copied, *consumed = ev.consumed;
    for (int i = 0; i < 2; ++i) {
        if (hipEventCreateWithFlags(&copied[i], hipEventDisableTiming) != hipSuccess) return QK_E_HIP;
        if (hipEventCreateWithFlags(&consumed[i], hipEventDisableTiming) != hipSuccess) return QK_E_HIP;
    }
    // zero the accumulating partial
    QK_HIP_TRY(hipMemsetAsync(ctx->d_small, 0, words * 8, ks));
    bool used[2] = {false, false};
    for (size_t off = 0, c = 0; off < n; off += chunk_ids, ++c) {
        const int slot = (int)(c & 1);
        const size_t m = std::min(chunk_ids, n - off);
        if (used[slot]) {
            // the kernel that read d_stage[slot] (and the copy that read
            // h_stage[slot]) must be done before we overwrite them
            QK_HIP_TRY(hipStreamWaitEvent(cs, consumed[slot], 0));
            if (!pinned) QK_HIP_TRY(hipEventSynchronize(copied[slot]));
        }
        const void *src = h_ids + off;
        if (!pinned) {
            staging_copy(ctx->h_stage[slot], h_ids + off, m * sizeof(IdT));
            src = ctx->h_stage[slot];
        }
        QK_HIP_TRY(hipMemcpyAsync(ctx->d_stage[slot], src, m * sizeof(IdT), hipMemcpyHostToDevice, cs));
        QK_HIP_TRY(hipEventRecord(copied[slot], cs));
        QK_HIP_TRY(hipStreamWaitEvent(ks, copied[slot], 0));
        rc = launch(ctx, (const IdT *)ctx->d_stage[slot], m, t, ctx->d_small, ks);
        if (rc) return rc;
        QK_HIP_TRY(hipEventRecord(consumed[slot], ks));
        used[slot] = true;
    }
    QK_HIP_TRY(hipMemcpyAsync(partial_out, ctx->d_small, words * 8, hipMemcpyDeviceToHost, ks));
    QK_HIP_TRY(hipStreamSynchronize(ks));
    QK_HIP_TRY(hipStreamSynchronize(cs));
    return QK_OK;
}

// Root test in two phases, so that several devices (a multi-GPU
// communicator, comm.hip) can have theirs in flight at once.
// root_test_begin enqueues on s: counters + coefficients (or root set) H2D,
// the kernel, and for Horner the counters and first hits D2H (the scan
// writes its hits and stops into pinned host memory itself, so no copy
// trails the kernel).  root_test_finish waits for s, reruns once with a larger hit
// buffer if the kernel ran out of room, and returns the hit positions sorted
// ascending (every hit of the log, not cut at the stop) and the first stop
// position (n if none or !use_stop).
// Root test by the root-set scan (decode.hip k_root_scan) or by Horner
// (k_root_test_*): the same hit list (P(x) == 0 <=> x mod p is a root of P).
// The scan costs the host root finding (roots.cpp, ~c d^2) plus an HBM-bound
// pass; Horner costs d multiply steps per candidate.  Cost model in
// microseconds from the measurements in DESIGN.md §3.4 (MI355X kernels,
// EPYC host root finding): the scan is taken when it is cheaper.
template <typename T> static bool rt_use_scan(const qk_ctx *ctx, uint32_t d, size_t n) {
    if (d < 2 || d > RT_SCAN_MAXD) return false;          // d = 1: the root is -c_1, Horner is one step
    if (ctx->knobs.root_test == 1) return false;
    if (ctx->knobs.root_test == 2) return true;
    const double nn = (double)n, dd = (double)d;
    const bool w32 = sizeof(T) == 4;
    const double horner = nn * dd * (w32 ? 1.43e-7 : 3.8e-7);
    const double scan = nn * (w32 ? 0.7e-6 : 1.4e-6) + dd * dd * (w32 ? 0.025 : 0.055);
    return scan < horner;
}

template <typename T> int root_test_plan(const qk_ctx *ctx, const T *coeffs, uint32_t d, size_t n, RtPlan<T> &plan) {
    plan = RtPlan<T>{};
    if (!n || !rt_use_scan<T>(ctx, d, n)) return QK_OK;
    std::vector<T> r(d);
    uint32_t k = 0;
    int rc;
    if constexpr (sizeof(T) == 4) rc = qk_u32_roots(coeffs, d, r.data(), d, &k);
    else rc = qk_u64_roots(coeffs, d, r.data(), d, &k);
    if (rc) return rc;
    plan.scan = rt_scan_table<T>(r.data(), k, plan.set, plan.tab, false) &&
                plan.set.words * sizeof(T) <= (SMALL_NHITS - RT_C) * 8;
    if (!plan.scan) plan.tab.clear();
    return QK_OK;
}

template <typename T>
int root_test_begin(qk_ctx *ctx, const RtPlan<T> &plan, const T *coeffs, uint32_t d, const T *d_log, size_t n,
                    int use_stop, T stop_value, hipStream_t s) {
    // d_small: [0] hit count, [1] stop index, [2] finished workgroups, from
    // [RT_C] the coefficients or the root set (ctx.h)
    uint64_t *d_counters = ctx->d_small;
    T *d_c = (T *)(ctx->d_small + RT_C);
    uint64_t *h_c = ctx->h_small + RT_C;
    const bool scan = n && plan.scan;
    size_t cbytes = (size_t)d * sizeof(T);
    if (scan) {
        cbytes = (size_t)plan.set.words * sizeof(T);
        memcpy(h_c, plan.tab.data(), cbytes);
    } else if constexpr (sizeof(T) == 8) {
        if (rt64_use_bsgs(ctx, d)) cbytes = rt64_bsgs_table(coeffs, d, h_c) * 8;   // limb-shifted table
        else memcpy(h_c, coeffs, cbytes);
    } else {
        memcpy(h_c, coeffs, cbytes);
    }
    // one copy carries the zeroed counters, the scan's hash multipliers and
    // the table (or coefficients): no counter-initialising launch
    ctx->h_small[0] = 0;
    ctx->h_small[1] = ~0ull;
    ctx->h_small[2] = scan ? (uint64_t)plan.set.m1 | (uint64_t)plan.set.m2 << 32 : 0;
    ctx->h_small[3] = 0;
    if (scan) {   // the scan's host slots (decode.hip rt_record): empty, no overflow
        std::fill(ctx->h_small + SMALL_HITPF, ctx->h_small + SMALL_WORDS, ~0ull);
        ctx->h_small[SMALL_OVF] = 0;
    }
    ctx->rt_slots_clean = false;   // this call's hits / stops (or Horner's copy) land in the slots
    QK_HIP_TRY(hipMemcpyAsync(ctx->d_small, ctx->h_small, (RT_C + (cbytes + 7) / 8) * sizeof(uint64_t),
                              hipMemcpyHostToDevice, s));
    if (int rc = ensure_hits(ctx, 4096, s)) return rc;
    if (n) {
        if (scan) {
            // the scan writes its hits and stops into h_small's slots itself
            // (rt_record); root_test_finish derives count and stop from them
            // (a D2H copy of the counters and hits instead measured slower,
            // profiles/r05/decode_nt/)
            return launch_root_scan<T>(ctx, d_c, plan.set, d_log, n, use_stop, stop_value, ctx->d_hits,
                                       (uint64_t)ctx->hits_cap, d_counters, ctx->h_small_dev + SMALL_NHITS, s);
        }
        int (*launch)(qk_ctx *, const T *, uint32_t, const T *, size_t, int, T, uint64_t *, uint64_t, uint64_t *,
                      hipStream_t);
        if constexpr (sizeof(T) == 4) launch = launch_root_test_u32;
        else launch = launch_root_test_u64;
        if (int rc = launch(ctx, d_c, d, d_log, n, use_stop, stop_value, ctx->d_hits, (uint64_t)ctx->hits_cap,
                            d_counters, s))
            return rc;
    }
    QK_HIP_TRY(hipMemcpyAsync(ctx->h_small + SMALL_NHITS, d_counters, 16, hipMemcpyDeviceToHost, s));
    // and the first hits with them: a decode finds ~d hits, so one
    // synchronisation (not a second, pageable, round trip) returns them
    QK_HIP_TRY(hipMemcpyAsync(ctx->h_small + SMALL_HITPF, ctx->d_hits,
                              std::min<size_t>(ctx->hits_cap, SMALL_HITPF_N) * 8, hipMemcpyDeviceToHost, s));
    return QK_OK;
}

template <typename T>
int root_test_finish(qk_ctx *ctx, const RtPlan<T> &plan, const T *coeffs, uint32_t d, const T *d_log, size_t n,
                     int use_stop, T stop_value, hipStream_t s, std::vector<uint64_t> &hits, uint64_t &stop_index) {
    // count and stop into h_small[SMALL_NHITS], [SMALL_STOP]: the Horner
    // form copied them; the scan has its slots, or on overflow the device
    // counters are copied now
    auto counts = [&]() -> int {
        QK_HIP_TRY(hipStreamSynchronize(s));
        if (!(n && plan.scan)) return QK_OK;
        uint64_t *h = ctx->h_small;
        if (h[SMALL_OVF]) {
            QK_HIP_TRY(hipMemcpyAsync(h + SMALL_NHITS, ctx->d_small, 16, hipMemcpyDeviceToHost, s));
            QK_HIP_TRY(hipStreamSynchronize(s));
            return QK_OK;
        }
        uint64_t c = 0;
        while (c < SMALL_HITPF_N && h[SMALL_HITPF + c] != ~0ull) ++c;
        uint64_t st = ~0ull;
        for (uint32_t k = 0; k < RT_NSTOP; ++k) st = std::min(st, h[SMALL_STOPS + k]);
        h[SMALL_NHITS] = c;
        h[SMALL_STOP] = st;
        return QK_OK;
    };
    if (int rc = counts()) return rc;
    uint64_t cnt = ctx->h_small[SMALL_NHITS];
    if (cnt > ctx->hits_cap) {   // grow and rerun once (the kernel counts every hit)
        if (int rc = ensure_hits(ctx, (size_t)cnt, s)) return rc;
        if (int rc = root_test_begin<T>(ctx, plan, coeffs, d, d_log, n, use_stop, stop_value, s)) return rc;
        if (int rc = counts()) return rc;
        cnt = ctx->h_small[SMALL_NHITS];
        if (cnt > ctx->hits_cap) return QK_E_HIP;
    }
    const uint64_t stop = ctx->h_small[SMALL_STOP];
    hits.resize(cnt);
    if (cnt && cnt <= std::min<size_t>(ctx->hits_cap, SMALL_HITPF_N)) {
        memcpy(hits.data(), ctx->h_small + SMALL_HITPF, cnt * 8);
    } else if (cnt) {
        QK_HIP_TRY(hipMemcpyAsync(hits.data(), ctx->d_hits, cnt * 8, hipMemcpyDeviceToHost, s));
        QK_HIP_TRY(hipStreamSynchronize(s));
    }
    std::sort(hits.begin(), hits.end());
    stop_index = use_stop ? std::min<uint64_t>(stop, (uint64_t)n) : (uint64_t)n;
    return QK_OK;
}
template int root_test_plan<uint32_t>(const qk_ctx *, const uint32_t *, uint32_t, size_t, RtPlan<uint32_t> &);
template int root_test_plan<uint64_t>(const qk_ctx *, const uint64_t *, uint32_t, size_t, RtPlan<uint64_t> &);
template int root_test_begin<uint32_t>(qk_ctx *, const RtPlan<uint32_t> &, const uint32_t *, uint32_t,
                                       const uint32_t *, size_t, int, uint32_t, hipStream_t);
template int root_test_begin<uint64_t>(qk_ctx *, const RtPlan<uint64_t> &, const uint64_t *, uint32_t,
                                       const uint64_t *, size_t, int, uint64_t, hipStream_t);
template int root_test_finish<uint32_t>(qk_ctx *, const RtPlan<uint32_t> &, const uint32_t *, uint32_t,
                                        const uint32_t *, size_t, int, uint32_t, hipStream_t, std::vector<uint64_t> &,
                                        uint64_t &);
template int root_test_finish<uint64_t>(qk_ctx *, const RtPlan<uint64_t> &, const uint64_t *, uint32_t,
                                        const uint64_t *, size_t, int, uint64_t, hipStream_t, std::vector<uint64_t> &,
                                        uint64_t &);

// The root-set scan with its set in the kernel arguments (single GPU, sets
// of at most RT_KTAB_BYTES: the compact layout, k = 32 roots -> 256 buckets,
// 1 KB u32 / 2 KB u64): the host finds the roots, builds the set and
// launches — no H2D
// copy and no counter reset in front of the scan (the hit / stop tickets
// run on from the values the previous call left, ctx->rt_hbase / rt_sbase,
// in their own words of d_small, SMALL_KT).  The scan hands its hits and
// stops over through the pinned slots; a slot overflow (more than the slots
// hold) returns 1, the caller reruns by the two-phase form, and the tickets
// are reset before the next kernel-argument call.
template <typename T>
static int root_test_scan_k(qk_ctx *ctx, const T *coeffs, uint32_t d, const T *d_log, size_t n, int use_stop,
                            T stop_value, hipStream_t s, std::vector<uint64_t> &h, uint64_t &stop) {
    std::vector<T> r(d);
    uint32_t k = 0;
    int rc;
    if constexpr (sizeof(T) == 4) rc = qk_u32_roots(coeffs, d, r.data(), d, &k);
    else rc = qk_u64_roots(coeffs, d, r.data(), d, &k);
    if (rc) return rc;
    RtScanSet set;
    std::vector<T> tab;
    if (!rt_scan_table<T>(r.data(), k, set, tab, true) || set.words * sizeof(T) > RT_KTAB_BYTES) return 1;
    if (int e = ensure_hits(ctx, 4096, s)) return e;
    uint64_t *hs = ctx->h_small;
    if (!ctx->rt_bases_valid) {   // after a two-phase call (or none): reset the tickets once
        QK_HIP_TRY(hipMemsetAsync(ctx->d_small + SMALL_KT, 0, 4 * sizeof(uint64_t), s));
        ctx->rt_hbase = ctx->rt_sbase = 0;
    }
    if (!ctx->rt_slots_clean) {
        std::fill(hs + SMALL_HITPF, hs + SMALL_WORDS, ~0ull);
        hs[SMALL_OVF] = 0;
    }
    ctx->rt_slots_clean = false;
    const uint64_t gen = ++ctx->rt_gen;
    if (int e = launch_root_scan_k<T>(ctx, tab, set, d_log, n, use_stop, stop_value, ctx->d_hits,
                                      (uint64_t)ctx->hits_cap, ctx->d_small + SMALL_KT, ctx->h_small_dev + SMALL_NHITS,
                                      ctx->rt_hbase, ctx->rt_sbase, ctx->d_small + RT_DONE, gen, s)) {
        ctx->rt_bases_valid = false;
        return e;
    }
    ctx->rt_bases_valid = true;
    // wait by polling the completion mark the kernel's last workgroup writes
    // (decode.hip k_root_scan_k: the result is in the slots ~3-5 µs before
    // the stream reports the kernel done), the stream asked now and then: an
    // error fails the call; a finished stream without the mark (completion
    // tickets left off by an earlier aborted launch) still has the result,
    // and the tickets are cleared for the next launch
    const volatile uint64_t *done = hs + SMALL_DONE;
    for (unsigned spin = 0;; ++spin) {
        if (*done == gen) break;
        if ((spin & 63) == 63) {
            const hipError_t q = hipStreamQuery(s);
            if (q != hipSuccess && q != hipErrorNotReady) {
                ctx->rt_bases_valid = false;
                return QK_E_HIP;
            }
            if (q == hipSuccess) {
                if (*done == gen) break;
                QK_HIP_TRY(hipMemsetAsync(ctx->d_small + RT_DONE, 0, (SMALL_DEV_WORDS - RT_DONE) * sizeof(uint64_t), s));
                break;
            }
        }
        if (spin >= 200000) std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    if (hs[SMALL_OVF]) {   // past the slots: the two-phase form reruns it (and resets the tickets)
        ctx->rt_bases_valid = false;
        return 1;
    }
    uint64_t c = 0;
    while (c < SMALL_HITPF_N && hs[SMALL_HITPF + c] != ~0ull) ++c;
    uint64_t st = ~0ull, ns = 0;
    for (uint32_t q = 0; q < RT_NSTOP; ++q) {
        st = std::min(st, hs[SMALL_STOPS + q]);
        ns += hs[SMALL_STOPS + q] != ~0ull;
    }
    ctx->rt_hbase += c;
    ctx->rt_sbase += ns;
    h.assign(hs + SMALL_HITPF, hs + SMALL_HITPF + c);
    // the next call finds the slots empty: the c hit slots and the stop
    // slots back to ~0 (the kernel wrote no others: no overflow)
    std::fill(hs + SMALL_HITPF, hs + SMALL_HITPF + c, ~0ull);
    std::fill(hs + SMALL_STOPS, hs + SMALL_WORDS, ~0ull);
    ctx->rt_slots_clean = true;
    std::sort(h.begin(), h.end());
    stop = use_stop ? std::min<uint64_t>(st, (uint64_t)n) : (uint64_t)n;
    return QK_OK;
}

template <typename T>
static int root_test_impl(qk_ctx *ctx, const T *coeffs, uint32_t d, const T *d_log, size_t n, int use_stop,
                          T stop_value, uint64_t *hits, size_t cap, size_t *n_hits, void *stream,
                          uint64_t *stop_index = nullptr) {
    if (!ctx || !n_hits || (d && !coeffs) || (n && !d_log)) return QK_E_INVAL;
    *n_hits = 0;
    if (stop_index) *stop_index = n;
    if (n == 0) return QK_OK;
    if (d == 0) {
        if (!stop_index || !use_stop) return QK_OK; // P == 1 has no roots
        // no roots, but a shard caller still needs the stop position: the
        // degree-0 launch tests nothing and only records the stop
    }
    if (d > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if (!is_device_ptr(d_log)) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = pick_stream(ctx, stream);
    std::vector<uint64_t> h;
    uint64_t stop = n;
    int ov = 1;
    if (ctx->knobs.rt_karg && rt_use_scan<T>(ctx, d, n)) {
        ov = root_test_scan_k<T>(ctx, coeffs, d, d_log, n, use_stop, stop_value, s, h, stop);
        if (ov < 0) return ov;
    }
    if (ov) {   // Horner, a set too large for the kernel arguments, or a slot overflow
        RtPlan<T> plan;
        if (int rc = root_test_plan<T>(ctx, coeffs, d, n, plan)) return rc;
        if (int rc = root_test_begin<T>(ctx, plan, coeffs, d, d_log, n, use_stop, stop_value, s)) return rc;
        if (int rc = root_test_finish<T>(ctx, plan, coeffs, d, d_log, n, use_stop, stop_value, s, h, stop)) return rc;
    }
    const size_t m = (size_t)(std::lower_bound(h.begin(), h.end(), stop) - h.begin());
    if (stop_index) *stop_index = stop;
    *n_hits = m;
    if (m > cap || (m && !hits)) return QK_E_CAPACITY;
    std::copy(h.begin(), h.begin() + m, hits);
    return QK_OK;
}

} // namespace qk

// =========================================================================
extern "C" {

int qk_device_count(int *n) {
    if (!n) return QK_E_INVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) {
        (void)hipGetLastError();
        *n = 0;
        return QK_E_NO_DEVICE;
    }
    *n = c;
    return c > 0 ? QK_OK : QK_E_NO_DEVICE;
}

int qk_ctx_create(int device, qk_ctx **out) {
    if (!out) return QK_E_INVAL;
    *out = nullptr;
    int n = 0;
    if (qk_device_count(&n) != QK_OK || device < 0 || device >= n) return QK_E_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return QK_E_NO_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return QK_E_NO_DEVICE; // code objects are gfx950-only
    if (hipSetDevice(device) != hipSuccess) return QK_E_HIP;
    qk_ctx *ctx = new (std::nothrow) qk_ctx();
    if (!ctx) return QK_E_NOMEM;
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount;
    if (prop.maxThreadsPerMultiProcessor > 0) ctx->max_threads_per_cu = prop.maxThreadsPerMultiProcessor;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&ctx->d_small, SMALL_DEV_WORDS * sizeof(uint64_t)) != hipSuccess ||
        hipHostMalloc(&ctx->h_small, SMALL_WORDS * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&ctx->h_flow, 8 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess ||
        hipHostGetDevicePointer((void **)&ctx->h_small_dev, ctx->h_small, 0) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->stage_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->stage_ev[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->scratch_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->flow_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->flow_ev[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->flow_ev[2], hipEventDisableTiming) != hipSuccess) {
        qk_ctx_destroy(ctx);
        return QK_E_HIP;
    }
    // every code object resident and the pageable-copy path set up now, not
    // inside the caller's first batch (ctx.h QK_WARM_KERNEL); the per-flow
    // work-item buffer (1 MiB) allocated
    uint64_t pageable[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (ensure_items(ctx, (size_t)1 << 20) || warm_api(ctx->stream) || warm_encode(ctx->stream) || warm_decode(ctx->stream) ||
        warm_packets(ctx->stream) || warm_flows(ctx->stream) || warm_segments(ctx->stream) || warm_comm(ctx->stream) ||
        hipMemsetAsync(ctx->d_small, 0, SMALL_DEV_WORDS * sizeof(uint64_t), ctx->stream) != hipSuccess ||
        hipMemcpyAsync(ctx->d_small, pageable, sizeof pageable, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
        hipMemcpyAsync(pageable, ctx->d_small, sizeof pageable, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
        qk_ctx_destroy(ctx);
        return QK_E_HIP;
    }
    *out = ctx;
    return QK_OK;
}

void qk_ctx_destroy(qk_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    for (auto &pr : ctx->prof_pending) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
    for (auto e : ctx->ev_pool) hipEventDestroy(e);
    for (int i = 0; i < 2; ++i) {
        if (ctx->h_stage[i]) hipHostFree(ctx->h_stage[i]);
        if (ctx->d_stage[i]) hipFree(ctx->d_stage[i]);
        if (ctx->stage_ev[i]) hipEventDestroy(ctx->stage_ev[i]);
    }
    if (ctx->scratch_ev) hipEventDestroy(ctx->scratch_ev);
    for (hipEvent_t e : ctx->flow_ev)
        if (e) hipEventDestroy(e);
    if (ctx->d_scratch) hipFree(ctx->d_scratch);
    if (ctx->d_hits) hipFree(ctx->d_hits);
    for (void *f : ctx->d_flow)
        if (f) hipFree(f);
    for (void *r : ctx->retired) hipFree(r);
    if (ctx->d_small) hipFree(ctx->d_small);
    if (ctx->h_small) hipHostFree(ctx->h_small);
    if (ctx->h_flow) hipHostFree(ctx->h_flow);
    if (ctx->h_items) hipHostFree(ctx->h_items);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    if (ctx->copy_stream) hipStreamDestroy(ctx->copy_stream);
    delete ctx;
}

int qk_ctx_synchronize(qk_ctx *ctx, void *stream) {
    if (!ctx) return QK_E_INVAL;
    QK_HIP_TRY(hipStreamSynchronize(pick_stream(ctx, stream)));
    return QK_OK;
}

int qk_ctx_set_profiling(qk_ctx *ctx, int on) {
    if (!ctx) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    ctx->profiling = on != 0;
    return QK_OK;
}

int qk_ctx_kernel_stats(qk_ctx *ctx, double *total_ms, uint64_t *launches) {
    if (!ctx || !total_ms || !launches) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    double tot = 0;
    uint64_t cnt = 0;
    int rc = QK_OK;
    for (auto &pr : ctx->prof_pending) {
        if (hipEventSynchronize(pr.second) != hipSuccess) rc = QK_E_HIP;
        float ms = 0;
        if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) { tot += ms; ++cnt; }
        ctx->ev_pool.push_back(pr.first);
        ctx->ev_pool.push_back(pr.second);
    }
    ctx->prof_pending.clear();
    *total_ms = tot;
    *launches = cnt;
    return rc;
}

int qk_ctx_trim(qk_ctx *ctx) {
    if (!ctx) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (ctx->retired.empty()) return QK_OK;
    QK_HIP_TRY(hipSetDevice(ctx->device));
    int rc = QK_OK;
    for (void *r : ctx->retired)
        if (hipFree(r) != hipSuccess) rc = QK_E_HIP;   // synchronises the device
    ctx->retired.clear();
    return rc;
}

int qk_ctx_set_grid(qk_ctx *ctx, uint32_t blocks) {
    if (!ctx) return QK_E_INVAL;
    ctx->grid_override = blocks;
    return QK_OK;
}

int qk_ctx_set_knob(qk_ctx *ctx, const char *name, int64_t value) {
    if (!ctx || !name) return QK_E_INVAL;
    struct K {
        const char *name;
        int qk_knobs::*field;
        int64_t lo, hi;
    };
    static const K table[] = {
        {"grid_mult", &qk_knobs::grid_mult, 1, 8},
        {"flow_hist", &qk_knobs::flow_hist, 0, 1 << 20},
        {"flow_byslot", &qk_knobs::flow_byslot, 0, 2},
        {"root_test", &qk_knobs::root_test, 0, 2},
        {"comm_fault", &qk_knobs::comm_fault, 0, 1 << 20},
        {"comm_delay_ms", &qk_knobs::comm_delay_ms, 0, 600000},
        {"rt_karg", &qk_knobs::rt_karg, 0, 1},
    };
    for (const K &k : table)
        if (strcmp(k.name, name) == 0) {
            if (value < k.lo || value > k.hi) return QK_E_INVAL;
            std::lock_guard<std::mutex> g(ctx->mu);
            ctx->knobs.*(k.field) = (int)value;
            return QK_OK;
        }
    return QK_E_INVAL;
}

// one wave: wall time from s_memrealtime (100 MHz), shader cycles from
// s_memtime; s_sleep between samples keeps the probe off the issue ports
__global__ void k_clock_probe(uint64_t *out, uint64_t ticks) {
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t c1, r1;
    do {
        __builtin_amdgcn_s_sleep(32);
        c1 = __builtin_amdgcn_s_memtime();
        r1 = __builtin_amdgcn_s_memrealtime();
    } while (r1 - r0 < ticks);
    if (threadIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = r1 - r0;
    }
}

int qk_clock_probe(qk_ctx *ctx, uint32_t microseconds, uint64_t *d_out, void *stream) {
    if (!ctx || !d_out || !microseconds || microseconds > 10000000u) return QK_E_INVAL;
    if (!is_device_ptr(d_out)) return QK_E_INVAL;
    QK_HIP_TRY(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, d_out, (uint64_t)microseconds * 100);
    QK_HIP_TRY(hipGetLastError());
    return QK_OK;
}

int qk_host_alloc(size_t bytes, void **out) {
    if (!out) return QK_E_INVAL;
    if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) { *out = nullptr; return QK_E_NOMEM; }
    return QK_OK;
}
int qk_host_free(void *p) {
    if (p && hipHostFree(p) != hipSuccess) return QK_E_HIP;
    return QK_OK;
}

// ------------------------------------------------------------ encode
int qk_u32_encode_device_async(qk_ctx *ctx, const uint32_t *d_ids, size_t n, uint32_t t, uint64_t *d_partial,
                               void *stream) {
    if (!ctx || !d_partial || (n && !d_ids)) return QK_E_INVAL;
    if (t == 0 || t > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if ((n && !is_device_ptr(d_ids)) || !is_device_ptr(d_partial)) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    return launch_encode_u32(ctx, d_ids, n, t, d_partial, pick_stream(ctx, stream));
}

int qk_u64_encode_device_async(qk_ctx *ctx, const uint64_t *d_ids, size_t n, uint32_t t, uint64_t *d_partial,
                               void *stream) {
    if (!ctx || !d_partial || (n && !d_ids)) return QK_E_INVAL;
    if (t == 0 || t > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if ((n && !is_device_ptr(d_ids)) || !is_device_ptr(d_partial)) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    return launch_encode_u64(ctx, d_ids, n, t, d_partial, pick_stream(ctx, stream));
}

int qk_u32_encode_device(qk_ctx *ctx, const uint32_t *d_ids, size_t n, qk_u32 *q, void *stream) {
    if (!ctx || !q || (n && !d_ids)) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    if (t == 0 || t > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if (n == 0) return QK_OK;
    if (!is_device_ptr(d_ids)) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = pick_stream(ctx, stream);
    int rc = launch_encode_u32(ctx, d_ids, n, t, ctx->d_small, s);
    if (rc) return rc;
    const size_t w = qk_u32_partial_words(t);
    QK_HIP_TRY(hipMemcpyAsync(ctx->h_small, ctx->d_small, w * 8, hipMemcpyDeviceToHost, s));
    QK_HIP_TRY(hipStreamSynchronize(s));
    return qk_u32_merge_partial(q, ctx->h_small, 1, (uint32_t)ctx->h_small[t + 1]);
}

int qk_u64_encode_device(qk_ctx *ctx, const uint64_t *d_ids, size_t n, qk_u64 *q, void *stream) {
    if (!ctx || !q || (n && !d_ids)) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    if (t == 0 || t > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if (n == 0) return QK_OK;
    if (!is_device_ptr(d_ids)) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = pick_stream(ctx, stream);
    int rc = launch_encode_u64(ctx, d_ids, n, t, ctx->d_small, s);
    if (rc) return rc;
    const size_t w = qk_u64_partial_words(t);
    QK_HIP_TRY(hipMemcpyAsync(ctx->h_small, ctx->d_small, w * 8, hipMemcpyDeviceToHost, s));
    QK_HIP_TRY(hipStreamSynchronize(s));
    return qk_u64_merge_partial(q, ctx->h_small, 1, ctx->h_small[2 * t + 1]);
}

int qk_u32_encode_host(qk_ctx *ctx, const uint32_t *h_ids, size_t n, qk_u32 *q) {
    if (!ctx || !q || (n && !h_ids)) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    if (t == 0 || t > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if (n == 0) return QK_OK;
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    const size_t w = qk_u32_partial_words(t);
    int rc = encode_host_impl<uint32_t>(ctx, h_ids, n, t, w, launch_encode_u32_acc, ctx->h_small);
    if (rc) return rc;
    return qk_u32_merge_partial(q, ctx->h_small, 1, h_ids[n - 1]);
}

int qk_u64_encode_host(qk_ctx *ctx, const uint64_t *h_ids, size_t n, qk_u64 *q) {
    if (!ctx || !q || (n && !h_ids)) return QK_E_INVAL;
    const uint32_t t = q->threshold;
    if (t == 0 || t > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if (n == 0) return QK_OK;
    std::lock_guard<std::mutex> g(ctx->mu);
    QK_HIP_TRY(hipSetDevice(ctx->device));
    const size_t w = qk_u64_partial_words(t);
    int rc = encode_host_impl<uint64_t>(ctx, h_ids, n, t, w, launch_encode_u64_acc, ctx->h_small);
    if (rc) return rc;
    return qk_u64_merge_partial(q, ctx->h_small, 1, h_ids[n - 1]);
}

// ------------------------------------------------------------ root test
int qk_u32_root_test_device(qk_ctx *ctx, const uint32_t *coeffs, uint32_t d, const uint32_t *d_log, size_t n,
                            int stop_at_value, uint32_t stop_value, uint64_t *hits, size_t cap, size_t *n_hits,
                            void *stream) {
    return root_test_impl<uint32_t>(ctx, coeffs, d, d_log, n, stop_at_value, stop_value, hits, cap, n_hits, stream);
}

int qk_u64_root_test_device(qk_ctx *ctx, const uint64_t *coeffs, uint32_t d, const uint64_t *d_log, size_t n,
                            int stop_at_value, uint64_t stop_value, uint64_t *hits, size_t cap, size_t *n_hits,
                            void *stream) {
    return root_test_impl<uint64_t>(ctx, coeffs, d, d_log, n, stop_at_value, stop_value, hits, cap, n_hits, stream);
}

int qk_u32_root_test_shard_device(qk_ctx *ctx, const uint32_t *coeffs, uint32_t d, const uint32_t *d_log, size_t n,
                                  int stop_at_value, uint32_t stop_value, uint64_t *hits, size_t cap,
                                  size_t *n_hits, uint64_t *stop_index, void *stream) {
    if (!stop_index) return QK_E_INVAL;
    return root_test_impl<uint32_t>(ctx, coeffs, d, d_log, n, stop_at_value, stop_value, hits, cap, n_hits, stream,
                                    stop_index);
}

int qk_u64_root_test_shard_device(qk_ctx *ctx, const uint64_t *coeffs, uint32_t d, const uint64_t *d_log, size_t n,
                                  int stop_at_value, uint64_t stop_value, uint64_t *hits, size_t cap,
                                  size_t *n_hits, uint64_t *stop_index, void *stream) {
    if (!stop_index) return QK_E_INVAL;
    return root_test_impl<uint64_t>(ctx, coeffs, d, d_log, n, stop_at_value, stop_value, hits, cap, n_hits, stream,
                                    stop_index);
}

int qk_u32_decode_device(qk_ctx *ctx, const qk_u32 *diff, const uint32_t *d_log, size_t n, int stop_at_last,
                         uint64_t *hits, size_t cap, size_t *n_hits, void *stream) {
    if (!ctx || !diff || !n_hits) return QK_E_INVAL;
    *n_hits = 0;
    if (diff->count == 0) return QK_OK;
    std::vector<uint32_t> c(diff->threshold ? diff->threshold : 1);
    uint32_t d = 0;
    int rc = qk_u32_to_coeffs(diff, c.data(), (uint32_t)c.size(), &d);
    if (rc) return rc;
    return qk_u32_root_test_device(ctx, c.data(), d, d_log, n, stop_at_last && diff->has_last, diff->last_value,
                                   hits, cap, n_hits, stream);
}

int qk_u64_decode_device(qk_ctx *ctx, const qk_u64 *diff, const uint64_t *d_log, size_t n, int stop_at_last,
                         uint64_t *hits, size_t cap, size_t *n_hits, void *stream) {
    if (!ctx || !diff || !n_hits) return QK_E_INVAL;
    *n_hits = 0;
    if (diff->count == 0) return QK_OK;
    std::vector<uint64_t> c(diff->threshold ? diff->threshold : 1);
    uint32_t d = 0;
    int rc = qk_u64_to_coeffs(diff, c.data(), (uint32_t)c.size(), &d);
    if (rc) return rc;
    return qk_u64_root_test_device(ctx, c.data(), d, d_log, n, stop_at_last && diff->has_last, diff->last_value,
                                   hits, cap, n_hits, stream);
}

// ------------------------------------------------------------ fills
int qk_fill_splitmix_u32(qk_ctx *ctx, uint32_t *d_out, size_t n, uint64_t seed, uint64_t start, void *stream) {
    if (!ctx || (n && !d_out)) return QK_E_INVAL;
    if (n == 0) return QK_OK;
    if (!is_device_ptr(d_out)) return QK_E_INVAL;
    QK_HIP_TRY(hipSetDevice(ctx->device));
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, (uint64_t)ctx->num_cus * 16);
    hipLaunchKernelGGL(k_fill_u32, dim3((uint32_t)blocks), dim3(256), 0, pick_stream(ctx, stream), d_out,
                       (uint64_t)n, seed, start);
    QK_HIP_TRY(hipGetLastError());
    return QK_OK;
}

int qk_fill_splitmix_u64(qk_ctx *ctx, uint64_t *d_out, size_t n, uint64_t seed, uint64_t start, void *stream) {
    if (!ctx || (n && !d_out)) return QK_E_INVAL;
    if (n == 0) return QK_OK;
    if (!is_device_ptr(d_out)) return QK_E_INVAL;
    QK_HIP_TRY(hipSetDevice(ctx->device));
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, (uint64_t)ctx->num_cus * 16);
    hipLaunchKernelGGL(k_fill_u64, dim3((uint32_t)blocks), dim3(256), 0, pick_stream(ctx, stream), d_out,
                       (uint64_t)n, seed, start);
    QK_HIP_TRY(hipGetLastError());
    return QK_OK;
}

} // extern "C"
