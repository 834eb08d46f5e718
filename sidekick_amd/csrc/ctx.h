// ctx.h — internal: the device context behind qk_ctx* and launch helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <vector>

#include "quack_hip.h"

// Per-context knobs (qk_ctx_set_knob).  Round 6 removed every knob that
// selected a measured-and-rejected variant ("measured and
// removed"); what is left selects between live product paths — the defaults
// below are the product's own choices — or injects a test fault.
struct qk_knobs {
    int grid_mult = 3;     // encode launches: resident workgroups x this (1: one round; grid_for, encode.hip)
    int flow_hist = 32;    // per-flow batches of at most this many flows (and a table of <= 8192 slots) are
                           // grouped by per-workgroup slot histograms instead of the radix sort (0: never);
                           // 16 flows 2.76 vs 2.90 ms, 64: 3.17 vs 3.05, 1000: 5.80 vs 3.68
                           // (profiles/r05/flows_hist/)
    int flow_byslot = 0;   // per-flow grouping-sort key: 0 the pass-count rule (flows.hip), 1 force by slot,
                           // 2 force by flow rank (tests cover both product paths)
    int root_test = 0;     // 0: automatic (cost model, api.hip rt_use_scan), 1: Horner, 2: root-set scan
    int comm_fault = 0;    // k > 0 (tests): this rank's payload staging for the k-th collective of its
                           // next sharded operation fails, once (comm.hip fault_now)
    int rt_karg = 1;       // 1: a root-set scan whose set fits the kernel arguments takes them (api.hip
                           // root_test_scan_k; configs[4] u64 wall 172 -> 167 us, u32 even,
                           // profiles/r06/s6_karg_s1/); 0: always the set by an H2D copy (the path of
                           // larger sets and of the sharded decode; tests compare the two)
    int comm_delay_ms = 0; // k > 0 (tests): a k-ms kernel in front of this rank's next RCCL collective,
                           // once (comm.hip mark_pre: the bounded wait for pre-collective work)
};

struct qk_ctx {
    int device = 0;
    int num_cus = 256;
    int max_threads_per_cu = 2048;     // hipDeviceProp_t::maxThreadsPerMultiProcessor
    uint32_t max_blocks_per_cu(uint32_t block) const { return (uint32_t)max_threads_per_cu / block; }
    hipStream_t stream = nullptr;      // own stream (host-input pipeline, comm collectives); a NULL
                                       // stream argument is the HIP null stream, not this one
    hipStream_t copy_stream = nullptr; // second stream for the host-input pipeline
    uint32_t grid_override = 0;
    qk_knobs knobs;

    // scratch: block partials of the encode kernels, hit buffers of the root test
    void *d_scratch = nullptr;
    size_t scratch_bytes = 0;
    uint64_t *d_small = nullptr;       // partial output / hit counters (small, fixed)
    uint64_t *h_small = nullptr;       // pinned mirror of d_small
    uint64_t *h_small_dev = nullptr;   // h_small as the device addresses it
    // the kernel-argument root-set scan keeps its hit / stop tickets
    // (d_small[0], [3]) running across calls: their values now, when valid
    uint64_t rt_hbase = 0, rt_sbase = 0;
    bool rt_bases_valid = false;
    // the pinned hit / stop slots hold ~0 everywhere (the kernel-argument
    // scan restores the few it used instead of re-filling all 1020 words)
    bool rt_slots_clean = false;
    // k_root_scan_k<u32 / u64, 1> workgroups per CU (0: not yet asked)
    int rt_occ_k[2] = {0, 0};
    // the value the next kernel-argument scan's last workgroup writes to
    // h_small[SMALL_DONE] (the host polls that word, not the stream)
    uint64_t rt_gen = 0;
    uint64_t *d_hits = nullptr;
    size_t hits_cap = 0;

    // per-flow batches (flows.hip): per-packet arena (slots, ids, sort
    // buffers), per-flow arena (segment info, accumulators, work items) and
    // the flow hash table; grow-only, reused across calls (a stream-ordered
    // malloc/free of GBs per batch costs more than the whole pipeline).
    // flow_hint: distinct flows of the previous batch (sizes the table).
    void *d_flow[3] = {nullptr, nullptr, nullptr};
    size_t flow_bytes[3] = {0, 0, 0};
    size_t flow_hint = 0;
    // work items of the per-flow encode, written by the host into pinned
    // memory the kernels read directly (h_items_dev): no H2D copy — a
    // process's first pageable H2D copy cost 7 ms (SDMA set-up) inside its
    // first flow batch: 16 flows 9.97 ms against 2.89 steady, 3.23 after
    // (profiles/r06/s1/, s2/flows_cold.jsonl); grow-only, used only inside
    // synchronous calls
    void *h_items = nullptr;
    void *h_items_dev = nullptr;
    size_t h_items_bytes = 0;

    // host-input pipeline: pinned staging + device chunk buffers (2 slots)
    void *h_stage[2] = {nullptr, nullptr};
    void *d_stage[2] = {nullptr, nullptr};
    size_t stage_bytes = 0;
    hipEvent_t stage_ev[2] = {nullptr, nullptr};

    // profiling of the dominant kernel
    bool profiling = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_pending;
    std::vector<hipEvent_t> ev_pool;

    // scratch hand-off between streams: every launch that uses d_scratch /
    // d_small / d_hits waits for the previous user's event, then records its own
    hipEvent_t scratch_ev = nullptr;
    bool scratch_ev_valid = false;
    // per-flow batches: fork/join of the flow-key branch on the second stream
    hipEvent_t flow_ev[3] = {nullptr, nullptr, nullptr};
    uint64_t *h_flow = nullptr;   // pinned: the flow extract's counters (read back without a staging copy)

    // grown-out device buffers, freed by qk_ctx_trim / qk_ctx_destroy (hipFree
    // synchronises the whole device; growth must not)
    std::vector<void *> retired;

    std::mutex mu;
};

#define QK_HIP_TRY(expr)                                                                           \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) return QK_E_HIP;                                                     \
    } while (0)

namespace qk {

// Small-buffer layout (u64 words).  Root tests: d_small[0] hit count, [1]
// first stop, [3] stops recorded (root-set scan), [RT_C ..) the
// coefficients or the root set — one H2D copy of h_small[0 .. RT_C + words)
// sets all of it.  Results in h_small from SMALL_NHITS: count, stop, the
// overflow flag of the direct form, then from SMALL_HITPF the first hits and
// at the end RT_NSTOP stop slots.  Horner's arrive by D2H copies; the
// root-set scan writes its hits and stops there itself (decode.hip
// rt_record) and the host derives count and stop from the slots.
constexpr size_t SMALL_WORDS = 4096;   // >= max partial words (2*1024+2) plus counters
constexpr size_t RT_C = 4;             // root tests: coefficients / root set from d_small[RT_C]
constexpr size_t SMALL_NHITS = 3072;   // h_small: hit count
constexpr size_t SMALL_STOP = 3073;    // h_small: first stop index
constexpr size_t SMALL_OVF = 3074;     // h_small: a hit or stop slot past the direct form's room
constexpr size_t SMALL_DONE = 3075;    // h_small: the kernel-argument scan's completion mark
constexpr size_t SMALL_HITPF = 3076;   // h_small: the first hits
constexpr uint32_t RT_NSTOP = 16;      // stop slots of the direct form
constexpr size_t SMALL_STOPS = SMALL_WORDS - RT_NSTOP;
constexpr size_t SMALL_HITPF_N = SMALL_STOPS - SMALL_HITPF;
// the same slots relative to SMALL_NHITS (the kernel's hout)
constexpr size_t RT_STOP0 = SMALL_STOPS - SMALL_NHITS;
// d_small[SMALL_KT ..+4): the kernel-argument root-set scan's counters (hit
// ticket, stop minimum, -, stop ticket), apart from everything else that
// writes d_small (encode partials, the two-phase root test's header)
constexpr size_t SMALL_KT = SMALL_WORDS - 8;
// d_small[RT_DONE ..) (device only, past h_small's mirror): the scan's
// completion tickets, one 128-byte line per workgroup group and one for the
// groups (a single ticket that every workgroup of the grid takes at its end
// serialises: +15 µs); zeroed at context creation, each reset by its taker
constexpr uint32_t RT_DONE_GROUPS = 32;
constexpr size_t RT_DONE = SMALL_WORDS;
constexpr size_t SMALL_DEV_WORDS = RT_DONE + 16 * (RT_DONE_GROUPS + 1);

// One no-op kernel per translation unit.  HIP loads a translation unit's code
// object at the first launch of any of its kernels, and sets up its staging
// path for pageable copies at the first such copy; qk_ctx_create does both
// (warm_* and two 64-byte pageable copies) so that neither lands inside a
// caller's first batch (a process's first flow batch had a 7.7 ms idle gap
// before its first pageable hand-back, profiles/r05/final5/flows_per_call.txt:20).
#define QK_WARM_KERNEL(name)                                                                                     \
    __global__ void k_warm_##name(int *p) {                                                                      \
        if (p) p[threadIdx.x] = 0;                                                                               \
    }                                                                                                            \
    int warm_##name(hipStream_t s) {                                                                             \
        hipLaunchKernelGGL(k_warm_##name, dim3(1), dim3(64), 0, s, nullptr);                                     \
        return hipGetLastError() == hipSuccess ? QK_OK : QK_E_HIP;                                               \
    }
int warm_api(hipStream_t s);
int warm_encode(hipStream_t s);
int warm_decode(hipStream_t s);
int warm_packets(hipStream_t s);
int warm_flows(hipStream_t s);
int warm_segments(hipStream_t s);
int warm_comm(hipStream_t s);

hipStream_t pick_stream(qk_ctx *ctx, void *stream);
// order stream s after the previous user of the context's scratch buffers
int scratch_acquire(qk_ctx *ctx, hipStream_t s);
// mark the end of s's use of the scratch buffers
int scratch_release(qk_ctx *ctx, hipStream_t s);
// grow-only buffers; growth never synchronises the device (the old buffer is
// retired, api.hip regrow)
int ensure_scratch(qk_ctx *ctx, size_t bytes, hipStream_t s);
int ensure_hits(qk_ctx *ctx, size_t cap, hipStream_t s);
int ensure_flow(qk_ctx *ctx, int which, size_t bytes, hipStream_t s);
int ensure_stage(qk_ctx *ctx, size_t bytes);
int ensure_items(qk_ctx *ctx, size_t bytes);
bool is_device_ptr(const void *p);
hipEvent_t prof_begin(qk_ctx *ctx, hipStream_t s);
void prof_end(qk_ctx *ctx, hipStream_t s, hipEvent_t begin);

// encode launchers (encode.hip): enqueue main kernel + finalize writing the
// (t+2)-word / (2t+2)-word partial to d_partial.
int launch_encode_u32(qk_ctx *ctx, const uint32_t *d_ids, size_t n, uint32_t t, uint64_t *d_partial,
                      hipStream_t s);
int launch_encode_u64(qk_ctx *ctx, const uint64_t *d_ids, size_t n, uint32_t t, uint64_t *d_partial,
                      hipStream_t s);
// accumulate-variant used by the host pipeline: adds into d_partial instead
// of overwriting (words 0..t-1 / 0..2t-1 and the count word; last word set).
int launch_encode_u32_acc(qk_ctx *ctx, const uint32_t *d_ids, size_t n, uint32_t t,
                          uint64_t *d_partial, hipStream_t s);
int launch_encode_u64_acc(qk_ctx *ctx, const uint64_t *d_ids, size_t n, uint32_t t,
                          uint64_t *d_partial, hipStream_t s);

int launch_root_test_u32(qk_ctx *ctx, const uint32_t *d_c, uint32_t d, const uint32_t *log, size_t n,
                         int use_stop, uint32_t stop_value, uint64_t *hits, uint64_t cap, uint64_t *counters,
                         hipStream_t s);
// canonical power sums out[0..T) from per-block partials [power][block] (encode.hip)
int launch_finalize_powers_u32(const uint64_t *partials, uint32_t nblocks, uint32_t T, uint64_t *out,
                               hipStream_t s);
// u64 root test by baby-step/giant-step for these degrees (decode.hip); the
// coefficient buffer then holds rt64_bsgs_table's limb-shifted table
bool rt64_use_bsgs(const qk_ctx *ctx, uint32_t d);
// largest degree the root-set scan takes (its set must fit d_small)
constexpr uint32_t RT_SCAN_MAXD = 256;
size_t rt64_bsgs_table(const uint64_t *coeffs, uint32_t d, uint64_t *out);
int launch_root_test_u64(qk_ctx *ctx, const uint64_t *d_c, uint32_t d, const uint64_t *log, size_t n,
                         int use_stop, uint64_t stop_value, uint64_t *hits, uint64_t cap, uint64_t *counters,
                         hipStream_t s);

// root-set scan (decode.hip): the hash set of P's roots in LDS
struct RtScanSet {
    uint32_t S = 1, words = 0, m1 = 1, m2 = 1, shift = 28;
};
template <typename T>
bool rt_scan_table(const T *roots, uint32_t k, RtScanSet &set, std::vector<T> &out, bool compact = false);
// the root-set scan with its set in the kernel arguments (decode.hip)
constexpr size_t RT_KTAB_BYTES = 2048;
struct RtKTab {
    uint64_t w[RT_KTAB_BYTES / 8];
};
template <typename T>
int launch_root_scan_k(qk_ctx *ctx, const std::vector<T> &tab, const RtScanSet &set, const T *log, size_t n,
                       int use_stop, T stop_value, uint64_t *hits, uint64_t cap, uint64_t *counters, uint64_t *hout,
                       uint64_t hbase, uint64_t sbase, uint64_t *done, uint64_t gen, hipStream_t s);
template <typename T>
int launch_root_scan(qk_ctx *ctx, const T *d_tab, const RtScanSet &set, const T *log, size_t n, int use_stop,
                     T stop_value, uint64_t *hits, uint64_t cap, uint64_t *counters, uint64_t *hout,
                     hipStream_t s);

// root test in two phases (api.hip): root_test_plan picks Horner or the
// root-set scan for (d, n) and, for the scan, finds the roots on the host and
// builds the set (once per call, shared by every shard of a sharded decode);
// root_test_begin enqueues on s; root_test_finish waits and collects the
// sorted hit positions (all of them) and the first stop position
template <typename T> struct RtPlan {
    bool scan = false;    // the root-set scan, writing its hits into pinned host slots (else Horner)
    RtScanSet set;
    std::vector<T> tab;   // the root set (scan)
};
template <typename T> int root_test_plan(const qk_ctx *ctx, const T *coeffs, uint32_t d, size_t n, RtPlan<T> &plan);
template <typename T>
int root_test_begin(qk_ctx *ctx, const RtPlan<T> &plan, const T *coeffs, uint32_t d, const T *d_log, size_t n,
                    int use_stop, T stop_value, hipStream_t s);
template <typename T>
int root_test_finish(qk_ctx *ctx, const RtPlan<T> &plan, const T *coeffs, uint32_t d, const T *d_log, size_t n,
                     int use_stop, T stop_value, hipStream_t s, std::vector<uint64_t> &hits, uint64_t &stop_index);

} // namespace qk
