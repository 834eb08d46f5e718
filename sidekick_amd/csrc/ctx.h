// ctx.h — internal: the device context behind qk_ctx* and launch helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>

#include "quack_hip.h"

// Measurement knobs (qk_ctx_set_knob; only tools/ and tests set them — the
// defaults below are the product's choices, each backed by a measurement in
// DESIGN.md).  Per context, so one process can compare variants.
struct qk_knobs {
    int bsgs_sg = -1;      // u32 BSGS: scalar-counted wrap groups (-1: the per-shape default)
    int u32_passes = 1;    // 0: u32 t > 80 on the power chain instead of BSGS passes
    int bsgs_shapes = 1;   // 0: the round-2 u32 BSGS shapes (t 17..36, 41..42, 65..72)
    int bsgs_prio = 1;     // 0: u32 BSGS without wave priority over the accumulation (bsgs.h Cfg PRIO 4)
    int grid_mult = 3;     // encode launches: resident workgroups x this (1: one round; grid_for, encode.hip)
    int u32_xcache = 1;    // 0: u32 offset passes raise x^8 to base/8 themselves (no per-id x^base cache)
    int bsgs64_sg = -1;    // u64 BSGS MAC mode override (-1: default)
    int bsgs64_off = 0;    // 1: u64 on the power chain instead of BSGS
    int bsgs64_shapes = 1; // 0: u64 t = 14..20, 25..28, 33..36 with 8 babies per id instead of 4
    int bsgs64_prio = 1;   // 0: u64 BSGS without s_setprio in the MAC step and without paired MACs (round 3)
    int bsgs64_tmin = 14;  // lowest u64 threshold on BSGS (below: the power chain; round 2: 21)
    int u64_passes = 1;    // 0: u64 t > 80 on the power chain instead of BSGS passes
    int u64_xcache = 1;    // 0: u64 offset passes raise x^8 to base/8 themselves (no per-id x^base cache)
    int u64_kmax = 40;     // u64 power chain: accumulators per lane
    int flow_load = 4;     // flow-table slots per expected flow
    int flow_wgpc = 12;    // flow extract: workgroups per CU
    int flow_hist = 32;    // batches of at most this many flows (and a table of <= 8192 slots) are grouped by
                           // per-workgroup slot histograms instead of the radix sort (0: never); 16 flows
                           // 2.76 vs 2.90 ms, 64: 3.17 vs 3.05, 1000: 5.80 vs 3.68 (profiles/r05/flows_hist/)
    int flow_sort = 2;     // grouping sort (radix.h, flows.hip rs_sort): 1: 8-bit digits, 256 threads, two arrays
                           // throughout; 2: pair arrays between the first and last pass; 3 / 4: 512 / 1024
                           // threads; 5 / 6: 11-bit digits, 512 / 1024 threads; 7-9: as 2, 5, 6 without LDS
                           // staging (direct scatter)
    int pkt_nt = 1;        // the packet-batch kernels: records read nontemporal (t = 32, 1e8 records:
                           // 1.83-1.84 -> 1.74-1.76 ms, profiles/r05/packets_nt/)
    int flow_nd = 1;       // 1: each radix scatter writes the next pass's digit bytes (count from them); 0: count from the pairs
    int flow_bail = 64;    // the flow extract stops on its own overflow, or on any (flag read every flow_bail-th tile); 0: never
    int flow_byslot = 0;   // grouping sort key: 0 by the pass-count rule, 1 slot, 2 flow rank (A/B)
    int flow_spec = 0;     // flow batches: the by-slot grouping sort launched before the host reads the
                           // extract's counters (16 / 1e4 / 1e6 flows: equal within 0.5 %,
                           // profiles/r05/flows_spec/: the launch gap it removes is not on the path)
    int flow_side_lo = 0;  // flow batches: the key-ranking branch on the lowest-priority stream (1e6 flows
                           // 5.92 vs 5.89 ms, 1e4 equal: no contention to speak of, profiles/r05/flows_side/)
    int flow_rs_nt = 1;    // grouping-sort scatters: bit 0 input read, bit 1 output written nontemporal
                           // (bit 0: 1e6 flows 6.16 -> 6.02 ms, 1e4 4.01 -> 3.89; bit 1: +15 %,
                           // profiles/r05/flows_nt/ab_rsnt.jsonl)
    int flow_nt = 1;       // k_flow_extract: records read / (slot, id) written nontemporal (1e6 flows
                           // 6.04 -> 5.93 ms, 16 flows 2.88 -> 2.81 ms, profiles/r05/flows_nt/)
    int flow_pipe = 0;     // 1: the flow extract reads its table one tile ahead (k_flow_extract_pipe: slower,
                           // 1e6 flows 7.14 vs 6.25 ms, 1e4 4.42 vs 4.11; profiles/r05/check4/ab_pipe.log)
    int flow_fuse0 = 1;    // 0: the grouping sort's first-digit counts by its own pass, not fused into the extract
                           // (1e6 flows 6.71 vs 6.61 ms, 1e4 4.46 vs 4.42; profiles/r05/check4/ab_fuse0.log)
    int flow_prio = 0;     // 1: per-flow encode kernels with s_setprio around the MACs (1e6 flows: 7.57 vs
                           // 6.80 ms, 16 / 1e4 flows even; profiles/r04/prio/ab_flows_prio.jsonl)
    int pkt_wgpc = 4;      // packet batches: workgroups per CU
    int pkt_fused = 1;     // 0: packet batches t 5..12 in two passes (extract, encode)
    int rt64_horner = 0;   // 1: u64 root test by Horner instead of baby-step/giant-step
    int root_test = 0;     // 0: automatic, 1: Horner, 2: root-set scan (decode.hip)
    int rt_scan_nt = 1;    // root-set scan: nontemporal 16-byte loads of the log (u32 kernel 72 -> 66 us,
                           // u64 135 -> 125 us at configs[4], profiles/r05/decode_nt/)
    int rt_scan_u = 1;     // root-set scan: 16-byte loads per lane per iteration (1, 2, 4; 3 runs as 2; 1: u32
                           // kernel 70 vs 84 / 78 us at 2 / 4, profiles/r04/decode_scan_u/)
    int rt_direct = 1;     // 0: the root-set scan's results by D2H copies instead of its host slots
    int comm_fault = 0;    // k > 0 (tests): this rank's payload staging for the k-th collective of its
                           // next sharded operation fails, once (comm.hip fault_now)
};

struct qk_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;      // own stream (host-input pipeline, comm collectives); a NULL
                                       // stream argument is the HIP null stream, not this one
    hipStream_t copy_stream = nullptr; // second stream for the host-input pipeline
    hipStream_t side_stream = nullptr; // lowest-priority stream: the flow batches' key-ranking branch
    uint32_t grid_override = 0;
    qk_knobs knobs;

    // scratch: block partials of the encode kernels, hit buffers of the root test
    void *d_scratch = nullptr;
    size_t scratch_bytes = 0;
    uint64_t *d_small = nullptr;       // partial output / hit counters (small, fixed)
    uint64_t *h_small = nullptr;       // pinned mirror of d_small
    uint64_t *h_small_dev = nullptr;   // h_small as the device addresses it
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
constexpr size_t SMALL_HITPF = 3076;   // h_small: the first hits
constexpr uint32_t RT_NSTOP = 16;      // stop slots of the direct form
constexpr size_t SMALL_STOPS = SMALL_WORDS - RT_NSTOP;
constexpr size_t SMALL_HITPF_N = SMALL_STOPS - SMALL_HITPF;
// the same slots relative to SMALL_NHITS (the kernel's hout)
constexpr size_t RT_STOP0 = SMALL_STOPS - SMALL_NHITS;

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
template <typename T> bool rt_scan_table(const T *roots, uint32_t k, RtScanSet &set, std::vector<T> &out);
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
    bool scan = false;
    bool direct = false;  // the scan writes its hits into pinned host slots (knob rt_direct, read once at plan time)
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
