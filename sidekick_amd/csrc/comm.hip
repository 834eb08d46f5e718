// comm.hip — multi-GPU sharding of the encode and decode paths over RCCL
// (xGMI), behind the C ABI (include/quack_hip.h "Multi-GPU").
//
// The sketch is additive, so one stream cut into contiguous shards (one per
// GPU, in global rank order) encodes shard by shard and the partial vectors
// are summed.  Per sharded encode:
//   each local rank   encode its shard into its payload buffer (the
//                     ordinary encode kernel + finalize), then k_comm_pack
//                     turns [S.., n, last] into [S.., n, slots, failed]:
//                     slot r = (has_last, last) of rank r, zero elsewhere;
//                     failed = 1 on a rank whose local work failed (its
//                     payload is otherwise zero: it still joins the reduce)
//   ONE ncclReduce    (sum, uint64) of the payload to the root rank:
//                     the summed power-sum words cannot overflow (canonical
//                     residues / 32-bit limbs, < 2^27 ranks), the count word
//                     sums the shard sizes, every slot has exactly one
//                     contributor, and the last word counts failed ranks
//   root              nonzero failed count -> QK_E_PEER, q untouched; else
//                     fold mod p, count mod 2^32, last_value = the last id of
//                     the highest non-empty rank
// Payload at t = 32 on 8 GPUs: 33 + 16 + 1 words = 400 B — latency-bound; the
// xGMI bandwidth is irrelevant.
//
// Sharded decode (the log cut the same way):
//   ncclBroadcast     [status, d, stop flag, stop value, c_1..c_d] from the
//                     root, which ran to_coeffs (host, O(t^2))
//   each local rank   the root test over its log shard (api.hip phases, all
//                     local GPUs in flight at once)
//   ncclAllGather     (n, first stop position, hits below it, status) per rank
//   ncclAllGather     the hit positions (+ shard base), padded, in chunks of
//                     a fixed size; every rank cuts at the global stop
// so every rank returns the single-GPU answer for the whole log.
//
// Collective safety (one process per GPU: a rank that returned early would
// leave its peers blocked in the next collective forever).  Every rank enters
// every collective of an operation; the only early returns precede the first
// collective and test arguments every rank passes alike by contract
// (threshold, root).  A local failure travels as data — the failed word of
// the encode payload, the status word of every decode exchange — and the
// gathered statuses decide, identically on every rank, whether a further
// collective runs: a rank that fails to stage its payload (the local copy
// into the collective buffer) sends the failure marker instead and keeps
// joining.  No buffer is allocated between collectives (the payload buffer is
// sized for the largest operation at init; hits travel in fixed-size chunks).
// A collective that fails, or a rank that cannot read what a collective
// delivered (so cannot follow the rest of the protocol), marks the
// communicator broken: its RCCL communicators are aborted (ncclCommAbort) and
// every later call returns QK_E_COMM.  An abort releases only this process's
// ranks: peers in other processes are released by their own timeout — every
// wait on an RCCL collective polls ncclCommGetAsyncError and gives up after
// the communicator's timeout (qk_comm_set_timeout, default 300 s), aborting
// in turn; a host channel's callbacks carry their own timeout.
// Collectives go through RCCL (device buffers, the context's stream) or,
// for a communicator made by qk_comm_init_host, through the caller's host
// callbacks on the pinned mirror of the payload buffer: the same protocol
// with a host channel (several ranks rehearsed on one GPU — RCCL refuses two
// ranks on one device — or ranks RCCL cannot connect).
//
// Streams: each local rank's work runs on its qk_ctx's own stream, ordered
// after the caller's stream (event) and, for the async encode, with the
// caller's stream ordered after it again.
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <thread>
#include <rccl/rccl.h>
#include <vector>

#include "ctx.h"
#include "field.h"

#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

static_assert(sizeof(ncclUniqueId) == QK_COMM_ID_BYTES, "unique id size");

struct qk_comm {
    struct Local {
        int rank = 0, device = 0;
        qk_ctx *ctx = nullptr;
        ncclComm_t nc = nullptr;
        uint64_t *d_coll = nullptr;   // collective payload (device), coll_cap(world) words
        uint64_t *h_coll = nullptr;   // pinned host mirror
        hipEvent_t ev_in = nullptr, ev_out = nullptr;
        hipEvent_t ev_pre = nullptr;  // the local work before the RCCL collective in flight
        bool pre = false;             // ev_pre recorded and not yet waited on
        hipStream_t user = nullptr;   // caller stream of the operation in flight
    };
    int world = 1;
    std::vector<Local> local;
    bool host = false;                // collectives through ops (qk_comm_init_host)
    qk_comm_host_ops ops{};
    bool broken = false;              // a collective failed: unusable
    bool abort_pending = false;       // broken by local work that outlasted its limit: abort at destroy
    int64_t timeout_ms = 300000;      // waits on RCCL collectives give up (and abort) after this; 0: never
    int step = 0;                     // collectives of the operation in progress (fault injection)
    // sharded encode in flight (qk_*_encode_sharded_async -> _wait)
    int pend_bits = 0;
    uint32_t pend_t = 0;
    int pend_root = -1;
    int pend_rc = QK_OK;              // local / collective status of the async half
    std::mutex mu;
};

namespace qk {

QK_WARM_KERNEL(comm)

using Local = qk_comm::Local;

// Words of every payload buffer: the largest encode payload, the decode
// header, the decode status gather, and hit chunks of >= 64 positions per rank.
static size_t coll_cap(int world) {
    const size_t W = (size_t)world;
    size_t c = 8192;
    c = std::max(c, 2 * (size_t)QK_MAX_THRESHOLD + 1 + 2 * W + 1);
    c = std::max(c, 4 + (size_t)QK_MAX_THRESHOLD);
    c = std::max(c, 4 + 4 * W);
    c = std::max(c, 64 * (W + 1));
    return c;
}

// summed words of the partial vector
static size_t reduce_words(int bits, uint32_t t) { return bits == 32 ? (size_t)t + 1 : 2 * (size_t)t + 1; }

// [S.., n, last] -> [S.., n, slot_0 .. slot_{world-1}, failed = 0]
// (R = the summed words, n at R - 1, last at R; slot = (has_last, last))
__global__ void k_comm_pack(uint64_t *buf, uint32_t R, uint32_t world, uint32_t rank) {
    const uint64_t n = buf[R - 1], last = buf[R];
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < 2 * world + 1; j += blockDim.x) buf[R + j] = 0;
    __syncthreads();
    if (threadIdx.x == 0 && n) {
        buf[R + 2 * rank] = 1;
        buf[R + 2 * rank + 1] = last;
    }
}

// the payload of a rank whose local work failed: zeros, failed = 1
__global__ void k_comm_fail(uint64_t *buf, uint32_t words) {
    for (uint32_t j = threadIdx.x; j < words; j += blockDim.x) buf[j] = j + 1 == words ? 1 : 0;
}

static int init_local(Local &L, int device, int world) {
    L.device = device;
    if (int rc = qk_ctx_create(device, &L.ctx)) return rc;
    QK_HIP_TRY(hipSetDevice(device));
    QK_HIP_TRY(hipEventCreateWithFlags(&L.ev_in, hipEventDisableTiming));
    QK_HIP_TRY(hipEventCreateWithFlags(&L.ev_out, hipEventDisableTiming));
    QK_HIP_TRY(hipEventCreateWithFlags(&L.ev_pre, hipEventDisableTiming));
    const size_t w = coll_cap(world);
    if (hipMalloc(&L.d_coll, w * 8) != hipSuccess) return QK_E_NOMEM;
    if (hipHostMalloc(&L.h_coll, w * 8, hipHostMallocDefault) != hipSuccess) return QK_E_NOMEM;
    return QK_OK;
}

enum class Op { Bcast, Gather };

// a rank's failure marker in a decode exchange payload: the status word
__global__ void k_comm_mark(uint64_t *buf, uint32_t idx, uint64_t value) {
    if (threadIdx.x == 0) buf[idx] = value;
}

// order the local rank's stream after the caller's stream
static int enter(Local &L) {
    QK_HIP_TRY(hipSetDevice(L.device));
    QK_HIP_TRY(hipEventRecord(L.ev_in, L.user));
    QK_HIP_TRY(hipStreamWaitEvent(L.ctx->stream, L.ev_in, 0));
    return QK_OK;
}
// and the caller's stream after the local rank's work
static int leave(Local &L) {
    QK_HIP_TRY(hipSetDevice(L.device));
    QK_HIP_TRY(hipEventRecord(L.ev_out, L.ctx->stream));
    QK_HIP_TRY(hipStreamWaitEvent(L.user, L.ev_out, 0));
    return QK_OK;
}

static int abort_comm(qk_comm *c) {
    c->broken = true;
    for (auto &L : c->local)
        if (L.nc) {
            ncclCommAbort(L.nc);
            L.nc = nullptr;
        }
    return QK_E_COMM;
}

// Test knob comm_delay_ms = k on a local rank's context: a one-wave kernel
// that spins k ms (s_memrealtime, 100 MHz; s_sleep between reads) is put in
// front of that rank's next collective, once — slow or hung local work
// before a collective (wait_local's bounded pre-collective wait).
__global__ void k_comm_delay(uint64_t ticks) {
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - r0 < ticks) __builtin_amdgcn_s_sleep(64);
}

// Mark the end of a local rank's own work (its encode, the caller's work
// ordered in by enter, the payload staging) just before an RCCL collective.
static void mark_pre(Local &L) {
    (void)hipSetDevice(L.device);
    int &dl = L.ctx->knobs.comm_delay_ms;
    if (dl > 0) {
        hipLaunchKernelGGL(k_comm_delay, dim3(1), dim3(64), 0, L.ctx->stream, (uint64_t)dl * 100000ull);
        (void)hipGetLastError();
        dl = 0;
    }
    L.pre = hipEventRecord(L.ev_pre, L.ctx->stream) == hipSuccess;
}

// Poll until `done` reports completion; every poll also reads the
// communicator's asynchronous error.  On an asynchronous error, or past
// limit_ms (0: none) with abort_late, the communicator is aborted: QK_E_COMM.
// Past the limit without abort_late it is only marked broken (QK_E_COMM,
// every later call fails at once) and aborted by qk_comm_destroy: RCCL's
// abort frees its buffers, and hipFree waits for the device — here, for the
// very local work that outlasted the limit.
template <class Done> static int poll_bounded(qk_comm *c, Local &L, int64_t limit_ms, bool abort_late, Done done) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0;; ++spin) {
        const hipError_t q = done();
        if (q == hipSuccess) return QK_OK;
        if (q != hipErrorNotReady) return QK_E_HIP;
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(L.nc, &ae) != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress))
            return abort_comm(c);
        if (limit_ms > 0 &&
            std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count() >
                limit_ms) {
            if (abort_late) return abort_comm(c);
            c->broken = true;
            c->abort_pending = true;
            return QK_E_COMM;
        }
        if (spin >= 256) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// Drain the local rank's stream.  With RCCL work in it, the wait polls the
// communicator's asynchronous error and gives up after the timeout (a peer
// that never reaches the collective): the communicator is aborted, QK_E_COMM.
// The local work recorded before the collective (mark_pre) is waited for
// first under its own, longer limit — PRE_TIMEOUT_MULT x the timeout: slow
// local work is not a missing peer, but local work that never ends (a hung
// kernel, a caller stream waiting on an event that never fires) must not
// hang the rank either.
constexpr int64_t PRE_TIMEOUT_MULT = 4;
static int wait_local(qk_comm *c, Local &L) {
    QK_HIP_TRY(hipSetDevice(L.device));
    if (c->host || !L.nc) {
        QK_HIP_TRY(hipStreamSynchronize(L.ctx->stream));
        return QK_OK;
    }
    if (L.pre) {
        L.pre = false;
        if (int rc = poll_bounded(c, L, c->timeout_ms * PRE_TIMEOUT_MULT, false,
                                  [&] { return hipEventQuery(L.ev_pre); }))
            return rc;
    }
    return poll_bounded(c, L, c->timeout_ms, true, [&] { return hipStreamQuery(L.ctx->stream); });
}

// Test knob comm_fault = k on a local rank's context (qk_ctx_set_knob): the
// staging of that rank's payload for the k-th collective of its next
// operation fails, once — the path a failed local copy takes.
static bool fault_now(qk_comm *c, Local &L) {
    int &k = L.ctx->knobs.comm_fault;
    if (k > 0 && k == c->step) {
        k = 0;
        return true;
    }
    return false;
}

// Sum-reduce of d_coll[0..w) to the root (the encode payload; the barrier's
// one word).  A rank whose payload cannot be staged (host channel: the copy
// to the pinned mirror) sends the failed payload instead — zeros, last word 1
// (k_comm_fail's layout) — and reports the error in lerr[i].  The result is
// in the root's d_coll (RCCL) or h_coll (host channel).  Returns QK_E_COMM
// when the collective itself fails (the communicator is then broken).
static int reduce_payload(qk_comm *c, size_t w, int root, std::vector<int> &lerr) {
    if (c->broken) return QK_E_COMM;
    ++c->step;
    if (c->host) {
        Local &L = c->local[0];
        hipStream_t s = L.ctx->stream;
        if (fault_now(c, L) || hipSetDevice(L.device) != hipSuccess ||
            hipMemcpyAsync(L.h_coll, L.d_coll, w * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            memset(L.h_coll, 0, w * 8);   // still take part: the peers are in the collective
            L.h_coll[w - 1] = 1;
            if (!lerr[0]) lerr[0] = QK_E_HIP;
        }
        if (c->ops.reduce_sum_u64(c->ops.user, L.h_coll, w, root) != 0) {
            c->broken = true;
            return QK_E_COMM;
        }
        return QK_OK;
    }
    for (size_t i = 0; i < c->local.size(); ++i) {
        Local &L = c->local[i];
        if (fault_now(c, L)) {
            (void)hipSetDevice(L.device);
            hipLaunchKernelGGL(k_comm_fail, dim3(1), dim3(256), 0, L.ctx->stream, L.d_coll, (uint32_t)w);
            (void)hipGetLastError();
            if (!lerr[i]) lerr[i] = QK_E_HIP;
        }
    }
    for (auto &L : c->local) mark_pre(L);
    bool ok = ncclGroupStart() == ncclSuccess;
    for (auto &L : c->local) {
        if (!ok) break;
        ok = ncclReduce(L.d_coll, L.d_coll, w, ncclUint64, ncclSum, root, L.nc, L.ctx->stream) == ncclSuccess;
    }
    if (ncclGroupEnd() != ncclSuccess) ok = false;
    return ok ? QK_OK : abort_comm(c);
}

// Broadcast / all-gather of host payloads (the decode's exchanges): every
// local rank's h_coll[0..w) is sent; a broadcast delivers the root's into
// h_coll[0..w), an all-gather rank r's into h_coll[w + r*w .. w + (r+1)*w).
// Word `sidx` of a payload is its rank's status: a rank whose payload cannot
// be staged (RCCL: the copy to the device buffer) sends QK_E_HIP there
// (k_comm_mark) and records it in ls[i] — it keeps joining.  A rank that
// cannot read what the collective delivered cannot follow the rest of the
// protocol: the communicator is broken (abort; peers are released by their
// own timeout).  Returns QK_OK or QK_E_COMM.
static int exchange(qk_comm *c, Op op, size_t w, int root, size_t sidx, std::vector<int> &ls) {
    if (c->broken) return QK_E_COMM;
    ++c->step;
    if (c->host) {
        Local &L = c->local[0];
        if (fault_now(c, L)) {
            L.h_coll[sidx] = (uint64_t)(int64_t)QK_E_HIP;
            if (!ls[0]) ls[0] = QK_E_HIP;
        }
        const int cb = op == Op::Bcast ? c->ops.broadcast_u64(c->ops.user, L.h_coll, w, root)
                                       : c->ops.allgather_u64(c->ops.user, L.h_coll, L.h_coll + w, w);
        if (cb != 0) {
            c->broken = true;
            return QK_E_COMM;
        }
        return QK_OK;
    }
    for (size_t i = 0; i < c->local.size(); ++i) {
        Local &L = c->local[i];
        (void)hipSetDevice(L.device);
        if (fault_now(c, L) ||
            hipMemcpyAsync(L.d_coll, L.h_coll, w * 8, hipMemcpyHostToDevice, L.ctx->stream) != hipSuccess) {
            hipLaunchKernelGGL(k_comm_mark, dim3(1), dim3(64), 0, L.ctx->stream, L.d_coll, (uint32_t)sidx,
                               (uint64_t)(int64_t)QK_E_HIP);
            (void)hipGetLastError();
            if (!ls[i]) ls[i] = QK_E_HIP;
        }
    }
    for (auto &L : c->local) mark_pre(L);
    bool ok = ncclGroupStart() == ncclSuccess;
    for (auto &L : c->local) {
        if (!ok) break;
        const ncclResult_t r = op == Op::Bcast
                                   ? ncclBroadcast(L.d_coll, L.d_coll, w, ncclUint64, root, L.nc, L.ctx->stream)
                                   : ncclAllGather(L.d_coll, L.d_coll + w, w, ncclUint64, L.nc, L.ctx->stream);
        ok = r == ncclSuccess;
    }
    if (ncclGroupEnd() != ncclSuccess) ok = false;
    if (!ok) return abort_comm(c);
    const size_t off = op == Op::Gather ? w : 0, words = op == Op::Gather ? w * (size_t)c->world : w;
    for (auto &L : c->local) {
        (void)hipSetDevice(L.device);
        if (hipMemcpyAsync(L.h_coll + off, L.d_coll + off, words * 8, hipMemcpyDeviceToHost, L.ctx->stream) !=
            hipSuccess)
            return abort_comm(c);
    }
    for (auto &L : c->local)
        if (int e = wait_local(c, L)) return e == QK_E_COMM ? e : abort_comm(c);
    return QK_OK;
}

template <int BITS>
static int encode_sharded_async(qk_comm *c, const void *const *d_ids, const size_t *n, uint32_t t, int root,
                                void *const *streams) {
    if (c->broken) return QK_E_COMM;
    // arguments every rank passes alike (the collective contract): failing
    // them returns before any collective, on every rank
    if (t == 0 || t > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if (root < 0 || root >= c->world) return QK_E_INVAL;
    c->step = 0;
    const size_t esz = BITS == 32 ? 4 : 8;
    const size_t R = reduce_words(BITS, t), W = R + 2 * (size_t)c->world + 1;
    // per-rank arguments and local work: a failure still joins the reduce,
    // with the failed payload
    std::vector<int> lerr(c->local.size(), QK_OK);
    for (size_t i = 0; i < c->local.size(); ++i) {
        Local &L = c->local[i];
        L.user = streams ? (hipStream_t)streams[i] : nullptr;
        int e = QK_OK;
        if (!d_ids || !n) {
            e = QK_E_INVAL;
        } else if (n[i] && (!d_ids[i] || ((uintptr_t)d_ids[i] & (esz - 1)) || n[i] >= (1ull << 40) ||
                            !is_device_ptr(d_ids[i]))) {
            e = QK_E_INVAL;
        }
        if (!e) e = enter(L);
        if (!e) {
            std::lock_guard<std::mutex> g(L.ctx->mu);
            e = BITS == 32 ? launch_encode_u32(L.ctx, (const uint32_t *)d_ids[i], n[i], t, L.d_coll, L.ctx->stream)
                           : launch_encode_u64(L.ctx, (const uint64_t *)d_ids[i], n[i], t, L.d_coll, L.ctx->stream);
        }
        if (!e) {
            hipLaunchKernelGGL(k_comm_pack, dim3(1), dim3(64), 0, L.ctx->stream, L.d_coll, (uint32_t)R,
                               (uint32_t)c->world, (uint32_t)L.rank);
            if (hipGetLastError() != hipSuccess) e = QK_E_HIP;
        }
        if (e) {
            (void)hipSetDevice(L.device);
            hipLaunchKernelGGL(k_comm_fail, dim3(1), dim3(256), 0, L.ctx->stream, L.d_coll, (uint32_t)W);
            (void)hipGetLastError();
            lerr[i] = e;
        }
    }
    const int crc = reduce_payload(c, W, root, lerr);
    int rc = QK_OK;
    for (size_t i = 0; i < c->local.size(); ++i) {
        Local &L = c->local[i];
        if (lerr[i] && !rc) rc = lerr[i];
        (void)hipSetDevice(L.device);
        // the root's sum to its pinned mirror (a host channel left it there)
        if (!crc && !c->host && L.rank == root &&
            hipMemcpyAsync(L.h_coll, L.d_coll, W * 8, hipMemcpyDeviceToHost, L.ctx->stream) != hipSuccess && !rc)
            rc = QK_E_HIP;
        if (int e = leave(L); e && !rc) rc = e;
    }
    c->pend_bits = BITS;
    c->pend_t = t;
    c->pend_root = root;
    c->pend_rc = crc ? crc : rc;
    return c->pend_rc;
}

template <int BITS, typename Q>
static int encode_sharded_wait(qk_comm *c, Q *q) {
    if (c->pend_bits != BITS) return QK_E_INVAL;   // nothing in flight for this id width
    const uint32_t t = c->pend_t;
    const int root = c->pend_root, prc = c->pend_rc;
    c->pend_bits = 0;
    int rc = QK_OK;
    for (auto &L : c->local)
        if (int e = wait_local(c, L); e && !rc) rc = e;
    if (prc) return prc;                           // q untouched
    if (rc) return rc;
    for (auto &L : c->local) {
        if (L.rank != root) continue;
        if (!q) return QK_E_INVAL;
        if (q->threshold != t) return QK_E_MISMATCH;
        const size_t R = reduce_words(BITS, t);
        const uint64_t *h = L.h_coll;
        if (h[R + 2 * (size_t)c->world]) return QK_E_PEER;   // a rank failed: q untouched
        int has = 0;
        uint64_t last = 0;
        for (int r = c->world - 1; r >= 0; --r)
            if (h[R + 2 * r]) {
                has = 1;
                last = h[R + 2 * r + 1];
                break;
            }
        if constexpr (BITS == 32) return qk_u32_merge_partial(q, h, has, (uint32_t)last);
        else return qk_u64_merge_partial(q, h, has, last);
    }
    return QK_OK;   // not the root: q is untouched
}

// the lowest failing rank's status among W gathered payloads of `w` words
// with the status at word sidx (0 if none failed) — the same on every rank
static int gathered_status(const uint64_t *g, size_t W, size_t w, size_t sidx) {
    for (size_t r = 0; r < W; ++r)
        if (g[r * w + sidx]) return (int)(int64_t)g[r * w + sidx];
    return QK_OK;
}

template <typename T, typename Q>
static int decode_sharded(qk_comm *c, const Q *diff, int root, const T *const *d_log, const size_t *n,
                          int stop_at_last, uint64_t *hits, size_t cap, size_t *n_hits, void *const *streams) {
    if (c->broken) return QK_E_COMM;
    if (root < 0 || root >= c->world) return QK_E_INVAL;   // alike on every rank
    c->step = 0;
    if (n_hits) *n_hits = 0;
    const size_t nl = c->local.size(), W = (size_t)c->world, B = 4 + QK_MAX_THRESHOLD;
    // local status per local rank: travels in the status word of every exchange
    std::vector<int> ls(nl, QK_OK);
    for (size_t i = 0; i < nl; ++i) {
        Local &L = c->local[i];
        L.user = streams ? (hipStream_t)streams[i] : nullptr;
        if (!d_log || !n || !n_hits) ls[i] = QK_E_INVAL;
        else if (n[i] && (!d_log[i] || ((uintptr_t)d_log[i] & (sizeof(T) - 1)) || !is_device_ptr(d_log[i])))
            ls[i] = QK_E_INVAL;
        if (int e = enter(L); e && !ls[i]) ls[i] = e;
    }
    auto finish = [&](int status) {
        int rc = status;
        for (auto &L : c->local)
            if (int e = leave(L); e && !rc) rc = e;
        return rc;
    };

    // 1. [status, d, stop flag, stop value, c_1..c_d] from the root
    for (size_t i = 0; i < nl; ++i) {
        Local &L = c->local[i];
        uint64_t *h = L.h_coll;
        memset(h, 0, B * 8);
        if (L.rank != root) continue;
        int64_t status = ls[i];
        uint32_t d = 0;
        if (!status && !diff) status = QK_E_INVAL;
        if (!status && diff->count != 0) {
            std::vector<T> cf(std::max<uint32_t>(diff->threshold, 1));
            if constexpr (sizeof(T) == 4) status = qk_u32_to_coeffs(diff, cf.data(), (uint32_t)cf.size(), &d);
            else status = qk_u64_to_coeffs(diff, cf.data(), (uint32_t)cf.size(), &d);
            if (status == QK_OK && d > QK_MAX_THRESHOLD) status = QK_E_THRESHOLD;
            if (status == QK_OK)
                for (uint32_t k = 0; k < d; ++k) h[4 + k] = (uint64_t)cf[k];
        }
        h[0] = (uint64_t)status;
        h[1] = status == QK_OK ? d : 0;
        h[2] = !status && stop_at_last && diff->has_last ? 1 : 0;
        h[3] = !status ? (uint64_t)diff->last_value : 0;
    }
    if (int e = exchange(c, Op::Bcast, B, root, 0, ls)) return finish(e);
    std::vector<std::vector<uint64_t>> hdr(nl);
    for (size_t i = 0; i < nl; ++i) {
        hdr[i].assign(c->local[i].h_coll, c->local[i].h_coll + B);
        if (!ls[i] && hdr[i][0]) ls[i] = (int)(int64_t)hdr[i][0];   // the root's status
    }

    // 2. root test of every local shard, all GPUs in flight; the plan (the
    //    host roots for the root-set scan) once per call for every local rank
    std::vector<std::vector<uint64_t>> lh(nl);
    std::vector<uint64_t> lstop(nl, 0);
    std::vector<char> began(nl, 0);
    std::vector<T> coeffs;
    RtPlan<T> plan;
    uint32_t d = 0;
    int use_stop = 0;
    T stop_value = 0;
    {
        size_t first = nl, nmax = 0;
        for (size_t i = 0; i < nl; ++i)
            if (!ls[i]) {
                if (first == nl) first = i;
                nmax = std::max(nmax, n[i]);
            }
        if (first < nl) {   // every local rank holds the same broadcast header
            const uint64_t *hd = hdr[first].data();
            d = (uint32_t)std::min<uint64_t>(hd[1], QK_MAX_THRESHOLD);
            use_stop = (int)hd[2];
            stop_value = (T)hd[3];
            coeffs.assign(std::max<uint32_t>(d, 1), 0);
            for (uint32_t k = 0; k < d; ++k) coeffs[k] = (T)hd[4 + k];
            if (d > 0 && nmax)
                if (int e = root_test_plan<T>(c->local[first].ctx, coeffs.data(), d, nmax, plan))
                    for (size_t i = 0; i < nl; ++i)
                        if (!ls[i]) ls[i] = e;
        }
    }
    for (size_t i = 0; i < nl; ++i) {
        Local &L = c->local[i];
        lstop[i] = n ? n[i] : 0;
        if (ls[i]) continue;
        if (!(d > 0 || use_stop) || !n[i]) continue;
        std::lock_guard<std::mutex> g(L.ctx->mu);
        if (hipSetDevice(L.device) != hipSuccess) {
            ls[i] = QK_E_HIP;
            continue;
        }
        if (int e = root_test_begin<T>(L.ctx, plan, coeffs.data(), d, d_log[i], n[i], use_stop, stop_value,
                                       L.ctx->stream))
            ls[i] = e;
        else
            began[i] = 1;
    }
    for (size_t i = 0; i < nl; ++i) {
        if (!began[i]) continue;
        Local &L = c->local[i];
        std::lock_guard<std::mutex> g(L.ctx->mu);
        (void)hipSetDevice(L.device);
        if (int e = root_test_finish<T>(L.ctx, plan, coeffs.data(), d, d_log[i], n[i], use_stop, stop_value,
                                        L.ctx->stream, lh[i], lstop[i])) {
            ls[i] = e;
            lh[i].clear();
            continue;
        }
        // hits at or past this shard's own stop are past the global one too
        lh[i].resize((size_t)(std::lower_bound(lh[i].begin(), lh[i].end(), lstop[i]) - lh[i].begin()));
    }

    // 3. (n, stop, hits, status) of every rank
    for (size_t i = 0; i < nl; ++i) {
        uint64_t *h = c->local[i].h_coll;
        h[0] = ls[i] ? 0 : n[i];
        h[1] = ls[i] ? 0 : lstop[i];
        h[2] = ls[i] ? 0 : lh[i].size();
        h[3] = (uint64_t)(int64_t)ls[i];
    }
    if (int e = exchange(c, Op::Gather, 4, root, 3, ls)) return finish(e);
    // every local rank received the same words
    const uint64_t *m = c->local[0].h_coll + 4;
    int gstatus = gathered_status(m, W, 4, 3);
    if (gstatus) return finish(gstatus);
    std::vector<uint64_t> base(W + 1, 0), cnt(W, 0);
    uint64_t gstop = UINT64_MAX, M = 0;
    for (size_t r = 0; r < W; ++r) {
        base[r + 1] = base[r] + m[4 * r];
        if (m[4 * r + 1] < m[4 * r]) gstop = std::min(gstop, base[r] + m[4 * r + 1]);
        cnt[r] = m[4 * r + 2];
    }
    for (size_t r = 0; r < W; ++r) {
        if (base[r] >= gstop) cnt[r] = 0;   // wholly past the global stop
        M = std::max(M, cnt[r]);
    }

    // 4. the hit positions, in rounds of C per rank (padded) plus the rank's
    //    status word; C fixed by the payload capacity: no allocation between
    //    collectives.  Every rank joins all rounds (M is known to all); a
    //    failure in a round travels in its status word.
    std::vector<uint64_t> all;
    const size_t C = coll_cap(c->world) / (W + 1) - 1, w = C + 1;
    for (uint64_t off = 0; off < M; off += C) {
        for (size_t i = 0; i < nl; ++i) {
            Local &L = c->local[i];
            uint64_t *h = L.h_coll;
            const uint64_t b = base[L.rank];
            for (size_t k = 0; k < C; ++k) {
                const size_t j = (size_t)off + k;
                h[k] = j < lh[i].size() && j < cnt[L.rank] ? b + lh[i][j] : UINT64_MAX;
            }
            h[C] = (uint64_t)(int64_t)ls[i];
        }
        if (int e = exchange(c, Op::Gather, w, root, C, ls)) return finish(e);
        const uint64_t *g = c->local[0].h_coll + w;
        if (!gstatus) gstatus = gathered_status(g, W, w, C);
        if (gstatus) continue;   // keep joining the remaining rounds
        for (size_t r = 0; r < W; ++r)
            for (size_t k = 0; k < C && off + k < cnt[r]; ++k) {
                const uint64_t p = g[r * w + k];
                if (p < gstop) all.push_back(p);
            }
    }
    if (int e = finish(gstatus)) return e;
    std::sort(all.begin(), all.end());   // rounds arrive rank-major: restore log order
    *n_hits = all.size();
    if (all.size() > cap || (!all.empty() && !hits)) return QK_E_CAPACITY;
    std::copy(all.begin(), all.end(), hits);
    return QK_OK;
}

static void destroy_local(Local &L) {
    if (L.ctx) (void)hipSetDevice(L.device);
    if (L.nc) ncclCommDestroy(L.nc);
    if (L.d_coll) hipFree(L.d_coll);
    if (L.h_coll) hipHostFree(L.h_coll);
    if (L.ev_in) hipEventDestroy(L.ev_in);
    if (L.ev_out) hipEventDestroy(L.ev_out);
    if (L.ev_pre) hipEventDestroy(L.ev_pre);
    if (L.ctx) qk_ctx_destroy(L.ctx);
    L = Local{};
}

} // namespace qk

using namespace qk;

extern "C" {

int qk_comm_unique_id(uint8_t id[QK_COMM_ID_BYTES]) {
    if (!id) return QK_E_INVAL;
    int n = 0;
    if (qk_device_count(&n) != QK_OK) return QK_E_NO_DEVICE;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return QK_E_COMM;
    memcpy(id, &u, sizeof(u));
    return QK_OK;
}

int qk_comm_create(int ndev, const int *devices, qk_comm **out) {
    if (!out || ndev < 1 || !devices) return QK_E_INVAL;
    *out = nullptr;
    for (int i = 0; i < ndev; ++i)
        for (int j = 0; j < i; ++j)
            if (devices[i] == devices[j]) return QK_E_INVAL;   // one rank per GPU
    qk_comm *c = new (std::nothrow) qk_comm();
    if (!c) return QK_E_NOMEM;
    c->world = ndev;
    c->local.resize(ndev);
    for (int i = 0; i < ndev; ++i) {
        c->local[i].rank = i;
        if (int rc = init_local(c->local[i], devices[i], ndev)) {
            qk_comm_destroy(c);
            return rc;
        }
    }
    std::vector<ncclComm_t> nc(ndev, nullptr);
    if (ncclCommInitAll(nc.data(), ndev, devices) != ncclSuccess) {
        qk_comm_destroy(c);
        return QK_E_COMM;
    }
    for (int i = 0; i < ndev; ++i) c->local[i].nc = nc[i];
    *out = c;
    return QK_OK;
}

int qk_comm_init_rank(const uint8_t id[QK_COMM_ID_BYTES], int rank, int world, int device, qk_comm **out) {
    if (!out || !id || world < 1 || rank < 0 || rank >= world) return QK_E_INVAL;
    *out = nullptr;
    qk_comm *c = new (std::nothrow) qk_comm();
    if (!c) return QK_E_NOMEM;
    c->world = world;
    c->local.resize(1);
    c->local[0].rank = rank;
    if (int rc = init_local(c->local[0], device, world)) {
        qk_comm_destroy(c);
        return rc;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&c->local[0].nc, world, u, rank) != ncclSuccess) {
        c->local[0].nc = nullptr;
        qk_comm_destroy(c);
        return QK_E_COMM;
    }
    *out = c;
    return QK_OK;
}

int qk_comm_init_host(const qk_comm_host_ops *ops, int rank, int world, int device, qk_comm **out) {
    if (!out || !ops || !ops->reduce_sum_u64 || !ops->broadcast_u64 || !ops->allgather_u64 || world < 1 ||
        rank < 0 || rank >= world)
        return QK_E_INVAL;
    *out = nullptr;
    qk_comm *c = new (std::nothrow) qk_comm();
    if (!c) return QK_E_NOMEM;
    c->world = world;
    c->host = true;
    c->ops = *ops;
    c->local.resize(1);
    c->local[0].rank = rank;
    if (int rc = init_local(c->local[0], device, world)) {
        qk_comm_destroy(c);
        return rc;
    }
    *out = c;
    return QK_OK;
}

void qk_comm_destroy(qk_comm *comm) {
    if (!comm) return;
    if (comm->abort_pending) {
        // the collective never started (its local work outlasted the limit):
        // abort now — this waits until that local work has drained (hipFree)
        for (auto &L : comm->local)
            if (L.nc) {
                (void)hipSetDevice(L.device);
                ncclCommAbort(L.nc);
                L.nc = nullptr;
            }
    }
    for (auto &L : comm->local)
        if (L.ctx) (void)wait_local(comm, L);   // (a peer that never arrives: the timeout aborts)
    for (auto &L : comm->local) destroy_local(L);
    delete comm;
}

int qk_comm_info(const qk_comm *comm, int *world, int *nlocal, int *first_rank) {
    if (!comm) return QK_E_INVAL;
    if (world) *world = comm->world;
    if (nlocal) *nlocal = (int)comm->local.size();
    if (first_rank) *first_rank = comm->local.empty() ? 0 : comm->local[0].rank;
    return QK_OK;
}

int qk_comm_context(qk_comm *comm, int local, qk_ctx **out) {
    if (!comm || !out || local < 0 || local >= (int)comm->local.size()) return QK_E_INVAL;
    *out = comm->local[local].ctx;
    return QK_OK;
}

int qk_comm_barrier(qk_comm *comm) {
    if (!comm) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    if (comm->broken) return QK_E_COMM;
    comm->step = 0;
    std::vector<int> lerr(comm->local.size(), QK_OK);
    for (size_t i = 0; i < comm->local.size(); ++i) {
        Local &L = comm->local[i];
        (void)hipSetDevice(L.device);
        if (hipMemsetAsync(L.d_coll, 0, 8, L.ctx->stream) != hipSuccess) lerr[i] = QK_E_HIP;
    }
    if (int e = reduce_payload(comm, 1, 0, lerr)) return e;
    int rc = QK_OK;
    for (size_t i = 0; i < comm->local.size(); ++i) {
        if (lerr[i] && !rc) rc = lerr[i];
        if (int e = wait_local(comm, comm->local[i]); e && !rc) rc = e;
    }
    return rc;
}

int qk_comm_set_timeout(qk_comm *comm, int64_t ms) {
    if (!comm || ms < 0) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    comm->timeout_ms = ms;
    return QK_OK;
}

int qk_comm_rccl_info(const qk_comm *comm, int local, int *count, int *device, int *rank) {
    if (!comm || local < 0 || local >= (int)comm->local.size()) return QK_E_INVAL;
    const Local &L = comm->local[local];
    if (comm->host || !L.nc) return QK_E_INVAL;   // no RCCL communicator (host channel, or aborted)
    int k = 0, d = 0, r = 0;
    if (ncclCommCount(L.nc, &k) != ncclSuccess || ncclCommCuDevice(L.nc, &d) != ncclSuccess ||
        ncclCommUserRank(L.nc, &r) != ncclSuccess)
        return QK_E_COMM;
    if (count) *count = k;
    if (device) *device = d;
    if (rank) *rank = r;
    return QK_OK;
}

int qk_u32_encode_sharded_async(qk_comm *comm, const uint32_t *const *d_ids, const size_t *n, uint32_t threshold,
                                int root, void *const *streams) {
    if (!comm) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    return encode_sharded_async<32>(comm, (const void *const *)d_ids, n, threshold, root, streams);
}
int qk_u64_encode_sharded_async(qk_comm *comm, const uint64_t *const *d_ids, const size_t *n, uint32_t threshold,
                                int root, void *const *streams) {
    if (!comm) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    return encode_sharded_async<64>(comm, (const void *const *)d_ids, n, threshold, root, streams);
}
int qk_u32_encode_sharded_wait(qk_comm *comm, qk_u32 *q) {
    if (!comm) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    return encode_sharded_wait<32>(comm, q);
}
int qk_u64_encode_sharded_wait(qk_comm *comm, qk_u64 *q) {
    if (!comm) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    return encode_sharded_wait<64>(comm, q);
}
// q is read for its threshold on every rank (a NULL q on a non-root rank
// would make that rank skip the collective: it is an argument error, alike
// on every rank by contract)
int qk_u32_encode_sharded(qk_comm *comm, const uint32_t *const *d_ids, const size_t *n, qk_u32 *q, int root,
                          void *const *streams) {
    if (!comm || !q) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    const int rc = encode_sharded_async<32>(comm, (const void *const *)d_ids, n, q->threshold, root, streams);
    const int w = encode_sharded_wait<32>(comm, q);
    return rc ? rc : w;
}
int qk_u64_encode_sharded(qk_comm *comm, const uint64_t *const *d_ids, const size_t *n, qk_u64 *q, int root,
                          void *const *streams) {
    if (!comm || !q) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    const int rc = encode_sharded_async<64>(comm, (const void *const *)d_ids, n, q->threshold, root, streams);
    const int w = encode_sharded_wait<64>(comm, q);
    return rc ? rc : w;
}

int qk_u32_decode_sharded(qk_comm *comm, const qk_u32 *diff, int root, const uint32_t *const *d_log, const size_t *n,
                          int stop_at_last, uint64_t *hits, size_t cap, size_t *n_hits, void *const *streams) {
    if (!comm) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    return decode_sharded<uint32_t>(comm, diff, root, d_log, n, stop_at_last, hits, cap, n_hits, streams);
}
int qk_u64_decode_sharded(qk_comm *comm, const qk_u64 *diff, int root, const uint64_t *const *d_log, const size_t *n,
                          int stop_at_last, uint64_t *hits, size_t cap, size_t *n_hits, void *const *streams) {
    if (!comm) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    return decode_sharded<uint64_t>(comm, diff, root, d_log, n, stop_at_last, hits, cap, n_hits, streams);
}

} // extern "C"
