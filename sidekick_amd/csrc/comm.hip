// comm.hip — multi-GPU sharding of the encode and decode paths over RCCL
// (xGMI), behind the C ABI (include/quack_hip.h "Multi-GPU").
//
// The sketch is additive, so one stream cut into contiguous shards (one per
// GPU, in global rank order) encodes shard by shard and the partial vectors
// are summed.  Per sharded encode:
//   each local rank   encode its shard into its payload buffer (the
//                     ordinary encode kernel + finalize), then k_comm_pack
//                     turns [S.., n, last] into [S.., n, slots]: slot r =
//                     (has_last, last) of rank r, zero elsewhere
//   ONE ncclReduce    (sum, uint64) of the payload to the root rank:
//                     the summed power-sum words cannot overflow (canonical
//                     residues / 32-bit limbs, < 2^27 ranks), the count word
//                     sums the shard sizes, and every slot has exactly one
//                     contributor, so the root reads each rank's last id
//   root              fold mod p, count mod 2^32, last_value = the last
//                     id of the highest non-empty rank
// Payload at t = 32 on 8 GPUs: 33 + 16 words = 392 B — latency-bound; the
// xGMI bandwidth is irrelevant.
//
// Sharded decode (the log cut the same way):
//   ncclBroadcast     [status, d, stop flag, stop value, c_1..c_d] from the
//                     root, which ran to_coeffs (host, O(t^2))
//   each local rank   the root test over its log shard (api.hip phases, all
//                     local GPUs in flight at once)
//   ncclAllGather     (n, first stop position, hits below it) per rank
//   ncclAllGather     the hit positions (+ shard base), padded to the
//                     largest count; every rank cuts at the global stop
// so every rank returns the single-GPU answer for the whole log.
//
// Streams: each local rank's work runs on its qk_ctx's own stream, ordered
// after the caller's stream (event) and, for the async encode, with the
// caller's stream ordered after it again.
#include <string.h>

#include <algorithm>
#include <mutex>
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
        uint64_t *d_coll = nullptr;   // collective payload (device)
        uint64_t *h_coll = nullptr;   // pinned host mirror
        size_t coll_words = 0;
        hipEvent_t ev_in = nullptr, ev_out = nullptr;
        hipStream_t user = nullptr;   // caller stream of the operation in flight
    };
    int world = 1;
    std::vector<Local> local;
    // sharded encode in flight (qk_*_encode_sharded_async -> _wait)
    int pend_bits = 0;
    uint32_t pend_t = 0;
    int pend_root = -1;
    std::mutex mu;
};

#define QK_NCCL_TRY(expr)                                                                          \
    do {                                                                                           \
        if ((expr) != ncclSuccess) return QK_E_COMM;                                               \
    } while (0)

namespace qk {

using Local = qk_comm::Local;

// [S.., n, last] -> [S.., n, slot_0 .. slot_{world-1}], slot = (has_last, last)
// (R = the summed words, n at R - 1, last at R)
__global__ void k_comm_pack(uint64_t *buf, uint32_t R, uint32_t world, uint32_t rank) {
    const uint64_t n = buf[R - 1], last = buf[R];
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < 2 * world; j += blockDim.x) buf[R + j] = 0;
    __syncthreads();
    if (threadIdx.x == 0 && n) {
        buf[R + 2 * rank] = 1;
        buf[R + 2 * rank + 1] = last;
    }
}

static int ensure_coll(Local &L, size_t words) {
    if (words <= L.coll_words) return QK_OK;
    // grown only between operations (every comm call drains its streams
    // before returning, except the async encode, whose size is fixed per t)
    QK_HIP_TRY(hipStreamSynchronize(L.ctx->stream));
    if (L.d_coll) hipFree(L.d_coll);
    if (L.h_coll) hipHostFree(L.h_coll);
    L.d_coll = nullptr;
    L.h_coll = nullptr;
    L.coll_words = 0;
    const size_t w = std::max<size_t>(words, 4096);
    if (hipMalloc(&L.d_coll, w * 8) != hipSuccess) return QK_E_NOMEM;
    if (hipHostMalloc(&L.h_coll, w * 8, hipHostMallocDefault) != hipSuccess) return QK_E_NOMEM;
    L.coll_words = w;
    return QK_OK;
}

// order the local rank's stream after the caller's stream
static int enter(Local &L, void *user) {
    QK_HIP_TRY(hipSetDevice(L.device));
    L.user = (hipStream_t)user;
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

static int init_local(Local &L, int device) {
    L.device = device;
    if (int rc = qk_ctx_create(device, &L.ctx)) return rc;
    QK_HIP_TRY(hipSetDevice(device));
    QK_HIP_TRY(hipEventCreateWithFlags(&L.ev_in, hipEventDisableTiming));
    QK_HIP_TRY(hipEventCreateWithFlags(&L.ev_out, hipEventDisableTiming));
    return ensure_coll(L, 4096);
}

// summed words of the partial vector
static size_t reduce_words(int bits, uint32_t t) { return bits == 32 ? (size_t)t + 1 : 2 * (size_t)t + 1; }

template <int BITS>
static int encode_sharded_async(qk_comm *c, const void *const *d_ids, const size_t *n, uint32_t t, int root,
                                void *const *streams) {
    if (!c || !d_ids || !n) return QK_E_INVAL;
    if (t == 0 || t > QK_MAX_THRESHOLD) return QK_E_THRESHOLD;
    if (root < 0 || root >= c->world) return QK_E_INVAL;
    const size_t esz = BITS == 32 ? 4 : 8;
    for (size_t i = 0; i < c->local.size(); ++i) {
        if (n[i] && (!d_ids[i] || !is_device_ptr(d_ids[i]) || ((uintptr_t)d_ids[i] & (esz - 1)))) return QK_E_INVAL;
        if (n[i] >= (1ull << 40)) return QK_E_INVAL;
    }
    const size_t R = reduce_words(BITS, t), W = R + 2 * (size_t)c->world;
    for (auto &L : c->local)
        if (int rc = ensure_coll(L, W)) return rc;
    // every check that can fail before the collective has run: from here on a
    // local failure still joins the reduce (the other ranks would wait in it)
    int rc = QK_OK;
    for (size_t i = 0; i < c->local.size(); ++i) {
        Local &L = c->local[i];
        int e = enter(L, streams ? streams[i] : nullptr);
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
        if (e && !rc) rc = e;
    }
    if (ncclGroupStart() != ncclSuccess) return QK_E_COMM;
    int nrc = QK_OK;
    for (auto &L : c->local)
        if (ncclReduce(L.d_coll, L.d_coll, W, ncclUint64, ncclSum, root, L.nc, L.ctx->stream) != ncclSuccess)
            nrc = QK_E_COMM;
    if (ncclGroupEnd() != ncclSuccess) nrc = QK_E_COMM;
    for (auto &L : c->local) {
        if (L.rank == root && hipMemcpyAsync(L.h_coll, L.d_coll, W * 8, hipMemcpyDeviceToHost, L.ctx->stream) !=
                                  hipSuccess && !rc)
            rc = QK_E_HIP;
        if (int e = leave(L); e && !rc) rc = e;
    }
    c->pend_bits = BITS;
    c->pend_t = t;
    c->pend_root = root;
    return rc ? rc : nrc;
}

template <int BITS, typename Q>
static int encode_sharded_wait(qk_comm *c, Q *q) {
    if (!c) return QK_E_INVAL;
    if (c->pend_bits != BITS) return QK_E_INVAL;   // nothing in flight for this id width
    const uint32_t t = c->pend_t;
    const int root = c->pend_root;
    c->pend_bits = 0;
    int rc = QK_OK;
    for (auto &L : c->local) {
        (void)hipSetDevice(L.device);
        if (hipStreamSynchronize(L.ctx->stream) != hipSuccess) rc = QK_E_HIP;
    }
    if (rc) return rc;
    for (auto &L : c->local) {
        if (L.rank != root) continue;
        if (!q) return QK_E_INVAL;
        if (q->threshold != t) return QK_E_MISMATCH;
        const size_t R = reduce_words(BITS, t);
        const uint64_t *h = L.h_coll;
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

template <typename T, typename Q>
static int decode_sharded(qk_comm *c, const Q *diff, int root, const T *const *d_log, const size_t *n,
                          int stop_at_last, uint64_t *hits, size_t cap, size_t *n_hits, void *const *streams) {
    if (!c || !d_log || !n || !n_hits) return QK_E_INVAL;
    if (root < 0 || root >= c->world) return QK_E_INVAL;
    *n_hits = 0;
    const size_t nl = c->local.size(), W = (size_t)c->world;
    for (size_t i = 0; i < nl; ++i)
        if (n[i] && (!d_log[i] || !is_device_ptr(d_log[i]) || ((uintptr_t)d_log[i] & (sizeof(T) - 1))))
            return QK_E_INVAL;
    const size_t B = 4 + QK_MAX_THRESHOLD;   // broadcast header + coefficients
    for (auto &L : c->local)
        if (int rc = ensure_coll(L, std::max(B, 6 * W + 6))) return rc;

    // 1. coefficients from the root (status travels with them, so an
    //    undecodable difference fails on every rank alike)
    for (size_t i = 0; i < nl; ++i) {
        Local &L = c->local[i];
        if (int e = enter(L, streams ? streams[i] : nullptr)) return e;
        if (L.rank != root) continue;
        uint64_t *h = L.h_coll;
        memset(h, 0, B * 8);
        int64_t status = QK_OK;
        uint32_t d = 0;
        if (!diff) status = QK_E_INVAL;
        else if (diff->count != 0) {
            std::vector<T> cf(std::max<uint32_t>(diff->threshold, 1));
            if constexpr (sizeof(T) == 4) status = qk_u32_to_coeffs(diff, cf.data(), (uint32_t)cf.size(), &d);
            else status = qk_u64_to_coeffs(diff, cf.data(), (uint32_t)cf.size(), &d);
            if (status == QK_OK && d > QK_MAX_THRESHOLD) status = QK_E_THRESHOLD;
            if (status == QK_OK)
                for (uint32_t k = 0; k < d; ++k) h[4 + k] = (uint64_t)cf[k];
        }
        h[0] = (uint64_t)status;
        h[1] = status == QK_OK ? d : 0;
        h[2] = diff && stop_at_last && diff->has_last ? 1 : 0;
        h[3] = diff ? (uint64_t)diff->last_value : 0;
        QK_HIP_TRY(hipMemcpyAsync(L.d_coll, h, B * 8, hipMemcpyHostToDevice, L.ctx->stream));
    }
    QK_NCCL_TRY(ncclGroupStart());
    for (auto &L : c->local)
        QK_NCCL_TRY(ncclBroadcast(L.d_coll, L.d_coll, B, ncclUint64, root, L.nc, L.ctx->stream));
    QK_NCCL_TRY(ncclGroupEnd());
    for (auto &L : c->local) {
        QK_HIP_TRY(hipMemcpyAsync(L.h_coll, L.d_coll, B * 8, hipMemcpyDeviceToHost, L.ctx->stream));
        QK_HIP_TRY(hipStreamSynchronize(L.ctx->stream));
    }
    const uint64_t *hdr = c->local[0].h_coll;
    const int status = (int)(int64_t)hdr[0];
    const uint32_t d = (uint32_t)hdr[1];
    const int use_stop = (int)hdr[2];
    const T stop_value = (T)hdr[3];
    std::vector<T> coeffs(std::max<uint32_t>(d, 1));
    for (uint32_t k = 0; k < d; ++k) coeffs[k] = (T)hdr[4 + k];
    if (status != QK_OK) return status;

    // 2. root test of every local shard, all GPUs in flight
    const bool test = d > 0 || use_stop;
    std::vector<std::vector<uint64_t>> lh(nl);
    std::vector<uint64_t> lstop(nl);
    for (size_t i = 0; i < nl; ++i) {
        Local &L = c->local[i];
        lstop[i] = n[i];
        if (!test || !n[i]) continue;
        std::lock_guard<std::mutex> g(L.ctx->mu);
        QK_HIP_TRY(hipSetDevice(L.device));
        if (int e = root_test_begin<T>(L.ctx, coeffs.data(), d, d_log[i], n[i], use_stop, stop_value, L.ctx->stream))
            return e;
    }
    for (size_t i = 0; i < nl; ++i) {
        Local &L = c->local[i];
        if (!test || !n[i]) continue;
        std::lock_guard<std::mutex> g(L.ctx->mu);
        QK_HIP_TRY(hipSetDevice(L.device));
        if (int e = root_test_finish<T>(L.ctx, coeffs.data(), d, d_log[i], n[i], use_stop, stop_value, L.ctx->stream,
                                        lh[i], lstop[i]))
            return e;
        // hits at or past this shard's own stop are past the global one too
        lh[i].resize((size_t)(std::lower_bound(lh[i].begin(), lh[i].end(), lstop[i]) - lh[i].begin()));
    }

    // 3. (n, stop, hits) of every rank
    for (size_t i = 0; i < nl; ++i) {
        Local &L = c->local[i];
        uint64_t *h = L.h_coll;
        h[0] = n[i];
        h[1] = lstop[i];
        h[2] = lh[i].size();
        QK_HIP_TRY(hipMemcpyAsync(L.d_coll, h, 24, hipMemcpyHostToDevice, L.ctx->stream));
    }
    QK_NCCL_TRY(ncclGroupStart());
    for (auto &L : c->local)
        QK_NCCL_TRY(ncclAllGather(L.d_coll, L.d_coll + 3, 3, ncclUint64, L.nc, L.ctx->stream));
    QK_NCCL_TRY(ncclGroupEnd());
    for (auto &L : c->local) {
        QK_HIP_TRY(hipMemcpyAsync(L.h_coll, L.d_coll + 3, 3 * W * 8, hipMemcpyDeviceToHost, L.ctx->stream));
        QK_HIP_TRY(hipStreamSynchronize(L.ctx->stream));
    }
    std::vector<uint64_t> base(W + 1, 0), cnt(W);
    uint64_t gstop = UINT64_MAX, M = 0;
    {
        const uint64_t *m = c->local[0].h_coll;
        for (size_t r = 0; r < W; ++r) {
            base[r + 1] = base[r] + m[3 * r];
            if (m[3 * r + 1] < m[3 * r]) gstop = std::min(gstop, base[r] + m[3 * r + 1]);
            cnt[r] = m[3 * r + 2];
            M = std::max(M, cnt[r]);
        }
    }

    // 4. the hit positions, padded to the largest count
    std::vector<uint64_t> all;
    if (M) {
        for (size_t i = 0; i < nl; ++i) {
            Local &L = c->local[i];
            if (int e = ensure_coll(L, M * (W + 1))) return e;
            uint64_t *h = L.h_coll;
            const uint64_t b = base[L.rank];
            for (size_t k = 0; k < M; ++k) h[k] = k < lh[i].size() ? b + lh[i][k] : UINT64_MAX;
            QK_HIP_TRY(hipMemcpyAsync(L.d_coll, h, M * 8, hipMemcpyHostToDevice, L.ctx->stream));
        }
        QK_NCCL_TRY(ncclGroupStart());
        for (auto &L : c->local)
            QK_NCCL_TRY(ncclAllGather(L.d_coll, L.d_coll + M, M, ncclUint64, L.nc, L.ctx->stream));
        QK_NCCL_TRY(ncclGroupEnd());
        Local &L0 = c->local[0];
        QK_HIP_TRY(hipMemcpyAsync(L0.h_coll, L0.d_coll + M, M * W * 8, hipMemcpyDeviceToHost, L0.ctx->stream));
        for (auto &L : c->local) QK_HIP_TRY(hipStreamSynchronize(L.ctx->stream));
        for (size_t r = 0; r < W; ++r)
            for (uint64_t k = 0; k < cnt[r]; ++k) {
                const uint64_t p = L0.h_coll[r * M + k];
                if (p < gstop) all.push_back(p);
            }
    } else {
        for (auto &L : c->local) QK_HIP_TRY(hipStreamSynchronize(L.ctx->stream));
    }
    for (auto &L : c->local)
        if (int e = leave(L)) return e;
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
    QK_NCCL_TRY(ncclGetUniqueId(&u));
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
        if (int rc = init_local(c->local[i], devices[i])) {
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
    if (int rc = init_local(c->local[0], device)) {
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

void qk_comm_destroy(qk_comm *comm) {
    if (!comm) return;
    for (auto &L : comm->local) {
        if (L.ctx) {
            (void)hipSetDevice(L.device);
            (void)hipStreamSynchronize(L.ctx->stream);
        }
    }
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
    for (auto &L : comm->local) {
        QK_HIP_TRY(hipSetDevice(L.device));
        QK_HIP_TRY(hipMemsetAsync(L.d_coll, 0, 8, L.ctx->stream));
    }
    QK_NCCL_TRY(ncclGroupStart());
    for (auto &L : comm->local)
        QK_NCCL_TRY(ncclAllReduce(L.d_coll, L.d_coll, 1, ncclUint64, ncclSum, L.nc, L.ctx->stream));
    QK_NCCL_TRY(ncclGroupEnd());
    for (auto &L : comm->local) QK_HIP_TRY(hipStreamSynchronize(L.ctx->stream));
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
int qk_u32_encode_sharded(qk_comm *comm, const uint32_t *const *d_ids, const size_t *n, qk_u32 *q, int root,
                          void *const *streams) {
    if (!comm || !q) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    int rc = encode_sharded_async<32>(comm, (const void *const *)d_ids, n, q->threshold, root, streams);
    const int w = encode_sharded_wait<32>(comm, q);
    return rc ? rc : w;
}
int qk_u64_encode_sharded(qk_comm *comm, const uint64_t *const *d_ids, const size_t *n, qk_u64 *q, int root,
                          void *const *streams) {
    if (!comm || !q) return QK_E_INVAL;
    std::lock_guard<std::mutex> g(comm->mu);
    int rc = encode_sharded_async<64>(comm, (const void *const *)d_ids, n, q->threshold, root, streams);
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
