/*
 * quack_hip.h — C ABI of the MI355X-native quACK power-sum engine
 * (libquack_hip.so).
 *
 * This is the drop-in boundary for the `quack` crate's encode/decode path.
 * The reference exposes it as a Rust crate API, not an FFI;
 * each entry point below names the reference call it replaces, and
 * INTEGRATION.md shows the Rust `extern "C"` binding a maintainer adds so
 * sidekick/ and media/ keep compiling against `quack::PowerSumQuackU32`.
 *
 * Conventions
 *   - Plain C types only; every buffer is caller-owned.  No ownership crosses
 *     the ABI except the opaque qk_ctx (create/destroy).
 *   - Every function returns an int status (QK_OK == 0, negative on error)
 *     unless documented otherwise.  No C++ exception crosses the ABI.
 *   - Sketch state is a POD with a flexible array; size it with
 *     qk_u32_size()/qk_u64_size().  Copying the bytes is Clone
 *     (sidekick.rs:203-205).  The state is not internally synchronised
 *     (the reference guards it with a Mutex: sidekick.rs:107).
 *   - "device" functions run hand-written gfx950 kernels.  They never fall
 *     back to the CPU: with no GPU they return QK_E_NO_DEVICE.
 *   - `stream` is a hipStream_t passed as void*; NULL is the HIP null
 *     (legacy default) stream, so work is ordered with the caller's
 *     default-stream work.  "_async" functions only enqueue on that stream.
 *
 * Field and semantics:  p32 = 2^32-5, p64 = 2^64-59; an id is
 * mapped to x = id mod p; S[k-1] = sum_i x_i^k mod p for k = 1..threshold;
 * count is a wrapping u32; last_value is the last inserted (unreduced) id.
 */
#ifndef QUACK_HIP_H
#define QUACK_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QK_P32 4294967291u
#define QK_P64 18446744073709551557ull
#define QK_MAX_THRESHOLD 1024u /* largest threshold the device kernels accept */

enum {
    QK_OK = 0,
    QK_E_INVAL = -1,        /* bad argument (null pointer, host pointer where device expected, ...) */
    QK_E_THRESHOLD = -2,    /* threshold 0 on insert/remove, or > QK_MAX_THRESHOLD on device */
    QK_E_MISMATCH = -3,     /* thresholds of two sketches differ (reference panics) */
    QK_E_UNDECODABLE = -4,  /* count > threshold: caller must reset (media_client.rs:258-261) */
    QK_E_CAPACITY = -5,     /* output buffer too small; *n_out holds the required size */
    QK_E_HIP = -6,          /* a HIP runtime call failed */
    QK_E_NO_DEVICE = -7,    /* no usable gfx950 device */
    QK_E_NOMEM = -8,
    QK_E_FORMAT = -9,       /* malformed serialized bytes */
    QK_E_COMM = -10,        /* a collective failed: the communicator is aborted and unusable */
    QK_E_PEER = -11         /* another rank of the communicator failed (its own call reports why) */
};

const char *qk_strerror(int status);
const char *qk_version(void);

/* ------------------------------------------------------------------------
 * Sketch state (PowerSumQuackU32 / PowerSumQuackU64)
 * ---------------------------------------------------------------------- */
typedef struct qk_u32 {
    uint32_t threshold;
    uint32_t count;       /* wrapping */
    uint32_t has_last;    /* Option tag of last_value */
    uint32_t last_value;
    uint32_t power_sums[]; /* threshold entries, canonical (< QK_P32) */
} qk_u32;

typedef struct qk_u64 {
    uint32_t threshold;
    uint32_t count;
    uint32_t has_last;
    uint32_t reserved;
    uint64_t last_value;
    uint64_t power_sums[]; /* threshold entries, canonical (< QK_P64) */
} qk_u64;

size_t qk_u32_size(uint32_t threshold);                 /* bytes of a qk_u32 */
size_t qk_u64_size(uint32_t threshold);

/* PowerSumQuackU32::new(threshold)   — sidekick/src/sidekick.rs:32 */
int qk_u32_init(qk_u32 *q, uint32_t threshold);
int qk_u64_init(qk_u64 *q, uint32_t threshold);

/* ---- host scalar path (per packet; a kernel launch costs more than an
 *      insert, so these never touch the GPU) ---------------------------- */
/* quack.insert(id)                   — sidekick.rs:42, sidekick_multi.rs:82 */
int qk_u32_insert(qk_u32 *q, uint32_t id);
int qk_u64_insert(qk_u64 *q, uint64_t id);
/* my_quack.remove(id)                — media_client.rs:319 */
int qk_u32_remove(qk_u32 *q, uint32_t id);
int qk_u64_remove(qk_u64 *q, uint64_t id);
/* diff_quack.sub_assign(quack)       — media_client.rs:296 (keeps q->last_value) */
int qk_u32_sub_assign(qk_u32 *q, const qk_u32 *rhs);
int qk_u64_sub_assign(qk_u64 *q, const qk_u64 *rhs);
/* union of two disjoint streams, `later` following q in stream order
 * (additivity): sums add, counts add, last from `later`. */
int qk_u32_merge(qk_u32 *q, const qk_u32 *later);
int qk_u64_merge(qk_u64 *q, const qk_u64 *later);
/* diff_quack.to_coeffs()             — media_client.rs:304.
 * Writes d = q->count coefficients c_1..c_d of prod(z - x_missing).
 * d > threshold -> QK_E_UNDECODABLE; cap < d -> QK_E_CAPACITY (*d set). */
int qk_u32_to_coeffs(const qk_u32 *q, uint32_t *coeffs, uint32_t cap, uint32_t *d);
int qk_u64_to_coeffs(const qk_u64 *q, uint64_t *coeffs, uint32_t cap, uint32_t *d);
/* quack::arithmetic::eval(&coeffs, x).value()   — media_client.rs:310.
 * Returns the canonical value of the monic polynomial at x (d == 0 -> 1). */
uint32_t qk_u32_eval(const uint32_t *coeffs, uint32_t d, uint32_t x);
uint64_t qk_u64_eval(const uint64_t *coeffs, uint32_t d, uint64_t x);

/* decode_with_log over a HOST-resident log (the receiver's short logs,
 * media_client.rs:304-313): to_coeffs, then the root test on the CPU; same
 * contract as qk_u32_decode_device (hits = log positions ascending, cut at
 * the first entry equal to diff->last_value when stop_at_last). */
int qk_u32_decode_host(const qk_u32 *diff, const uint32_t *log, size_t n, int stop_at_last, uint64_t *hits,
                       size_t cap, size_t *n_hits);
int qk_u64_decode_host(const qk_u64 *diff, const uint64_t *log, size_t n, int stop_at_last, uint64_t *hits,
                       size_t cap, size_t *n_hits);

/* bincode 1.3 image of the serde-derived struct
 * {power_sums: Vec<ModularInteger>, last_value: Option<T>, count: u32}
 * (sidekick.rs:187, media_client.rs:227; layout [RECALL]). */
size_t qk_u32_serialized_size(const qk_u32 *q);
int qk_u32_serialize(const qk_u32 *q, uint8_t *buf, size_t cap, size_t *len);
/* Reads the threshold from the bytes; *threshold_out lets the caller size q
 * first (call with q == NULL), then qk_*_init(q, threshold) and call again:
 * q->threshold must equal the serialized threshold (else QK_E_MISMATCH and q
 * is untouched). */
int qk_u32_deserialize(const uint8_t *buf, size_t len, qk_u32 *q, uint32_t *threshold_out);
size_t qk_u64_serialized_size(const qk_u64 *q);
int qk_u64_serialize(const qk_u64 *q, uint8_t *buf, size_t cap, size_t *len);
int qk_u64_deserialize(const uint8_t *buf, size_t len, qk_u64 *q, uint32_t *threshold_out);

/* ------------------------------------------------------------------------
 * Device context
 * ---------------------------------------------------------------------- */
typedef struct qk_ctx qk_ctx;

int qk_device_count(int *n);
int qk_ctx_create(int device, qk_ctx **out);
void qk_ctx_destroy(qk_ctx *ctx);
int qk_ctx_synchronize(qk_ctx *ctx, void *stream);
/* When on, every launch of the dominant kernel (encode / root test) is
 * bracketed by hipEvents on its stream; qk_ctx_kernel_stats() waits for them
 * and returns the summed duration and launch count, then resets. */
int qk_ctx_set_profiling(qk_ctx *ctx, int on);
int qk_ctx_kernel_stats(qk_ctx *ctx, double *total_ms, uint64_t *launches);
/* Growing a context's scratch never synchronises the device: grown-out
 * buffers are retired, not freed (hipFree synchronises every stream).
 * qk_ctx_trim frees them — a device-wide synchronisation, so call it when
 * that is acceptable (qk_ctx_destroy does it too). */
int qk_ctx_trim(qk_ctx *ctx);
/* Tuning knobs (0 = automatic): workgroups per launch. */
int qk_ctx_set_grid(qk_ctx *ctx, uint32_t blocks);
/* Knobs of this context that select between live product paths (DESIGN.md
 * §3; the defaults are the product's measured choices — tools/ and the
 * tests set them): "grid_mult" (1..8: encode grids of that many rounds of
 * resident workgroups), "flow_hist" (per-flow batches of at most this many
 * flows are grouped by slot histograms, 0: never), "flow_byslot" (0 the
 * rule, 1 / 2 force the by-slot / by-rank grouping key), "root_test" (0
 * automatic, 1 Horner, 2 root-set scan), "comm_fault" (tests: the k-th
 * collective's payload staging of this context's rank fails once),
 * "comm_delay_ms" (tests: a kernel of that many ms runs before this rank's
 * next RCCL collective, once), "rt_karg" (1: a root-set scan whose set fits
 * the kernel arguments takes them; 0: always by copy).
 * Unknown name or out-of-range value -> QK_E_INVAL. */
int qk_ctx_set_knob(qk_ctx *ctx, const char *name, int64_t value);
/* Shader-clock probe (measurement): one wave on `stream` spins for
 * `microseconds` of wall time and writes d_out[0] = shader-clock ticks
 * (s_memtime) and d_out[1] = 100 MHz ticks (s_memrealtime) elapsed, so the
 * clock is d_out[0] / d_out[1] * 100 MHz.  Launched beside running kernels it
 * reads the clock the chip holds under their load. */
int qk_clock_probe(qk_ctx *ctx, uint32_t microseconds, uint64_t *d_out, void *stream);
/* Pinned host memory for the host-input path: ids written here by the
 * sniffer are DMA'd without a staging copy. */
int qk_host_alloc(size_t bytes, void **out);
int qk_host_free(void *p);

/* ------------------------------------------------------------------------
 * Batch encode — the hot path.  Replaces the per-id loop
 *   for id in ids { quack.insert(id) }   (sidekick.rs:42 under :76-124;
 *   media_client.rs:247-252; quack benchmark_construct) for an id array.
 * ---------------------------------------------------------------------- */
/* Partial vector written by the _async encoders, u64 words:
 *   u32: [S_1..S_t (canonical), n, last_id]            (t + 2 words)
 *   u64: [lo32(S_k), hi32(S_k) for k = 1..t, n, last_id] (2t + 2 words)
 * The first t+1 (u32) / 2t+1 (u64) words of several partials may be summed
 * elementwise as unsigned 64-bit integers (e.g. an RCCL sum-reduce) without
 * overflow for up to 2^27 partials; qk_*_from_partial folds such a sum. */
size_t qk_u32_partial_words(uint32_t threshold);
size_t qk_u64_partial_words(uint32_t threshold);

int qk_u32_encode_device_async(qk_ctx *ctx, const uint32_t *d_ids, size_t n, uint32_t threshold,
                               uint64_t *d_partial, void *stream);
int qk_u64_encode_device_async(qk_ctx *ctx, const uint64_t *d_ids, size_t n, uint32_t threshold,
                               uint64_t *d_partial, void *stream);
/* Fold a (possibly summed) host copy of the partial into q as the stream that
 * follows q: sums and count add; last_value taken from `last` if has_last. */
int qk_u32_merge_partial(qk_u32 *q, const uint64_t *partial, int has_last, uint32_t last);
int qk_u64_merge_partial(qk_u64 *q, const uint64_t *partial, int has_last, uint64_t last);

/* Synchronous: encode device-resident ids and merge them into q (as if
 * inserted in array order after q's existing content). */
int qk_u32_encode_device(qk_ctx *ctx, const uint32_t *d_ids, size_t n, qk_u32 *q, void *stream);
int qk_u64_encode_device(qk_ctx *ctx, const uint64_t *d_ids, size_t n, qk_u64 *q, void *stream);
/* Synchronous: encode HOST-resident ids (the sniffed-packet case): chunked
 * H2D through pinned staging on two streams, overlapped with the kernel. */
int qk_u32_encode_host(qk_ctx *ctx, const uint32_t *h_ids, size_t n, qk_u32 *q);
int qk_u64_encode_host(qk_ctx *ctx, const uint64_t *h_ids, size_t n, qk_u64 *q);

/* ------------------------------------------------------------------------
 * Packet batches: identifier extraction fused in front of the encode
 * (SURVEY.md §8f rank 2).  Replaces the sniff loop of sidekick.rs:76-124 for
 * a batch of captured buffers: per packet, in order,
 *   skip unless sll_pkttype is PACKET_HOST/PACKET_OTHERHOST      (:78-80)
 *   skip unless sll_protocol == htons(ETH_P_IP)                    (:81-84)
 *   skip unless buf[23] == IPPROTO_UDP      (buffer.rs:80-83)      (:85-88)
 *   dst ip buf[30..34] == my_ipv4 -> reset the quACK               (:92-96)
 *   skip unless the capture length == QK_BUFFER_SIZE               (:99-102)
 *   insert the big-endian u32 at byte QK_ID_OFFSET (buffer.rs:99-106)
 * Buffers are `stride`-byte records (the reference reads QK_BUFFER_SIZE = 67
 * bytes per packet) in device memory; meta may be NULL (all packets incoming
 * IPv4 of full length).  my_ipv4 may be NULL (no packet resets).
 * ---------------------------------------------------------------------- */
#define QK_ID_OFFSET 63u
#define QK_BUFFER_SIZE 67u
typedef struct qk_pkt_meta {
    uint8_t pkttype;      /* sockaddr_ll.sll_pkttype */
    uint8_t reserved;
    uint16_t protocol_be; /* sockaddr_ll.sll_protocol (network byte order, as stored) */
    uint32_t len;         /* bytes returned by recvfrom */
} qk_pkt_meta;
typedef struct qk_pkt_stats {
    uint64_t inserted;    /* inserts that reached the final state (after the last reset) */
    uint64_t discarded;   /* inserts wiped by a later reset in the same batch */
    uint64_t resets;
    uint64_t filtered;    /* packets skipped by the filters */
    int64_t last_reset_index; /* -1 if no reset */
} qk_pkt_stats;
int qk_u32_encode_packets_device(qk_ctx *ctx, const uint8_t *d_bufs, size_t n, size_t stride,
                                 const qk_pkt_meta *d_meta, const uint8_t my_ipv4[4], qk_u32 *q,
                                 qk_pkt_stats *stats, void *stream);

/* ------------------------------------------------------------------------
 * Segmented multi-flow encode: one quACK per flow.
 * ---------------------------------------------------------------------- */
/* AddrKey of sidekick_multi.rs:13 / buffer.rs:91-95:
 * [src ip (4), src port (2), dst ip (4), dst port (2)], bytes as on the wire. */
typedef struct qk_flow_key {
    uint8_t addr[12];
} qk_flow_key;
/* SidekickMulti over a packet batch (sidekick_multi.rs:65-90,101-143): every
 * Insert goes to its AddrKey's quACK (created on first use).  Output: the
 * batch's flows in ascending key order, keys[i] and sketches record i
 * (qk_u32_size(threshold) bytes each, ready for qk_u32_merge into the
 * caller's table).  my_addr = own dst ip:port (6 bytes) or NULL.  A Reset
 * packet (dst ip:port == my_addr) wipes EVERY flow, as the sniff loops do
 * (`senders = HashMap::new()`, sidekick_multi.rs:205,265): the output holds
 * only the inserts after the batch's last reset, stats.discarded counts the
 * inserts before it, stats.last_reset_index is its position, and a caller
 * with stats.resets > 0 must clear its own table before merging the output.
 * cap < flows -> QK_E_CAPACITY with *n_flows set.  keys and sketches may
 * both be host memory (two D2H copies at the end) or both device memory of
 * ctx's GPU (written in place by the finalize kernel: nothing crosses PCIe;
 * the caller synchronises `stream` before reading them); mixed -> QK_E_INVAL. */
int qk_u32_encode_flows_device(qk_ctx *ctx, const uint8_t *d_bufs, size_t n, size_t stride,
                               const qk_pkt_meta *d_meta, const uint8_t my_addr[6], uint32_t threshold,
                               qk_flow_key *keys, uint8_t *sketches, size_t cap, size_t *n_flows,
                               qk_pkt_stats *stats, void *stream);
/* The segmented primitive: ids already grouped by flow (device array,
 * segment g = [offsets[g], offsets[g+1]), host offsets, stream order within a
 * segment) -> nseg sketches (qk_u32_size(threshold) bytes each). */
int qk_u32_encode_segments_device(qk_ctx *ctx, const uint32_t *d_ids, const uint64_t *offsets, size_t nseg,
                                  uint32_t threshold, uint8_t *sketches, void *stream);

/* ------------------------------------------------------------------------
 * Decode-missing root test.  Replaces media_client.rs:306-313:
 *   for id in log { if arithmetic::eval(&coeffs, id).value() == 0 { hit } }
 * Hit positions (indices into the log) are returned ascending (log order);
 * every log entry congruent to a root is a hit, duplicates included.
 * With stop_at_value != 0 only positions before the first entry equal to
 * stop_value are returned (the `break` at media_client.rs:307-309).
 * *n_hits is set to the number of hits; cap < *n_hits -> QK_E_CAPACITY.
 * ---------------------------------------------------------------------- */
int qk_u32_root_test_device(qk_ctx *ctx, const uint32_t *coeffs, uint32_t d, const uint32_t *d_log,
                            size_t n, int stop_at_value, uint32_t stop_value, uint64_t *hits,
                            size_t cap, size_t *n_hits, void *stream);
int qk_u64_root_test_device(qk_ctx *ctx, const uint64_t *coeffs, uint32_t d, const uint64_t *d_log,
                            size_t n, int stop_at_value, uint64_t stop_value, uint64_t *hits,
                            size_t cap, size_t *n_hits, void *stream);
/* Shard form of the root test for a log cut into contiguous shards across
 * ranks: as above on this shard, and *stop_index is set to the
 * position of the first entry equal to stop_value in the shard, or n when
 * there is none (or stop_at_value == 0).  The global result is the union of
 * shard hits (offset by shard base) below the smallest shard_base+stop_index;
 * sidekick_amd/dist.py: root_test_sharded does that merge with two small
 * collectives. */
int qk_u32_root_test_shard_device(qk_ctx *ctx, const uint32_t *coeffs, uint32_t d, const uint32_t *d_log,
                                  size_t n, int stop_at_value, uint32_t stop_value, uint64_t *hits,
                                  size_t cap, size_t *n_hits, uint64_t *stop_index, void *stream);
int qk_u64_root_test_shard_device(qk_ctx *ctx, const uint64_t *coeffs, uint32_t d, const uint64_t *d_log,
                                  size_t n, int stop_at_value, uint64_t stop_value, uint64_t *hits,
                                  size_t cap, size_t *n_hits, uint64_t *stop_index, void *stream);
/* The distinct roots in GF(p), ascending, of the monic polynomial
 * z^d + c_1 z^(d-1) + ... + c_d (coeffs as qk_*_to_coeffs writes them; any
 * value is taken mod p).  An entry x of a log is a root-test hit
 * (media_client.rs:310, eval(&coeffs, x) == 0) exactly when x mod p is one of
 * them: the device root test scans the log against this set (O(1) per entry)
 * when that beats d Horner steps per entry.  gcd(P, z^(p-1) - 1) and
 * Cantor-Zassenhaus splitting on the host, O(d^2 log p).  *k = number of
 * roots (<= d); cap < *k -> QK_E_CAPACITY. */
int qk_u32_roots(const uint32_t *coeffs, uint32_t d, uint32_t *roots, uint32_t cap, uint32_t *k);
int qk_u64_roots(const uint64_t *coeffs, uint32_t d, uint64_t *roots, uint32_t cap, uint32_t *k);
/* decode_with_log on the device: to_coeffs(diff) on the host (O(t^2)), then
 * the root test over the device-resident log.  diff->count == 0 -> no hits;
 * diff->count > threshold -> QK_E_UNDECODABLE. */
int qk_u32_decode_device(qk_ctx *ctx, const qk_u32 *diff, const uint32_t *d_log, size_t n,
                         int stop_at_last, uint64_t *hits, size_t cap, size_t *n_hits, void *stream);
int qk_u64_decode_device(qk_ctx *ctx, const qk_u64 *diff, const uint64_t *d_log, size_t n,
                         int stop_at_last, uint64_t *hits, size_t cap, size_t *n_hits, void *stream);

/* ------------------------------------------------------------------------
 * Multi-GPU: the id stream cut into contiguous shards, one
 * per GPU in global rank order, merged with ONE RCCL reduce over xGMI.
 * The reference callers are single processes (sidekick.rs:58-127,
 * sender.rs:80-116), so a communicator can drive several GPUs from one
 * process; one process per GPU works the same way.
 *   - one process, several GPUs:  qk_comm_create(ndev, devices)
 *     (ncclCommInitAll; local rank i = global rank i = devices[i]);
 *   - one process per GPU:        rank 0 calls qk_comm_unique_id and ships
 *     the QK_COMM_ID_BYTES bytes to the other ranks by any channel, then
 *     every rank calls qk_comm_init_rank(id, rank, world, device);
 *   - collectives over a host channel: qk_comm_init_host (below).
 * Each local rank owns its own qk_ctx.  Array arguments (d_ids, n, d_log,
 * streams) have one entry per LOCAL rank (qk_comm_info's nlocal), in local
 * rank order.  streams may be NULL (every local rank uses its device's null
 * stream); the work runs on the context's stream, ordered after the given
 * stream, and the given stream is ordered after it.  Every rank of the
 * communicator must make the same sequence of collective calls with the same
 * threshold and root.
 * Failure semantics: a rank whose own arguments or local work fail — including
 * the staging copy of its payload into a collective — still takes part in
 * every collective of the call (its failure travels as data), so no peer is
 * left blocked; see each call for what every rank returns.  A failed
 * collective, or a rank that cannot read what a collective delivered, aborts
 * the communicator (ncclCommAbort): that call and every later one return
 * QK_E_COMM; destroy it.  An abort releases this process's ranks only; a peer
 * in another process is released by its own timeout: every wait on an RCCL
 * collective polls ncclCommGetAsyncError and aborts after the communicator's
 * timeout (qk_comm_set_timeout; a host channel's callbacks time out
 * themselves), and the rank's own work in front of the collective is waited
 * for under 4 x that timeout, also polling the asynchronous error.
 * ---------------------------------------------------------------------- */
typedef struct qk_comm qk_comm;
#define QK_COMM_ID_BYTES 128
int qk_comm_unique_id(uint8_t id[QK_COMM_ID_BYTES]);
int qk_comm_create(int ndev, const int *devices, qk_comm **out);
int qk_comm_init_rank(const uint8_t id[QK_COMM_ID_BYTES], int rank, int world, int device, qk_comm **out);
/* One rank on `device` whose collectives run through the caller's host
 * channel instead of RCCL: the identical sharded protocol, every collective
 * staged through pinned host memory (the async encode completes before it
 * returns).  For more ranks than GPUs (RCCL takes one rank per device) and for
 * ranks RCCL cannot connect.  Each callback acts as the collective of its name
 * over all ranks (uint64 elements, wrapping sums; allgather: recv[r*n .. r*n+n)
 * = rank r's send) and returns 0, nonzero on failure (-> QK_E_COMM). */
typedef struct qk_comm_host_ops {
    void *user;
    int (*reduce_sum_u64)(void *user, uint64_t *buf, size_t n, int root);
    int (*broadcast_u64)(void *user, uint64_t *buf, size_t n, int root);
    int (*allgather_u64)(void *user, const uint64_t *send, uint64_t *recv, size_t n);
} qk_comm_host_ops;
int qk_comm_init_host(const qk_comm_host_ops *ops, int rank, int world, int device, qk_comm **out);
void qk_comm_destroy(qk_comm *comm);
/* world size, local ranks in this process, global rank of local rank 0 */
int qk_comm_info(const qk_comm *comm, int *world, int *nlocal, int *first_rank);
/* the qk_ctx of a local rank (owned by the communicator, valid until
 * qk_comm_destroy: profiling, grid knobs, and the single-GPU calls on that
 * device) */
int qk_comm_context(qk_comm *comm, int local, qk_ctx **out);
/* all ranks reach this point (one 8-byte reduce), then the local streams drain */
int qk_comm_barrier(qk_comm *comm);
/* Waits on RCCL collectives give up after `ms` milliseconds (0: never;
 * default 300 000), abort the communicator and return QK_E_COMM — the bound
 * on how long a rank waits for a peer that failed in another process. */
int qk_comm_set_timeout(qk_comm *comm, int64_t ms);
/* What RCCL itself reports for local rank `local`: ncclCommCount (ranks),
 * ncclCommCuDevice (device), ncclCommUserRank (rank) — e.g. to check that a
 * multi-process launch joined one communicator of the expected size.
 * QK_E_INVAL for a host-channel communicator (no RCCL communicator). */
int qk_comm_rccl_info(const qk_comm *comm, int local, int *count, int *device, int *rank);

/* Sharded encode: local rank i encodes d_ids[i][0 .. n[i]) on its GPU, then
 * one ncclReduce(sum, uint64) of its partial to global rank `root`:
 * (t + 1) power-sum/count words (u64 ids: 2t + 1, 32-bit limbs), a
 * (has_last, last) slot per rank, so the root learns the last id of the last
 * non-empty shard without a second collective, and a failed-rank count.  The
 * root merges the whole stream into q (as if inserted after q's content);
 * other ranks leave q untouched.  _async only enqueues; _wait (every rank)
 * drains the local streams and merges on the root.
 * Failures: a rank whose shard argument is bad (non-device, misaligned) or
 * whose encode fails returns that error from _async and _wait and sends a
 * failed payload; the root then returns QK_E_PEER (or its own error) and
 * leaves q untouched. */
int qk_u32_encode_sharded_async(qk_comm *comm, const uint32_t *const *d_ids, const size_t *n, uint32_t threshold,
                                int root, void *const *streams);
int qk_u64_encode_sharded_async(qk_comm *comm, const uint64_t *const *d_ids, const size_t *n, uint32_t threshold,
                                int root, void *const *streams);
int qk_u32_encode_sharded_wait(qk_comm *comm, qk_u32 *q);
int qk_u64_encode_sharded_wait(qk_comm *comm, qk_u64 *q);
int qk_u32_encode_sharded(qk_comm *comm, const uint32_t *const *d_ids, const size_t *n, qk_u32 *q, int root,
                          void *const *streams);
int qk_u64_encode_sharded(qk_comm *comm, const uint64_t *const *d_ids, const size_t *n, qk_u64 *q, int root,
                          void *const *streams);
/* Sharded decode over a candidate log cut the same way (log shard i on local
 * rank i): the root turns diff into coefficients (diff is read on the root
 * only; other ranks may pass NULL) and broadcasts them, every rank
 * root-tests its shard, the shards' stop positions, hit counts and statuses
 * are all-gathered, then the hits.  Every rank returns the single-GPU
 * qk_*_decode_device result for the whole log (global positions, ascending,
 * cut at the first entry equal to diff->last_value when stop_at_last).  Any
 * failure — an undecodable diff on the root, a bad log shard or a failed root
 * test on any rank — makes every rank return the same status (the lowest
 * failing rank's). */
int qk_u32_decode_sharded(qk_comm *comm, const qk_u32 *diff, int root, const uint32_t *const *d_log, const size_t *n,
                          int stop_at_last, uint64_t *hits, size_t cap, size_t *n_hits, void *const *streams);
int qk_u64_decode_sharded(qk_comm *comm, const qk_u64 *diff, int root, const uint64_t *const *d_log, const size_t *n,
                          int stop_at_last, uint64_t *hits, size_t cap, size_t *n_hits, void *const *streams);

/* ------------------------------------------------------------------------
 * Synthetic identifier streams (benchmarks/tests): counter-based splitmix64,
 * id_i = mix(seed + (start+i+1)*0x9E3779B97F4A7C15); u32 ids = high 32 bits.
 * ---------------------------------------------------------------------- */
int qk_fill_splitmix_u32(qk_ctx *ctx, uint32_t *d_out, size_t n, uint64_t seed, uint64_t start,
                         void *stream);
int qk_fill_splitmix_u64(qk_ctx *ctx, uint64_t *d_out, size_t n, uint64_t seed, uint64_t start,
                         void *stream);

#ifdef __cplusplus
}
#endif
#endif /* QUACK_HIP_H */
