/*
 * quack_oracle.c — scalar C restatement of the quACK power-sum path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load this (as liboracle.so via ctypes); the
 * product library libquack_hip.so never links or calls it.
 *
 * PARITY STATUS: parity unpinned against the reference (the `quack` crate is
 * an empty, un-vendored submodule: /root/reference/.gitmodules:9-11; no Rust
 * toolchain here).  Pinned instead by algebraic known-answer tests and by
 * agreement with the independent Python big-int restatement
 * (oracle/quack_oracle.py) — see tests/test_oracle.py and DESIGN.md §1.
 *
 * The per-id loop mirrors the reference insert as called from
 * sidekick/src/sidekick.rs:42 and sidekick_multi.rs:82: x = id mod p, then
 * t-1 dependent modular multiplies and t modular adds, reducing with a plain
 * `%` by the constant prime after every multiply and a compare-subtract after
 * every add (the crate's ModularInteger arithmetic).  No SIMD, no threads:
 * it is also the single-core CPU baseline that bench.py times.
 *
 * Decode (media_client.rs:295-313): Newton's identities (to_coeffs) and the
 * Horner root test (arithmetic::eval(&coeffs, id).value() == 0).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define QO_P32 4294967291u                 /* 2^32 - 5  */
#define QO_P64 18446744073709551557ull     /* 2^64 - 59 */
#define QO_GAMMA 0x9E3779B97F4A7C15ull

typedef unsigned __int128 u128;

static inline uint64_t qo_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t qo_splitmix64_at(uint64_t seed, uint64_t i) { return qo_mix(seed + (i + 1) * QO_GAMMA); }

void qo_splitmix_u32(uint64_t seed, uint64_t start, uint64_t n, uint32_t *out) {
    for (uint64_t i = 0; i < n; ++i) out[i] = (uint32_t)(qo_mix(seed + (start + i + 1) * QO_GAMMA) >> 32);
}

void qo_splitmix_u64(uint64_t seed, uint64_t start, uint64_t n, uint64_t *out) {
    for (uint64_t i = 0; i < n; ++i) out[i] = qo_mix(seed + (start + i + 1) * QO_GAMMA);
}

/* ---- GF(p32) ---------------------------------------------------------- */
/* The conditional subtract as a mask, not a branch: s >= p is a coin flip
 * per add for random operands, and gcc compiled the ternary into a jump that
 * mispredicted every other power (~8 of the ~24 core cycles per power of the
 * insert loop; the crate's LLVM build selects instead). */
static inline uint32_t add32(uint32_t a, uint32_t b) {
    const uint64_t s = (uint64_t)a + b;
    const uint64_t m = (uint64_t)0 - (uint64_t)(s >= QO_P32);
    return (uint32_t)(s - (m & QO_P32));
}
static inline uint32_t sub32(uint32_t a, uint32_t b) { return a >= b ? a - b : (uint32_t)((uint64_t)a + QO_P32 - b); }
static inline uint32_t mul32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) % QO_P32); }
static uint32_t pow32(uint32_t a, uint32_t e) {
    uint32_t r = 1;
    while (e) { if (e & 1) r = mul32(r, a); a = mul32(a, a); e >>= 1; }
    return r;
}

static inline void insert32(uint32_t *S, uint32_t t, uint32_t id) {
    uint32_t x = id % QO_P32, y = x;
    for (uint32_t k = 0; k + 1 < t; ++k) { S[k] = add32(S[k], y); y = mul32(y, x); }
    S[t - 1] = add32(S[t - 1], y);
}

/* S (length t, canonical, accumulated in place) += power sums of ids. */
void qo_encode_u32(const uint32_t *ids, uint64_t n, uint32_t t, uint32_t *S) {
    if (t == 0) return;
    for (uint64_t i = 0; i < n; ++i) insert32(S, t, ids[i]);
}

/* Same, over the synthetic stream ids[start..start+n) of `seed` without
 * materialising it (bench.py cpu_baseline). */
void qo_encode_u32_seed(uint64_t seed, uint64_t start, uint64_t n, uint32_t t, uint32_t *S) {
    if (t == 0) return;
    for (uint64_t i = 0; i < n; ++i) insert32(S, t, (uint32_t)(qo_mix(seed + (start + i + 1) * QO_GAMMA) >> 32));
}

void qo_remove_u32(uint32_t *S, uint32_t t, uint32_t id) {
    uint32_t x = id % QO_P32, y = x;
    for (uint32_t k = 0; k < t; ++k) { S[k] = sub32(S[k], y); y = mul32(y, x); }
}

/* Newton's identities: c[i] = -(S[i] + sum_{j<i} S[j] c[i-j-1]) / (i+1). */
void qo_to_coeffs_u32(const uint32_t *S, uint32_t d, uint32_t *c) {
    for (uint32_t i = 0; i < d; ++i) {
        uint32_t acc = S[i];
        for (uint32_t j = 0; j < i; ++j) acc = add32(acc, mul32(S[j], c[i - j - 1]));
        c[i] = mul32(sub32(0, acc), pow32(i + 1, QO_P32 - 2));
    }
}

uint32_t qo_eval_u32(const uint32_t *c, uint32_t d, uint32_t id) {
    if (d == 0) return 1;
    uint32_t x = id % QO_P32, r = x;
    for (uint32_t i = 0; i + 1 < d; ++i) r = mul32(add32(r, c[i]), x);
    return add32(r, c[d - 1]);
}

/* Hit positions in log order; returns the number of hits (may exceed cap,
 * only the first cap are written). */
uint64_t qo_root_test_u32(const uint32_t *c, uint32_t d, const uint32_t *log, uint64_t n,
                          int64_t *hits, uint64_t cap) {
    uint64_t nh = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (qo_eval_u32(c, d, log[i]) == 0) { if (nh < cap) hits[nh] = (int64_t)i; ++nh; }
    return nh;
}

/* ---- GF(p64) ---------------------------------------------------------- */
static inline uint64_t add64(uint64_t a, uint64_t b) {   /* as add32: a mask, not a branch */
    const u128 s = (u128)a + b;
    const u128 m = (u128)0 - (u128)(s >= QO_P64);
    return (uint64_t)(s - (m & QO_P64));
}
static inline uint64_t sub64(uint64_t a, uint64_t b) { return a >= b ? a - b : (uint64_t)((u128)a + QO_P64 - b); }
static inline uint64_t mul64(uint64_t a, uint64_t b) { return (uint64_t)(((u128)a * b) % QO_P64); }
static uint64_t pow64(uint64_t a, uint64_t e) {
    uint64_t r = 1;
    while (e) { if (e & 1) r = mul64(r, a); a = mul64(a, a); e >>= 1; }
    return r;
}

static inline void insert64(uint64_t *S, uint32_t t, uint64_t id) {
    uint64_t x = id % QO_P64, y = x;
    for (uint32_t k = 0; k + 1 < t; ++k) { S[k] = add64(S[k], y); y = mul64(y, x); }
    S[t - 1] = add64(S[t - 1], y);
}

void qo_encode_u64(const uint64_t *ids, uint64_t n, uint32_t t, uint64_t *S) {
    if (t == 0) return;
    for (uint64_t i = 0; i < n; ++i) insert64(S, t, ids[i]);
}

void qo_encode_u64_seed(uint64_t seed, uint64_t start, uint64_t n, uint32_t t, uint64_t *S) {
    if (t == 0) return;
    for (uint64_t i = 0; i < n; ++i) insert64(S, t, qo_mix(seed + (start + i + 1) * QO_GAMMA));
}

void qo_to_coeffs_u64(const uint64_t *S, uint32_t d, uint64_t *c) {
    for (uint32_t i = 0; i < d; ++i) {
        uint64_t acc = S[i];
        for (uint32_t j = 0; j < i; ++j) acc = add64(acc, mul64(S[j], c[i - j - 1]));
        c[i] = mul64(sub64(0, acc), pow64(i + 1, QO_P64 - 2));
    }
}

uint64_t qo_eval_u64(const uint64_t *c, uint32_t d, uint64_t id) {
    if (d == 0) return 1;
    uint64_t x = id % QO_P64, r = x;
    for (uint32_t i = 0; i + 1 < d; ++i) r = mul64(add64(r, c[i]), x);
    return add64(r, c[d - 1]);
}

uint64_t qo_root_test_u64(const uint64_t *c, uint32_t d, const uint64_t *log, uint64_t n,
                          int64_t *hits, uint64_t cap) {
    uint64_t nh = 0;
    for (uint64_t i = 0; i < n; ++i)
        if (qo_eval_u64(c, d, log[i]) == 0) { if (nh < cap) hits[nh] = (int64_t)i; ++nh; }
    return nh;
}


/* ---- all-cores CPU baseline: the same scalar insert loop on
 * nthreads threads, one partial sketch per thread over a contiguous slice,
 * merged at the end (the sketch is additive). */
typedef struct {
    uint64_t seed, start, n;
    uint32_t t, bits;
    void *S;
    const void *ids;   /* pre-generated ids (slice [start, start + n)), or NULL: splitmix inline */
} qo_job;

static void *qo_worker(void *arg) {
    qo_job *j = (qo_job *)arg;
    if (j->ids) {
        if (j->bits == 32) qo_encode_u32((const uint32_t *)j->ids + j->start, j->n, j->t, (uint32_t *)j->S);
        else qo_encode_u64((const uint64_t *)j->ids + j->start, j->n, j->t, (uint64_t *)j->S);
    } else if (j->bits == 32) {
        qo_encode_u32_seed(j->seed, j->start, j->n, j->t, (uint32_t *)j->S);
    } else {
        qo_encode_u64_seed(j->seed, j->start, j->n, j->t, (uint64_t *)j->S);
    }
    return 0;
}

static int qo_encode_mt_impl(uint32_t bits, const void *ids, uint64_t seed, uint64_t start, uint64_t n, uint32_t t,
                             uint32_t nthreads, void *S) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    qo_job job[256];
    const size_t esz = bits == 32 ? 4 : 8;
    uint8_t *parts = (uint8_t *)calloc((size_t)nthreads * t, esz);
    if (!parts) return -1;
    uint32_t started = 0;
    for (uint32_t i = 0; i < nthreads; ++i, ++started) {
        const uint64_t b = n * i / nthreads, e = n * (i + 1) / nthreads;
        job[i] = (qo_job){seed, start + b, e - b, t, bits, parts + (size_t)i * t * esz, ids};
        if (pthread_create(&th[i], 0, qo_worker, &job[i])) break;
    }
    for (uint32_t i = 0; i < started; ++i) pthread_join(th[i], 0);
    if (started < nthreads) { free(parts); return -2; }
    for (uint32_t i = 0; i < nthreads; ++i)
        for (uint32_t k = 0; k < t; ++k) {
            if (bits == 32) ((uint32_t *)S)[k] = add32(((uint32_t *)S)[k], ((uint32_t *)parts)[(size_t)i * t + k]);
            else ((uint64_t *)S)[k] = add64(((uint64_t *)S)[k], ((uint64_t *)parts)[(size_t)i * t + k]);
        }
    free(parts);
    return 0;
}

/* returns 0 on success */
int qo_encode_seed_mt(uint32_t bits, uint64_t seed, uint64_t start, uint64_t n, uint32_t t, uint32_t nthreads,
                      void *S) {
    return qo_encode_mt_impl(bits, 0, seed, start, n, t, nthreads, S);
}
/* over a pre-generated id array (the crate's benchmark times inserts of
 * pre-generated ids) */
int qo_encode_mt(uint32_t bits, const void *ids, uint64_t n, uint32_t t, uint32_t nthreads, void *S) {
    return qo_encode_mt_impl(bits, ids, 0, 0, n, t, nthreads, S);
}

/* ---- reference-shape microbenchmark (BASELINE.md "Reference-shape row"):
 * the shape of the quack crate's `benchmark_construct` runs quoted there
 * (`-e 1000`, per-trial time / ids): each trial draws n fresh ids, then
 * times constructing an empty sketch of threshold t and inserting them.
 * Returns the summed timed nanoseconds; the folded sketches go to *sink so
 * the work cannot be elided.  The crate itself is absent (parity unpinned),
 * so this times the restatement's insert loop, not the crate. */
static uint64_t qo_now_ns(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

uint64_t qo_bench_construct(uint32_t bits, uint64_t seed, uint64_t n, uint32_t t, uint32_t trials, uint64_t *sink) {
    const size_t esz = bits == 32 ? 4 : 8;
    void *ids = malloc(n ? n * esz : 1), *S = malloc(t ? t * esz : 1);
    if (!ids || !S || t == 0) { free(ids); free(S); return 0; }
    uint64_t total = 0, fold = 0;
    for (uint32_t r = 0; r < trials; ++r) {
        if (bits == 32) qo_splitmix_u32(seed, (uint64_t)r * n, n, (uint32_t *)ids);
        else qo_splitmix_u64(seed, (uint64_t)r * n, n, (uint64_t *)ids);
        const uint64_t t0 = qo_now_ns();
        memset(S, 0, t * esz);
        if (bits == 32) qo_encode_u32((const uint32_t *)ids, n, t, (uint32_t *)S);
        else qo_encode_u64((const uint64_t *)ids, n, t, (uint64_t *)S);
        total += qo_now_ns() - t0;
        fold ^= bits == 32 ? ((uint32_t *)S)[t - 1] : ((uint64_t *)S)[t - 1];
    }
    if (sink) *sink = fold;
    free(ids);
    free(S);
    return total;
}

/* The crate's own unit: benchmark_construct reports avg_cycles, rdtsc
 * around its insert loop (zip:nsdi24/quack/threshold_vs_encode_time/32.txt:
 * 1-3; parsed by figures/fig2_microbenchmarks.py:48-69).  This times the
 * restatement's insert loop over pre-generated ids with the TSC and with
 * CLOCK_MONOTONIC around the same region, so the TSC rate comes from the
 * same run.  *tsc = 0 where there is no TSC (not x86-64). */
#if defined(__x86_64__)
#include <x86intrin.h>
static inline uint64_t qo_tsc(void) {
    _mm_lfence();
    const uint64_t v = __rdtsc();
    _mm_lfence();
    return v;
}
#else
static inline uint64_t qo_tsc(void) { return 0; }
#endif
void qo_encode_timed(uint32_t bits, const void *ids, uint64_t n, uint32_t t, void *S, uint64_t *tsc, uint64_t *ns) {
    const uint64_t n0 = qo_now_ns(), c0 = qo_tsc();
    if (bits == 32) qo_encode_u32((const uint32_t *)ids, n, t, (uint32_t *)S);
    else qo_encode_u64((const uint64_t *)ids, n, t, (uint64_t *)S);
    const uint64_t c1 = qo_tsc(), n1 = qo_now_ns();
    *tsc = c1 - c0;
    *ns = n1 - n0;
}

/* The same region read in core cycles, so that the baseline can say how its
 * TSC figure relates to the work the core did (a TSC tick is not a core
 * cycle on a boosting CPU):
 *   out[0] core cycles, out[1] instructions retired (perf_event_open,
 *          user-mode only, this thread; 0 where the kernel refuses —
 *          perf_event_paranoid, a container's seccomp),
 *   out[2] TSC ticks, out[3] ns (as qo_encode_timed),
 *   out[4] the core clock in kHz from a chain of dependent adds (1 cycle
 *          each) timed just before and just after the loop — an unprivileged
 *          reading of the clock the core runs at, whatever perf allows,
 *   out[5] errno of a refused perf_event_open (0 if it opened). */
#if defined(__linux__)
#include <errno.h>
#include <linux/perf_event.h>
#include <sys/ioctl.h>
#include <sys/syscall.h>
#include <unistd.h>
static int qo_perf_open(uint64_t config, int group) {
    struct perf_event_attr a;
    memset(&a, 0, sizeof a);
    a.type = PERF_TYPE_HARDWARE;
    a.size = sizeof a;
    a.config = config;
    a.disabled = group < 0;
    a.exclude_kernel = 1;
    a.exclude_hv = 1;
    return (int)syscall(SYS_perf_event_open, &a, 0, -1, group, 0);
}
#endif
/* kHz of this core: 2^26 dependent adds (1 cycle each on x86-64) */
static uint64_t qo_clock_khz(void) {
#if defined(__x86_64__)
    uint64_t best = 0;
    for (int rep = 0; rep < 3; ++rep) {
        uint64_t x = 0, k = 1u << 22;
        const uint64_t t0 = qo_now_ns();
        uint64_t one = 1;
        __asm__ volatile("" : "+r"(one));   /* a register operand: no immediate-add folding in the renamer */
        for (uint64_t i = 0; i < k; ++i)
            __asm__ volatile("add %1, %0\n\tadd %1, %0\n\tadd %1, %0\n\tadd %1, %0\n\t"
                             "add %1, %0\n\tadd %1, %0\n\tadd %1, %0\n\tadd %1, %0\n\t"
                             "add %1, %0\n\tadd %1, %0\n\tadd %1, %0\n\tadd %1, %0\n\t"
                             "add %1, %0\n\tadd %1, %0\n\tadd %1, %0\n\tadd %1, %0"
                             : "+r"(x)
                             : "r"(one));
        const uint64_t dt = qo_now_ns() - t0;
        const uint64_t khz = dt ? x * 1000000ull / dt : 0;   /* x adds in dt ns */
        if (khz > best) best = khz;
    }
    return best;
#else
    return 0;
#endif
}
void qo_encode_cycles(uint32_t bits, const void *ids, uint64_t n, uint32_t t, void *S, uint64_t *out) {
    memset(out, 0, 6 * sizeof(uint64_t));
    const uint64_t khz0 = qo_clock_khz();
    int fc = -1, fi = -1;
#if defined(__linux__)
    fc = qo_perf_open(PERF_COUNT_HW_CPU_CYCLES, -1);
    if (fc < 0) out[5] = (uint64_t)errno;
    else fi = qo_perf_open(PERF_COUNT_HW_INSTRUCTIONS, fc);
    if (fc >= 0) {
        ioctl(fc, PERF_EVENT_IOC_RESET, PERF_IOC_FLAG_GROUP);
        ioctl(fc, PERF_EVENT_IOC_ENABLE, PERF_IOC_FLAG_GROUP);
    }
#endif
    const uint64_t n0 = qo_now_ns(), c0 = qo_tsc();
    if (bits == 32) qo_encode_u32((const uint32_t *)ids, n, t, (uint32_t *)S);
    else qo_encode_u64((const uint64_t *)ids, n, t, (uint64_t *)S);
    const uint64_t c1 = qo_tsc(), n1 = qo_now_ns();
#if defined(__linux__)
    if (fc >= 0) {
        ioctl(fc, PERF_EVENT_IOC_DISABLE, PERF_IOC_FLAG_GROUP);
        uint64_t v = 0;
        if (read(fc, &v, sizeof v) == (ssize_t)sizeof v) out[0] = v;
        if (fi >= 0 && read(fi, &v, sizeof v) == (ssize_t)sizeof v) out[1] = v;
        close(fc);
        if (fi >= 0) close(fi);
    }
#endif
    const uint64_t khz1 = qo_clock_khz();
    out[2] = c1 - c0;
    out[3] = n1 - n0;
    out[4] = (khz0 + khz1) / 2;
}

/* CPU port of quack's benchmark_decode (figures/fig2_microbenchmarks.py:
 * 134-141,175-183; timed region [RECALL]): sender sketch of n ids, receiver
 * missing d of them (evenly spread), threshold t = d; each trial times
 * diff = sender - receiver, to_coeffs, and the root test over the n-id log.
 * Returns the summed timed nanoseconds; *found = hits of the last trial. */
uint64_t qo_bench_decode(uint32_t bits, uint64_t n, uint32_t d, uint32_t trials, uint64_t *found) {
    const size_t esz = bits == 32 ? 4 : 8;
    void *log = malloc(n ? n * esz : 1), *SA = calloc(d, esz), *SB = calloc(d, esz), *S = calloc(d, esz),
         *c = calloc(d, esz);
    int64_t *hits = malloc((n + 1) * sizeof(int64_t));
    if (!log || !SA || !SB || !S || !c || !hits || d == 0) return 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t v = qo_mix(0xDEC0DEull + (i + 1) * QO_GAMMA);
        const int dropped = (i * d) % n < d;
        if (bits == 32) {
            ((uint32_t *)log)[i] = (uint32_t)(v >> 32);
            insert32((uint32_t *)SA, d, (uint32_t)(v >> 32));
            if (!dropped) insert32((uint32_t *)SB, d, (uint32_t)(v >> 32));
        } else {
            ((uint64_t *)log)[i] = v;
            insert64((uint64_t *)SA, d, v);
            if (!dropped) insert64((uint64_t *)SB, d, v);
        }
    }
    uint64_t total = 0, nh = 0;
    for (uint32_t r = 0; r < trials; ++r) {
        const uint64_t t0 = qo_now_ns();
        if (bits == 32) {
            for (uint32_t k = 0; k < d; ++k) ((uint32_t *)S)[k] = sub32(((uint32_t *)SA)[k], ((uint32_t *)SB)[k]);
            qo_to_coeffs_u32((const uint32_t *)S, d, (uint32_t *)c);
            nh = qo_root_test_u32((const uint32_t *)c, d, (const uint32_t *)log, n, hits, n + 1);
        } else {
            for (uint32_t k = 0; k < d; ++k) ((uint64_t *)S)[k] = sub64(((uint64_t *)SA)[k], ((uint64_t *)SB)[k]);
            qo_to_coeffs_u64((const uint64_t *)S, d, (uint64_t *)c);
            nh = qo_root_test_u64((const uint64_t *)c, d, (const uint64_t *)log, n, hits, n + 1);
        }
        total += qo_now_ns() - t0;
    }
    if (found) *found = nh;
    free(log); free(SA); free(SB); free(S); free(c); free(hits);
    return total;
}
