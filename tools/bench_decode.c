#define _POSIX_C_SOURCE 199309L
/* bench_decode.c — the reference's decode microbenchmark shapes through the
 * C ABI (plain C against include/quack_hip.h, as the Rust FFI would bind it;
 * not product code).
 *
 *   bench_decode BITS MODE TRIALS n:d [n:d ...]     MODE = host | device
 *
 * Mirrors quack's benchmark_decode (figures/fig2_microbenchmarks.py:134-141,
 * 175-183; [RECALL] timed region): a sender sketch of n ids (threshold t =
 * d), a receiver sketch missing d of them; each trial times
 *     diff = clone(sender); diff.sub_assign(receiver); decode over the n-id log
 * with the host path (qk_*_decode_host) or the device path
 * (qk_*_decode_device, log resident in HBM).  Prints one JSON line per point.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "quack_hip.h"

static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double now_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

#define DIE(...) do { fprintf(stderr, __VA_ARGS__); exit(1); } while (0)

int main(int argc, char **argv) {
    if (argc < 5) DIE("usage: %s BITS host|device TRIALS n:d ...\n", argv[0]);
    const int bits = atoi(argv[1]);
    const int dev = strcmp(argv[2], "device") == 0;
    const int trials = atoi(argv[3]);
    qk_ctx *ctx = NULL;
    if (dev && qk_ctx_create(0, &ctx) != QK_OK) DIE("no device\n");
    for (int a = 4; a < argc; ++a) {
        unsigned long n = 0, d = 0;
        if (sscanf(argv[a], "%lu:%lu", &n, &d) != 2 || d == 0 || d > n) DIE("bad point %s\n", argv[a]);
        const size_t esz = bits == 32 ? 4 : 8;
        const size_t qsz = bits == 32 ? qk_u32_size((uint32_t)d) : qk_u64_size((uint32_t)d);
        void *log = malloc(n * esz), *A = malloc(qsz), *B = malloc(qsz), *D = malloc(qsz);
        uint64_t *hits = malloc((n + 1) * 8);
        if (bits == 32) { qk_u32_init(A, (uint32_t)d); qk_u32_init(B, (uint32_t)d); }
        else { qk_u64_init(A, (uint32_t)d); qk_u64_init(B, (uint32_t)d); }
        for (unsigned long i = 0; i < n; ++i) {
            const uint64_t v = mix(0xDEC0DEull + (i + 1) * 0x9E3779B97F4A7C15ull);
            const int dropped = (i * d) % n < d;                 /* d evenly spread drops */
            if (bits == 32) {
                ((uint32_t *)log)[i] = (uint32_t)(v >> 32);
                qk_u32_insert(A, (uint32_t)(v >> 32));
                if (!dropped) qk_u32_insert(B, (uint32_t)(v >> 32));
            } else {
                ((uint64_t *)log)[i] = v;
                qk_u64_insert(A, v);
                if (!dropped) qk_u64_insert(B, v);
            }
        }
        void *dlog = NULL;
        if (dev) {
            if (hipMalloc(&dlog, n * esz) != hipSuccess) DIE("hipMalloc\n");
            if (hipMemcpy(dlog, log, n * esz, hipMemcpyHostToDevice) != hipSuccess) DIE("hipMemcpy\n");
        }
        size_t nh = 0;
        double best = 1e30, total = 0;
        for (int r = -3; r < trials; ++r) {   /* 3 warmup trials */
            const double t0 = now_us();
            memcpy(D, A, qsz);
            int rc;
            if (bits == 32) {
                qk_u32_sub_assign(D, B);
                rc = dev ? qk_u32_decode_device(ctx, D, dlog, n, 0, hits, n + 1, &nh, NULL)
                         : qk_u32_decode_host(D, log, n, 0, hits, n + 1, &nh);
            } else {
                qk_u64_sub_assign(D, B);
                rc = dev ? qk_u64_decode_device(ctx, D, dlog, n, 0, hits, n + 1, &nh, NULL)
                         : qk_u64_decode_host(D, log, n, 0, hits, n + 1, &nh);
            }
            const double dt = now_us() - t0;
            if (rc != QK_OK) DIE("decode rc=%d (%s)\n", rc, qk_strerror(rc));
            if (r >= 0) { total += dt; if (dt < best) best = dt; }
        }
        if (nh < d) DIE("only %zu of %lu missing ids found\n", nh, d);
        printf("{\"bits\": %d, \"mode\": \"%s\", \"n\": %lu, \"d\": %lu, \"t\": %lu, \"trials\": %d, "
               "\"avg_us\": %.3f, \"min_us\": %.3f, \"hits\": %zu}\n",
               bits, dev ? "device" : "host", n, d, d, trials, total / trials, best, nh);
        fflush(stdout);
        if (dlog) hipFree(dlog);
        free(log); free(A); free(B); free(D); free(hits);
    }
    if (ctx) qk_ctx_destroy(ctx);
    return 0;
}
