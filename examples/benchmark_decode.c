#define _POSIX_C_SOURCE 199309L
/* benchmark_decode — drop-in for the quack crate's example of the same name,
 * as the reference's figure script runs it
 * (figures/fig2_microbenchmarks.py:85-95,134-141,175-183):
 *
 *   benchmark_decode power-sum -n N -d D -t T -b {32,64} --trials K [--montgomery]
 *
 * A sender sketch of the N logged ids and a receiver sketch missing D of them
 * (threshold T >= D); each trial times what media_client.rs:295-313 does on a
 * quACK: diff = sender - receiver, the coefficients of the missing ids, and
 * the root test over the N-id log — through the C ABI (include/quack_hip.h).
 * Prints the crate's SUMMARY lines (bench_common.h).
 *
 * Paths: default = host decode (qk_*_decode_host); --gpu = the gfx950 root
 * test over the log resident in HBM (qk_*_decode_device, launch-bound at the
 * figure's sizes).  Out of scope: -b 16 / --precompute and
 * --factor (the libpari factoring decoder).
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bench_common.h"
#include "quack_hip.h"

static void usage(const char *p) {
    fprintf(stderr, "usage: %s power-sum -n N -d D [-t T] [-b 32|64] [--trials K] [--montgomery] [--gpu]\n", p);
    exit(2);
}

int main(int argc, char **argv) {
    unsigned long n = 1000, d = 20, t = 0, trials = 10;
    int bits = 32, gpu = 0;
    if (argc < 2) usage(argv[0]);
    if (strcmp(argv[1], "power-sum") != 0) {
        fprintf(stderr, "%s: only the power-sum sketch is provided (strawmen are out of scope)\n", argv[0]);
        return 2;
    }
    for (int i = 2; i < argc; ++i) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
        if ((!strcmp(a, "-n") || !strcmp(a, "--num-packets")) && v) { n = strtoul(v, 0, 10); ++i; }
        else if ((!strcmp(a, "-d") || !strcmp(a, "--num-drop")) && v) { d = strtoul(v, 0, 10); ++i; }
        else if ((!strcmp(a, "-t") || !strcmp(a, "--threshold")) && v) { t = strtoul(v, 0, 10); ++i; }
        else if ((!strcmp(a, "-b") || !strcmp(a, "--num-bits-id")) && v) { bits = atoi(v); ++i; }
        else if (!strcmp(a, "--trials") && v) { trials = strtoul(v, 0, 10); ++i; }
        else if (!strcmp(a, "--montgomery")) { /* the canonical values do not depend on the representation */ }
        else if (!strcmp(a, "--gpu")) gpu = 1;
        else if (!strcmp(a, "--factor")) { fprintf(stderr, "--factor (libpari) is out of scope\n"); return 2; }
        else if (!strcmp(a, "--precompute")) { fprintf(stderr, "--precompute (u16 power table) is out of scope\n"); return 2; }
        else usage(argv[0]);
    }
    if (!t) t = d;
    if (bits != 32 && bits != 64) { fprintf(stderr, "-b %d: u32 and u64 identifiers only\n", bits); return 2; }
    if (d == 0 || d > n || t < d || t > QK_MAX_THRESHOLD || trials == 0) usage(argv[0]);

    const size_t esz = bits == 32 ? 4 : 8;
    const size_t qsz = bits == 32 ? qk_u32_size((uint32_t)t) : qk_u64_size((uint32_t)t);
    void *log = malloc(n * esz), *A = malloc(qsz), *B = malloc(qsz), *D = malloc(qsz);
    uint64_t *hits = malloc((n + 1) * 8);
    if (bits == 32) { qk_u32_init(A, (uint32_t)t); qk_u32_init(B, (uint32_t)t); }
    else { qk_u64_init(A, (uint32_t)t); qk_u64_init(B, (uint32_t)t); }
    for (unsigned long i = 0; i < n; ++i) {
        const uint64_t v = bench_mix(0xDEC0DEull + (i + 1) * 0x9E3779B97F4A7C15ull);
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
    qk_ctx *ctx = NULL;
    void *dlog = NULL;
    if (gpu) {
        int rc = qk_ctx_create(0, &ctx);
        if (rc != QK_OK) { fprintf(stderr, "--gpu: %s\n", qk_strerror(rc)); return 1; }
        if (hipMalloc(&dlog, n * esz) != hipSuccess || hipMemcpy(dlog, log, n * esz, hipMemcpyHostToDevice) != hipSuccess) {
            fprintf(stderr, "hipMalloc/hipMemcpy failed\n");
            return 1;
        }
    }
    size_t nh = 0;
    double total_ns = 0;
    uint64_t total_cycles = 0;
    for (long r = -2; r < (long)trials; ++r) {   /* 2 untimed warmup trials */
        const uint64_t c0 = bench_cycles();
        const double t0 = bench_now_ns();
        memcpy(D, A, qsz);
        int rc;
        if (bits == 32) {
            qk_u32_sub_assign(D, B);
            rc = gpu ? qk_u32_decode_device(ctx, D, dlog, n, 0, hits, n + 1, &nh, NULL)
                     : qk_u32_decode_host(D, log, n, 0, hits, n + 1, &nh);
        } else {
            qk_u64_sub_assign(D, B);
            rc = gpu ? qk_u64_decode_device(ctx, D, dlog, n, 0, hits, n + 1, &nh, NULL)
                     : qk_u64_decode_host(D, log, n, 0, hits, n + 1, &nh);
        }
        const double dt = bench_now_ns() - t0;
        const uint64_t dc = bench_cycles() - c0;
        if (rc != QK_OK) { fprintf(stderr, "decode failed: %s\n", qk_strerror(rc)); return 1; }
        if (r >= 0) { total_ns += dt; total_cycles += dc; }
    }
    if (nh < d) { fprintf(stderr, "only %zu of %lu missing ids found\n", nh, d); return 1; }
    bench_summary("benchmark_decode", trials, total_ns / trials, total_cycles / trials, n);
    if (dlog) hipFree(dlog);
    if (ctx) qk_ctx_destroy(ctx);
    free(log); free(A); free(B); free(D); free(hits);
    return 0;
}
