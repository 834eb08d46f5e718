#define _POSIX_C_SOURCE 199309L
/* benchmark_construct — drop-in for the quack crate's example of the same
 * name, as the reference's figure script runs it
 * (figures/fig2_microbenchmarks.py:205-213):
 *
 *   benchmark_construct power-sum -e 1000 --trials 100 -t T -b {32,64} [--montgomery]
 *
 * Each trial builds a fresh sketch of threshold T and inserts e random ids
 * through the C ABI (include/quack_hip.h); the timed region is the trial.
 * The two SUMMARY lines have the crate's format, which the figure's parsers
 * read (fig2_microbenchmarks.py:25-69: "avg = <duration>" and
 * "(per-packet): <duration>/packet").
 *
 * Paths: default = the per-packet host insert (qk_*_insert, what the
 * reference times); --gpu = one batch insert on the MI355X per trial from
 * host memory (qk_*_encode_host); --gpu-resident = ids already in HBM
 * (qk_*_encode_device).  Out of scope here: -b 16 /
 * --precompute (the u16 power table) and the strawman sketches.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bench_common.h"
#include "quack_hip.h"

static void usage(const char *p) {
    fprintf(stderr,
            "usage: %s power-sum [-e N] [--trials K] [-t T] [-b 32|64] [--montgomery] [--gpu|--gpu-resident]\n", p);
    exit(2);
}

int main(int argc, char **argv) {
    unsigned long n = 1000, trials = 10, t = 20;
    int bits = 32, gpu = 0, resident = 0;
    if (argc < 2) usage(argv[0]);
    if (strcmp(argv[1], "power-sum") != 0) {
        fprintf(stderr, "%s: only the power-sum sketch is provided (strawmen are out of scope)\n", argv[0]);
        return 2;
    }
    for (int i = 2; i < argc; ++i) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
        if ((!strcmp(a, "-e") || !strcmp(a, "-n") || !strcmp(a, "--num-packets")) && v) { n = strtoul(v, 0, 10); ++i; }
        else if (!strcmp(a, "--trials") && v) { trials = strtoul(v, 0, 10); ++i; }
        else if ((!strcmp(a, "-t") || !strcmp(a, "--threshold")) && v) { t = strtoul(v, 0, 10); ++i; }
        else if ((!strcmp(a, "-b") || !strcmp(a, "--num-bits-id")) && v) { bits = atoi(v); ++i; }
        else if (!strcmp(a, "--montgomery")) { /* the canonical sums do not depend on the representation */ }
        else if (!strcmp(a, "--gpu")) gpu = 1;
        else if (!strcmp(a, "--gpu-resident")) gpu = resident = 1;
        else if (!strcmp(a, "--precompute")) { fprintf(stderr, "--precompute (u16 power table) is out of scope\n"); return 2; }
        else usage(argv[0]);
    }
    if (bits != 32 && bits != 64) { fprintf(stderr, "-b %d: u32 and u64 identifiers only\n", bits); return 2; }
    if (t == 0 || t > QK_MAX_THRESHOLD || n == 0 || trials == 0) usage(argv[0]);

    const size_t esz = bits == 32 ? 4 : 8;
    const size_t qsz = bits == 32 ? qk_u32_size((uint32_t)t) : qk_u64_size((uint32_t)t);
    void *q = malloc(qsz), *ids = malloc((size_t)n * trials * esz);
    for (unsigned long i = 0; i < n * trials; ++i) {
        const uint64_t v = bench_mix(0xC0E5ull + (i + 1) * 0x9E3779B97F4A7C15ull);
        if (bits == 32) ((uint32_t *)ids)[i] = (uint32_t)(v >> 32);
        else ((uint64_t *)ids)[i] = v;
    }
    qk_ctx *ctx = NULL;
    void *dids = NULL;
    if (gpu) {
        int rc = qk_ctx_create(0, &ctx);
        if (rc != QK_OK) { fprintf(stderr, "--gpu: %s\n", qk_strerror(rc)); return 1; }
        if (resident) {
            if (hipMalloc(&dids, (size_t)n * trials * esz) != hipSuccess ||
                hipMemcpy(dids, ids, (size_t)n * trials * esz, hipMemcpyHostToDevice) != hipSuccess) {
                fprintf(stderr, "hipMalloc/hipMemcpy failed\n");
                return 1;
            }
        }
    }
    double total_ns = 0;
    uint64_t total_cycles = 0;
    uint64_t check = 0;
    for (long r = -2; r < (long)trials; ++r) {   /* 2 untimed warmup trials */
        const unsigned long k = r < 0 ? 0 : (unsigned long)r;
        const void *src = (const char *)ids + k * n * esz;
        const uint64_t c0 = bench_cycles();
        const double t0 = bench_now_ns();
        int rc = QK_OK;
        if (bits == 32) {
            qk_u32_init(q, (uint32_t)t);
            if (!gpu) for (unsigned long i = 0; i < n; ++i) rc |= qk_u32_insert(q, ((const uint32_t *)src)[i]);
            else if (!resident) rc = qk_u32_encode_host(ctx, src, n, q);
            else rc = qk_u32_encode_device(ctx, (const uint32_t *)dids + k * n, n, q, NULL);
        } else {
            qk_u64_init(q, (uint32_t)t);
            if (!gpu) for (unsigned long i = 0; i < n; ++i) rc |= qk_u64_insert(q, ((const uint64_t *)src)[i]);
            else if (!resident) rc = qk_u64_encode_host(ctx, src, n, q);
            else rc = qk_u64_encode_device(ctx, (const uint64_t *)dids + k * n, n, q, NULL);
        }
        const double dt = bench_now_ns() - t0;
        const uint64_t dc = bench_cycles() - c0;
        if (rc != QK_OK) { fprintf(stderr, "insert failed: %s\n", qk_strerror(rc)); return 1; }
        check ^= bits == 32 ? ((qk_u32 *)q)->power_sums[t - 1] : ((qk_u64 *)q)->power_sums[t - 1];
        if (r >= 0) { total_ns += dt; total_cycles += dc; }
    }
    bench_summary("benchmark_construct", trials, total_ns / trials, total_cycles / trials, n);
    if (dids) hipFree(dids);
    if (ctx) qk_ctx_destroy(ctx);
    free(q);
    free(ids);
    return check == 0xFFFFFFFFFFFFFFFFull;   /* keeps the sums live; never true in practice */
}
