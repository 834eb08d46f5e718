/* bench_common.h — shared helpers of the drop-in microbenchmark programs
 * (benchmark_construct.c, benchmark_decode.c): the id generator, clocks, and
 * the crate's SUMMARY lines.  The durations are printed the way Rust's
 * `Debug` for `Duration` prints them ("34.676µs", "1.2ms", "834ns"), since
 * the reference's figure script parses exactly that text
 * (figures/fig2_microbenchmarks.py:25-69). */
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

static inline uint64_t bench_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline double bench_now_ns(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e9 + ts.tv_nsec;
}

static inline uint64_t bench_cycles(void) {
#if defined(__x86_64__)
    return __builtin_ia32_rdtsc();
#else
    return (uint64_t)bench_now_ns();
#endif
}

/* Rust Debug of Duration::from_nanos(ns) */
static inline void bench_fmt_duration(uint64_t ns, char *out, size_t cap) {
    uint64_t whole, frac, scale;
    int digits;
    const char *unit;
    if (ns >= 1000000000ull) { scale = 1000000000ull; digits = 9; unit = "s"; }
    else if (ns >= 1000000ull) { scale = 1000000ull; digits = 6; unit = "ms"; }
    else if (ns >= 1000ull) { scale = 1000ull; digits = 3; unit = "µs"; }
    else { snprintf(out, cap, "%lluns", (unsigned long long)ns); return; }
    whole = ns / scale;
    frac = ns % scale;
    if (!frac) { snprintf(out, cap, "%llu%s", (unsigned long long)whole, unit); return; }
    char f[16];
    snprintf(f, sizeof f, "%0*llu", digits, (unsigned long long)frac);
    for (int i = (int)strlen(f) - 1; i > 0 && f[i] == '0'; --i) f[i] = 0;
    snprintf(out, cap, "%llu.%s%s", (unsigned long long)whole, f, unit);
}

static inline void bench_log_prefix(const char *name) {
    char ts[32];
    time_t now = time(NULL);
    struct tm tmv;
    gmtime_r(&now, &tmv);
    strftime(ts, sizeof ts, "%Y-%m-%dT%H:%M:%SZ", &tmv);
    fprintf(stderr, "[%s WARN  %s] ", ts, name);
}

/* the crate's two summary lines for `trials` trials of `n` packets each */
static inline void bench_summary(const char *name, unsigned long trials, double avg_ns, uint64_t avg_cycles,
                                 unsigned long n) {
    const uint64_t avg = (uint64_t)avg_ns;
    const uint64_t per = avg / n;
    char a[48], p[48];
    bench_fmt_duration(avg, a, sizeof a);
    bench_fmt_duration(per, p, sizeof p);
    bench_log_prefix(name);
    fprintf(stderr, "SUMMARY: num_trials = %lu, avg_cycles = %llu, avg = %s\n", trials,
            (unsigned long long)avg_cycles, a);
    bench_log_prefix(name);
    fprintf(stderr, "SUMMARY (per-packet): %s/packet = %llu packets/s = %llu cycles/packet\n", p,
            (unsigned long long)(per ? 1000000000ull / per : 0), (unsigned long long)(avg_cycles / n));
    fflush(stderr);
}
