// field_check.cpp — CPU checks of sidekick_amd/csrc/field.h (the arithmetic
// the gfx950 kernels and the host path share), and a search for identifiers
// that force the rare "wrapped" branch of the baby-step/giant-step encode.
//
//   field_check check            -> exhaustive edge + random congruence/bound checks
//   field_check find NB NA COUNT START
//                                -> first COUNT ids >= START whose lazy power
//                                   computation wraps for the (NB, NA) kernel
// Built and run by tests/test_field_native.py (g++ -O2); test infrastructure.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <initializer_list>

#include "../../sidekick_amd/csrc/field.h"

using namespace qk;
typedef unsigned __int128 u128;

static uint64_t rng_state = 0x1234567;
static uint64_t rnd() {
    rng_state += 0x9E3779B97F4A7C15ull;
    return splitmix_mix(rng_state);
}
static uint32_t r32() { return (uint32_t)(rnd() >> 32); }
static int fails = 0;
#define EXPECT(c, ...)                                                                             \
    do {                                                                                           \
        if (!(c)) {                                                                                \
            if (fails < 20) { printf("FAIL %s:%d: ", __FILE__, __LINE__); printf(__VA_ARGS__); printf("\n"); } \
            ++fails;                                                                               \
        }                                                                                          \
    } while (0)

static uint32_t ref_mul32(uint64_t a, uint64_t b) { return (uint32_t)((u128)a * b % P32); }

static void check_tstep(uint32_t lo, uint32_t hi, uint32_t x, uint32_t c) {
    const uint32_t x5 = times5_32(x);
    EXPECT(x5 == ref_mul32(x, 5), "times5 x=%u", x);
    const uint64_t t = lo + ((uint64_t)hi << 32);
    uint32_t l2 = lo, h2 = hi;
    tstep32(l2, h2, x, x5, c);
    const uint64_t t2 = l2 + ((uint64_t)h2 << 32);
    EXPECT(h2 <= 5, "tstep hi bound lo=%u hi=%u x=%u c=%u -> hi=%u", lo, hi, x, c, h2);
    EXPECT(t2 % P32 == ((u128)t * x + c) % P32, "tstep congruence lo=%u hi=%u x=%u c=%u", lo, hi, x, c);
    EXPECT(tstep32p(t, x, x5, c) == t2, "tstep32p != tstep32");
}

static void check_tstep64(uint64_t lo, uint32_t hi, uint64_t x) {
    const uint64_t x59 = mul64(x, C64);
    uint32_t t0 = (uint32_t)lo, t1 = (uint32_t)(lo >> 32), th = hi;
    tstep64(t0, t1, th, (uint32_t)x, (uint32_t)(x >> 32), (uint32_t)x59, (uint32_t)(x59 >> 32));
    const u128 v = ((u128)hi << 64) + lo, v2 = ((u128)th << 64) + (((uint64_t)t1 << 32) | t0);
    EXPECT(th <= 59, "tstep64 th bound hi=%u -> %u", hi, th);
    EXPECT((uint64_t)(v2 % P64) == (uint64_t)(v % P64 * x % P64), "tstep64 congruence");
}

static void check_mulfold(uint32_t y, uint32_t x) {
    uint32_t w = 0;
    const uint32_t f = mulfold32_fast(y, x, w);
    const uint32_t e = mulfold32_exact(y, x);
    EXPECT(e % P32 == ref_mul32(y, x) % P32 || canon32(e) == ref_mul32(y, x), "exact y=%u x=%u", y, x);
    EXPECT(canon32(e) == ref_mul32(y, x), "exact canon y=%u x=%u", y, x);
    if (!w) EXPECT(f == e, "fast != exact without wrap y=%u x=%u", y, x);
    EXPECT(canon32(mul32_lazy(y, x)) == ref_mul32(y, x), "mul32_lazy y=%u x=%u", y, x);
    EXPECT(canon32(mad32_lazy(y, x, 7)) == (uint32_t)(((u128)y * x + 7) % P32), "mad32_lazy");
    // min-tracked form (bsgs.h FOLD == 1): a wrap always leaves r < 25, and
    // any r >= 25 is the exact lazy product
    uint32_t mn = 0xFFFFFFFFu;
    const uint32_t m = mulfold32_min(y, x, mn);
    EXPECT(mn == m, "mulfold32_min tracks its result");
    if (w) EXPECT(m < 25, "wrapped fold left r=%u >= 25 (y=%u x=%u)", m, y, x);
    if (m >= 25) EXPECT(m == e, "min form != exact with r >= 25 y=%u x=%u", y, x);
}

static int run_check() {
    const uint32_t edges32[] = {0, 1, 2, 3, 4, 5, 6, P32 - 2, P32 - 1, P32, P32 + 1, P32 + 4, 0xFFFFFFFFu,
                                0x80000000u, 0x7FFFFFFFu, 0xFFFFFFF0u};
    const uint32_t canon_edges[] = {0, 1, 2, 5, P32 - 2, P32 - 1, 0x80000000u, 0x7FFFFFFFu};
    for (uint32_t lo : edges32)
        for (uint32_t hi = 0; hi <= 5; ++hi)
            for (uint32_t x : canon_edges)
                for (uint32_t c : canon_edges) check_tstep(lo, hi, x, c);
    for (int i = 0; i < 2000000; ++i) {
        const uint32_t x = r32() % P32, c = (i & 1) ? r32() % P32 : 0;
        check_tstep(r32(), r32() % 6, x, c);
    }
    for (uint32_t y : edges32)
        for (uint32_t x : edges32) check_mulfold(y, x);
    for (int i = 0; i < 2000000; ++i) check_mulfold(r32(), r32());
    for (uint32_t x : edges32) EXPECT(canon32(x) == x % P32, "canon32 %u", x);
    // 64-bit accumulator folds
    const uint64_t a64[] = {0, 1, ~0ull, ~0ull - 1, 1ull << 63, (1ull << 32) - 1, 1ull << 32, P32, 25ull << 32};
    for (uint64_t a : a64) EXPECT(canon32(fold64_32(a)) == a % P32, "fold64_32 %llu", (unsigned long long)a);
    for (int i = 0; i < 1000000; ++i) {
        const uint64_t a = rnd();
        EXPECT(canon32(fold64_32(a)) == a % P32, "fold64_32 rnd");
    }
    // GF(p64)
    const uint64_t e64[] = {0, 1, 58, 59, P64 - 1, P64, P64 + 1, ~0ull, 1ull << 63, 1ull << 32};
    for (uint64_t a : e64) {
        EXPECT(canon64(a) == a % P64, "canon64");
        for (uint64_t b : e64) {
            EXPECT(canon64(mul64_lazy(a, b)) == (uint64_t)((u128)a * b % P64), "mul64_lazy");
            EXPECT(canon64(mad64_lazy(a, b, 12345)) == (uint64_t)(((u128)a * b + 12345) % P64), "mad64_lazy");
        }
    }
    for (int i = 0; i < 500000; ++i) {
        const uint64_t a = rnd(), b = rnd(), c = rnd();
        EXPECT(canon64(mul64_lazy(a, b)) == (uint64_t)((u128)a * b % P64), "mul64_lazy rnd");
        EXPECT(canon64(mad64_lazy(a, b, c)) == (uint64_t)(((u128)a * b + c) % P64), "mad64_lazy rnd");
        const uint32_t h = r32();
        EXPECT(canon64(fold96_64(h, a)) == (uint64_t)((((u128)h << 64) + a) % P64), "fold96_64 rnd");
    }
    // u64 t-form step: edges of every operand, then random
    for (uint64_t lo : e64)
        for (uint32_t hi : {0u, 1u, 58u, 59u})
            for (uint64_t x : std::initializer_list<uint64_t>{0, 1, 59, P64 - 1, P64 - 2, 1ull << 63, 0xFFFFFFFFull, 1ull << 32})
                check_tstep64(lo, hi, x);
    for (int i = 0; i < 1000000; ++i) check_tstep64(rnd(), r32() % 60, rnd() % P64);
    printf("field_check: %s (%d failures)\n", fails ? "FAIL" : "ok", fails);
    return fails ? 1 : 0;
}

// mirror of encode.hip bsgs_powers: does any lazy fold wrap for this id?
static bool bsgs_wraps(uint32_t id, int NB, int NA) {
    uint32_t B[64], A[64], w = 0;
    B[0] = canon32(id);
    for (int b = 1; b < NB; ++b) B[b] = mulfold32_fast(B[b - 1], B[0], w);
    if (NA > 1) {
        A[0] = B[NB - 1];
        for (int a = 1; a < NA - 1; ++a) A[a] = mulfold32_fast(A[a - 1], A[0], w);
    }
    return w != 0;
}

int main(int argc, char **argv) {
    if (argc >= 2 && !strcmp(argv[1], "check")) return run_check();
    if (argc >= 6 && !strcmp(argv[1], "find")) {
        const int NB = atoi(argv[2]), NA = atoi(argv[3]);
        long want = atol(argv[4]);
        uint64_t id = strtoull(argv[5], 0, 0);
        for (; want > 0 && id <= 0xFFFFFFFFull; ++id)
            if (bsgs_wraps((uint32_t)id, NB, NA)) { printf("%llu\n", (unsigned long long)id); --want; }
        return 0;
    }
    fprintf(stderr, "usage: field_check check | find NB NA COUNT START\n");
    return 2;
}
