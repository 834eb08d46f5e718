// roots_paths.cpp — the host root finding's vector paths against its scalar
// path (sidekick_amd/csrc/roots.cpp, included whole so its internals are
// reachable).  The library takes one path per CPU (IFMA on the GPU box's
// EPYC and on this container's Xeon); this program runs all of them on the
// same inputs and requires identical results:
//   the u64 squaring mod f:   scalar / AVX-512 (vpmuludq) / IFMA (52-bit limbs)
//   the u32 squaring mod f:   scalar / AVX-512
//   the u64 row operation d = alpha d - beta s:  scalar / AVX-512 / IFMA
// over degrees 8 .. 70 (vector tails of every length), random and edge
// coefficients (0, 1, p - 1, 2^52 - 1, 2^52), 2000 cases each.
// Exit 0 iff all agree (prints the case on the first mismatch).
#include <cstdio>

#include "../../sidekick_amd/csrc/roots.cpp"

static uint64_t sm = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() { return splitmix_mix(sm += GAMMA); }

template <class F> static typename F::T pick() {
    using T = typename F::T;
    const uint64_t r = rnd();
    switch (r % 11) {
    case 0: return 0;
    case 1: return 1;
    case 2: return F::neg(1);
    case 3: return F::W == 64 ? (T)((1ull << 52) - 1) : (T)0xFFFFFFFAu;
    case 4: return F::W == 64 ? (T)(1ull << 52) : (T)P32 - 2;
    default: return F::canon_any((T)rnd());
    }
}

template <class F> static int check_sqr(const char *name) {
    using T = typename F::T;
    for (int c = 0; c < 2000; ++c) {
        const size_t m = 8 + rnd() % 63;
        Poly<F> f(m + 1);
        for (size_t i = 0; i < m; ++i) f[i] = pick<F>();
        f[m] = 1;
        std::vector<T> a(m);
        for (size_t i = 0; i < m; ++i) a[i] = pick<F>();
        ModRing<F> R(f);
        std::vector<T> want = a;
        const bool vec = R.vec, ifma = R.ifma;
        R.vec = false;
        R.sqr(want);
        for (int mode = 1; mode <= 2; ++mode) {
            if (!vec || (mode == 2 && !ifma) || (mode == 2 && F::W == 32)) continue;
            std::vector<T> got = a;
            R.vec = true;
            R.ifma = mode == 2;
            R.sqr(got);
            if (got != want) {
                printf("%s sqr mismatch: m=%zu mode=%d case=%d\n", name, m, mode, c);
                return 1;
            }
        }
    }
    return 0;
}

static int check_axmy64() {
    if (!cpu_has_avx512()) return 0;
    for (int c = 0; c < 2000; ++c) {
        const size_t m = 1 + rnd() % 70;
        std::vector<uint64_t> d(m), s(m);
        for (size_t i = 0; i < m; ++i) {
            d[i] = pick<F64>();
            s[i] = pick<F64>();
        }
        const uint64_t alpha = rnd() % 3 == 0 ? 1 : pick<F64>(), beta = pick<F64>();
        std::vector<uint64_t> want = d;
        for (size_t i = 0; i < m; ++i) want[i] = F64::sub(alpha == 1 ? d[i] : F64::mul(d[i], alpha), F64::mul(beta, s[i]));
        std::vector<uint64_t> g1 = d;
        axmy64_avx512(g1.data(), s.data(), m, alpha, beta);
        if (g1 != want) {
            printf("axmy64 avx512 mismatch m=%zu case=%d\n", m, c);
            return 1;
        }
        if (cpu_has_ifma()) {
            std::vector<uint64_t> g2 = d;
            axmy64_ifma(g2.data(), s.data(), m, alpha, beta);
            if (g2 != want) {
                printf("axmy64 ifma mismatch m=%zu case=%d\n", m, c);
                return 1;
            }
        }
    }
    return 0;
}

int main() {
    int rc = check_sqr<F64>("u64") | check_sqr<F32>("u32") | check_axmy64();
    printf("avx512=%d ifma=%d %s\n", (int)cpu_has_avx512(), (int)cpu_has_ifma(), rc ? "FAIL" : "ok");
    return rc;
}
