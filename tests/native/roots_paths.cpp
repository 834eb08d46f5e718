// roots_paths.cpp — the host root finding's vector paths against its scalar
// path (sidekick_amd/csrc/roots.cpp, included whole so its internals are
// reachable).  The library takes one path per CPU (IFMA on the GPU box's
// EPYC and on this container's Xeon); this program runs all of them on the
// same inputs and requires identical results:
//   the u64 squaring and product mod f:   scalar / AVX-512 (vpmuludq; the
//     product: scalar) / IFMA (52-bit limbs)
//   the u32 squaring and product mod f:   scalar / AVX-512
//   the multiplication by (z + c) mod f: scalar / AVX-512 (u32) / IFMA (u64)
//   the u64 row operation d = alpha d - beta s:  scalar / AVX-512 / IFMA
//   the small-modulus squaring and product (degree 2 .. 7): unrolled / loops
//   the gcd of operands of <= 40 coefficients: register rows / row calls
//   the field inverses: addition chains / field.h's binary ladders
// over degrees 8 .. 70 (vector tails of every length), random and edge
// coefficients (0, 1, p - 1, 2^52 - 1, 2^52), 2000 cases each, and up to the
// vector paths' largest degree (all coefficients p - 1: the largest sums).
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

// the squaring and the product mod f on every path against the scalar one:
// 2000 cases of degree 8..70, then 12 of degree up to the vector paths'
// limits with every coefficient p - 1 (the largest column sums) or random
template <class F> static int check_sqr(const char *name) {
    using T = typename F::T;
    for (int c = 0; c < 2012; ++c) {
        const bool big = c >= 2000;
        const size_t mmax = F::W == 64 ? IFMA_MAX : 1024;
        const size_t m = big ? (c % 2 ? mmax : mmax - 1 - rnd() % 400) : 8 + rnd() % 63;
        const bool worst = big && c % 3 == 0;
        Poly<F> f(m + 1);
        for (size_t i = 0; i < m; ++i) f[i] = worst ? F::neg(1) : pick<F>();
        f[m] = 1;
        std::vector<T> a(m), b(m);
        for (size_t i = 0; i < m; ++i) {
            a[i] = worst ? F::neg(1) : pick<F>();
            b[i] = worst ? F::neg(1) : pick<F>();
        }
        ModRing<F> R(f);
        std::vector<T> want = a, wantm = a, wantl = a;
        const T cl = pick<F>();
        const bool vec = R.vec, ifma = R.ifma;
        R.vec = false;
        R.ifma = false;
        R.sqr(want);
        R.mul(wantm, b);
        R.mul_lin(wantl, cl);
        for (int mode = 1; mode <= 2; ++mode) {
            if (!vec || (mode == 2 && !ifma) || (mode == 2 && F::W == 32)) continue;
            std::vector<T> got = a, gotm = a, gotl = a;
            R.vec = true;
            R.ifma = mode == 2;
            R.sqr(got);
            R.mul(gotm, b);
            R.mul_lin(gotl, cl);
            if (got != want || gotm != wantm || gotl != wantl) {
                printf("%s %s mismatch: m=%zu mode=%d case=%d\n", name,
                       got != want ? "sqr" : gotm != wantm ? "mul" : "mul_lin", m, mode, c);
                return 1;
            }
        }
    }
    return 0;
}

// the unrolled small-modulus squaring and product (degree 2 .. SMALL_MAX,
// ModRing::small) against the generic scalar loops
template <class F> static int check_small(const char *name) {
    using T = typename F::T;
    for (int c = 0; c < 6000; ++c) {
        const size_t m = 2 + c % (SMALL_MAX - 1);
        const bool worst = c % 7 == 0;
        Poly<F> f(m + 1);
        for (size_t i = 0; i < m; ++i) f[i] = worst ? F::neg(1) : pick<F>();
        f[m] = 1;
        std::vector<T> a(m), b(m);
        for (size_t i = 0; i < m; ++i) {
            a[i] = worst ? F::neg(1) : pick<F>();
            b[i] = worst ? F::neg(1) : pick<F>();
        }
        ModRing<F> R(f);
        if (!R.small) {
            printf("%s: degree %zu ring not on the small path\n", name, m);
            return 1;
        }
        std::vector<T> got = a, gotm = a, want = a, wantm = a;
        R.sqr(got);
        R.mul(gotm, b);
        R.small = false;
        R.sqr(want);
        R.mul(wantm, b);
        if (got != want || gotm != wantm) {
            printf("%s small %s mismatch: m=%zu case=%d\n", name, got != want ? "sqr" : "mul", m, c);
            return 1;
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

// gcd of operands up to 40 coefficients (the register path) against the
// row path: random pairs with a planted common factor of random degree
template <class F> static int check_gcd(const char *name) {
    using T = typename F::T;
    for (int c = 0; c < 3000; ++c) {
        const size_t dc = rnd() % 12, da = rnd() % (40 - dc), db = rnd() % (40 - dc);
        Poly<F> h{1}, a, b;
        for (size_t i = 0; i < dc; ++i) {   // h *= (z - r)
            const T r = pick<F>();
            Poly<F> t(h.size() + 1, 0);
            for (size_t k = 0; k < h.size(); ++k) {
                t[k + 1] = F::add(t[k + 1], h[k]);
                t[k] = F::sub(t[k], F::mul(h[k], r));
            }
            h = t;
        }
        for (int which = 0; which < 2; ++which) {
            Poly<F> x(which ? db : da);
            for (auto &v : x) v = pick<F>();
            Poly<F> y(x.size() + h.size() - 1 + (x.empty() ? 1 : 0), 0);
            if (x.empty()) y = h;
            else
                for (size_t i = 0; i < x.size(); ++i)
                    for (size_t j = 0; j < h.size(); ++j) y[i + j] = F::add(y[i + j], F::mul(x[i], h[j]));
            (which ? b : a) = y;
        }
        const Poly<F> g1 = gcd_rows<F>(a, b, true), g2 = gcd_rows<F>(a, b, false);
        if (g1 != g2) {
            printf("%s gcd mismatch: sizes %zu %zu case=%d\n", name, a.size(), b.size(), c);
            return 1;
        }
    }
    return 0;
}

// the inverse chains against the binary ladders of field.h
static int check_inv() {
    for (int c = 0; c < 20000; ++c) {
        const uint32_t a = c < 8 ? (uint32_t)(P32 - 1 - c) : F32::canon_any((uint32_t)rnd());
        const uint64_t b = c < 8 ? P64 - 1 - c : F64::canon_any(rnd());
        if ((a && inv32_chain(a) != inv32(a)) || (b && inv64_chain(b) != inv64(b))) {
            printf("inverse mismatch case=%d\n", c);
            return 1;
        }
    }
    return 0;
}

int main() {
    int rc = check_inv() | check_sqr<F64>("u64") | check_sqr<F32>("u32") | check_small<F64>("u64") |
             check_small<F32>("u32") | check_axmy64() | check_gcd<F32>("u32") | check_gcd<F64>("u64");
    printf("avx512=%d ifma=%d %s\n", (int)cpu_has_avx512(), (int)cpu_has_ifma(), rc ? "FAIL" : "ok");
    return rc;
}
