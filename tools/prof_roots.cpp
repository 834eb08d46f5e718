// prof_roots.cpp — where the host root finding's time goes (roots.cpp,
// included whole).  For d distinct random roots: the whole roots() call, the
// ModRing set-up, one squaring and one product mod the degree-d product, the
// top-level exponentiation (z + a)^((p-1)/L), and one gcd of the product
// with w - 1.
// Min over reps (a shared host); one JSON line per field.
//   make -C tools prof_roots   (the product library's flags: baseline x86-64,
//   the vector paths behind target attributes and a CPU check)
//   ./prof_roots [d] [reps]
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "../sidekick_amd/csrc/roots.cpp"

static uint64_t sm = 0x5EEDull;
static uint64_t rnd() { return splitmix_mix(sm += GAMMA); }

template <class Fn> static double best_us(int reps, Fn &&fn) {
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        fn();
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        if (us < best) best = us;
    }
    return best;
}

template <class F> static void prof(const char *name, uint32_t d, int reps) {
    using T = typename F::T;
    Poly<F> f{1};
    for (uint32_t i = 0; i < d; ++i) {   // f *= (z - r)
        const T r = F::canon_any((T)rnd());
        Poly<F> g(f.size() + 1, 0);
        for (size_t k = 0; k < f.size(); ++k) {
            g[k + 1] = F::add(g[k + 1], f[k]);
            g[k] = F::sub(g[k], F::mul(f[k], r));
        }
        f = g;
    }
    std::vector<T> c(d);
    for (uint32_t i = 1; i <= d; ++i) c[i - 1] = f[d - i];
    volatile size_t sink = 0;
    const double t_all = best_us(reps, [&] { sink += roots<F>(c.data(), d).size(); });
    const double t_ring = best_us(reps, [&] { ModRing<F> R(f); sink += R.m; });
    ModRing<F> R(f);
    std::vector<T> a(R.m);
    for (auto &v : a) v = F::canon_any((T)rnd());
    const double t_sqr = best_us(reps, [&] {
        for (int i = 0; i < 16; ++i) R.sqr(a);
    }) / 16;
    std::vector<T> b(R.m);
    for (auto &v : b) v = F::canon_any((T)rnd());
    const double t_mul = best_us(reps, [&] {
        for (int i = 0; i < 16; ++i) R.mul(a, b);
    }) / 16;
    std::vector<T> w;
    const double t_pow = best_us(reps, [&] { w = R.pow_lin(F::canon_any((T)12345), F::PM1 / F::L); });
    Poly<F> w1 = to_poly<F>(w);
    if (w1.empty()) w1.push_back(0);
    w1[0] = F::sub(w1[0], 1);
    const double t_gcd = best_us(reps, [&] { sink += gcd<F>(f, w1).size(); });
    printf("{\"field\": \"%s\", \"d\": %u, \"roots_us\": %.2f, \"ring_setup_us\": %.2f, \"sqr_us\": %.3f, \"mul_us\": %.3f, "
           "\"pow_us\": %.2f, \"gcd_us\": %.2f, \"vec\": %d, \"ifma\": %d}\n",
           name, d, t_all, t_ring, t_sqr, t_mul, t_pow, t_gcd, (int)R.vec, (int)R.ifma);
    // the top-level split of f by Splitter's steps (E = 4 / 2 / 1 as F::E)
    const Splitter<F> S{};
    const std::vector<T> wv = R.pow_lin(F::canon_any((T)777), F::PM1 / F::L);
    const Poly<F> wp = to_poly<F>(wv);
    std::vector<T> vv;
    const double t_v = best_us(reps, [&] { vv = F::LO > 1 ? R.pow(wv, F::LO) : wv; });
    Poly<F> A, B;
    std::vector<T> qv = vv;
    if (F::E == 4) R.sqr(qv);
    const double t_cut = best_us(reps, [&] { S.cut(f, to_poly<F>(qv), 1, A, B); });
    std::vector<Poly<F>> parts;
    const double t_classes = best_us(reps, [&] {
        parts.clear();
        S.classes(A, wp, 0, F::canon_any((T)777), parts);
        S.classes(B, wp, 1, F::canon_any((T)777), parts);
    });
    const double t_inv = best_us(reps, [&] {
        T x = 3;
        for (int i = 0; i < 16; ++i) x = F::inv(F::add(x, 1));
        sink += x;
    }) / 16;
    printf("{\"field\": \"%s\", \"d\": %u, \"v_us\": %.2f, \"cut_us\": %.2f, \"classes_us\": %.2f, "
           "\"parts\": %zu, \"deg_A\": %zu, \"inv_us\": %.3f}\n",
           name, d, t_v, t_cut, t_classes, parts.size(), A.size() ? A.size() - 1 : 0, t_inv);
}

int main(int argc, char **argv) {
    const uint32_t d = argc > 1 ? (uint32_t)atoi(argv[1]) : 32;
    const int reps = argc > 2 ? atoi(argv[2]) : 200;
    prof<F32>("u32", d, reps);
    prof<F64>("u64", d, reps);
    return 0;
}
