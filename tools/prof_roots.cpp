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
#include <string>

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
    {   // split() settings, alternated, over 8 root sets (the mean of their minima)
        std::vector<std::vector<T>> cs(8, std::vector<T>(d));
        for (auto &cv : cs) {
            Poly<F> h{1};
            for (uint32_t i = 0; i < d; ++i) {
                const T r = F::canon_any((T)rnd());
                Poly<F> g(h.size() + 1, 0);
                for (size_t k = 0; k < h.size(); ++k) {
                    g[k + 1] = F::add(g[k + 1], h[k]);
                    g[k] = F::sub(g[k], F::mul(h[k], r));
                }
                h = g;
            }
            for (uint32_t i = 1; i <= d; ++i) cv[i - 1] = h[d - i];
        }
        const size_t vs[] = {0, 4, 6, 8};   // small_split_deg (u32: factors split 10 ways up to it)
        const size_t keep = small_split_deg;
        printf("{\"field\": \"%s\", \"ab\": [", name);
        for (int r = 0; r < 4; ++r)
            for (int v = 0; v < 4; ++v) {
                small_split_deg = vs[v];
                double t = 0;
                for (auto &cv : cs) t += best_us(reps, [&] { sink += roots<F>(cv.data(), d).size(); }) / cs.size();
                printf("%s{\"small_split_deg\": %zu, \"roots_us\": %.2f}", r + v ? ", " : "", vs[v], t);
            }
        printf("]}\n");
        small_split_deg = keep;
    }
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
    if constexpr (F::W == 64) {   // the IFMA squaring's two stages: the products, the reduction mod f
        if (R.ifma) {
            const size_t cw = 2 * ((R.m + 7) & ~(size_t)7) + 16;
            uint64_t *c0 = R.cols.data() + ((8 - ((uintptr_t)R.cols.data() / 8) % 8) % 8);
            std::vector<T> x = a;
            R.sqr(x);   // leaves the last product's columns in c0 / c1 / c2
            std::vector<uint64_t> keep(c0, c0 + 3 * cw);
            const double t_red = best_us(reps, [&] {
                for (int i = 0; i < 16; ++i) {
                    std::copy(keep.begin(), keep.end(), c0);
                    red64_tab((uint64_t *)x.data(), R.m, R.tl0, R.tl1, c0, c0 + cw, c0 + 2 * cw);
                }
            }) / 16;
            const double t_cp = best_us(reps, [&] {
                for (int i = 0; i < 16; ++i) std::copy(keep.begin(), keep.end(), c0);
            }) / 16;
            double t_sq[2];
            for (int v = 0; v < 2; ++v) {
                reg_sqr = v;
                t_sq[v] = best_us(reps, [&] {
                    for (int i = 0; i < 16; ++i) R.sqr(x);
                }) / 16;
            }
            reg_sqr = true;
            printf("{\"field\": \"%s\", \"m\": %zu, \"sqr_mem_us\": %.3f, \"sqr_reg_us\": %.3f, \"red64_tab_us\": %.3f, "
                   "\"copy_us\": %.3f}\n",
                   name, R.m, t_sq[0], t_sq[1], t_red, t_cp);
        }
    }
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
    // the real top-level split (Splitter::run: exponentiation, v = w^LO, the
    // E-cuts, the classes of each part) and, for E = 4, the classes of the
    // four parts alone
    std::vector<Poly<F>> rp;
    const double t_run = best_us(reps, [&] {
        rp.clear();
        S.run(R, f, F::canon_any((T)777), rp);
    });
    if constexpr (F::E == 4) {
        Poly<F> A0, A2, B1, B3;
        const Poly<F> v = to_poly<F>(vv);
        if (A.size() > 2) S.cut(A, v, 1, A0, A2);
        else A2 = A;
        if (B.size() > 2) S.cut(B, v, F::pow(root_of_unity<F>(), F::LO), B1, B3);
        else B3 = B;
        std::vector<Poly<F>> p4;
        const double t_parts = best_us(reps, [&] {
            p4.clear();
            S.classes(A0, wp, 0, F::canon_any((T)777), p4);
            S.classes(A2, wp, 2, F::canon_any((T)777), p4);
            S.classes(B1, wp, 1, F::canon_any((T)777), p4);
            S.classes(B3, wp, 3, F::canon_any((T)777), p4);
        });
        // one class gcd on part B1 against one product mod B1 (scalar)
        Poly<F> wr = wp;
        rem_monic<F>(wr, B1);
        wr[0] = F::sub(wr[0], 5);
        const double t_g8 = best_us(reps, [&] {
            for (int i = 0; i < 16; ++i) sink += gcd_rows<F>(B1, wr, true, false).size();
        }) / 16;
        const size_t m8 = B1.size() - 1;
        std::vector<typename F::A> acc(2 * m8);
        Poly<F> pr = wr;
        pr.resize(m8, 0);
        const double t_m8 = best_us(reps, [&] {
            for (int it = 0; it < 16; ++it) {
                std::fill(acc.begin(), acc.end(), typename F::A(0));
                for (size_t i = 0; i < m8; ++i)
                    for (size_t j = 0; j < m8; ++j) F::mac(acc[i + j], pr[i], wr[j < wr.size() ? j : 0]);
                for (size_t k = 2 * m8 - 1; k-- > m8;) {
                    const T q = F::red(acc[k]);
                    for (size_t i = 0; i < m8; ++i) F::mac(acc[k - m8 + i], q, F::neg(B1[i]));
                }
                for (size_t i = 0; i < m8; ++i) pr[i] = F::red(acc[i]);
            }
        }) / 16;
        sink += pr[0];
        // the 11 class gcds of part B1: one at a time against one batch
        std::vector<Poly<F>> wrs;
        for (int j = 0; j < (int)F::LO; ++j) {
            wrs.push_back(wp);
            rem_monic<F>(wrs.back(), B1);
            if (wrs.back().empty()) wrs.back().push_back(0);
            wrs.back()[0] = F::sub(wrs.back()[0], (T)(1000 + j));
        }
        const double t_seq = best_us(reps, [&] {
            for (auto &b : wrs) sink += gcd_rows<F>(B1, b, true, false).size();
        });
        const double t_bat = best_us(reps, [&] { sink += gcd_many<F>(B1, wrs).size(); });
        const double t_rem = best_us(reps, [&] {
            Poly<F> wg = wp;
            rem_monic<F>(wg, B1);
            sink += wg.size();
        });
        std::vector<Poly<F>> p1;
        const double t_cl1 = best_us(reps, [&] {
            p1.clear();
            S.classes(B1, wp, 1, F::canon_any((T)777), p1);
        });
        printf("{\"field\": \"%s\", \"class_gcds_seq_us\": %.3f, \"class_gcds_batch_us\": %.3f, \"rem_w_us\": %.3f, "
               "\"classes_B1_us\": %.3f, \"B1_parts\": %zu}\n",
               name, t_seq, t_bat, t_rem, t_cl1, p1.size());
        printf("{\"field\": \"%s\", \"deg\": %zu, \"gcd_part_us\": %.3f, \"mulmod_part_us\": %.3f}\n", name, m8,
               t_g8, t_m8);
        printf("{\"field\": \"%s\", \"d\": %u, \"run_us\": %.2f, \"run_parts\": %zu, \"classes4_us\": %.2f, "
               "\"parts4\": %zu, \"deg\": [%zu, %zu, %zu, %zu]}\n",
               name, d, t_run, rp.size(), t_parts, p4.size(), A0.size() ? A0.size() - 1 : 0,
               A2.size() ? A2.size() - 1 : 0, B1.size() ? B1.size() - 1 : 0, B3.size() ? B3.size() - 1 : 0);
    }
    // what follows the top-level split in split(): the parts of >= 3 roots
    // (a ring and a split each), the quadratics (a square root each) — the
    // parts of the real top-level split above
    {
        std::vector<Poly<F>> big, quad;
        for (auto &p : rp)
            if (p.size() > 3) big.push_back(p);
            else if (p.size() == 3) quad.push_back(p);
        const double t_big = best_us(reps, [&] {
            for (auto g : big) {
                make_monic<F>(g);
                ModRing<F> R2(g);
                std::vector<Poly<F>> sp;
                S.run(R2, g, F::canon_any((T)4242), sp);
                sink += sp.size();
            }
        });
        const double t_quad = best_us(reps, [&] {
            for (auto &g : quad) {
                T r;
                sink += F::sqrt(F::sub(F::mul(g[1], g[1]), F::mul(F::mul(4, g[2]), g[0])), r);
                sink += r;
            }
        });
        double t_ring2 = 0, t_pow2 = 0;
        if (!big.empty()) {
            Poly<F> g = big[0];
            make_monic<F>(g);
            t_ring2 = best_us(reps, [&] { ModRing<F> R2(g); sink += R2.m; });
            ModRing<F> R2(g);
            t_pow2 = best_us(reps, [&] { sink += R2.pow_lin(F::canon_any((T)4242), F::PM1 / F::L)[0]; });
        }
        printf("{\"field\": \"%s\", \"part0_ring_us\": %.2f, \"part0_pow_us\": %.2f}\n", name, t_ring2, t_pow2);
        std::string degs;
        for (auto &p : big) degs += std::to_string(p.size() - 1) + " ";
        printf("{\"field\": \"%s\", \"big_parts_us\": %.2f, \"big_degs\": \"%s\", \"quadratics\": %zu, "
               "\"quad_us\": %.2f}\n",
               name, t_big, degs.c_str(), quad.size(), t_quad);
    }
    const double t_inv = best_us(reps, [&] {
        T x = 3;
        for (int i = 0; i < 16; ++i) x = F::inv(F::add(x, 1));
        sink += x;
    }) / 16;
    printf("{\"field\": \"%s\", \"d\": %u, \"v_us\": %.2f, \"cut_us\": %.2f, \"classes_us\": %.2f, "
           "\"parts\": %zu, \"deg_A\": %zu, \"inv_us\": %.3f}\n",
           name, d, t_v, t_cut, t_classes, parts.size(), A.size() ? A.size() - 1 : 0, t_inv);
}

// IFMA issue rate: 16 independent vpmadd52luq chains (ns per instruction),
// and one dependent chain (ns of latency); best of 20
QK_IFMA static void ifma_rate() {
    __m512i acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = _mm512_set1_epi64(i);
    const __m512i x = _mm512_set1_epi64(12345), y = _mm512_set1_epi64(678);
    const int N = 1 << 16;
    double t_thr = 1e30, t_lat = 1e30;
    __m512i c = acc[0];
    for (int r = 0; r < 20; ++r) {
        auto t0 = std::chrono::steady_clock::now();
        for (int it = 0; it < N; ++it)
            for (int i = 0; i < 16; ++i) acc[i] = _mm512_madd52lo_epu64(acc[i], x, y);
        for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(acc[i]));
        auto t1 = std::chrono::steady_clock::now();
        for (int it = 0; it < N * 4; ++it) c = _mm512_madd52lo_epu64(c, x, y);
        asm volatile("" : "+v"(c));
        auto t2 = std::chrono::steady_clock::now();
        t_thr = std::min(t_thr, std::chrono::duration<double, std::nano>(t1 - t0).count());
        t_lat = std::min(t_lat, std::chrono::duration<double, std::nano>(t2 - t1).count());
    }
    long long sink = _mm512_reduce_add_epi64(c);
    for (int i = 0; i < 16; ++i) sink += _mm512_reduce_add_epi64(acc[i]);
    printf("{\"ifma_ns_per_instr_independent\": %.4f, \"ifma_ns_latency\": %.4f, \"sink\": %lld}\n",
           t_thr / (16.0 * N), t_lat / (4.0 * N), sink & 1);
}

int main(int argc, char **argv) {
    if (cpu_has_ifma()) ifma_rate();
    const uint32_t d = argc > 1 ? (uint32_t)atoi(argv[1]) : 32;
    const int reps = argc > 2 ? atoi(argv[2]) : 200;
    prof<F32>("u32", d, reps);
    prof<F64>("u64", d, reps);
    return 0;
}
