// Sprt::verify (word runs + no-crossing certificates) against Sprt::verify_plain (the reference's
// per-point loop, sprt.hpp:191-317) on random pool-order masks: decisions, counts, scores, the
// rolling pool index and the history must agree call for call.  Built and run by
// tests/test_sprt_walk.py (g++, host only).
#include <chrono>
#include <cstdio>
#include <random>
#include "usac_host.hpp"

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 300;
    std::mt19937_64 g(12345);
    long calls = 0, accepted = 0;
    double ta = 0, tb = 0;
    for (int t = 0; t < trials; t++) {
        const int est = 1 + (int)(g() % 4);
        const uint32_t n = t % 10 == 0 ? 1 + (uint32_t)(g() % 64)
                         : t % 10 == 1 ? 50000 + (uint32_t)(g() % 150000) : 100 + (uint32_t)(g() % 12000);
        const uint32_t nw = (n + 31) / 32, stride = 1 + (uint32_t)(g() % 3);
        usac::GlibcRandom ra((unsigned)t), rb((unsigned)t);
        usac::Sprt a(ra, est, n, 7, 100000, 20), b(rb, est, n, 7, 100000, 20);
        b.set_plain_walk(true);
        a.set_plain_walk(false);
        std::vector<uint32_t> w((size_t)nw * stride);
        uint32_t best = 0;
        for (int k = 0; k < 60; k++) {
            // inlier rate: mostly bad models, some good ones, some near the decision boundary
            const double r = std::uniform_real_distribution<double>(0, 1)(g);
            const double p = r < 0.5 ? 0.02 + 0.1 * r : r < 0.8 ? 0.15 + 0.5 * (r - 0.5) : 0.9 * (r - 0.8) + 0.3;
            std::bernoulli_distribution bit(p);
            for (uint32_t i = 0; i < nw; i++) {
                uint32_t v = 0;
                for (uint32_t b2 = 0; b2 < 32 && 32 * i + b2 < n; b2++) v |= (bit(g) ? 1u : 0u) << b2;
                w[(size_t)i * stride] = v;
            }
            int ca = -7, cb = -7;
            float sa = -7.f, sb = -7.f;
            const int hyp = (int)(g() % 40);
            const auto t0 = std::chrono::steady_clock::now();
            const bool ga = a.verify(w.data(), hyp, best, ca, sa, stride);
            const auto t1 = std::chrono::steady_clock::now();
            const bool gb = b.verify(w.data(), hyp, best, cb, sb, stride);
            ta += std::chrono::duration<double>(t1 - t0).count();
            tb += std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
            calls++;
            if (ga != gb || ca != cb || sa != sb || a.pool_index() != b.pool_index() ||
                a.histories() != b.histories() ||
                a.history().back().epsilon != b.history().back().epsilon ||
                a.history().back().delta != b.history().back().delta || a.history().back().A != b.history().back().A ||
                a.history().back().k != b.history().back().k) {
                printf("MISMATCH trial %d call %d n %u est %d: good %d/%d count %d/%d idx %u/%u hist %zu/%zu\n", t, k, n,
                       est, ga, gb, ca, cb, a.pool_index(), b.pool_index(), a.histories(), b.histories());
                return 1;
            }
            if (ga) {
                accepted++;
                if ((uint32_t)ca > best) best = (uint32_t)ca;
            }
        }
    }
    printf("OK calls %ld accepted %ld; walk time %.1f ms (per-point %.1f ms)\n", calls, accepted, ta * 1e3, tb * 1e3);
    return 0;
}
