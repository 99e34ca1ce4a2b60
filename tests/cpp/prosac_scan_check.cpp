// prosac_scan_check.cpp -- CPU check (tests/test_prosac_scan.py): usac::ProsacTerminationCriteria's
// scan with its lazily applied maximality updates (usac_host.hpp) against the plain scan it
// replaces (every candidate's standard-termination value computed and applied in place, as in
// prosac_termination_criteria.hpp:148-201), and its sorted-inlier-list variant, over random call
// sequences: every returned bound and every termination length equal.  Prints "ok <calls>" or the first difference.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "usac_host.hpp"

namespace {

struct PlainScan {  // the scan before the lazy updates, state kept here
    usac::StandardTerminationCriteria std_;
    std::vector<uint32_t> growth_, non_random_, maximality_;
    uint32_t n_, term_len_;
    PlainScan(const std::vector<uint32_t> &growth, float p, uint32_t m, uint32_t n, uint32_t max_iters)
        : std_(p, m, n, max_iters), growth_(growth),
          non_random_(usac::ProsacTerminationCriteria::table(n, m)), maximality_(n, 10000), n_(n), term_len_(n) {}
    uint32_t scan(uint32_t hypCount, const std::vector<char> &inl, uint32_t largest) {
        constexpr uint32_t kMin = 20;
        uint32_t max_samples = maximality_[term_len_ - 1];
        uint32_t count = 0;
        for (uint32_t i = 0; i < kMin; i++) count += inl[i] ? 1 : 0;
        bool cur = inl[kMin], nxt = false;
        for (uint32_t i = kMin; i < n_; ++i) {
            if (i != n_ - 1) nxt = inl[i + 1];
            count += cur ? 1 : 0;
            if (non_random_[i] < count) {
                non_random_[i] = count;
                if (i == n_ - 1 || (cur && !nxt)) {
                    uint32_t samples = std_.getUpBoundIterations(count, i + 1);
                    if (i + 1 < largest) samples += hypCount - growth_[i];
                    if (samples < maximality_[i]) {
                        maximality_[i] = samples;
                        if (samples < max_samples || (samples == max_samples && i + 1 >= term_len_)) {
                            term_len_ = i + 1;
                            max_samples = samples;
                        }
                    }
                }
            }
            cur = nxt;
        }
        return max_samples;
    }
};

}  // namespace

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 300;
    std::mt19937 g(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long calls = 0;
    for (int t = 0; t < trials; t++) {
        const uint32_t n = 100 + (uint32_t)(U(g) * 9900), m = (t % 3 == 0) ? 4u : (t % 3 == 1) ? 7u : 5u;
        const uint32_t max_iters = (t % 4 == 0) ? 1000u : 10000u;
        const float p = (t % 5 == 0) ? 0.99f : 0.95f;
        usac::ProsacSampler pro(t + 1, n, m);
        usac::ProsacTerminationCriteria lazy(pro.growth(), p, m, n, max_iters);
        usac::ProsacTerminationCriteria sorted(pro.growth(), p, m, n, max_iters);
        PlainScan plain(pro.growth(), p, m, n, max_iters);
        uint32_t hyp = 1 + (uint32_t)(U(g) * 20);
        const int ncalls = 1 + (int)(U(g) * 8);
        double quality = 0.2 + 0.7 * U(g);
        for (int k = 0; k < ncalls; k++) {
            std::vector<char> inl(n);
            const double front = quality * (0.5 + 0.5 * U(g)), noise = 0.05 * U(g);
            for (uint32_t i = 0; i < n; i++) {
                const double pr = front * (1.0 - (double)i / n) + noise;
                inl[i] = U(g) < pr ? 1 : 0;
            }
            switch ((t + k) % 23) {  // edge patterns now and then
                case 0: std::fill(inl.begin(), inl.end(), 1); break;                              // all
                case 1: std::fill(inl.begin() + 20, inl.end(), 0); break;                         // below kMin only
                case 2: inl[n - 1] = 1; inl[n - 2] = 0; break;                                    // last alone
                case 3: for (uint32_t i = 0; i < n; i++) inl[i] = (char)(i % 2); break;           // alternating
                case 4: std::fill(inl.begin(), inl.end(), 0); inl[n - 1] = 1; break;              // only the last
                case 5: std::fill(inl.begin(), inl.end() - n / 3, 1); break;                      // a tail run
                default: break;
            }
            const uint32_t largest = m + (uint32_t)(U(g) * (U(g) < 0.5 ? 50 : n));
            const uint32_t a = plain.scan(hyp, inl, largest);
            const uint32_t b = lazy.getUpBoundIterations(hyp, [&](uint32_t i) { return inl[i] != 0; }, largest);
            std::vector<int32_t> idx;
            for (uint32_t i = 0; i < n; i++)
                if (inl[i]) idx.push_back((int32_t)i);
            const uint32_t c = sorted.getUpBoundIterationsSorted(hyp, idx.data(), (uint32_t)idx.size(), largest);
            calls++;
            if (a != b || a != c || plain.term_len_ != lazy.terminationLength() ||
                plain.term_len_ != sorted.terminationLength()) {
                printf("diff trial %d call %d n %u m %u: bound %u / %u / %u, term_len %u / %u / %u\n", t, k, n, m, a,
                       b, c, plain.term_len_, lazy.terminationLength(), sorted.terminationLength());
                return 1;
            }
            hyp += 1 + (uint32_t)(U(g) * 200);
            quality = std::min(0.95, quality * (1.0 + 0.3 * U(g)));
        }
    }
    printf("ok %ld\n", calls);
    return 0;
}
