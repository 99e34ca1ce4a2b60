// usac_host.hpp -- host-side mirror of the reference's plugin surface (C++17), the layer
// a reference-style driver talks to.  Names and argument meaning follow the reference;
// the work is done by the device (usac_api.cpp / kernels*.hip).
//
//   usac::Score                      quality.hpp:16-37
//   usac::UniformSampler             uniform_sampler.hpp:49-95 over a private glibc
//                                    random_r TYPE_3 state (= random()/srandom() stream)
//   usac::StandardTerminationCriteria standard_termination_criteria.hpp:10-74
//   usac::Mt19937 / UniformIntDist   std::mt19937 + uniform_int_distribution<int>
//                                    (uniform_random_generator.hpp:16-63)
//   usac::ProsacSampler              prosac_sampler.hpp:62-172
//   usac::ProsacTerminationCriteria  prosac_termination_criteria.hpp:44-201
//   usac::Sprt                       sprt.hpp:89-491 (decisions on device inlier masks)
//   usac::GridNeighbors              nearest_neighbors.cpp:160-202
//   usac::NapsacSampler              napsac_sampler.hpp:40-158 (grid), array_random_generator.hpp
//   usac::NapsacKnnSampler           napsac_sampler.hpp:76-98 (KNN rows from usac_knn)
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace usac {

struct Score {
    int inlier_number = 0;
    float score = 0.f;
    bool bigger(const Score &o) const {
        if (inlier_number > o.inlier_number) return true;
        if (inlier_number == o.inlier_number) return score > o.score;
        return false;
    }
};

// glibc random() stream with private state: initstate_r with a 128-byte buffer selects
// TYPE_3 and seeds it exactly as srandom(seed) seeds the default state.
class GlibcRandom {
   public:
    explicit GlibcRandom(unsigned int seed) {
        memset(&data_, 0, sizeof(data_));
        memset(state_, 0, sizeof(state_));
        initstate_r(seed, state_, sizeof(state_), &data_);
    }
    uint32_t next() {
        int32_t r;
        random_r(&data_, &r);
        return (uint32_t)r;
    }
    // the generator's state, saved and restored in place (random_data points into state_,
    // so a state only goes back into the object it came from)
    struct Saved {
        char state[128];
        struct random_data data;
    };
    void save(Saved &o) const {
        memcpy(o.state, state_, sizeof(state_));
        o.data = data_;
    }
    void restore(const Saved &o) {
        memcpy(state_, o.state, sizeof(state_));
        data_ = o.data;
    }

   private:
    char state_[128];
    struct random_data data_;
};

class UniformSampler {
   public:
    UniformSampler(unsigned int seed, uint32_t points_size, uint32_t sample_size)
        : own_(seed), rng_(own_), pool_(points_size), max_((int)points_size), n_(points_size), m_(sample_size) {
        for (uint32_t i = 0; i < points_size; i++) pool_[i] = i;
    }
    // sampler drawing from a shared stream (the reference's global random(): the SPRT pool
    // shuffle and the sampler consume the same sequence)
    UniformSampler(GlibcRandom &shared, uint32_t points_size, uint32_t sample_size)
        : own_(1), rng_(shared), pool_(points_size), max_((int)points_size), n_(points_size), m_(sample_size) {
        for (uint32_t i = 0; i < points_size; i++) pool_[i] = i;
    }
    // uniform_sampler.hpp:42-54: persistent pool; refill when max reaches 0 (also
    // mid-sample)
    void generateSample(int32_t *sample) {
        for (uint32_t i = 0; i < m_; i++) {
            if (max_ == 0) max_ = (int)n_;
            uint32_t idx = rng_.next() % (uint32_t)max_;
            uint32_t v = pool_[idx];
            max_--;
            pool_[idx] = pool_[max_];
            pool_[max_] = v;
            sample[i] = (int32_t)v;
            if (journal_on_) journal_.push_back({idx, (uint32_t)max_});
        }
    }
    // speculative draws (the loop's next batch drawn ahead): mark the state, draw, and either
    // keep the draws (commit) or undo them (rollback: the pool swaps in reverse order, the
    // generator and the pool size restored)
    void mark() {
        rng_.save(mark_rng_);
        mark_max_ = max_;
        journal_.clear();
        journal_on_ = true;
    }
    void commit() {
        journal_on_ = false;
        journal_.clear();
    }
    void rollback() {
        for (auto it = journal_.rbegin(); it != journal_.rend(); ++it) std::swap(pool_[it->first], pool_[it->second]);
        max_ = mark_max_;
        rng_.restore(mark_rng_);
        commit();
    }

   private:
    GlibcRandom own_;
    GlibcRandom &rng_;
    std::vector<uint32_t> pool_;
    int max_;
    uint32_t n_, m_;
    bool journal_on_ = false;
    std::vector<std::pair<uint32_t, uint32_t>> journal_;
    GlibcRandom::Saved mark_rng_;
    int mark_max_ = 0;
};

// standard_termination_criteria.hpp:24-31, 52-62 (fp32 ratio power, 0.0005f floor,
// double log of (1 - q), truncation to unsigned: SURVEY Q14)
class StandardTerminationCriteria {
   public:
    StandardTerminationCriteria(float desired_prob, uint32_t sample_size, uint32_t points_size,
                                uint32_t max_iterations)
        : log_1_p_((float)std::log((double)(1 - desired_prob))),
          m_(sample_size),
          n_(points_size),
          max_(max_iterations) {}
    uint32_t getUpBoundIterations(uint32_t inlier_size) const { return getUpBoundIterations(inlier_size, n_); }
    // two-argument overload (standard_termination_criteria.hpp:64-74), used by PROSAC
    uint32_t getUpBoundIterations(uint32_t inlier_size, uint32_t points_size) const {
        float inl_ratio = (float)inlier_size / (float)points_size;
        float inl_prob = inl_ratio * inl_ratio;
        int k = (int)m_;
        while (k > 2) {
            inl_prob *= inl_ratio;
            k--;
        }
        if (inl_prob < 0.0005f) return max_;
        double r = (double)log_1_p_ / std::log((double)(1 - inl_prob));
        return (uint32_t)r;
    }
    // A lower bound of the two-argument getUpBoundIterations without its log: the value itself
    // (exact = true) below the 0.0005 floor, else floor(|log(1-p)| y / (1 - y) (1 - 2^-40)) with
    // y = the same float 1 - w^m: -ln y <= (1 - y) / y, and the log (< 1 ulp) and the two
    // roundings of r are far inside the 2^-40 slack.
    uint32_t lowerBound(uint32_t inlier_size, uint32_t points_size, bool &exact) const {
        float inl_ratio = (float)inlier_size / (float)points_size;
        float inl_prob = inl_ratio * inl_ratio;
        int k = (int)m_;
        while (k > 2) {
            inl_prob *= inl_ratio;
            k--;
        }
        exact = inl_prob < 0.0005f;
        if (exact) return max_;
        const double y = (double)(1 - inl_prob), x = 1.0 - y;  // (x exact: y is a float in (0, 1))
        if (!(x > 0.0)) return 0;                             // (no bound: p rounded to 0 in 1 - p)
        const double lb = -(double)log_1_p_ * y / x * (1.0 - 9.094947017729282e-13);  // 2^-40
        return lb >= 4294967295.0 ? 4294967295u : (uint32_t)lb;
    }

   private:
    float log_1_p_;
    uint32_t m_, n_, max_;
};

// ---------------------------------------------------------------- PROSAC
// std::mt19937 (32-bit Mersenne twister, default tempering) -- the reference's PROSAC
// generator; seeded here with the run seed (the reference uses std::random_device).
class Mt19937 {
   public:
    explicit Mt19937(uint32_t seed) {
        s_[0] = seed;
        for (int i = 1; i < kN; i++) s_[i] = 1812433253u * (s_[i - 1] ^ (s_[i - 1] >> 30)) + (uint32_t)i;
        pos_ = kN;
    }
    uint32_t operator()() {
        if (pos_ == kN) twist();
        uint32_t y = s_[pos_++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        return y ^ (y >> 18);
    }

   private:
    static constexpr int kN = 624, kM = 397;
    void twist() {
        for (int k = 0; k < kN; k++) {
            const uint32_t y = (s_[k] & 0x80000000u) | (s_[(k + 1) % kN] & 0x7fffffffu);
            s_[k] = s_[(k + kM) % kN] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        pos_ = 0;
    }
    uint32_t s_[kN];
    int pos_;
};

// uniform_int_distribution<int>(0, hi) as libstdc++ implemented it through GCC 10
// (downscaling by the generator range; the toolchain of the reference's era).
inline int uniform_int(Mt19937 &g, uint32_t hi) {
    const uint64_t range = 0xFFFFFFFFull;
    if ((uint64_t)hi == range) return (int)g();
    const uint64_t buckets = (uint64_t)hi + 1, scale = range / buckets, limit = buckets * scale;
    uint64_t r;
    do r = g(); while (r >= limit);
    return (int)(r / scale);
}

// UniformRandomGenerator::generateUniqueRandomSet(sample, k, hi): k distinct draws from
// the closed range <0; hi>, a repeat is redrawn (uniform_random_generator.hpp:44-54)
inline void unique_set(Mt19937 &g, int32_t *sample, uint32_t k, uint32_t hi) {
    for (uint32_t i = 0; i < k; i++) {
        const int v = uniform_int(g, hi);
        bool dup = false;
        for (uint32_t j = 0; j < i; j++) dup |= sample[j] == v;
        if (dup) i--;
        else sample[i] = v;
    }
}

class ProsacSampler {
   public:
    // prosac_sampler.hpp:62-114 (T_N = 200000)
    ProsacSampler(uint32_t seed, uint32_t points_size, uint32_t sample_size)
        : rng_(seed), growth_(growth_table(points_size, sample_size)), n_(points_size), m_(sample_size) {
        largest_ = subset_ = m_;
        hyp_ = 1;
    }
    // the growth function depends on (n, m) alone: computed once per shape and shared (a dependent
    // chain of n fp64 divisions, ~0.1 ms at n = 10 k -- a tenth of a cfg3 run when rebuilt per run;
    // snapshots of the sampler share it too)
    static std::shared_ptr<const std::vector<uint32_t>> growth_table(uint32_t n, uint32_t m) {
        static std::mutex mu;
        static std::map<std::pair<uint32_t, uint32_t>, std::shared_ptr<const std::vector<uint32_t>>> cache;
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = cache.find({n, m});
            if (it != cache.end()) return it->second;
        }
        auto t = std::make_shared<std::vector<uint32_t>>(n);
        std::vector<uint32_t> &growth = *t;
        double T_n = kGrowthMax;
        for (uint32_t i = 0; i < m; ++i) T_n *= (double)(m - i) / (n - i);
        uint32_t T_prime = 1;
        for (uint32_t i = 0; i < n; ++i) {
            if (i + 1 <= m) {
                growth[i] = T_prime;
                continue;
            }
            const double T_next = (double)(i + 1) * T_n / (i + 1 - m);
            growth[i] = T_prime + (uint32_t)std::ceil(T_next - T_n);
            T_n = T_next;
            T_prime = growth[i];
        }
        std::lock_guard<std::mutex> g(mu);
        if (cache.size() > 64) cache.clear();
        cache[{n, m}] = t;
        return t;
    }
    // prosac_sampler.hpp:117-172 with the current termination_length
    void generateSample(int32_t *sample, uint32_t termination_length) {
        if (hyp_ > kGrowthMax) {
            unique_set(rng_, sample, m_, n_);  // closed range (reference), guarded by the caller
            return;
        }
        if (subset_ > termination_length) {
            unique_set(rng_, sample, m_, termination_length);  // closed range, SURVEY Q15
            return;
        }
        if (hyp_ > (*growth_)[subset_ - 1]) {
            if (++subset_ > n_) subset_ = n_;
            largest_ = std::max(largest_, subset_);
        }
        unique_set(rng_, sample, m_ - 1, subset_ - 2);
        sample[m_ - 1] = (int32_t)subset_ - 1;
        hyp_++;
    }
    const std::vector<uint32_t> &growth() const { return *growth_; }
    uint32_t largest() const { return largest_; }
    uint32_t subset() const { return subset_; }
    static constexpr uint32_t kGrowthMax = 200000;

   private:
    Mt19937 rng_;
    std::shared_ptr<const std::vector<uint32_t>> growth_;
    uint32_t n_, m_, largest_, subset_, hyp_;
};

class ProsacTerminationCriteria {
   public:
    // prosac_termination_criteria.hpp:44-119: non-random inlier minima (beta 0.05,
    // Psi 0.05, tabulated up to n = 1001 then held), maximality samples = 10000
    ProsacTerminationCriteria(const std::vector<uint32_t> &growth, float desired_prob, uint32_t sample_size,
                              uint32_t points_size, uint32_t max_iterations)
        : std_(desired_prob, sample_size, points_size, max_iterations),
          growth_(growth),
          non_random_(table(points_size, sample_size)),
          maximality_(points_size, 10000),
          pend_(points_size, 0),
          n_(points_size),
          term_len_(points_size) {}

    // the non-random inlier minima depend on (n, m) alone: computed once per shape and kept (the
    // reference recomputes them in every ctor, O(1000^2) pow / div, ~1.4 ms a run)
    static std::vector<uint32_t> table(uint32_t points_size, uint32_t sample_size) {
        static std::mutex mu;
        static std::map<std::pair<uint32_t, uint32_t>, std::vector<uint32_t>> cache;
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = cache.find({points_size, sample_size});
            if (it != cache.end()) return it->second;
        }
        std::vector<uint32_t> t = non_random_table(points_size, sample_size);
        std::lock_guard<std::mutex> g(mu);
        if (cache.size() > 64) cache.clear();
        cache[{points_size, sample_size}] = t;
        return t;
    }
    static std::vector<uint32_t> non_random_table(uint32_t n_, uint32_t m_) {
        std::vector<uint32_t> non_random_(n_, 0);
        const float psi = 0.95f, beta = 0.05f;
        std::vector<double> pn(n_);
        for (size_t n = m_ + 1; n <= n_; ++n) {
            if (n - 1 > 1000) {
                non_random_[n - 1] = non_random_[n - 2];
                continue;
            }
            std::fill(pn.begin(), pn.begin() + n, 0.0);  // entries [0, n) are the ones read
            pn[m_] = beta * std::pow((double)1 - beta, (double)n - m_ - 1) * (n - m_);
            double prev = pn[m_];
            for (size_t i = m_ + 2; i <= n; ++i) {
                if (i == n) {
                    pn[n - 1] = std::pow((double)beta, (double)n - m_);
                    break;
                }
                pn[i - 1] = prev * (beta / (1 - beta)) * ((double)(n - i) / (i - m_ + 1));
                prev = pn[i - 1];
            }
            double acc = 0.0;
            uint32_t imin = 0;
            for (size_t i = n; i >= m_ + 1; --i) {
                acc += pn[i - 1];
                if (acc < 1 - psi) imin = (uint32_t)i;
                else break;
            }
            non_random_[n - 1] = imin;
        }
        return non_random_;
    }
    uint32_t terminationLength() const { return term_len_; }
    // prosac_termination_criteria.hpp:148-201; inlier(i) = error of point i < threshold for
    // the new best model, largest = the sampler's largest_sample_size at that iteration
    //
    // The standard-termination value of a candidate (a log each, ~1 800 on a first scan at
    // n = 10 k) is computed only where it can decide something now: a candidate whose value is
    // provably above the running max_samples (StandardTerminationCriteria::lowerBound) cannot
    // move term_len / max_samples, and its maximality update -- min(maximality_[i], value) -- is
    // recorded as pending (the count) and applied when maximality_[i] is next read.  The results
    // and the state are the reference's, value for value (tests/test_prosac_scan.py runs both).
    template <class Flags>
    uint32_t getUpBoundIterations(uint32_t hypCount, const Flags &inlier, uint32_t largest) {
        uint32_t max_samples = maximality(term_len_ - 1);
        uint32_t count = 0;
        for (uint32_t i = 0; i < kMin; i++) count += inlier(i) ? 1 : 0;
        bool cur = inlier(kMin), nxt = false;
        for (uint32_t i = kMin; i < n_; ++i) {
            if (i != n_ - 1) nxt = inlier(i + 1);
            count += cur ? 1 : 0;
            if (non_random_[i] < count) {
                non_random_[i] = count;
                if (i == n_ - 1 || (cur && !nxt)) candidate(i, count, hypCount, largest, max_samples);
            }
            cur = nxt;
        }
        return max_samples;
    }
    // The same scan from the new best's inlier indices in ascending order (idx[0 .. cnt)): the
    // count is constant between consecutive inliers, so each stretch of outliers is one max()
    // pass over non_random_, and the candidates -- the last inlier of a run, and point n - 1 --
    // are visited in the same order as above.
    uint32_t getUpBoundIterationsSorted(uint32_t hypCount, const int32_t *idx, uint32_t cnt, uint32_t largest) {
        uint32_t max_samples = maximality(term_len_ - 1);
        uint32_t k = 0;  // inliers below i
        while (k < cnt && (uint32_t)idx[k] < kMin) k++;
        uint32_t i = kMin;
        while (i < n_) {
            while (k < cnt && (uint32_t)idx[k] < i) k++;  // (only a list out of order: always progress)
            if (k < cnt && (uint32_t)idx[k] == i) {  // an inlier: count k + 1
                const uint32_t count = k + 1;
                const bool last = i == n_ - 1 || k + 1 == cnt || (uint32_t)idx[k + 1] != i + 1;
                if (non_random_[i] < count) {
                    non_random_[i] = count;
                    if (last) candidate(i, count, hypCount, largest, max_samples);
                }
                k++;
                i++;
                continue;
            }
            // outliers i .. e - 1 at count k; of them only point n - 1 can be a candidate
            const uint32_t e = k < cnt ? (uint32_t)idx[k] : n_;
            const uint32_t e1 = e == n_ ? n_ - 1 : e;
            uint32_t *nr = non_random_.data();
            for (uint32_t j = i; j < e1; j++) nr[j] = nr[j] < k ? k : nr[j];
            if (e == n_ && nr[n_ - 1] < k) {
                nr[n_ - 1] = k;
                candidate(n_ - 1, k, hypCount, largest, max_samples);
            }
            i = e;
        }
        return max_samples;
    }

   private:
    static constexpr uint32_t kMin = 20;
    // candidate i (count inliers up to it) after its non-random update: its standard-termination
    // value, maximality and the running minimum (prosac_termination_criteria.hpp:170-195)
    void candidate(uint32_t i, uint32_t count, uint32_t hypCount, uint32_t largest, uint32_t &max_samples) {
        uint32_t samples;
        if (i + 1 < largest) {
            samples = std_.getUpBoundIterations(count, i + 1) + (hypCount - growth_[i]);
        } else {
            bool exact;
            const uint32_t lb = std_.lowerBound(count, i + 1, exact);
            if (!exact && lb > max_samples) {
                if (pend_[i]) maximality(i);  // an older pending update first
                pend_[i] = count;
                return;
            }
            samples = exact ? lb : std_.getUpBoundIterations(count, i + 1);
        }
        if (samples < maximality(i)) {
            maximality_[i] = samples;
            if (samples < max_samples || (samples == max_samples && i + 1 >= term_len_)) {
                term_len_ = i + 1;
                max_samples = samples;
            }
        }
    }
    // maximality_[i] with its pending update applied
    uint32_t maximality(uint32_t i) {
        if (pend_[i]) {
            const uint32_t v = std_.getUpBoundIterations(pend_[i], i + 1);
            if (v < maximality_[i]) maximality_[i] = v;
            pend_[i] = 0;
        }
        return maximality_[i];
    }
    StandardTerminationCriteria std_;
    std::vector<uint32_t> growth_;  // the sampler's growth function (a copy: samplers are rewound by value)
    std::vector<uint32_t> non_random_, maximality_;
    std::vector<uint32_t> pend_;    // a pending maximality update's inlier count (0: none)
    uint32_t n_, term_len_;
};

// ---------------------------------------------------------------- SPRT
// sprt.hpp:89-491.  The walk over the random pool runs here, in fp64 with the host libm
// (as the reference); the device supplies each model's inlier flags in pool order as
// 32-bit words (bit b of word w = pool position 32 w + b).
class Sprt {
   public:
    struct History {
        double epsilon, delta, A;
        int k;
    };
    // ctor (sprt.hpp:89-175): pool shuffle with points_size draws of the shared stream
    // defer_pool: the shuffle waits for shuffle_pool() -- for a caller whose next draws of rng
    // come after it anyway (PROSAC draws from its own generator), to overlap it with device work
    Sprt(GlibcRandom &rng, int estimator, uint32_t points_size, uint32_t sample_size, uint32_t max_iterations,
         int max_hypothesis_test_before_sprt = 20, bool defer_pool = false)
        : pool_(points_size), n_(points_size), m_(sample_size), max_iters_(max_iterations),
          max_before_(max_hypothesis_test_before_sprt), rng_(&rng) {
        if (!defer_pool) shuffle_pool();
        double eps0, delta0;
        switch (estimator) {
            case 2: delta0 = 0.01; eps0 = 0.1; t_M_ = 200; m_S_ = 1; break;        // homography
            case 3: delta0 = 0.05; eps0 = 0.2; t_M_ = 200; m_S_ = 2.48; break;     // fundamental
            case 4: delta0 = 0.05; eps0 = 0.2; t_M_ = 300; m_S_ = 4; break;        // essential
            default: delta0 = 0.0001; eps0 = 0.001; t_M_ = 100; m_S_ = 1; break;   // line2d
        }
        hist_.push_back(History{eps0, delta0, thresholdA(eps0, delta0), 0});
    }
    void shuffle_pool() {
        if (!rng_) return;
        for (uint32_t i = 0; i < n_; i++) pool_[i] = i;
        int max = (int)n_;
        for (uint32_t i = 0; i < n_; i++) {
            const uint32_t r = rng_->next() % (uint32_t)max;
            const uint32_t t = pool_[r];
            max--;
            pool_[r] = pool_[max];
            pool_[max] = t;
        }
        rng_ = nullptr;
    }
    bool pool_ready() const { return rng_ == nullptr; }
    const std::vector<uint32_t> &pool() const { return pool_; }
    size_t histories() const { return hist_.size(); }
    double thresholdA0() const { return hist_[0].A; }
    double epsilon0() const { return hist_[0].epsilon; }
    double delta0() const { return hist_[0].delta; }

    // verifyModelAndGetModelScore (sprt.hpp:191-317).  words = the model's pool-order flags, word
    // w at words[w * stride] (the device's [word][model] layout read in place: a walk touches a
    // few words, not all n / 32); count/score are written when the reference writes them.
    bool verify(const uint32_t *words, int current_hypothese, uint32_t maximum_score, int &count, float &score,
                size_t stride = 1) {
        if (plain_) return verify_plain(words, current_hypothese, maximum_score, count, score, stride);
        const History &h = hist_[cur_];
        const double epsilon = h.epsilon, delta = h.delta, A = h.A;
        const double up = delta / epsilon, down = (1 - delta) / (1 - epsilon);
        double lambda = 1;
        uint32_t tested = 0, inl = 0;
        bool good = true;
        // the reference's per-point walk, a word's run of positions at a time (the fp64 product
        // chain is the same sequence of multiplications); at growing intervals the rest of the
        // walk is tried for a certificate that lambda cannot pass A (no_crossing): then the
        // remaining points are only counted -- the same decision, count and pool index
        uint32_t next_cert = 32;
        while (tested < n_) {
            if (idx_ >= n_) idx_ = 0;
            const uint32_t b = idx_ & 31;
            const uint32_t len = std::min(std::min(32 - b, n_ - idx_), n_ - tested);
            uint32_t bits = words[(size_t)(idx_ >> 5) * stride] >> b;
            uint32_t k = 0;
            for (; k < len; k++, bits >>= 1) {
                const uint32_t in = bits & 1u;
                const double next = lambda * (in ? up : down);
                inl += in;
                if (next > A) {
                    good = false;
                    k++;
                    break;
                }
                lambda = next;
            }
            tested += k;
            idx_ += k;
            if (!good) break;
            if (tested >= next_cert && tested < n_) {
                if (idx_ >= n_) idx_ = 0;
                if (no_crossing(words, stride, lambda, A, up, down, idx_, n_ - tested)) {
                    inl += count_range(words, stride, idx_, n_ - tested);
                    idx_ = last_of(idx_, n_ - tested) + 1;  // as the per-point walk leaves it
                    tested = n_;
                    break;
                }
                next_cert *= 4;
            }
        }
        if (good) {
            count = (int)inl;
            score = (float)count;
        } else if (current_hypothese < max_before_) {
            uint32_t after = 0;
            if (tested < n_) {
                if (idx_ >= n_) idx_ = 0;
                after = count_range(words, stride, idx_, n_ - tested);
                idx_ = last_of(idx_, n_ - tested) + 1;
            }
            count = (int)(inl + after);
            score = (float)count;
        }
        if (good) {
            if (inl > maximum_score) {
                const double eps = (float)inl / n_;
                push(eps, delta, current_hypothese);
            }
        } else {
            const float dest = (float)inl / tested;
            if (dest > 0 && std::fabs(delta - dest) / delta > 0.05) push(epsilon, dest, current_hypothese);
        }
        return good;
    }

    // the same, one point per step throughout (the reference's loop as written): the check of
    // verify()'s word runs and certificates (tests/test_sprt_walk.py), USAC_SPRT_PLAIN_WALK=1
    bool verify_plain(const uint32_t *words, int current_hypothese, uint32_t maximum_score, int &count, float &score,
                      size_t stride = 1) {
        const History &h = hist_[cur_];
        const double epsilon = h.epsilon, delta = h.delta, A = h.A;
        const double up = delta / epsilon, down = (1 - delta) / (1 - epsilon);
        double lambda = 1;
        uint32_t tested = 0, inl = 0;
        bool good = true;
        for (tested = 0; tested < n_; tested++) {
            if (idx_ >= n_) idx_ = 0;
            const bool in = (words[(idx_ >> 5) * stride] >> (idx_ & 31)) & 1u;
            const double next = in ? lambda * up : lambda * down;
            inl += in ? 1 : 0;
            idx_++;
            if (next > A) {
                good = false;
                tested++;
                break;
            }
            lambda = next;
        }
        if (good) {
            count = (int)inl;
            score = (float)count;
        } else if (current_hypothese < max_before_) {
            uint32_t after = 0;
            for (uint32_t p = tested; p < n_; p++) {
                if (idx_ >= n_) idx_ = 0;
                after += (words[(idx_ >> 5) * stride] >> (idx_ & 31)) & 1u;
                idx_++;
            }
            count = (int)(inl + after);
            score = (float)count;
        }
        if (good) {
            if (inl > maximum_score) {
                const double eps = (float)inl / n_;
                push(eps, delta, current_hypothese);
            }
        } else {
            const float dest = (float)inl / tested;
            if (dest > 0 && std::fabs(delta - dest) / delta > 0.05) push(epsilon, dest, current_hypothese);
        }
        return good;
    }
    void set_plain_walk(bool v) { plain_ = v; }
    uint32_t pool_index() const { return idx_; }
    const std::vector<History> &history() const { return hist_; }

    // getUpperBoundIterations (sprt.hpp:371-393)
    uint32_t getUpperBoundIterations(int inliers_size) const {
        const double epsilon = (double)inliers_size / n_;
        const double P_g = std::pow(epsilon, m_);
        double log_eta = 0;
        for (uint32_t t = 0; t < cur_; t++) {
            const double h = exponentH(hist_[t].epsilon, epsilon, hist_[t].delta);
            log_eta += std::log(1 - P_g * (1 - std::pow(hist_[t].A, -h))) * hist_[t].k;
        }
        const double num = std::log(0.05) - log_eta;
        if (num >= 0) return 0;
        const double den = std::log(1 - P_g * (1 - 1 / hist_[cur_].A));
        if (std::isnan(den) || std::fabs(den) < 0.00001) return max_iters_;
        const uint32_t k = (uint32_t)(num / den);
        return std::min(k, max_iters_);
    }

    // estimateThresholdA (sprt.hpp:332-355)
    double thresholdA(double epsilon, double delta) const {
        const double C = (1 - delta) * std::log((1 - delta) / (1 - epsilon)) + delta * (std::log(delta / epsilon));
        const double K = (t_M_ * C) / m_S_ + 1;
        double prev = K, An = K;
        for (int i = 0; i < 10; ++i) {
            An = K + std::log(prev);
            if (std::fabs(An - prev) < 1.5e-8) break;
            prev = An;
        }
        return An;
    }

   private:
    // pool position of the last of r >= 1 positions walked from p (< n_), wrapping at n_
    uint32_t last_of(uint32_t p, uint32_t r) const {
        const uint64_t q = (uint64_t)p + r - 1;
        return (uint32_t)(q < n_ ? q : q - n_);
    }
    // inlier bits at pool positions [lo, hi) (hi <= n_)
    static uint32_t count_linear(const uint32_t *words, size_t stride, uint32_t lo, uint32_t hi) {
        uint32_t c = 0;
        while (lo < hi) {
            const uint32_t b = lo & 31, len = std::min(32 - b, hi - lo);
            const uint32_t w = words[(size_t)(lo >> 5) * stride] >> b;
            c += (uint32_t)__builtin_popcount(len == 32 ? w : w & ((1u << len) - 1));
            lo += len;
        }
        return c;
    }
    // inlier bits of the r positions from p, wrapping at n_
    uint32_t count_range(const uint32_t *words, size_t stride, uint32_t p, uint32_t r) const {
        const uint32_t first = std::min(r, n_ - p);
        return count_linear(words, stride, p, p + first) + count_linear(words, stride, 0, r - first);
    }
    // Certificate that the per-point walk from lambda over the r positions from p never sees
    // next > A.  L bounds log(computed lambda) step by step: a product rounds up by at most a
    // factor (1 + 2^-53) while normal, and a subnormal or zero result is below T = 2^-1000, so
    // L_j = max(L_{j-1} + log f_j + u, log T) holds (f = up | down, u >= log(1 + 2^-53)).
    // Over a run of i inliers and o outliers the process stays below its start (floored at
    // log T) plus the run's positive terms, and ends below max(start + run sum, log T + the
    // positive terms).  Runs are the words; the test keeps a margin far above the bound's own
    // rounding.  false: not proven (the exact walk continues).
    bool no_crossing(const uint32_t *words, size_t stride, double lambda, double A, double up, double down,
                     uint32_t p, uint32_t r) const {
        if (!(A > 0) || !(lambda >= 0)) return false;
        const double lu = std::log(up), ld = std::log(down), logT = -1000 * 0.6931471805599453;
        const double la = std::log(A), u = 2.3e-16;
        const double margin = 1e-6 + 1e-12 * (double)r * (std::fabs(lu) + std::fabs(ld) + 1);
        if (!std::isfinite(ld) || std::isnan(lu)) return false;
        double L = lambda > 0 ? std::max(std::log(lambda), logT) : logT;
        auto runs = [&](uint32_t lo, uint32_t hi) -> bool {
            while (lo < hi) {
                const uint32_t b = lo & 31, len = std::min(32 - b, hi - lo);
                const uint32_t w = words[(size_t)(lo >> 5) * stride] >> b;
                const uint32_t i = (uint32_t)__builtin_popcount(len == 32 ? w : w & ((1u << len) - 1)), o = len - i;
                const double pos = (o ? (ld > 0 ? o * ld : 0.0) : 0.0) + (i && lu > 0 ? i * lu : 0.0) + len * u;
                const double start = std::max(L, logT);
                if (!(start + pos + margin < la)) return false;
                const double sum = (i ? i * lu : 0.0) + (o ? o * ld : 0.0) + len * u;  // lu may be -inf
                L = std::max(start + sum, logT + pos);
                lo += len;
            }
            return true;
        };
        const uint32_t first = std::min(r, n_ - p);
        return runs(p, p + first) && runs(0, r - first);
    }
    void push(double eps, double delta, int current_hypothese) {
        hist_.push_back(History{eps, delta, thresholdA(eps, delta), current_hypothese - last_update_});
        last_update_ = current_hypothese;
        cur_++;
    }
    // computeExponentH (sprt.hpp:442-491)
    static double exponentH(double epsilon, double epsilon_new, double delta) {
        const double a = std::log(delta / epsilon);
        const double b = std::log((1 - delta) / (1 - epsilon));
        const double x0 = std::log(1 / (1 - epsilon_new)) / b;
        const double v0 = epsilon_new * std::exp(x0 * a);
        const double x1 = std::log((1 - 2 * v0) / (1 - epsilon_new)) / b;
        const double v1 = epsilon_new * std::exp(x1 * a) + (1 - epsilon_new) * std::exp(x1 * b);
        const double h = x0 - (x0 - x1) / (1 + v0 - v1) * v0;
        return std::isnan(h) ? 0 : h;
    }

    std::vector<uint32_t> pool_;
    std::vector<History> hist_;
    uint32_t n_, m_, max_iters_, idx_ = 0, cur_ = 0;
    int max_before_, last_update_ = 0;
    double t_M_ = 0, m_S_ = 0;
    bool plain_ = getenv("USAC_SPRT_PLAIN_WALK") != nullptr;
    GlibcRandom *rng_;  // set until the pool is shuffled
};

// ---------------------------------------------------------------- NAPSAC (grid)
// Grid neighbours: cell = ((int)(x1/cs), (int)(y1/cs), (int)(x2/cs), (int)(y2/cs)) with fp32
// division and truncation; a point's neighbours are the other points of its cell in
// ascending index order (what the reference's pair loop over each cell produces).  CSR.
class GridNeighbors {
   public:
    // neighbours of point i = the other points of its 4-D cell, ascending index.  Stored as
    // the cells' member lists (O(n), not the O(sum cell^2) pair lists): point i knows its
    // cell and its rank in it, and neighbour k skips that rank.
    GridNeighbors(const float *pts, uint32_t n, int cell_size) : cell_(n), rank_(n), members_(n) {
        struct Key {
            int c[4];
            bool operator==(const Key &o) const {
                return c[0] == o.c[0] && c[1] == o.c[1] && c[2] == o.c[2] && c[3] == o.c[3];
            }
        };
        struct Hash {
            size_t operator()(const Key &k) const {
                uint64_t h = 0x9e3779b97f4a7c15ull;
                for (int j = 0; j < 4; j++) {
                    h ^= (uint32_t)k.c[j];
                    h *= 0xff51afd7ed558ccdull;
                    h ^= h >> 32;
                }
                return (size_t)h;
            }
        };
        std::vector<uint32_t> size;
        std::vector<Key> keys(n);
        bool packable = true;
        for (uint32_t i = 0; i < n; i++)
            for (int j = 0; j < 4; j++) {
                const int v = (int)(pts[4 * (size_t)i + j] / (float)cell_size);
                keys[i].c[j] = v;
                packable &= v >= -32768 && v <= 32767;
            }
        if (packable) {  // open addressing on the 64-bit packed cell
            size_t cap = 16;
            while (cap < 2 * (size_t)n) cap <<= 1;
            std::vector<uint64_t> slot_key(cap);
            std::vector<uint32_t> slot_id(cap, UINT32_MAX);
            for (uint32_t i = 0; i < n; i++) {
                uint64_t k = 0;
                for (int j = 0; j < 4; j++) k = (k << 16) | (uint16_t)(int16_t)keys[i].c[j];
                size_t h = (size_t)((k * 0x9e3779b97f4a7c15ull) >> 20) & (cap - 1);
                while (slot_id[h] != UINT32_MAX && slot_key[h] != k) h = (h + 1) & (cap - 1);
                if (slot_id[h] == UINT32_MAX) {
                    slot_key[h] = k;
                    slot_id[h] = (uint32_t)size.size();
                    size.push_back(0);
                }
                cell_[i] = slot_id[h];
                rank_[i] = size[cell_[i]]++;
            }
        } else {
            std::unordered_map<Key, uint32_t, Hash> ids;
            ids.reserve(n);
            for (uint32_t i = 0; i < n; i++) {
                auto it = ids.emplace(keys[i], (uint32_t)size.size());
                if (it.second) size.push_back(0);
                cell_[i] = it.first->second;
                rank_[i] = size[cell_[i]]++;
            }
        }
        start_.assign(size.size() + 1, 0);
        for (size_t c = 0; c < size.size(); c++) start_[c + 1] = start_[c] + size[c];
        for (uint32_t i = 0; i < n; i++) members_[start_[cell_[i]] + rank_[i]] = (int32_t)i;
    }
    // the same CSR built on the device (build_grid, kernels_grid.hip)
    GridNeighbors(std::vector<uint32_t> cell, std::vector<uint32_t> rank, std::vector<uint32_t> start,
                  std::vector<int32_t> members)
        : cell_(std::move(cell)), rank_(std::move(rank)), start_(std::move(start)), members_(std::move(members)) {}
    uint32_t count(uint32_t i) const { return start_[cell_[i] + 1] - start_[cell_[i]] - 1; }
    // the CSR itself (cells in order of first appearance, members ascending)
    const std::vector<uint32_t> &cells() const { return cell_; }
    const std::vector<uint32_t> &ranks() const { return rank_; }
    const std::vector<uint32_t> &starts() const { return start_; }
    const std::vector<int32_t> &members() const { return members_; }
    int32_t at(uint32_t i, uint32_t k) const { return members_[start_[cell_[i]] + (k < rank_[i] ? k : k + 1)]; }

   private:
    std::vector<uint32_t> cell_, rank_, start_;
    std::vector<int32_t> members_;
};

// NapsacSampler (grid): ArrayRandomGenerator pool over [0, n) on the shared glibc stream
// (its member `max` starts at 0); an initial point needs >= m neighbours (Q18);
// after n failed draws the sampler turns uniform and, as the reference, then rewrites only
// sample[0] (generateUniqueRandomSet with subset size 1).
class NapsacSampler {
   public:
    NapsacSampler(GlibcRandom &rng, const GridNeighbors &g, uint32_t n, uint32_t m)
        : rng_(rng), g_(g), array_(n), next_(n, 0), n_(n), m_(m) {
        for (uint32_t i = 0; i < n; i++) array_[i] = (int32_t)i;
    }
    void generateSample(int32_t *sample) {
        if (uniform_) {
            sample[0] = draw();
            return;
        }
        uint32_t i;
        int32_t init = 0;
        for (i = 0; i < n_; i++) {
            init = draw();
            if (g_.count((uint32_t)init) < m_) continue;
            break;
        }
        if (i == n_) {
            uniform_ = true;
            return;
        }
        sample[0] = init;
        const uint32_t sz = g_.count((uint32_t)init);
        if (journal_on_) cursor_.push_back({(uint32_t)init, next_[init]});
        for (uint32_t k = 1; k < m_; k++) {
            sample[k] = g_.at((uint32_t)init, next_[init]);
            if (++next_[init] >= sz) next_[init] = 0;
        }
    }
    // speculative draws, as UniformSampler: the pool swaps and the cursors undone in reverse
    void mark() {
        rng_.save(mark_rng_);
        mark_max_ = max_;
        mark_uniform_ = uniform_;
        swaps_.clear();
        cursor_.clear();
        journal_on_ = true;
    }
    void commit() {
        journal_on_ = false;
        swaps_.clear();
        cursor_.clear();
    }
    void rollback() {
        for (auto it = cursor_.rbegin(); it != cursor_.rend(); ++it) next_[it->first] = it->second;
        for (auto it = swaps_.rbegin(); it != swaps_.rend(); ++it) std::swap(array_[it->first], array_[it->second]);
        max_ = mark_max_;
        uniform_ = mark_uniform_;
        rng_.restore(mark_rng_);
        commit();
    }

   private:
    int32_t draw() {
        if (max_ == 0) max_ = n_;
        const uint32_t k = rng_.next() % max_;
        const int32_t v = array_[k];
        max_--;
        array_[k] = array_[max_];
        array_[max_] = v;
        if (journal_on_) swaps_.push_back({k, max_});
        return v;
    }
    GlibcRandom &rng_;
    const GridNeighbors &g_;
    std::vector<int32_t> array_;
    std::vector<uint32_t> next_;
    uint32_t n_, m_, max_ = 0;
    bool uniform_ = false;
    bool journal_on_ = false, mark_uniform_ = false;
    std::vector<std::pair<uint32_t, uint32_t>> swaps_, cursor_;
    GlibcRandom::Saved mark_rng_;
    uint32_t mark_max_ = 0;
};

// NapsacSampler::generateSampleKNN (napsac_sampler.hpp:76-98): the initial point from the
// ArrayRandomGenerator pool on the shared glibc stream (member max = 0), then m - 1
// neighbours walking the point's KNN row (ascending distance) from the farthest, backwards
// and cyclically; the per-point cursor persists across samples.
class NapsacKnnSampler {
   public:
    NapsacKnnSampler(GlibcRandom &rng, const int32_t *nb, uint32_t n, uint32_t m, uint32_t knn)
        : rng_(rng), nb_(nb), array_(n), next_(n, 0), n_(n), m_(m), knn_((int)knn) {
        for (uint32_t i = 0; i < n; i++) array_[i] = (int32_t)i;
    }
    void generateSample(int32_t *sample) {
        if (max_ == 0) max_ = n_;
        const uint32_t k = rng_.next() % max_;
        const int32_t init = array_[k];
        max_--;
        array_[k] = array_[max_];
        array_[max_] = init;
        sample[0] = init;
        for (uint32_t i = 1; i < m_; i++) {
            sample[i] = nb_[(size_t)knn_ * (size_t)init + (size_t)(next_[init] + knn_ - 1)];
            if (--next_[init] == -knn_) next_[init] = 0;
        }
    }

   private:
    GlibcRandom &rng_;
    const int32_t *nb_;
    std::vector<int32_t> array_;
    std::vector<int> next_;
    uint32_t n_, m_, max_ = 0;
    int knn_;
};

}  // namespace usac
