// usac_host.hpp -- host-side mirror of the reference's plugin surface (C++17), the layer
// a reference-style driver talks to.  Names and argument meaning follow the reference;
// the work is done by the device (usac_api.cpp / kernels*.hip).
//
//   usac::Score                      quality.hpp:16-37
//   usac::UniformSampler             uniform_sampler.hpp:49-95 over a private glibc
//                                    random_r TYPE_3 state (= random()/srandom() stream)
//   usac::StandardTerminationCriteria standard_termination_criteria.hpp:10-74
//   usac::Ransac (batched replay)    ransac.cpp:14-238
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
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

   private:
    char state_[128];
    struct random_data data_;
};

class UniformSampler {
   public:
    UniformSampler(unsigned int seed, uint32_t points_size, uint32_t sample_size)
        : rng_(seed), pool_(points_size), max_((int)points_size), n_(points_size), m_(sample_size) {
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
        }
    }

   private:
    GlibcRandom rng_;
    std::vector<uint32_t> pool_;
    int max_;
    uint32_t n_, m_;
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
    uint32_t getUpBoundIterations(uint32_t inlier_size) const {
        float inl_ratio = (float)inlier_size / (float)n_;
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

   private:
    float log_1_p_;
    uint32_t m_, n_, max_;
};

}  // namespace usac
