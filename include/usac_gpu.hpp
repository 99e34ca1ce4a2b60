/*
 * usac_gpu.hpp -- C++ plugin layer over the C-ABI (usac_gpu.h), header-only, C++11.
 *
 * Mirrors the reference's plugin surface so that its callers read the same:
 *   usac_gpu::Model          usac/model.hpp:10-139 (fields, enums, setters; the cv::Mat
 *                            descriptor becomes 9 floats -- 3 for the line)
 *   usac_gpu::Score          usac/quality/quality.hpp:16-37 (bigger, copyFrom)
 *   usac_gpu::GpuEstimator   usac/estimator/estimator.hpp:14-41 (EstimateModel,
 *                            EstimateModelNonMinimalSample, LeastSquaresFitting,
 *                            SampleNumber) -- plus the batched EstimateModels
 *   usac_gpu::GpuQuality     usac/quality/quality.hpp:40-147 (init, getNumberInliers,
 *                            getInliers, static getInliers) -- plus the batched scoreModels
 *   usac_gpu::RansacOutput   usac/ransac/ransac_output.hpp:11-99 (getters)
 *   usac_gpu::Ransac         usac/ransac/ransac.hpp:18-117 + ransac.cpp:14-238 (Ransac(model,
 *                            points); run(); getRansacOutput()), the loop on the device
 *                            (usac_ransac_run), or hypothesis-sharded over ranks (runSharded)
 *   usac_gpu::Context        one usac_ctx (device, HIP stream, resident points)
 *   usac_gpu::RandomGenerator  the global glibc random() stream the samplers / SPRT share
 *   usac_gpu::Sampler        usac/sampler/sampler.hpp:11-35 (Uniform / Prosac / Napsac)
 *   usac_gpu::TerminationCriteria, ProsacTerminationCriteria
 *                            termination_criteria.hpp:16-17, prosac_termination_criteria.hpp:44-201
 *   usac_gpu::SPRT           usac/sprt.hpp:89-491 (verifyModelAndGetModelScore,
 *                            getUpperBoundIterations; replay = usac_sprt_replay)
 *   usac_gpu::LocalOptimization  local_optimization.hpp:19 (InItLORsc / InItFLORsc / GC)
 *
 * Errors: the C-ABI's negative status codes become usac_gpu::Error (code + usac_last_error);
 * USAC_ERR_NO_MODEL (-111) is the reference's exit(111) of ransac.cpp:143-147.
 * No CPU fallback: Context throws when no GPU is usable.
 */
#ifndef USAC_GPU_HPP
#define USAC_GPU_HPP

#include <array>
#include <cstdint>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "usac_gpu.h"

namespace usac_gpu {

// usac/model.hpp:10-13 (same numeric values as the C-ABI's USAC_* enums)
enum ESTIMATOR { NullE, Line2d, Homography, Fundamental, Essential };
enum SAMPLER { NullS, Uniform, ProgressiveNAPSAC, Napsac, Prosac, Evsac, ProsacNapsac };
enum NeighborsSearch { NullN, Nanoflann, Grid };
enum LocOpt { NullLO, InItLORsc, InItFLORsc, GC, IRLS };

class Error : public std::runtime_error {
public:
    int code;
    Error(int code_, const std::string &what) : std::runtime_error(what), code(code_) {}
};

// usac/quality/quality.hpp:16-37
class Score {
public:
    int inlier_number = 0;
    float score = 0;
    bool bigger(const Score *const score2) const { return bigger(*score2); }
    bool bigger(const Score &score2) const {
        if (inlier_number > score2.inlier_number) return true;
        if (inlier_number == score2.inlier_number) return score > score2.score;
        return false;
    }
    void copyFrom(const Score *const s) {
        score = s->score;
        inlier_number = s->inlier_number;
    }
};

typedef std::array<float, 9> Descriptor;

// usac/model.hpp:15-139
class Model {
public:
    float threshold = 2;
    float desired_prob = 0.95f;
    unsigned int sample_size = 0;
    unsigned int min_iterations = 20;
    unsigned int max_iterations = 10000;
    unsigned int k_nearest_neighbors = 5;
    LocOpt lo = NullLO;
    unsigned int lo_sample_size = 14;
    unsigned int lo_iterative_iterations = 4;
    unsigned int lo_inner_iterations = 20;
    unsigned int lo_threshold_multiplier = 10;
    float spatial_coherence_gc = 0.1f;
    ESTIMATOR estimator = NullE;
    SAMPLER sampler = NullS;
    bool sprt = false;
    unsigned int max_hypothesis_test_before_sprt = 20;
    NeighborsSearch neighborsType = NullN;
    int cell_size = 50;
    bool reset_random_generator = true;
    // device-side knobs (no reference counterpart)
    uint32_t seed = 1;          // srandom(seed) when reset_random_generator is false
    int dlt_mode = USAC_DLT_THIN;
    uint32_t batch = 0;         // hypotheses per device batch (0 = library default)
    int device = 0;

    Model(float threshold_, unsigned int sample_number_, float desired_prob_, unsigned int knn, ESTIMATOR estimator_,
          SAMPLER sampler_)
        : threshold(threshold_), desired_prob(desired_prob_), sample_size(sample_number_),
          k_nearest_neighbors(knn), estimator(estimator_), sampler(sampler_) {}
    explicit Model(const Model *const m) { *this = *m; }

    void ResetRandomGenerator(bool reset) { reset_random_generator = reset; }
    void setNeighborsType(NeighborsSearch t) { neighborsType = t; }
    void setCellSize(int c) { cell_size = c; }
    void setSprt(bool s) { sprt = s; }
    void setLOParametres(unsigned int lo_iterative_iters, unsigned int lo_inner_iters, unsigned int lo_thresh_mult) {
        lo_iterative_iterations = lo_iterative_iters;
        lo_inner_iterations = lo_inner_iters;
        lo_threshold_multiplier = lo_thresh_mult;
    }
    void setThreshold(float t) { threshold = t; }
    void setSampleNumber(float n) { sample_size = (unsigned int)n; }
    void setDesiredProbability(float p) { desired_prob = p; }
    void setKNearestNeighbors(int k) { k_nearest_neighbors = (unsigned int)k; }
    void setDescriptor(const float *d) { std::memcpy(descriptor.data(), d, sizeof(float) * descriptorSize()); }
    const Descriptor &returnDescriptor() const { return descriptor; }
    unsigned int descriptorSize() const { return estimator == Line2d ? 3u : 9u; }

    usac_params params() const {
        usac_params p;
        std::memset(&p, 0, sizeof(p));
        p.threshold = threshold;
        p.desired_prob = desired_prob;
        p.max_iterations = max_iterations;
        p.seed = reset_random_generator ? (uint32_t)std::random_device{}() : seed;  // ransac.cpp srand(time)
        p.dlt_mode = dlt_mode;
        p.batch = batch;
        p.sampler = (int32_t)sampler;
        p.sprt = sprt ? 1 : 0;
        p.lo = (int32_t)lo;
        p.lo_sample_size = lo_sample_size;
        p.lo_iterative_iterations = lo_iterative_iterations;
        p.lo_inner_iterations = lo_inner_iterations;
        p.lo_threshold_multiplier = lo_threshold_multiplier;
        p.cell_size = cell_size;
        p.neighbors = (int32_t)neighborsType;
        p.knn = k_nearest_neighbors;
        p.spatial_coherence_gc = spatial_coherence_gc;
        p.max_hypothesis_test_before_sprt = max_hypothesis_test_before_sprt;
        return p;
    }

private:
    Descriptor descriptor = {{0, 0, 0, 0, 0, 0, 0, 0, 0}};
};

// One device context: points resident in HBM, one HIP stream.  Not copyable.
class Context {
public:
    Context(ESTIMATOR est, const float *points, unsigned int points_size, int device = 0) : est_(est) {
        const int rc = usac_create(&ctx_, device, (int)est, points, points_size, est == Line2d ? 2u : 4u);
        if (rc != USAC_OK) {
            const std::string msg = ctx_ ? usac_last_error(ctx_) : "usac_create failed";
            if (ctx_) usac_destroy(ctx_);
            ctx_ = nullptr;
            throw Error(rc, msg);
        }
    }
    ~Context() {
        if (ctx_) usac_destroy(ctx_);
    }
    Context(const Context &) = delete;
    Context &operator=(const Context &) = delete;

    usac_ctx *get() const { return ctx_; }
    ESTIMATOR estimator() const { return est_; }
    unsigned int pointsSize() const { return usac_num_points(ctx_); }
    unsigned int sampleSize() const { return usac_sample_size(ctx_); }
    // model slots per minimal sample (the 7-point solver returns up to 3 F)
    unsigned int modelSlots() const { return est_ == Fundamental ? 3u : 1u; }
    void check(int rc, const char *what) const {
        if (rc != USAC_OK) throw Error(rc, std::string(what) + ": " + usac_last_error(ctx_));
    }

private:
    usac_ctx *ctx_ = nullptr;
    ESTIMATOR est_;
};

// usac/estimator/estimator.hpp:14-41 on the device
class GpuEstimator {
public:
    explicit GpuEstimator(Context &ctx) : ctx_(ctx) {}
    virtual ~GpuEstimator() = default;

    // minimal model estimation: appends the sample's valid models, returns their number
    unsigned int EstimateModel(const int *const sample, std::vector<Descriptor> &models) {
        const unsigned int S = ctx_.modelSlots();
        std::vector<float> out(9 * S, 0.f);
        int32_t nm = 0;
        ctx_.check(usac_estimate_models(ctx_.get(), sample, 1, out.data(), &nm), "EstimateModel");
        for (int j = 0; j < nm; j++) {
            Descriptor d;
            std::memcpy(d.data(), &out[9 * j], sizeof(float) * 9);
            models.push_back(d);
        }
        return (unsigned int)nm;
    }
    // batched: samples B x m -> models B x slots x 9, n_models[B]
    void EstimateModels(const int *const samples, unsigned int B, float *models, int *n_models) {
        ctx_.check(usac_estimate_models(ctx_.get(), samples, B, models, n_models), "EstimateModels");
    }
    bool EstimateModelNonMinimalSample(const int *const sample, unsigned int sample_size, Descriptor &model) {
        const int rc = usac_nonminimal(ctx_.get(), sample, sample_size, model.data());
        if (rc == USAC_ERR_NO_MODEL) return false;
        ctx_.check(rc, "EstimateModelNonMinimalSample");
        return true;
    }
    // the weighted overload (estimator.hpp:26): weights[point index], homography / fundamental
    bool EstimateModelNonMinimalSample(const int *const sample, unsigned int sample_size, const float *const weights,
                                       Descriptor &model) {
        const int rc = usac_lsq_fit(ctx_.get(), sample, sample_size, weights, model.data());
        if (rc == USAC_ERR_NO_MODEL) return false;
        ctx_.check(rc, "EstimateModelNonMinimalSample(weights)");
        return true;
    }
    bool LeastSquaresFitting(const int *const sample, unsigned int sample_size, Descriptor &model) {
        return EstimateModelNonMinimalSample(sample, sample_size, model);
    }
    int SampleNumber() const { return (int)ctx_.sampleSize(); }
    Context &context() { return ctx_; }

private:
    Context &ctx_;
};

// usac/quality/quality.hpp:40-147 on the device: counts exact, Σerr the reference's
// sequential fp32 sum (quality.hpp:89-96), inliers ascending.
class GpuQuality {
protected:
    unsigned int points_size = 0;
    float threshold = 0;
    GpuEstimator *estimator = nullptr;
    bool isinit = false;

public:
    bool isInit() const { return isinit; }
    void init(unsigned int points_size_, float threshold_, GpuEstimator *estimator_) {
        points_size = points_size_;
        threshold = threshold_;
        estimator = estimator_;
        isinit = true;
    }
    // `parallel` is accepted for signature parity; the device path is always parallel
    void getNumberInliers(Score *score, const float *model, float thr = 0, bool get_inliers = false,
                          int *inliers = nullptr, bool /*parallel*/ = false) {
        if (thr == 0) thr = threshold;
        float m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        std::memcpy(m, model, sizeof(float) * modelFloats());
        Context &c = estimator->context();
        if (get_inliers) {
            uint32_t n = 0;
            c.check(usac_get_inliers(c.get(), m, thr, inliers, &n, &score->score), "getNumberInliers");
            score->inlier_number = (int)n;
        } else {
            c.check(usac_score_models(c.get(), m, 1, thr, &score->inlier_number, &score->score), "getNumberInliers");
        }
    }
    void getNumberInliers(Score *score, const Descriptor &model, float thr = 0, bool get_inliers = false,
                          int *inliers = nullptr) {
        getNumberInliers(score, model.data(), thr, get_inliers, inliers);
    }
    // batched getNumberInliers over n models (n x 9 floats)
    void scoreModels(const float *models, unsigned int n, float thr, int *counts, float *sums) {
        Context &c = estimator->context();
        c.check(usac_score_models(c.get(), models, n, thr == 0 ? threshold : thr, counts, sums), "scoreModels");
    }
    void getInliers(const float *model, int *inliers) {
        Score s;
        getNumberInliers(&s, model, threshold, true, inliers);
    }
    static void getInliers(GpuEstimator *est, const Descriptor &model, float thr, unsigned int points_size,
                           std::vector<int> &inliers) {
        inliers.assign(points_size, 0);
        uint32_t n = 0;
        float sum = 0;
        Context &c = est->context();
        c.check(usac_get_inliers(c.get(), model.data(), thr, inliers.data(), &n, &sum), "getInliers");
        inliers.resize(n);
    }

private:
    unsigned int modelFloats() const { return estimator->context().estimator() == Line2d ? 3u : 9u; }
};

// ---- the stateful plugins (usac_gpu.h ABI 11): what a caller keeping its own loop swaps in ----

// The reference's global glibc random() stream (srand(seed)): UniformSampler / NapsacSampler draw
// from it and the SPRT ctor shuffles its pool with it (uniform_sampler.hpp:22-54, sprt.hpp:93-104).
class RandomGenerator {
public:
    explicit RandomGenerator(uint32_t seed) {
        if (usac_random_create(seed, &h_) != USAC_OK) throw Error(USAC_ERR_ARG, "usac_random_create");
    }
    ~RandomGenerator() { usac_random_destroy(h_); }
    RandomGenerator(const RandomGenerator &) = delete;
    RandomGenerator &operator=(const RandomGenerator &) = delete;
    uint32_t next() { return usac_random_next(h_); }
    usac_random *get() const { return h_; }

private:
    usac_random *h_ = nullptr;
};

// usac/sampler/sampler.hpp:11-35, built as initSampler builds it for model.sampler: UniformSampler
// (persistent pool on rng), ProsacSampler (mt19937 seeded with model.seed), NapsacSampler (grid or KNN
// neighbours built on the device, on rng)
class Sampler {
public:
    Sampler(Context &ctx, const Model &model, RandomGenerator *rng) : ctx_(ctx) {
        const usac_params p = model.params();
        ctx_.check(usac_sampler_create(ctx_.get(), &p, rng ? rng->get() : nullptr, &h_), "Sampler");
    }
    virtual ~Sampler() { usac_sampler_destroy(h_); }
    Sampler(const Sampler &) = delete;
    Sampler &operator=(const Sampler &) = delete;
    void generateSample(int *sample) { ctx_.check(usac_sampler_generate(h_, sample), "generateSample"); }
    // count samples in a row (count x m; each row starts from the previous one, as the reused array)
    void generateSamples(unsigned int count, int *samples) {
        ctx_.check(usac_sampler_generate_batch(h_, count, samples), "generateSamples");
    }
    unsigned int getNumberOfIterations() const {
        uint64_t d = 0;
        usac_sampler_state(h_, &d, nullptr, nullptr);
        return (unsigned int)d;
    }
    bool isInit() const { return h_ != nullptr; }
    usac_sampler *get() const { return h_; }

private:
    Context &ctx_;
    usac_sampler *h_ = nullptr;
};

// usac/termination_criteria/termination_criteria.hpp:16-17 (StandardTerminationCriteria)
class TerminationCriteria {
public:
    TerminationCriteria(Context &ctx, const Model &model, Sampler *prosac_sampler = nullptr) : ctx_(ctx) {
        const usac_params p = model.params();
        ctx_.check(usac_termination_create(ctx_.get(), &p, prosac_sampler ? prosac_sampler->get() : nullptr, &h_),
                   "TerminationCriteria");
    }
    virtual ~TerminationCriteria() { usac_termination_destroy(h_); }
    TerminationCriteria(const TerminationCriteria &) = delete;
    TerminationCriteria &operator=(const TerminationCriteria &) = delete;
    unsigned int getUpBoundIterations(unsigned int inlier_size) { return usac_termination_bound(h_, inlier_size, 0); }
    unsigned int getUpBoundIterations(unsigned int inlier_size, unsigned int points_size) {
        return usac_termination_bound(h_, inlier_size, points_size);
    }

protected:
    Context &ctx_;
    usac_termination *h_ = nullptr;
};

// usac/termination_criteria/prosac_termination_criteria.hpp:44-201, linked to its PROSAC sampler
class ProsacTerminationCriteria : public TerminationCriteria {
public:
    ProsacTerminationCriteria(Context &ctx, const Model &model, Sampler &prosac_sampler)
        : TerminationCriteria(ctx, model, &prosac_sampler), termination_length(ctx.pointsSize()) {}
    using TerminationCriteria::getUpBoundIterations;
    // getUpBoundIterations(hypCount, model): the model's inliers over the quality-sorted points
    unsigned int getUpBoundIterations(unsigned int hypCount, const Descriptor &model) {
        uint32_t max_samples = 0;
        ctx_.check(usac_prosac_termination(h_, hypCount, model.data(), &max_samples, &termination_length),
                   "ProsacTerminationCriteria::getUpBoundIterations");
        return max_samples;
    }
    unsigned int *getStoppingLength() { return &termination_length; }

private:
    unsigned int termination_length;
};

// usac/sprt.hpp:89-491
class SPRT {
public:
    SPRT(Context &ctx, const Model &model, RandomGenerator &rng) : ctx_(ctx) {
        const usac_params p = model.params();
        ctx_.check(usac_sprt_create(ctx_.get(), &p, rng.get(), &h_), "SPRT");
    }
    ~SPRT() { usac_sprt_destroy(h_); }
    SPRT(const SPRT &) = delete;
    SPRT &operator=(const SPRT &) = delete;
    // verifyModelAndGetModelScore(model, current_hypothese, maximum_score, score) (sprt.hpp:191-317)
    bool verifyModelAndGetModelScore(const Descriptor &model, int current_hypothese, unsigned int maximum_score,
                                     Score *score) {
        int32_t good = 0;
        ctx_.check(usac_sprt_verify(h_, model.data(), current_hypothese, maximum_score, &good, &score->inlier_number,
                                    &score->score),
                   "SPRT::verifyModelAndGetModelScore");
        return good != 0;
    }
    unsigned int getUpperBoundIterations(int inlier_size) { return usac_sprt_upper_bound(h_, (uint32_t)inlier_size); }
    // the batch form of the loop body (usac_sprt_replay): models B x slots x 9, n_models[B]
    bool replay(const float *models, const int *n_models, unsigned int B, usac_sprt_state &state) {
        ctx_.check(usac_sprt_replay(h_, models, n_models, B, &state), "SPRT::replay");
        return state.found != 0;
    }
    unsigned int histories() const {
        uint32_t h = 0;
        usac_sprt_stats(h_, &h, nullptr);
        return h;
    }

private:
    Context &ctx_;
    usac_sprt *h_ = nullptr;
};

// usac/local_optimization/local_optimization.hpp:19, built as initLocalOptimization builds it for
// model.lo (InItLORsc / InItFLORsc: inner + iterative LO-RANSAC; GC: graph cut)
class LocalOptimization {
public:
    LocalOptimization(Context &ctx, const Model &model) : ctx_(ctx) {
        const usac_params p = model.params();
        ctx_.check(usac_lo_create(ctx_.get(), &p, &h_), "LocalOptimization");
    }
    ~LocalOptimization() { usac_lo_destroy(h_); }
    LocalOptimization(const LocalOptimization &) = delete;
    LocalOptimization &operator=(const LocalOptimization &) = delete;
    void GetModelScore(Model *best_model, Score *best_score) {
        Descriptor d = best_model->returnDescriptor();
        ctx_.check(usac_lo_get_model_score(h_, d.data(), &best_score->inlier_number, &best_score->score),
                   "LocalOptimization::GetModelScore");
        best_model->setDescriptor(d.data());
    }
    // (lo_inner_iters, lo_iterative_iters) -- GC: (gc_iterations, labellings)
    void iters(unsigned int &inner, unsigned int &iterative) const {
        uint32_t a = 0, b = 0;
        usac_lo_iters(h_, &a, &b);
        inner = a;
        iterative = b;
    }

private:
    Context &ctx_;
    usac_lo *h_ = nullptr;
};

// usac/ransac/ransac_output.hpp:11-99
class RansacOutput {
public:
    RansacOutput(const Model &model_, const usac_run_output &raw_, std::vector<int> inliers_,
                 std::vector<usac_record> records_)
        : model(model_), raw(raw_), inliers(std::move(inliers_)), records(std::move(records_)) {
        model.setDescriptor(raw.model);
        const bool gc = model_.lo == GC;
        lo_inner_iters = gc ? 0u : raw.lo_inner_iters;
        lo_iterative_iters = gc ? 0u : raw.lo_iterative_iters;
        gc_iters = gc ? raw.lo_inner_iters : 0u;
    }
    std::vector<int> getInliers() const { return inliers; }
    long getTimeMicroSeconds() const { return (long)raw.time_us; }
    unsigned int getNumberOfInliers() const { return (unsigned int)raw.inliers; }
    unsigned int getNumberOfMainIterations() const { return raw.iters; }
    unsigned int getLOIters() const { return lo_inner_iters + lo_iterative_iters + gc_iters; }
    unsigned int getLOInnerIters() const { return lo_inner_iters; }
    unsigned int getLOIterativeIters() const { return lo_iterative_iters; }
    unsigned int getGCIters() const { return gc_iters; }
    const Model *getModel() const { return &model; }
    // beyond the reference: the C-ABI's counters and the best-score updates in loop order
    const usac_run_output &getRaw() const { return raw; }
    const std::vector<usac_record> &getRecords() const { return records; }

private:
    Model model;
    usac_run_output raw;
    std::vector<int> inliers;
    std::vector<usac_record> records;
    unsigned int lo_inner_iters, lo_iterative_iters, gc_iters;
};

// usac/ransac/ransac.hpp:18-117: Ransac(model, points); run(); getRansacOutput().
class Ransac {
public:
    Ransac(Model *model_, const float *points, unsigned int points_size_)
        : model(model_), points_size(points_size_),
          own_(new Context(model_->estimator, points, points_size_, model_->device)), ctx(own_) {}
    // run on an existing context over the same points (e.g. the one holding the RCCL communicator)
    Ransac(Model *model_, Context &ctx_) : model(model_), points_size(ctx_.pointsSize()), ctx(&ctx_) {}
    ~Ransac() {
        delete out_;
        delete own_;
    }
    Ransac(const Ransac &) = delete;
    Ransac &operator=(const Ransac &) = delete;

    void run(uint32_t rec_cap = 4096) { runImpl(1, 0, nullptr, nullptr, false, rec_cap); }
    // hypothesis-sharded (usac_ransac_run_sharded): gather == nullptr -> RCCL on the context's
    // communicator (usac_comm_init); every rank's output equals run()'s
    void runSharded(int nranks, int rank, usac_allgather_fn gather, void *user, uint32_t rec_cap = 4096) {
        runImpl(nranks, rank, gather, user, true, rec_cap);
    }
    RansacOutput *getRansacOutput() { return out_; }
    Context &context() { return *ctx; }

private:
    void runImpl(int nranks, int rank, usac_allgather_fn gather, void *user, bool sharded, uint32_t rec_cap) {
        usac_params p = model->params();
        usac_run_output raw;
        std::memset(&raw, 0, sizeof(raw));
        std::vector<int> inl(points_size);
        std::vector<usac_record> recs(rec_cap);
        const int rc = sharded ? usac_ransac_run_sharded(ctx->get(), &p, nranks, rank, gather, user, &raw, inl.data(),
                                                         recs.data(), rec_cap)
                               : usac_ransac_run(ctx->get(), &p, &raw, inl.data(), recs.data(), rec_cap);
        ctx->check(rc, "Ransac::run");
        inl.resize((size_t)raw.inliers);
        recs.resize(raw.n_records < (int32_t)rec_cap ? (size_t)raw.n_records : rec_cap);
        delete out_;
        out_ = new RansacOutput(*model, raw, std::move(inl), std::move(recs));
    }

    Model *model;
    unsigned int points_size;
    Context *own_ = nullptr;
    Context *ctx;
    RansacOutput *out_ = nullptr;
};

}  // namespace usac_gpu

#endif  // USAC_GPU_HPP
