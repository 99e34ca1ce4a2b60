// consumer.cpp -- a reference-style C++ caller of the drop-in boundary, compiled with g++
// against include/usac_gpu.hpp (the usac_gpu:: plugin layer) over include/usac_gpu.h and
// linked with libransac_amd.so.  It does what INTEGRATION.md §1-2 describe a maintainer
// doing in the reference: Ransac::run replaced whole, and Quality::getNumberInliers /
// Estimator::EstimateModel / EstimateModelNonMinimalSample forwarded operator by operator.
// tests/test_gpu_cpp_consumer.py drives it and checks its output against the oracle.
//
//   consumer abi
//   consumer run <est> <n> <points.f32> <thr> <prob> <seed> <sampler> <sprt> <lo> <neighbors>
//   consumer quality <est> <n> <points.f32> <thr> <models.f32> <k> <samples.i32> <B>
//   consumer loop <est> <n> <points.f32> <thr> <prob> <seed> <sampler> <sprt> <lo> <neighbors> loop|batched
// est: 1 line2d, 2 homography, 3 fundamental, 4 essential (usac/model.hpp:10).
// Output: one JSON object on stdout; floats as their int32 bit patterns (bit-exact checks).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <algorithm>
#include <string>
#include <vector>

#include "usac_gpu.hpp"

using namespace usac_gpu;

template <typename T>
static std::vector<T> read_file(const char *path, size_t count) {
    std::vector<T> v(count);
    FILE *f = std::fopen(path, "rb");
    if (!f || std::fread(v.data(), sizeof(T), count, f) != count) {
        std::fprintf(stderr, "consumer: cannot read %zu items from %s\n", count, path);
        std::exit(2);
    }
    std::fclose(f);
    return v;
}

static int32_t bits(float f) {
    int32_t b;
    std::memcpy(&b, &f, 4);
    return b;
}

static void print_ints(const char *key, const int *v, size_t n, bool last = false) {
    std::printf("\"%s\": [", key);
    for (size_t i = 0; i < n; i++) std::printf(i ? ", %d" : "%d", v[i]);
    std::printf("]%s\n", last ? "" : ",");
}

static void print_bits(const char *key, const float *v, size_t n, bool last = false) {
    std::vector<int> b(n);
    for (size_t i = 0; i < n; i++) b[i] = bits(v[i]);
    print_ints(key, b.data(), n, last);
}

static unsigned int sample_size(ESTIMATOR e) {
    return e == Line2d ? 2 : e == Homography ? 4 : e == Fundamental ? 7 : 5;
}

// Ransac::run replaced by the device loop
static int cmd_run(int argc, char **argv) {
    if (argc != 12) return 2;
    const ESTIMATOR est = (ESTIMATOR)std::atoi(argv[2]);
    const unsigned int n = (unsigned int)std::atoi(argv[3]);
    std::vector<float> pts = read_file<float>(argv[4], (size_t)n * (est == Line2d ? 2 : 4));
    Model model(std::strtof(argv[5], nullptr), sample_size(est), std::strtof(argv[6], nullptr), 7, est,
                (SAMPLER)std::atoi(argv[8]));
    model.ResetRandomGenerator(false);
    model.seed = (uint32_t)std::atoi(argv[7]);
    model.setSprt(std::atoi(argv[9]) != 0);
    model.lo = (LocOpt)std::atoi(argv[10]);
    model.setNeighborsType((NeighborsSearch)std::atoi(argv[11]));
    Ransac ransac(&model, pts.data(), n);
    ransac.run();
    RansacOutput *out = ransac.getRansacOutput();
    const std::vector<int> inl = out->getInliers();
    std::vector<int> rec;
    for (const usac_record &r : out->getRecords()) {
        rec.push_back((int)r.hyp_index);
        rec.push_back(r.inliers);
        rec.push_back(bits(r.score));
    }
    std::printf("{\n\"iters\": %u,\n\"inliers\": %u,\n\"lo_inner\": %u,\n\"lo_iterative\": %u,\n\"gc\": %u,\n",
                out->getNumberOfMainIterations(), out->getNumberOfInliers(), out->getLOInnerIters(),
                out->getLOIterativeIters(), out->getGCIters());
    print_bits("model", out->getModel()->returnDescriptor().data(), out->getModel()->descriptorSize());
    print_ints("records", rec.data(), rec.size());
    print_ints("inlier_idx", inl.data(), inl.size(), true);
    std::printf("}\n");
    return 0;
}

// the reference loop kept, its hot operators forwarded
static int cmd_quality(int argc, char **argv) {
    if (argc != 10) return 2;
    const ESTIMATOR est = (ESTIMATOR)std::atoi(argv[2]);
    const unsigned int n = (unsigned int)std::atoi(argv[3]);
    std::vector<float> pts = read_file<float>(argv[4], (size_t)n * (est == Line2d ? 2 : 4));
    const float thr = std::strtof(argv[5], nullptr);
    const unsigned int k = (unsigned int)std::atoi(argv[7]);
    std::vector<float> models = read_file<float>(argv[6], (size_t)k * 9);
    const unsigned int B = (unsigned int)std::atoi(argv[9]);
    std::vector<int> samples = read_file<int>(argv[8], (size_t)B * sample_size(est));

    Context ctx(est, pts.data(), n);
    GpuEstimator estimator(ctx);
    GpuQuality quality;
    quality.init(n, thr, &estimator);

    // Quality::getNumberInliers, one model at a time as ransac.cpp calls it
    std::vector<int> counts(k);
    std::vector<float> sums(k);
    for (unsigned int i = 0; i < k; i++) {
        Score s;
        quality.getNumberInliers(&s, &models[9 * i]);
        counts[i] = s.inlier_number;
        sums[i] = s.score;
    }
    // ... and batched
    std::vector<int> bcounts(k);
    std::vector<float> bsums(k);
    quality.scoreModels(models.data(), k, 0, bcounts.data(), bsums.data());
    // get_inliers = true on the first model, then the non-minimal fit on those inliers
    std::vector<int> inl(n);
    Score s0;
    quality.getNumberInliers(&s0, models.data(), 0, true, inl.data());
    inl.resize((size_t)s0.inlier_number);
    std::vector<int> inl2;
    GpuQuality::getInliers(&estimator, Descriptor{{models[0], models[1], models[2], models[3], models[4], models[5],
                                                   models[6], models[7], models[8]}},
                           thr, n, inl2);
    Descriptor nm{};
    const bool nm_ok = estimator.EstimateModelNonMinimalSample(inl.data(), (unsigned int)inl.size(), nm);
    // Estimator::EstimateModel, sample by sample (the reference's per-iteration call) and batched
    std::vector<int> est_n(B);
    std::vector<float> est_models;
    for (unsigned int b = 0; b < B; b++) {
        std::vector<Descriptor> ms;
        est_n[b] = (int)estimator.EstimateModel(&samples[(size_t)b * estimator.SampleNumber()], ms);
        for (unsigned int j = 0; j < ctx.modelSlots(); j++)
            for (int c = 0; c < 9; c++) est_models.push_back(j < ms.size() ? ms[j][c] : 0.f);
    }
    std::vector<float> bmodels((size_t)B * ctx.modelSlots() * 9);
    std::vector<int> bn(B);
    estimator.EstimateModels(samples.data(), B, bmodels.data(), bn.data());

    std::printf("{\n\"first_count\": %d,\n\"first_sum\": %d,\n\"nonminimal_ok\": %d,\n", s0.inlier_number,
                bits(s0.score), nm_ok ? 1 : 0);
    print_ints("counts", counts.data(), k);
    print_bits("sums", sums.data(), k);
    print_ints("batch_counts", bcounts.data(), k);
    print_bits("batch_sums", bsums.data(), k);
    print_ints("first_inliers", inl.data(), inl.size());
    print_ints("first_inliers_static", inl2.data(), inl2.size());
    print_bits("nonminimal", nm.data(), 9);
    print_ints("est_n", est_n.data(), B);
    print_bits("est_models", est_models.data(), est_models.size());
    print_ints("batch_est_n", bn.data(), B);
    print_bits("batch_est_models", bmodels.data(), bmodels.size(), true);
    std::printf("}\n");
    return 0;
}

// the reference's own Ransac::run (ransac.cpp:14-238) kept as written, every
// plugin it calls replaced by the device one -- Sampler, Estimator, Quality, SPRT, termination
// criteria (standard or PROSAC), LocalOptimization -- in the reference's construction order
// (Ransac ctor: estimator, sampler, quality, LO, termination, SPRT; ransac.hpp:41-93).
// mode "loop": one call per plugin per model, as the reference; mode "batched": samples drawn
// and solved B at a time, the SPRT walk by SPRT::replay (usac_sprt_replay) -- same results.
static int cmd_loop(int argc, char **argv) {
    if (argc != 13) return 2;
    const bool batched = !std::strcmp(argv[12], "batched");
    const ESTIMATOR est = (ESTIMATOR)std::atoi(argv[2]);
    const unsigned int points_size = (unsigned int)std::atoi(argv[3]);
    std::vector<float> pts = read_file<float>(argv[4], (size_t)points_size * (est == Line2d ? 2 : 4));
    Model model(std::strtof(argv[5], nullptr), sample_size(est), std::strtof(argv[6], nullptr), 7, est,
                (SAMPLER)std::atoi(argv[8]));
    model.ResetRandomGenerator(false);
    model.seed = (uint32_t)std::atoi(argv[7]);
    model.setSprt(std::atoi(argv[9]) != 0);
    model.lo = (LocOpt)std::atoi(argv[10]);
    model.setNeighborsType((NeighborsSearch)std::atoi(argv[11]));

    Context ctx(est, pts.data(), points_size);
    GpuEstimator estimator(ctx);
    RandomGenerator random(model.seed);  // srand(seed): the stream the sampler and SPRT share
    Sampler sampler(ctx, model, &random);
    GpuQuality quality;
    quality.init(points_size, model.threshold, &estimator);
    std::unique_ptr<LocalOptimization> local_optimization;
    if (model.lo != NullLO) local_optimization.reset(new LocalOptimization(ctx, model));
    const bool is_prosac = model.sampler == Prosac;
    std::unique_ptr<TerminationCriteria> termination_criteria(
        is_prosac ? new ProsacTerminationCriteria(ctx, model, sampler) : new TerminationCriteria(ctx, model));
    std::unique_ptr<SPRT> sprt;
    if (model.sprt) sprt.reset(new SPRT(ctx, model, random));

    // ---- ransac.cpp:14-139
    Score best_score, current_score;
    Model best_model(&model);
    const unsigned int m = estimator.SampleNumber(), slots = ctx.modelSlots();
    std::vector<int> sample(m, 0), records;
    const bool is_sprt = model.sprt, LO = model.lo != NullLO;
    unsigned int iters = 0, max_iters = model.max_iterations;
    auto new_best = [&](const Descriptor &d) {  // ransac.cpp:103-135, after the score
        Model cur(&model);
        cur.setDescriptor(d.data());
        if (LO) local_optimization->GetModelScore(&cur, &current_score);
        best_score.copyFrom(&current_score);
        best_model.setDescriptor(cur.returnDescriptor().data());
        if (is_prosac)
            max_iters = static_cast<ProsacTerminationCriteria *>(termination_criteria.get())
                            ->getUpBoundIterations(iters, best_model.returnDescriptor());
        else
            max_iters = termination_criteria->getUpBoundIterations(best_score.inlier_number);
        if (is_sprt) max_iters = std::min(max_iters, sprt->getUpperBoundIterations(best_score.inlier_number));
        records.push_back((int)iters);
        records.push_back(best_score.inlier_number);
        records.push_back(bits(best_score.score));
    };
    if (!batched) {
        std::vector<Descriptor> models;
        while (iters < max_iters) {
            sampler.generateSample(sample.data());
            models.clear();
            const unsigned int number_of_models = estimator.EstimateModel(sample.data(), models);
            for (unsigned int i = 0; i < number_of_models; i++) {
                if (is_sprt) {
                    const bool is_good_model =
                        sprt->verifyModelAndGetModelScore(models[i], (int)iters, best_score.inlier_number, &current_score);
                    if (!is_good_model && iters >= model.max_hypothesis_test_before_sprt) {
                        iters++;
                        continue;
                    }
                } else {
                    quality.getNumberInliers(&current_score, models[i]);
                }
                if (current_score.bigger(best_score)) new_best(models[i]);
            }
            iters++;
        }
    } else {
        // B samples at a time: draw, solve on the device, then the loop body over the batch --
        // SPRT::replay walks it and stops at each new best; without SPRT the batch's exact scores
        // are compared in loop order.  PROSAC draws depend on the termination length, which a
        // new best may change, so it draws one sample per batch.
        const unsigned int B = is_prosac ? 1u : 64u;
        std::vector<int> smp((size_t)B * m), n_models(B);
        std::vector<float> mod((size_t)B * slots * 9);
        while (iters < max_iters) {
            sampler.generateSamples(B, smp.data());
            estimator.EstimateModels(smp.data(), B, mod.data(), n_models.data());
            if (is_sprt) {
                usac_sprt_state st;
                std::memset(&st, 0, sizeof(st));
                st.iters = iters;
                for (;;) {
                    st.max_iters = max_iters;
                    st.best_inliers = best_score.inlier_number;
                    st.best_score = best_score.score;
                    if (!sprt->replay(mod.data(), n_models.data(), B, st)) break;
                    iters = st.iters;
                    current_score.inlier_number = st.inliers;
                    current_score.score = st.score;
                    Descriptor d;
                    std::memcpy(d.data(), &mod[((size_t)st.found_sample * slots + st.found_slot) * 9], sizeof(float) * 9);
                    new_best(d);
                }
                iters = st.iters;
            } else {
                std::vector<int> cnt((size_t)B * slots);
                std::vector<float> sum((size_t)B * slots);
                quality.scoreModels(mod.data(), B * slots, 0, cnt.data(), sum.data());
                for (unsigned int b = 0; b < B && iters < max_iters; b++) {
                    for (int i = 0; i < n_models[b]; i++) {
                        current_score.inlier_number = cnt[(size_t)b * slots + i];
                        current_score.score = sum[(size_t)b * slots + i];
                        if (!current_score.bigger(best_score)) continue;
                        Descriptor d;
                        std::memcpy(d.data(), &mod[((size_t)b * slots + i) * 9], sizeof(float) * 9);
                        new_best(d);
                    }
                    iters++;
                }
            }
        }
    }
    if (best_score.inlier_number == 0) {
        std::fprintf(stderr, "consumer: best score is 0\n");
        return 4;
    }
    unsigned int lo_inner = 0, lo_iterative = 0;
    if (LO) local_optimization->iters(lo_inner, lo_iterative);
    if (model.lo == GC && lo_inner == 0) {  // ransac.cpp:149-153
        local_optimization->GetModelScore(&best_model, &best_score);
        local_optimization->iters(lo_inner, lo_iterative);
    }
    // ---- ransac.cpp:157-214: the non-minimal polish
    std::vector<int> max_inliers(points_size);
    quality.getInliers(best_model.returnDescriptor().data(), max_inliers.data());
    unsigned int previous_non_minimal_num_inlier = 0;
    Descriptor non_minimal{};
    for (unsigned int norm = 0; norm < 4; norm++) {
        if (!estimator.EstimateModelNonMinimalSample(max_inliers.data(), (unsigned int)best_score.inlier_number,
                                                     non_minimal))
            break;
        quality.getNumberInliers(&current_score, non_minimal, model.threshold, true, max_inliers.data());
        if ((float)current_score.inlier_number / best_score.inlier_number < 0.8) break;
        if ((unsigned int)current_score.inlier_number <= previous_non_minimal_num_inlier) break;
        previous_non_minimal_num_inlier = (unsigned int)current_score.inlier_number;
        best_score.copyFrom(&current_score);
        best_model.setDescriptor(non_minimal.data());
    }
    Score final_score;
    quality.getNumberInliers(&final_score, best_model.returnDescriptor(), model.threshold, true, max_inliers.data());
    max_inliers.resize((size_t)final_score.inlier_number);

    std::printf("{\n\"iters\": %u,\n\"inliers\": %d,\n\"lo_inner\": %u,\n\"lo_iterative\": %u,\n", iters,
                best_score.inlier_number, lo_inner, lo_iterative);
    if (sprt) std::printf("\"sprt_histories\": %u,\n", sprt->histories());
    if (is_prosac)
        std::printf("\"termination_length\": %u,\n",
                    *static_cast<ProsacTerminationCriteria *>(termination_criteria.get())->getStoppingLength());
    print_bits("model", best_model.returnDescriptor().data(), best_model.descriptorSize());
    print_ints("records", records.data(), records.size());
    print_ints("inlier_idx", max_inliers.data(), max_inliers.size(), true);
    std::printf("}\n");
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 2 && !std::strcmp(argv[1], "abi")) {
        std::printf("{\"abi\": %d, \"header\": %d}\n", usac_abi_version(), USAC_ABI_VERSION);
        return usac_abi_version() == USAC_ABI_VERSION ? 0 : 1;
    }
    try {
        if (argc >= 2 && !std::strcmp(argv[1], "run")) return cmd_run(argc, argv);
        if (argc >= 2 && !std::strcmp(argv[1], "quality")) return cmd_quality(argc, argv);
        if (argc >= 2 && !std::strcmp(argv[1], "loop")) return cmd_loop(argc, argv);
    } catch (const Error &e) {
        std::fprintf(stderr, "consumer: usac error %d: %s\n", e.code, e.what());
        return 3;
    }
    std::fprintf(stderr, "usage: consumer abi | run ... | quality ...\n");
    return 2;
}
