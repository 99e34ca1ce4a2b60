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
// est: 1 line2d, 2 homography, 3 fundamental, 4 essential (usac/model.hpp:10).
// Output: one JSON object on stdout; floats as their int32 bit patterns (bit-exact checks).
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

int main(int argc, char **argv) {
    if (argc >= 2 && !std::strcmp(argv[1], "abi")) {
        std::printf("{\"abi\": %d, \"header\": %d}\n", usac_abi_version(), USAC_ABI_VERSION);
        return usac_abi_version() == USAC_ABI_VERSION ? 0 : 1;
    }
    try {
        if (argc >= 2 && !std::strcmp(argv[1], "run")) return cmd_run(argc, argv);
        if (argc >= 2 && !std::strcmp(argv[1], "quality")) return cmd_quality(argc, argv);
    } catch (const Error &e) {
        std::fprintf(stderr, "consumer: usac error %d: %s\n", e.code, e.what());
        return 3;
    }
    std::fprintf(stderr, "usage: consumer abi | run ... | quality ...\n");
    return 2;
}
