/*
 * usac_oracle.h -- CPU ORACLE for the USAC hypothesize-and-verify hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product (ransac_amd/) never links, loads or calls it.
 *
 * This is a plain-C restatement of the reference's algorithm (MathsionYang/Ransac,
 * paths relative to the reference root); every function cites the file:line it
 * follows.  The reference itself cannot be compiled here (it needs OpenCV+contrib,
 * Eigen3, nanoflann: usac/precomp.hpp:25-41), so the OpenCV linear algebra it calls is
 * restated from its documented semantics (see DESIGN.md "Oracle").
 *
 * Pinning: the residual + 3x3-inverse path is pinned by the reference's own published
 * ground-truth inlier counts (results/homography/<cfg>.csv "GT Inl" column, 12 scenes,
 * tests/golden/homography_gt.json); the glibc sample stream by the glibc KAT; the
 * line2d loop statistically by results/line2d/uniform_000.csv.  Minimal-solver outputs
 * (OpenCV SVD) have no reference golden vector: "parity unpinned" at that boundary.
 */
#ifndef USAC_ORACLE_H
#define USAC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_LINE2D = 1, ORC_HOMOGRAPHY = 2, ORC_FUNDAMENTAL = 3, ORC_ESSENTIAL = 4 };
/* 4-pt DLT variant: ORC_DLT_THIN = reference semantics (vt.row(7) of the thin 8x9 SVD,
 * SURVEY Q1); ORC_DLT_NULLSPACE = true null vector. */
enum { ORC_DLT_THIN = 0, ORC_DLT_NULLSPACE = 1 };

/* glibc random() stream (the reference's sampler RNG, uniform_sampler.hpp:42) */
void orc_srandom(unsigned int seed);
long orc_random(void);
void orc_random_n(long *out, int n);

/* UniformSampler (usac/sampler/uniform_sampler.hpp:49-95) */
typedef struct orc_uniform orc_uniform;
orc_uniform *orc_uniform_new(unsigned int points_size, unsigned int sample_size);
void orc_uniform_free(orc_uniform *s);
void orc_uniform_sample(orc_uniform *s, int *sample);
void orc_uniform_samples(orc_uniform *s, int *out, int count);

/* Estimators (usac/estimator/<name>_estimator.hpp) */
typedef struct orc_est orc_est;
orc_est *orc_est_new(int kind, const float *points, unsigned int n, int dlt_mode);
void orc_est_free(orc_est *e);
int orc_est_sample_size(const orc_est *e);
/* models per EstimateModel call: 3 for the 7-point fundamental solver, else 1 */
int orc_est_max_models(const orc_est *e);
/* real roots (ascending) of c0 x^3 + c1 x^2 + c2 x + c3: the shared cubic spec of the 7-pt solver */
int orc_cubic_roots(double c0, double c1, double c2, double c3, double *roots);
/* EstimateModel: writes <= 3 models of 9 floats; returns number of models */
int orc_est_estimate(orc_est *e, const int *sample, float *models);
/* EstimateModelNonMinimalSample: returns 1 on success */
int orc_est_nonminimal(orc_est *e, const int *sample, unsigned int n, float *model);
void orc_est_set_model(orc_est *e, const float *model);
float orc_est_error(const orc_est *e, unsigned int pidx);

/* cv::Mat::inv() 3x3 closed form (fp64 intermediates) -- returns 0 if singular (dst zeroed) */
int orc_inv3x3(const float *src, float *dst);

/* Quality::getNumberInliers (usac/quality/quality.hpp:60-101); inliers nullable */
void orc_quality(orc_est *e, const float *model, float thr, int *count, float *sum, int *inliers);
/* batched helpers (tests / cpu baseline) */
void orc_score_models(orc_est *e, const float *models, int n_models, float thr, int *counts, float *sums);
void orc_estimate_batch(orc_est *e, const int *samples, int n_samples, float *models, int *n_models);
/* GT inlier count as dataset/GetImage.h:209-231 (max over H and H^-1) */
int orc_gt_inliers_homography(const float *points, unsigned int n, const float *model, float thr);

/* StandardTerminationCriteria::getUpBoundIterations (standard_termination_criteria.hpp:52-62) */
unsigned int orc_std_termination(unsigned int inliers, unsigned int points_size, unsigned int sample_size,
                                 float desired_prob, unsigned int max_iterations);

/* Ransac::run (usac/ransac/ransac.cpp:14-238), Uniform sampler, no LO / SPRT.
 * Sampler RNG seeded with srandom(seed) (ResetRandomGenerator(false) semantics).
 * rec_* (nullable, capacity rec_cap) receive the best-score updates in loop order:
 * (iteration index, model slot, inlier count, score).  Returns 0, or -111 when the best
 * score is 0 (ransac.cpp:143-147). */
typedef struct {
    float model[9];
    int inliers;          /* best_score->inlier_number */
    unsigned int iters;   /* main iterations */
    int n_records;
    int polish_passes;    /* accepted non-minimal passes */
    float minimal_model[9];
    int minimal_inliers;
} orc_result;

int orc_ransac_run(int kind, const float *points, unsigned int n, float threshold, float desired_prob,
                   unsigned int max_iterations, unsigned int seed, int dlt_mode, orc_result *out,
                   int *inliers_out, unsigned int *rec_iter, int *rec_count, float *rec_score, int rec_cap);

/* Reference-style hypothesis throughput loop for the CPU baseline: `count` hypotheses
 * of sample (glibc pool) + minimal solve + full score, no termination; returns best count. */
int orc_hypothesis_loop(orc_est *e, orc_uniform *s, int count, float thr, float *best_score_sum);

/* generator/generator.cpp:98-148 Generate2DLinePoints (glibc rand(), srand(seed) first) */
void orc_generate_line2d(unsigned int seed, float noise, int inliers, int outliers, int border_x, int border_y,
                         float *points_out, float *gt_model);

#ifdef __cplusplus
}
#endif
#endif
