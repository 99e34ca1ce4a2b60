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
/* real roots (ascending) of a[0] + a[1] z + ... + a[n] z^n: the 5-pt solver's root spec */
int orc_real_roots(const double *a, int n, double *roots);
int orc_asc_roots(const double *a, int n, double *roots);
int orc_rpoly_zeros(const double *a, int n, double *zr, double *zi);
double orc_jt_log(double x);
double orc_jt_exp(double y);
void orc_e5_poly(orc_est *e, const int *sample, double *a);
/* every real root's E of the 5-pt solver (<= 10 x 9) and its cheirality flag (test hook) */
int orc_e5_candidates(orc_est *e, const int *sample, float *cand, int *cand_ok);
/* real roots (ascending) of c0 x^3 + c1 x^2 + c2 x + c3: the shared cubic spec of the 7-pt solver */
int orc_cubic_roots(double c0, double c1, double c2, double c3, double *roots);
/* EstimateModel: writes <= 3 models of 9 floats; returns number of models */
int orc_est_estimate(orc_est *e, const int *sample, float *models);
/* EstimateModelNonMinimalSample: returns 1 on success */
int orc_est_nonminimal(orc_est *e, const int *sample, unsigned int n, float *model);
/* the LSQ fits' 9x9 eigen spec (inverse iteration, Jacobi fall-back): smallest-eigenvalue
 * eigenvector of the symmetric A (row-major 81); returns 1 if inverse iteration converged */
int orc_sym_eig_min(const double *A81, double *v);
/* the weighted overload (weights[point index]): homography / fundamental; -1 for the others */
int orc_est_nonminimal_weighted(orc_est *e, const int *sample, unsigned int n, const float *weights, float *model);
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
    int sprt_rejected;    /* models SPRT rejected */
    int sprt_histories;   /* SPRT tests designed (history length) */
    unsigned int prosac_term_len; /* final PROSAC termination_length (n without PROSAC) */
    unsigned int lo_inner_iters, lo_iterative_iters; /* RansacOutput LO counters */
} orc_result;

enum { ORC_SAMPLER_UNIFORM = 1, ORC_SAMPLER_NAPSAC = 3, ORC_SAMPLER_PROSAC = 4 }; /* = SAMPLER, usac/model.hpp:11 */
enum { ORC_LO_NONE = 0, ORC_LO_INITLORSC = 1, ORC_LO_INITFLORSC = 2, ORC_LO_GC = 3 }; /* = LocOpt, usac/model.hpp:13 */
typedef struct {
    float threshold, desired_prob;
    unsigned int max_iterations, seed;
    int dlt_mode;
    int sampler; /* ORC_SAMPLER_* (NAPSAC: grid neighbours of cell_size) */
    int sprt;    /* Model::setSprt */
    int lo;      /* ORC_LO_* */
    unsigned int lo_sample_size, lo_iterative_iterations, lo_inner_iterations, lo_threshold_multiplier; /* model.hpp:27-30 */
    int cell_size; /* model.hpp:43 */
    int neighbors;        /* ORC_NEIGHBORS_* (model.hpp:12,42): Grid, else nanoflann KNN */
    unsigned int knn;     /* model.hpp:23 k_nearest_neighbors (NAPSAC KNN, GC) */
    float spatial_coherence_gc; /* model.hpp:33 (0.1): used as given, 0 = no pairwise term -- set it */
} orc_config;
enum { ORC_NEIGHBORS_NULL = 0, ORC_NEIGHBORS_NANOFLANN = 1, ORC_NEIGHBORS_GRID = 2 }; /* = NeighborsSearch */

/* KNN neighbours (nearest_neighbors.cpp:69-128): idx/d2 n x k, self excluded, ties by index */
float orc_l2_dist(const float *a, const float *b, unsigned int cols);
void orc_knn(const float *pts, unsigned int n, unsigned int cols, unsigned int k, int *idx, float *d2);
typedef struct orc_napsac_knn orc_napsac_knn;
orc_napsac_knn *orc_napsac_knn_new(const int *nb, unsigned int n, unsigned int m, unsigned int knn);
void orc_napsac_knn_free(orc_napsac_knn *s);
void orc_napsac_knn_sample(orc_napsac_knn *s, int *sample);

/* Boykov-Kolmogorov max-flow (gco-v3.0 graph.h / maxflow.inl) and its energy.h terms */
typedef struct orc_bk orc_bk;
orc_bk *orc_bk_new(int n_nodes, int n_edges);
void orc_bk_free(orc_bk *g);
int orc_bk_add_node(orc_bk *g);
void orc_bk_add_tweights(orc_bk *g, int i, float cap_source, float cap_sink);
void orc_bk_add_edge(orc_bk *g, int i, int j, float cap, float rev_cap);
void orc_bk_add_term1(orc_bk *g, int x, float e0, float e1);
void orc_bk_add_term2(orc_bk *g, int x, int y, float A, float B, float C, float D);
float orc_bk_maxflow(orc_bk *g);
int orc_bk_is_sink(const orc_bk *g, int i);
float orc_bk_label(int n, const float *unary, int m, const int *ei, const int *ej, const float *e00,
                   const float *e01, const float *e10, const float *e11, int *sink_out);

/* grid neighbours (nearest_neighbors.cpp:160-202) and the NAPSAC grid sampler (napsac_sampler.hpp) */
typedef struct orc_grid orc_grid;
orc_grid *orc_grid_new(const float *pts, unsigned int n, int cell_size);
void orc_grid_free(orc_grid *g);
int orc_grid_count(const orc_grid *g, unsigned int i);
const int *orc_grid_list(const orc_grid *g, unsigned int i);
typedef struct orc_napsac orc_napsac;
orc_napsac *orc_napsac_new(const orc_grid *g, unsigned int n, unsigned int m);
void orc_napsac_free(orc_napsac *s);
void orc_napsac_sample(orc_napsac *s, int *sample);

/* Ransac::run with the sampler / SPRT of cfg (PROSAC: points sorted by quality; its
 * mt19937 is seeded with cfg->seed instead of std::random_device). */
/* test switch: rank-2 enforcement in the 8-point polish (older reference revision) */
void orc_set_f8_rank2(int on);
/* test switch: SPRT tests points in file order from point 0 (revision of results/line2d/uniform_001.csv) */
void orc_set_sprt_file_order(int on);
/* all-cores CPU baseline: wall seconds of `count` hypotheses on `threads` workers */
double orc_hypothesis_loop_mt(int kind, const float *points, unsigned int n, int dlt_mode, float thr,
                              unsigned int seed, int count, int threads, int *best_cnt);
int orc_ransac_run_cfg(int kind, const float *points, unsigned int n, const orc_config *cfg, orc_result *out,
                       int *inliers_out, unsigned int *rec_iter, int *rec_count, float *rec_score, int rec_cap);

/* std::mt19937 + uniform_int_distribution<int>(0, max) (libstdc++ downscaling) */
typedef struct {
    uint32_t mt[624];
    int i;
} orc_mt;
void orc_mt_seed(orc_mt *g, uint32_t seed);
uint32_t orc_mt_next(orc_mt *g);
int orc_mt_uniform(orc_mt *g, unsigned int max);

/* ProsacSampler (usac/sampler/prosac_sampler.hpp) */
typedef struct orc_prosac orc_prosac;
orc_prosac *orc_prosac_new(unsigned int sample_size, unsigned int points_size, uint32_t seed);
void orc_prosac_free(orc_prosac *p);
const unsigned int *orc_prosac_growth(const orc_prosac *p);
unsigned int orc_prosac_largest(const orc_prosac *p);
void orc_prosac_set_term_len(orc_prosac *p, unsigned int t);
void orc_prosac_sample(orc_prosac *p, int *sample);

/* ProsacTerminationCriteria (usac/termination_criteria/prosac_termination_criteria.hpp) */
typedef struct orc_prosac_term orc_prosac_term;
orc_prosac_term *orc_prosac_term_new(const unsigned int *growth, unsigned int points_size, unsigned int sample_size,
                                     float desired_prob, unsigned int max_iterations);
void orc_prosac_term_free(orc_prosac_term *t);
unsigned int orc_prosac_term_length(const orc_prosac_term *t);
unsigned int orc_prosac_term_update(orc_prosac_term *t, unsigned int hypCount, const unsigned char *flags,
                                    unsigned int largest);

/* the 5-point solver's polynomial matrix M(z) of a null basis (4 x 9) -> 10 x 10 (pinned against
 * the reference's mblock.hpp by tests/test_oracle_essential.py) */
void orc_e5_matrix(const double *N, double z, double *M);

/* SPRT (usac/sprt.hpp) */
typedef struct orc_sprt orc_sprt;
orc_sprt *orc_sprt_new(int kind, unsigned int points_size, unsigned int sample_size, unsigned int max_iterations,
                       int max_hypothesis_test_before_sprt);
void orc_sprt_free(orc_sprt *s);
const unsigned int *orc_sprt_pool(const orc_sprt *s);
double orc_sprt_A(const orc_sprt *s);
unsigned int orc_sprt_histories(const orc_sprt *s);
int orc_sprt_verify(orc_sprt *s, orc_est *e, float thr, int current_hypothese, unsigned int maximum_score,
                    int *count, float *score, unsigned int *tested_out);
unsigned int orc_sprt_upper_bound(const orc_sprt *s, int inliers_size);
/* the throughput SPRT's per-model test: fixed (epsilon, delta, A), given pool starts (tests) */
void orc_sprt_fixed_batch(orc_est *e, const unsigned int *pool, unsigned int n, float thr, const float *models,
                          const unsigned int *starts, int K, double epsilon, double delta, double A, int *good,
                          int *count, unsigned int *tested);

int orc_ransac_run(int kind, const float *points, unsigned int n, float threshold, float desired_prob,
                   unsigned int max_iterations, unsigned int seed, int dlt_mode, orc_result *out,
                   int *inliers_out, unsigned int *rec_iter, int *rec_count, float *rec_score, int rec_cap);

/* Reference-style hypothesis throughput loop for the CPU baseline: `count` hypotheses
 * of sample (glibc pool) + minimal solve + full score, no termination; returns best count. */
int orc_hypothesis_loop(orc_est *e, orc_uniform *s, int count, float thr, float *best_score_sum);

/* generator/generator.cpp:98-148 Generate2DLinePoints (glibc rand(), srand(seed) first) */
void orc_generate_line2d(unsigned int seed, float noise, int inliers, int outliers, int border_x, int border_y,
                         float *points_out, float *gt_model);
/* the same without reseeding (continues rand(); generate_syntectic_dataset, generator.cpp:6-67) */
void orc_generate_line2d_next(float noise, int inliers, int outliers, int border_x, int border_y,
                              float *points_out, float *gt_model);

#ifdef __cplusplus
}
#endif
#endif
