/*
 * usac_gpu.h -- C-ABI of the MI355X-native USAC hypothesize-and-verify engine
 * (libransac_amd.so).  Plain pointers and sizes, opaque handles, int status
 * (0 = ok, < 0 = error, message via usac_last_error), never exit().
 *
 * Each entry point replaces one reference interface (MathsionYang/Ransac paths):
 *
 *   usac_create / usac_destroy     Ransac(Model*, cv::InputArray) estimator+quality init
 *                                  (usac/ransac/ransac.hpp:41-93, init.cpp:3-20)
 *   usac_estimate_models           Estimator::EstimateModel, batched
 *                                  (usac/estimator/estimator.hpp:19; homography
 *                                  homography_estimator.hpp:47-56 -> dlt.cpp:7-52;
 *                                  fundamental fundamental_estimator.hpp:48-63 ->
 *                                  seven_points.cpp:49-156;
 *                                  line2d line2d_estimator.hpp:36-54)
 *   usac_score_models              Quality::getNumberInliers(score, model), batched over
 *                                  models (usac/quality/quality.hpp:60-101)
 *   usac_get_inliers               Quality::getNumberInliers(..., get_inliers=true, inliers)
 *                                  / Quality::getInliers (quality.hpp:80-87, 108-121)
 *   usac_nonminimal / usac_lsq_fit Estimator::EstimateModelNonMinimalSample (weighted: estimator.hpp:26)
 *                                  (estimator.hpp:21; normalized_dlt.cpp:7-23;
 *                                  eight_points.cpp:4-100;
 *                                  line2d_estimator.hpp:59-107)
 *   usac_hypothesize_score         Sampler::generateSample + Estimator::EstimateModel +
 *                                  Quality::getNumberInliers + Score::bigger, fused over a
 *                                  batch (the body of ransac.cpp:58-139)
 *   usac_std_termination           StandardTerminationCriteria::getUpBoundIterations
 *                                  (standard_termination_criteria.hpp:52-62)
 *   usac_set_sprt / usac_sprt_tested  SPRT::verifyModelAndGetModelScore as a batch test
 *                                  (sprt.hpp:191-317, 332-355)
 *   usac_prosac_samples            ProsacSampler::generateSample (prosac_sampler.hpp:117-172)
 *   usac_set_device_sampler        Sampler choice of the throughput batches (Uniform / PROSAC
 *   usac_draw_samples              schedule, prosac_sampler.hpp:62-172 / NAPSAC grid,
 *   usac_set_cell_size             napsac_sampler.hpp:100-138) and its samples
 *   usac_grid_neighbors            NearestNeighbors::getGridNearestNeighbors
 *                                  (nearest_neighbors.cpp:160-202) built on the device
 *   usac_sprt_pool                 SPRT ctor pool + A0 (sprt.hpp:89-175)
 *   usac_ransac_run                Ransac::run + RansacOutput (ransac.cpp:14-238,
 *                                  ransac_output.hpp:29-97), Uniform sampler
 *   usac_ransac_run_sharded        Ransac::run with hypothesis-sharded batches
 *   usac_comm_*                    new: one RCCL all-gather of best records per batch
 *   usac_random / usac_sampler /   the per-call plugin state (ABI 11): the glibc random() stream,
 *   usac_termination / usac_sprt / Sampler::generateSample (sampler.hpp:11-35), TerminationCriteria
 *   usac_lo                        (termination_criteria.hpp:16-17, prosac_termination_criteria.hpp:
 *                                  148-201), SPRT (sprt.hpp:191-393, + the batch replay
 *                                  usac_sprt_replay), LocalOptimization::GetModelScore
 *                                  (local_optimization.hpp:19)
 *
 * Threading: a context is bound to one device and one HIP stream and is not
 * thread-safe (one host thread / process per GPU).  Calls are synchronous with respect
 * to their outputs unless named *_async.
 */
#ifndef USAC_GPU_H
#define USAC_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define USAC_ABI_VERSION 14

/* = enum ESTIMATOR (usac/model.hpp:10) */
enum { USAC_LINE2D = 1, USAC_HOMOGRAPHY = 2, USAC_FUNDAMENTAL = 3, USAC_ESSENTIAL = 4 };
/* = enum SAMPLER (usac/model.hpp:11): Uniform, Napsac (grid neighbours), Prosac */
enum { USAC_SAMPLER_UNIFORM = 1, USAC_SAMPLER_NAPSAC = 3, USAC_SAMPLER_PROSAC = 4 };
/* = enum LocOpt (usac/model.hpp:13): inner + iterative LO-RANSAC (unlimited / limited), graph-cut
 * LO (graphcut.hpp) */
enum { USAC_LO_NONE = 0, USAC_LO_INITLORSC = 1, USAC_LO_INITFLORSC = 2, USAC_LO_GC = 3 };
/* = enum NeighborsSearch (usac/model.hpp:12): the Ransac ctor (ransac.hpp:60-78) builds Grid
 * neighbours for Grid and nanoflann KNN for any other value (NullN included) */
enum { USAC_NEIGHBORS_NULL = 0, USAC_NEIGHBORS_NANOFLANN = 1, USAC_NEIGHBORS_GRID = 2 };
/* 4-pt DLT: THIN = reference semantics (vt.row(7) of the thin 8x9 SVD, dlt.cpp:43-48);
 * NULLSPACE = true null vector. */
enum { USAC_DLT_THIN = 0, USAC_DLT_NULLSPACE = 1 };

enum {
    USAC_OK = 0,
    USAC_ERR_ARG = -1,
    USAC_ERR_HIP = -2,
    USAC_ERR_UNSUPPORTED = -3,
    USAC_ERR_NO_MODEL = -111 /* best score 0, ransac.cpp:143-147 (reference exit(111)) */
};

typedef struct usac_ctx usac_ctx;

/* A hypothesis record: Score {inlier_number, score} (quality.hpp:16-37) of model
 * `model` produced by hypothesis `hyp_index` (global sample index). */
typedef struct usac_record {
    uint64_t hyp_index;
    int32_t inliers;
    float score;
    float model[9];
    int32_t valid;
} usac_record;

/* Model (usac/model.hpp:15-45) fields the loop reads. */
typedef struct usac_params {
    float threshold;            /* model.hpp:17 (default 2) */
    float desired_prob;         /* model.hpp:18 (0.95) */
    uint32_t max_iterations;    /* model.hpp:22 (10000) */
    uint32_t seed;              /* glibc srandom(seed): ResetRandomGenerator(false) semantics;
                                   also seeds PROSAC's mt19937 (the reference uses random_device) */
    int32_t dlt_mode;           /* USAC_DLT_* */
    uint32_t batch;             /* hypotheses per device batch (0 = default: 1024, 2048, ... up to 8192; SPRT 1024) */
    int32_t sampler;            /* USAC_SAMPLER_UNIFORM | _NAPSAC (grid) | _PROSAC (points sorted by quality) */
    int32_t sprt;               /* Model::setSprt (model.hpp:104): SPRT verification, sprt.hpp */
    int32_t lo;                 /* USAC_LO_* (model.hpp:26) */
    uint32_t lo_sample_size;          /* model.hpp:27 (14) */
    uint32_t lo_iterative_iterations; /* model.hpp:28 (4) */
    uint32_t lo_inner_iterations;     /* model.hpp:29 (20) */
    uint32_t lo_threshold_multiplier; /* model.hpp:30 (10) */
    int32_t cell_size;                /* model.hpp:43 (50): NAPSAC grid cell */
    int32_t neighbors;                /* USAC_NEIGHBORS_* (model.hpp:42): NAPSAC Grid or KNN */
    uint32_t knn;                     /* model.hpp:23 k_nearest_neighbors (NAPSAC KNN / GC, 1..32) */
    float spatial_coherence_gc;       /* model.hpp:33 (0.1): GC pairwise weight, used as given
                                         (graphcut.hpp:43; 0 = no pairwise term) */
    uint32_t max_hypothesis_test_before_sprt; /* model.hpp:40 (20; ABI 12): a rejected model still counts
                                         as an iteration from this iteration on (ransac.cpp:81-83), and the
                                         SPRT's adaptive history starts then (sprt.hpp:243); 0 = 20 */
} usac_params;

/* RansacOutput getters (ransac_output.hpp:57-97) */
typedef struct usac_run_output {
    float model[9];
    int32_t inliers;            /* getNumberOfInliers */
    uint32_t iters;             /* getNumberOfMainIterations */
    int64_t time_us;            /* getTimeMicroSeconds (loop + polish, as ransac.cpp:15,209) */
    int32_t n_records;          /* best-score updates in the main loop */
    int32_t polish_passes;
    float minimal_model[9];     /* best model before the non-minimal polish */
    int32_t minimal_inliers;
    uint32_t batches;           /* device batches launched */
    int32_t sprt_rejected;      /* models rejected by SPRT */
    int32_t sprt_histories;     /* SPRT tests designed (sprt_histories.size()) */
    uint32_t prosac_term_len;   /* final PROSAC termination_length (n without PROSAC) */
    uint32_t rollbacks;         /* PROSAC speculative batches cut short by a termination_length change */
    uint32_t lo_inner_iters;    /* getLOIters (ransac_output.hpp): inner LO iterations (GC: gc_iterations) */
    uint32_t lo_iterative_iters; /* iterative LO iterations (GC: labellings) */
    uint32_t lo_rounds;         /* LO speculation rounds (batches of inner iterations run at once) */
    uint32_t lo_stages;         /* LO device stages (one batched fit or one batched scoring each) */
    uint32_t sum_models;        /* models whose exact sequential Σerr the replay needed */
    uint32_t lo_fits;           /* LO least-squares fits this rank ran (a sharded run splits the
                                   inner-iteration chains: the ranks' counts add up to the 1-rank run's) */
    uint32_t spec_batches;      /* batches drawn and solved ahead of the replay (speculation) */
    uint32_t spec_rollbacks;    /* of those, cut short by a smaller termination bound (sampler rolled back) */
    uint32_t spec_wasted;       /* hypotheses solved and scored ahead that the run never reached */
} usac_run_output;

/* ---- lifetime ----------------------------------------------------------------- */
/* pts: n rows of `cols` floats (2: line [x y]; 4: two-view [x1 y1 x2 y2]), host memory,
 * copied to the device at create (the caller may free it). */
int usac_create(usac_ctx **out, int device, int estimator, const float *pts, uint32_t n, uint32_t cols);
void usac_destroy(usac_ctx *ctx);
const char *usac_last_error(const usac_ctx *ctx);
int usac_abi_version(void);
int usac_set_dlt_mode(usac_ctx *ctx, int mode);
uint32_t usac_sample_size(const usac_ctx *ctx);
uint32_t usac_num_points(const usac_ctx *ctx);

/* ---- plugin operators ----------------------------------------------------------- */
/* samples: B x m int32 (host) -> models: B x S x 9 floats, n_models[B] valid models per
 * sample, S = model slots per sample (3 for USAC_FUNDAMENTAL -- SevenPointsAlgorithm returns
 * <= 3 F that pass the oriented constraint, fundamental_estimator.hpp:48-63 -- else 1);
 * empty slots are zero-filled. */
int usac_estimate_models(usac_ctx *ctx, const int32_t *samples, uint32_t B, float *models, int32_t *n_models);
/* models: n_models x 9 floats (host); counts/sums (host, sums nullable).  Counts are
 * exact; sums are the sequential fp32 sums of quality.hpp:89-96. */
int usac_score_models(usac_ctx *ctx, const float *models, uint32_t n_models, float thr, int32_t *counts,
                      float *sums);
/* One model: ascending inlier indices (idx capacity >= n points), count and sum. */
int usac_get_inliers(usac_ctx *ctx, const float *model, float thr, int32_t *idx, uint32_t *n, float *sum);
/* The graph-cut LO's min cut, host side (usac_maxflow.hpp; gco-v3.0 energy.h + maxflow.inl
 * semantics): n nodes with add_term1(i, unary[i], 0), add_term2(ei[k], ej[k], e00[k], e01[k],
 * e10[k], e11[k]) in order, BK max-flow; sink_out[i] = 1 iff what_segment(i) == SINK.
 * Returns the flow.  No device work (exposed for parity tests against the gco sources). */
float usac_bk_label(int n, const float *unary, int m, const int32_t *ei, const int32_t *ej, const float *e00,
                    const float *e01, const float *e10, const float *e11, int32_t *sink_out);
/* NearestNeighbors::getNearestNeighbors_nanoflann (nearest_neighbors.cpp:69-128) on the
 * device: the k nearest neighbours of every point (1 <= k <= 32; idx n x k, d2 n x k
 * squared distances, nullable) by nanoflann's float L2 distance, the point itself excluded,
 * ascending distance, equal distances by ascending index; -1 / +inf where n - 1 < k. */
int usac_knn(usac_ctx *ctx, uint32_t k, int32_t *idx, float *d2);
/* Non-minimal least squares on the listed points; returns USAC_OK and writes model. */
int usac_nonminimal(usac_ctx *ctx, const int32_t *idx, uint32_t n, float *model);
/* Estimator::EstimateModelNonMinimalSample with optional weights (estimator.hpp:21,26):
 * weights == NULL is usac_nonminimal; otherwise weights[i] belongs to point i of the context
 * (n_points floats, indexed by point index as the reference's weights[sample[i]]) and the fit
 * is the weighted overload -- homography: weighted NormalizedDLT (normalized_dlt.cpp:25-36),
 * fundamental: weighted EightPointsAlgorithm (eight_points.cpp:176-228), both through the
 * weighted GetNormalizingTransformation (normalizing_transformation.cpp:117-166).  Line and
 * essential estimators have no weighted overload (USAC_ERR_UNSUPPORTED). */
int usac_lsq_fit(usac_ctx *ctx, const int32_t *idx, uint32_t n, const float *weights, float *model);

/* Fused batch: samples (B x m host int32) or NULL => device xorshift sampler keyed by
 * (seed, first_hyp + i).  Per-model counts/sums (host, nullable, B x S entries: slot
 * b*S + j = j-th valid model of sample b, count -1 on an empty slot) and the batch best
 * under Score::bigger with the earliest (sample, slot) on exact ties (best, nullable;
 * best->hyp_index = first_hyp + sample). */
int usac_hypothesize_score(usac_ctx *ctx, const int32_t *samples, uint32_t B, uint64_t seed, uint64_t first_hyp,
                           float thr, int32_t *counts, float *sums, usac_record *best);
/* Asynchronous device-sampled batch for throughput runs: enqueues sample+solve+score+
 * argmax on the context stream; usac_fetch_best waits and returns the batch best. */
int usac_hypothesize_async(usac_ctx *ctx, uint32_t B, uint64_t seed, uint64_t first_hyp, float thr);
int usac_fetch_best(usac_ctx *ctx, usac_record *best);
/* Per-slot counts / sums (sums nullable) of the last batch as the score kernel left them (the
 * throughput kernels' chunked sums included): n <= B x slots.  Waits for the stream.  For tests.
 * USAC_ERR_ARG after a usac_ransac_run until the next batch (the run's buffers are not a batch's). */
int usac_last_counts(usac_ctx *ctx, int32_t *counts, float *sums, uint32_t n);
int usac_sync(usac_ctx *ctx);
/* Device time of the last async batch's kernels, measured with HIP events on the
 * context stream: [0] whole batch, [1] score kernel, [2] solve kernel (ms). */
int usac_last_timings(usac_ctx *ctx, float *ms3);
/* ABI 14: on = 0 stops usac_hypothesize_async recording those HIP events on this context (four
 * event records of host time per batch; usac_last_timings then keeps returning the last timed
 * batch's values); on = 1 (the default) records them again. */
int usac_set_timing(usac_ctx *ctx, int on);
/* Score-kernel split factor (point chunks per hypothesis tile, 1 = exact sequential sums):
 * 1, 2, 4, 8, 16; any of 1..128 for the fundamental / essential estimators (their chunks are
 * separate workgroups, combined in chunk order; default 96). */
int usac_set_score_chunks(usac_ctx *ctx, int chunks);
/* Homography score kernel: 0 = guard-band fast path with the hypothesis pre-sort (default; multi-
 * chunk batches -- the throughput and loop batches -- go through the matrix-core prefilter scorer
 * unless USAC_H16=0), 1 = exact reference expression for every pair, 2 = fast path without the
 * pre-sort, 3 = as 0, and usac_score_models also scores through the multi-chunk scorer (tests: exact
 * counts, Σ within its bound).  Every variant gives the same counts. */
int usac_set_score_variant(usac_ctx *ctx, int variant);

/* Throughput SPRT (sprt.hpp:191-317 as a batch test): with enable != 0 every later
 * batch (usac_hypothesize_score / _async) verifies each model by the SPRT with fixed
 * (epsilon, delta) -- <= 0 selects the reference's initial values for the estimator
 * (sprt.hpp:106-150) -- and threshold A = estimateThresholdA(epsilon, delta), over the
 * SPRT pool of srandom(seed) (sprt.hpp:93-104), each model from a pool position of its own
 * (usac_batch_sprt_info) instead of the rolling index, without the history updates.  Each
 * decision equals the reference's fp64 lambda product walk with those constants from that
 * position (certified in log space from exact counts, the sequential product where the
 * certificate fails; kernels_sprt.hip).  Rejected models get count -1; accepted ones count =
 * inliers over all points, score = (float)count (sprt.hpp:276-281).  usac_ransac_run always
 * replays the exact sequential SPRT (rolling index, history) instead. */
int usac_set_sprt(usac_ctx *ctx, int enable, uint32_t seed, double epsilon, double delta);
/* pool points the SPRT tested in the last batch (the scoring work actually done) */
int usac_sprt_tested(usac_ctx *ctx, uint64_t *points_tested);
/* The batch test's constants -- eps_delta_A[3] = epsilon, delta, A (nullable) -- and the first pool
 * position each model slot of the last batch was tested from (starts, n slots, nullable; slots of
 * the fundamental solver 3 per sample; n <= the last batch's slots; a slot the solver left empty
 * reads UINT32_MAX).  Every decision equals the reference's fp64 product walk (sprt.hpp:209-234)
 * with these constants from that position.  For tests. */
int usac_batch_sprt_info(usac_ctx *ctx, double *eps_delta_A, uint32_t *starts, uint32_t n);
/* Sampler of the throughput batches' device stream (usac_hypothesize_score with samples ==
 * NULL, usac_hypothesize_async): USAC_SAMPLER_UNIFORM (default), USAC_SAMPLER_NAPSAC (grid
 * neighbours of usac_set_cell_size's cell, default 50, built on the device: the initial point
 * uniform over the points with >= m neighbours, then m - 1 consecutive entries of its
 * neighbour list from a random phase -- napsac_sampler.hpp:100-138, whose cursor persists
 * across samples; uniform samples when no point qualifies; 4-column points) or
 * USAC_SAMPLER_PROSAC --
 * hypothesis h (the global index first_hyp + b) uses the reference's PROSAC subset schedule
 * (growth function prosac_sampler.hpp:62-114, termination_length = n; points must be sorted
 * by quality): the subset's last point plus m - 1 distinct points before it, for
 * h < T_N = 200000, uniform afterwards (prosac_sampler.hpp:117-172).  The random draws are
 * the device SplitMix64 stream, not the host mt19937 (usac_ransac_run keeps that one). */
int usac_set_device_sampler(usac_ctx *ctx, int sampler);
/* Grid cell size of the device NAPSAC sampler (model.hpp:43, default 50). */
int usac_set_cell_size(usac_ctx *ctx, int cell_size);
/* NearestNeighbors::getGridNearestNeighbors (nearest_neighbors.cpp:160-202) on the device:
 * cell ((int)(x1/cs), (int)(y1/cs), (int)(x2/cs), (int)(y2/cs)), fp32 division.  CSR (every
 * output nullable, host memory): cell[n] (cells numbered in order of first appearance),
 * rank[n] (position in the cell), start[n_cells + 1], members[n] (cells in order, ascending
 * index) -- point i's neighbours are its cell's members except itself, ascending -- and
 * eligible[n_eligible] = the points with >= sample-size neighbours (NAPSAC, Q18), ascending.
 * usac_ransac_run's NAPSAC / graph-cut grids are this one. */
int usac_grid_neighbors(usac_ctx *ctx, int cell_size, uint32_t *n_cells, uint32_t *cell, uint32_t *rank,
                        uint32_t *start, int32_t *members, int32_t *eligible, uint32_t *n_eligible);
/* The device stream's samples for hypotheses first_hyp .. first_hyp + B - 1 (B x m int32,
 * host memory): what the solve kernels draw.  For tests. */
int usac_draw_samples(usac_ctx *ctx, uint32_t B, uint64_t seed, uint64_t first_hyp, int32_t *out);

/* ---- loop --------------------------------------------------------------------- */
uint32_t usac_std_termination(uint32_t inliers, uint32_t points_size, uint32_t sample_size, float desired_prob,
                              uint32_t max_iterations);
/* Ransac::run (ransac.cpp:14-238) with the Uniform (glibc random() stream), NAPSAC (grid or
 * KNN neighbours, napsac_sampler.hpp), graph-cut LO (graphcut.hpp; KNN or grid neighbours;
 * not with NAPSAC, whose combination the reference leaves undefined) or PROSAC (prosac_sampler.hpp + prosac_termination_criteria.hpp)
 * sampler, optional SPRT (sprt.hpp; pool shuffle from the same glibc stream), optional
 * inner + iterative LO-RANSAC (inner_local_optimization.hpp, iterative_local_optimization.hpp;
 * its mt19937 seeded with seed + 1).  inliers_out (capacity n,
 * nullable): final inliers ascending.  records (nullable, capacity rec_cap): best-score
 * updates in loop order (hyp_index = iteration, SPRT double counting included). */
int usac_ransac_run(usac_ctx *ctx, const usac_params *params, usac_run_output *out, int32_t *inliers_out,
                    usac_record *records, uint32_t rec_cap);
/* All-gather of host bytes across the ranks of a sharded run: every rank passes `bytes` bytes at
 * `send`; `recv` (nranks x bytes) receives them in rank order.  Returns 0 on success. */
typedef int (*usac_allgather_fn)(void *user, const void *send, size_t bytes, void *recv);
/* Ransac::run with every batch's hypotheses sharded over nranks processes / GPUs:
 * each rank draws the same host sample stream (same params, same seed), solves and scores its
 * contiguous slice of the batch, and the slices' counts and models are all-gathered -- through
 * `gather` when non-null (e.g. a torch.distributed gloo group), else RCCL on the communicator of
 * usac_comm_init(ctx, nranks, rank, id).  Termination, LO, graph cut and polish are then replayed
 * on the merged batch identically on every rank, so every rank's output equals usac_ransac_run's.
 * With SPRT each rank also computes its slice's pool-order inlier words (the words the sequential
 * SPRT walk reads, sprt.hpp:191-317), all-gathered with the models; every rank replays the walk.
 * A rank that fails joins the all-gather with its status and every rank fails with it; a gather
 * callback must therefore fail (return non-zero) on every rank or on none. */
int usac_ransac_run_sharded(usac_ctx *ctx, const usac_params *params, int nranks, int rank, usac_allgather_fn gather,
                            void *gather_user, usac_run_output *out, int32_t *inliers_out, usac_record *records,
                            uint32_t rec_cap);
/* Host glibc-compatible UniformSampler stream (uniform_sampler.hpp:42-54): count x m
 * samples after srandom(seed).  Exposed for parity tests. */
int usac_uniform_samples(uint32_t seed, uint32_t n_points, uint32_t m, uint32_t count, int32_t *out);
/* Host ProsacSampler stream (prosac_sampler.hpp:117-172), mt19937 seeded with `seed`,
 * termination_length held at `termination_length`: count x m samples.  For parity tests. */
int usac_prosac_samples(uint32_t seed, uint32_t n_points, uint32_t m, uint32_t count, uint32_t termination_length,
                        int32_t *out);
/* SPRT random pool after srandom(seed) (sprt.hpp:89-104; n_points glibc draws) and the
 * first test's threshold A (sprt.hpp:332-355) for `estimator`.  For parity tests. */
int usac_sprt_pool(uint32_t seed, int estimator, uint32_t n_points, uint32_t m, uint32_t *pool, double *A0);

/* ---- stateful plugins: the reference's per-call surface (ABI 11) ----------------------
 * Handles that keep the reference's plugin state between calls, so a caller that keeps its
 * own Ransac::run loop (ransac.cpp:58-139) swaps each plugin for the device one:
 *   usac_random       the global glibc random() stream after srandom(seed) -- UniformSampler and
 *                     NapsacSampler draw from it, the SPRT ctor shuffles its pool with it
 *                     (uniform_sampler.hpp:22-54, array_random_generator.hpp:21-49, sprt.hpp:93-104)
 *   usac_sampler      Sampler::generateSample (sampler.hpp:11-35): Uniform (persistent pool),
 *                     PROSAC (growth function, termination length), NAPSAC (grid / KNN neighbours
 *                     built on the context's device)
 *   usac_termination  TerminationCriteria::getUpBoundIterations (termination_criteria.hpp:16-17) and
 *                     ProsacTerminationCriteria::getUpBoundIterations(hypCount, model)
 *                     (prosac_termination_criteria.hpp:148-201)
 *   usac_sprt         SPRT::verifyModelAndGetModelScore (sprt.hpp:191-317), getUpperBoundIterations
 *                     (sprt.hpp:371-393) and the batch replay of the loop body with SPRT
 *   usac_lo           LocalOptimization::GetModelScore (local_optimization.hpp:19): inner + iterative
 *                     LO-RANSAC or graph-cut LO
 * A handle created on a context uses that context's device, stream and buffers: it must be
 * destroyed before the context, and -- like the reference's plugins -- is not thread-safe.
 * Handles drawing from a usac_random keep a pointer to it (destroy them first). */
typedef struct usac_random usac_random;
typedef struct usac_sampler usac_sampler;
typedef struct usac_termination usac_termination;
typedef struct usac_sprt usac_sprt;
typedef struct usac_lo usac_lo;

int usac_random_create(uint32_t seed, usac_random **out);
uint32_t usac_random_next(usac_random *rng); /* random() */
void usac_random_destroy(usac_random *rng);

/* initSampler (ransac/init.cpp) for params->sampler:
 *   USAC_SAMPLER_UNIFORM  UniformSampler on rng: m draws without replacement from a persistent
 *                         pool, idx = random() % max, refilled when max reaches 0 (Q5)
 *   USAC_SAMPLER_PROSAC   ProsacSampler, its mt19937 seeded with params->seed (the reference:
 *                         std::random_device); points sorted by quality; sampling is limited to the
 *                         termination length of the PROSAC termination criteria created on it
 *                         (usac_termination_create), n before that (prosac_sampler.hpp:117-172)
 *   USAC_SAMPLER_NAPSAC   NapsacSampler on rng with grid neighbours (params->neighbors ==
 *                         USAC_NEIGHBORS_GRID, cell params->cell_size; 4-column points) or KNN
 *                         (params->knn), both built on ctx's device (napsac_sampler.hpp:40-158)
 * rng: required for Uniform / NAPSAC, ignored for PROSAC. */
int usac_sampler_create(usac_ctx *ctx, const usac_params *params, usac_random *rng, usac_sampler **out);
/* generateSample(sample): m indices into `sample`.  NAPSAC rewrites only sample[0] once it has
 * turned uniform (as the reference), so pass the same array every call, as the loop does. */
int usac_sampler_generate(usac_sampler *s, int32_t *sample);
/* count successive generateSample calls into samples (count x m; each row starts as a copy of
 * the previous one, the reference's reused sample array) */
int usac_sampler_generate_batch(usac_sampler *s, uint32_t count, int32_t *samples);
/* samples drawn so far; PROSAC: subset_size and largest_sample_size (else n, n) -- nullable */
int usac_sampler_state(const usac_sampler *s, uint64_t *drawn, uint32_t *subset_size, uint32_t *largest_sample_size);
void usac_sampler_destroy(usac_sampler *s);

/* initTerminationCriteria: StandardTerminationCriteria (params->desired_prob, ->max_iterations;
 * m and n from ctx), or -- prosac != NULL, a USAC_SAMPLER_PROSAC sampler -- ProsacTerminationCriteria
 * linked to it both ways as in the reference (the sampler reads its termination length, it reads
 * the sampler's growth function and largest sample size; prosac_termination_criteria.hpp:44-119). */
int usac_termination_create(usac_ctx *ctx, const usac_params *params, usac_sampler *prosac, usac_termination **out);
/* getUpBoundIterations(inlier_size) / (inlier_size, points_size) (standard_termination_criteria.hpp:
 * 52-74); points_size 0 = the context's n */
uint32_t usac_termination_bound(const usac_termination *t, uint32_t inlier_size, uint32_t points_size);
/* ProsacTerminationCriteria::getUpBoundIterations(hypCount, model): the model's inlier flags at
 * params->threshold over the quality-sorted points from the device, the non-randomness /
 * maximality scan on the host.  *max_iters = the new bound, *termination_length (nullable) = the
 * updated termination length (the linked sampler uses it from its next sample on). */
int usac_prosac_termination(usac_termination *t, uint32_t hyp_count, const float *model, uint32_t *max_iters,
                            uint32_t *termination_length);
void usac_termination_destroy(usac_termination *t);

/* SPRT ctor (sprt.hpp:89-175): the random pool from n draws of rng (the Ransac ctor creates it after
 * the sampler, before the sampler's first draw), the reference's initial epsilon / delta / t_M / m_S
 * for ctx's estimator; params->threshold, ->max_iterations, ->max_hypothesis_test_before_sprt. */
int usac_sprt_create(usac_ctx *ctx, const usac_params *params, usac_random *rng, usac_sprt **out);
/* verifyModelAndGetModelScore(model, current_hypothese, maximum_score, score), one model (9 floats;
 * line: 3): the model's inlier flags in pool order from the device, the reference's fp64 lambda walk
 * over the rolling pool index on the host.  *good = the decision; *count / *score written as the
 * reference writes them (accepted: inliers, (float)inliers; rejected while current_hypothese <
 * params->max_hypothesis_test_before_sprt (default 20): the full count; otherwise left untouched). */
int usac_sprt_verify(usac_sprt *s, const float *model, int32_t current_hypothese, uint32_t maximum_score,
                     int32_t *good, int32_t *count, float *score);
/* getUpperBoundIterations(inlier_size) (sprt.hpp:371-393) */
uint32_t usac_sprt_upper_bound(const usac_sprt *s, uint32_t inlier_size);
/* tests designed so far (sprt_histories.size()) and models rejected by this handle */
int usac_sprt_stats(const usac_sprt *s, uint32_t *histories, uint32_t *rejected);

/* The loop body of ransac.cpp:58-139 with SPRT over a batch of minimal samples (SURVEY §8(b)
 * usac_sprt_replay).  State in / out: */
typedef struct usac_sprt_state {
    uint32_t iters;        /* in/out: the loop's iteration counter (ransac.cpp:55) */
    uint32_t max_iters;    /* in: the bound in force (`while (iters < max_iters)`) */
    int32_t best_inliers;  /* in: best_score->inlier_number */
    float best_score;      /* in: best_score->score */
    uint32_t sample;       /* in/out cursor: the next sample of the batch ... */
    uint32_t slot;         /* ... and model slot to verify; (0, 0) starts a new batch */
    int32_t found;         /* out: 1 = stopped after a model bigger than the best (Score::bigger) */
    int32_t inliers;       /* out: that model's score (the caller updates its best, runs LO and */
    float score;           /*      the termination, sets max_iters / best_* and calls again) */
    uint32_t found_sample, found_slot;
    uint32_t rejected;     /* out: models rejected during this call */
} usac_sprt_state;
/* models: B x slots x 9 floats and n_models[B] (usac_estimate_models' layout; slots = 3 for the
 * 7-point solver, else 1).  From the cursor, in loop order: verify(model, iters, best_inliers); a
 * rejected model at iters >= max_hypothesis_test_before_sprt (the handle's params, default 20) counts an
 * iteration and is skipped (Q9); every other model is
 * compared with the best; after each sample iters++; before each sample `iters < max_iters` is
 * checked.  Returns with found = 1 at the first model bigger than the best (the cursor then points
 * past it), or found = 0 when the batch is exhausted (sample == B) or the loop bound is reached
 * (iters >= max_iters).  The batch's inlier words are computed on the device when the cursor is at
 * (0, 0); later calls for the same batch must pass the same models. */
int usac_sprt_replay(usac_sprt *s, const float *models, const int32_t *n_models, uint32_t B, usac_sprt_state *st);
void usac_sprt_destroy(usac_sprt *s);

/* initLocalOptimization for params->lo: USAC_LO_INITLORSC / _INITFLORSC (InnerLocalOptimization with
 * IterativeLocalOptimization, unlimited / limited; inner_local_optimization.hpp:40-133,
 * iterative_local_optimization.hpp:28-136; its mt19937 seeded with params->seed + 1) or USAC_LO_GC
 * (GraphCut, graphcut.hpp:99-153, KNN or grid neighbours built on ctx's device; params->neighbors,
 * ->knn, ->cell_size, ->spatial_coherence_gc).  The LO threshold persists across calls (Q11). */
int usac_lo_create(usac_ctx *ctx, const usac_params *params, usac_lo **out);
/* GetModelScore(best_model, best_score): model (9 floats), inliers and score improved in place */
int usac_lo_get_model_score(usac_lo *lo, float *model, int32_t *inliers, float *score);
/* lo_inner_iters / lo_iterative_iters (InnerLocalOptimization), or gc_iterations / labellings (GC) */
int usac_lo_iters(const usac_lo *lo, uint32_t *inner, uint32_t *iterative);
void usac_lo_destroy(usac_lo *lo);

/* ---- multi-GPU (RCCL over xGMI) --------------------------------------------------- */
/* 128-byte RCCL unique id (rank 0 creates, everyone receives it out of band). */
int usac_comm_unique_id(uint8_t *id128);
int usac_comm_init(usac_ctx *ctx, int nranks, int rank, const uint8_t *id128);
/* What RCCL itself reports for ctx's communicator (ABI 12): ncclCommCount / ncclCommUserRank /
 * ncclCommCuDevice -- a multi-GPU bench line states the rank count RCCL saw, not the one asked for. */
int usac_comm_count(usac_ctx *ctx, int *nranks, int *rank, int *device);
/* All-gather of one usac_record per rank on the context stream: all[nranks]. */
int usac_allgather_records(usac_ctx *ctx, const usac_record *local, usac_record *all);
/* The per-batch best exchange of the throughput pipeline, off the compute streams: the record
 * usac_hypothesize_async(batch) leaves on the device is all-gathered over ctx's communicator
 * on ctx's own exchange stream, ordered after `batch`'s stream by an event (neither stream
 * waits for the other's later work; no host staging), then copied to pinned host memory.
 * `slot` (< USAC_XRING) names the exchange in a ring; usac_exchange_best_wait(slot) returns
 * the nranks records (rank order) and frees the slot: at most USAC_XRING exchanges may be
 * outstanding.  Every rank must issue the exchanges -- and the context's other collectives
 * (usac_allgather_records, sharded runs on its communicator) -- in the same order; the two kinds
 * may be mixed: a collective on the context stream waits for the exchanges issued before it, an
 * exchange for the context-stream collectives issued before it (events, no host wait).
 * batch may be ctx itself or another context on the same device. */
#define USAC_XRING 8
int usac_exchange_best_async(usac_ctx *ctx, usac_ctx *batch, uint32_t slot);
int usac_exchange_best_wait(usac_ctx *ctx, uint32_t slot, usac_record *all);
/* Merge n records by Score::bigger, earliest hyp_index on exact ties. */
int usac_merge_records(const usac_record *recs, uint32_t n, usac_record *best);

/* ---- self-test hooks (ABI 13) ------------------------------------------------------- */
/* The essential 5-point solver's root step alone (five_points.cpp:139-157: rpoly_ak1's real zeros
 * in its order, usac_rpoly.hpp) on B host polynomials of 11 ascending coefficients each: roots
 * (B x 10 doubles, row h = polynomial h's real zeros in order) and their numbers.  Its correctly
 * rounded log / exp (rpoly.cpp:82,98) on n host arguments.  Device: the context's; no other state. */
int usac_selftest_rpoly(usac_ctx *ctx, const double *coeffs, uint32_t B, double *roots, int32_t *nroots);
int usac_selftest_logexp(usac_ctx *ctx, const double *x, uint32_t n, double *log_out, double *exp_out);

#ifdef __cplusplus
}
#endif
#endif
