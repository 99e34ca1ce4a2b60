// usac_kernels.h -- internal launchers (kernels.hip, kernels_nonmin.hip) used by the host
// side of the C-ABI (usac_api.cpp).  Every launcher enqueues on `st` and returns the
// launch status; none synchronises.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/usac_gpu.h"

namespace usac {

// Throughput-path sampler state (one per batch): the SplitMix64 stream keyed by (seed,
// hypothesis index), and optionally the PROSAC schedule -- prosac[h] = the subset size the
// reference's ProsacSampler uses for hypothesis h (prosac_sampler.hpp:117-172, growth
// function of :62-114, termination_length = N) for h < prosac_len; later hypotheses are
// uniform, as the reference's are after T_N = 200000.
//
// NAPSAC (grid, napsac_sampler.hpp:100-138) when nap_start != nullptr: the initial point is
// drawn uniformly from the points with >= m grid neighbours (the reference draws from its
// pool and skips the others, Q18 -- the same distribution), then m - 1 consecutive entries of
// its neighbour list from a random phase (the reference walks them from a cursor that
// persists across samples); no eligible point -> uniform samples (the reference turns
// uniform after n failed draws).  Grid CSR as built by build_grid.
struct DevSampler {
    uint64_t seed;
    const uint32_t *prosac;  // nullptr: uniform sampler
    uint32_t prosac_len;
    uint32_t nap_n_eligible;
    const uint32_t *nap_cell, *nap_rank, *nap_start;  // nap_start == nullptr: no NAPSAC
    const int32_t *nap_members, *nap_eligible;
};

// Grid neighbours on the device (kernels_grid.hip): CSR bit-identical to usac_host.hpp's
// GridNeighbors -- cell[n] (first-appearance numbering), rank[n], start[n_cells + 1],
// members[n] -- plus eligible[] = points with >= m neighbours, ascending.  cmin = the lowest
// cell of the dataset box per dimension, bits = each dimension's key width (its cell range
// plus an out-of-box sentinel; <= 63 bits in all).  Synchronises `st` once (the counts).
size_t grid_workspace_bytes(uint32_t n);
hipError_t build_grid(hipStream_t st, const float4 *pts, uint32_t n, int cell_size, int4 cmin, int4 bits, uint32_t m,
                      void *ws, uint32_t *cell, uint32_t *rank, uint32_t *start, int32_t *members, int32_t *eligible,
                      uint32_t *pinned2, uint32_t *n_cells_out, uint32_t *n_elig_out);

// device-drawn samples only (B x m int32), the stream the solve kernels use
hipError_t launch_draw_samples(hipStream_t st, int m, uint32_t n, uint32_t B, DevSampler ds, uint64_t first_hyp,
                               int32_t *out);

// thin mode: k_solve_h4 (QR + inverse iteration) then k_solve_h4_jac over its fall-back list
// (fb_list: B entries; fb_n: two counters, zero before the first use, reset by the kernel);
// nullspace mode: k_solve_h4_jac over all B (fb_list / fb_n unused)
struct H16Consts;
// emit (nullable): the solvers also write each hypothesis' matrix-core scorer rows and slack
// (usac_h16.hpp h16_rows_of; rows = B x 96 B, fm = B floats) for threshold thr
struct H16Emit {
    const H16Consts *k;
    float thr;
    void *rows;
    float *fm;
};
hipError_t launch_solve_h4(hipStream_t st, const float4 *pts, uint32_t n, const int32_t *samples_in,
                           int32_t *samples_out, uint32_t B, DevSampler ds, uint64_t first_hyp, int nullspace,
                           float *models, uint32_t *fb_list, uint32_t *fb_n, const H16Emit *emit = nullptr);
hipError_t launch_prepare_h(hipStream_t st, const float *in, uint32_t B, float *models);
hipError_t launch_score_h(hipStream_t st, int chunks, const float4 *pts, uint32_t n, const float *models, uint32_t B,
                          float thr, int32_t *counts, float *sums);

hipError_t launch_prepare_rec(hipStream_t st, const float4 *pts, uint32_t n, float thr, float4 *rec);
// ext = dataset box {max|x1|, max|y1|, max|x2|, max|y2|} (stage-A error bounds)
// perm (nullable, B + 2 uint32): hypothesis pre-sort scratch (k_presort_h)
// ysplit > 1 (throughput mode): every 64-hypothesis tile's points over chunks x ysplit waves in
// ysplit workgroups, partials in yscratch (8 B x ysplit x B) added in order by a second launch
// the fast scorer's hypothesis pre-sort buffer: region counters (zeroed once, when the buffer
// is allocated: every launch leaves them at 0), then B permutation entries
size_t presort_bytes(uint32_t B);
size_t presort_counter_bytes();
hipError_t launch_score_hf(hipStream_t st, int chunks, bool exact_sum, const float4 *rec, uint32_t n, float4 ext,
                           const float *models, uint32_t B, float thr, uint32_t *perm, int32_t *counts, float *sums,
                           uint32_t ysplit = 1, void *yscratch = nullptr);

// Matrix-core prefilter scorer of homographies (kernels_h16.hip, DESIGN.md §6 "h16"): the dataset
// constants -- every coordinate centred and scaled by a power of two, x1 = cx1 + s1 u, y1 = cy1 + s1 v,
// x2 = cx2 + s2 p, y2 = cy2 + s2 q -- and fmax[k] >= |f_k| over the finite points for the nine features
// f = (u, v, 1, p u, p v, p, q u, q v, q); ext = the dataset box of k_score_hf (its stage-A bounds).
struct H16Consts {
    double cx1, cy1, s1, cx2, cy2, s2;
    double fmax[9];
    float4 ext;
};
// device (one workgroup, once per context at the first h16 batch): the constants of n float4
// points into *out (no finite point: centres 0, scales 1, fmax 0 -- every feature is then NaN)
hipError_t launch_h16_consts(hipStream_t st, const float4 *pts, uint32_t n, float4 ext, H16Consts *out);
// fp16 point features in the MFMA B-operand layout, 1 KB per 32 points (h16_feature_bytes(n));
// points past n and non-finite points get NaN features (never kept)
size_t h16_feature_bytes(uint32_t n);
hipError_t launch_h16_points(hipStream_t st, const float4 *pts, uint32_t n, const H16Consts *k, void *feat);
// per batch: each hypothesis' three fp16 rows (96 B) and its prefilter slack (rows: B x 96 B, fm: B floats)
hipError_t launch_h16_rows(hipStream_t st, const float *models, uint32_t B, const H16Consts *k, float thr,
                           void *rows, float *fm);
// the scorer: counts / sums of B hypotheses (exact counts; Σ from fixed-point stage-B terms) over
// `chunks` point chunks; part = h16_part_bytes(B, chunks) scratch
size_t h16_part_bytes(uint32_t B, int chunks);
// finish = false: the chunk partials are left for launch_argmax_h16 (the batch argmax adds them)
hipError_t launch_score_h16(hipStream_t st, const void *feat, const float4 *pts, uint32_t n, const void *rows,
                            const float *fm, const float *models, uint32_t B, float thr, int chunks, void *part,
                            int32_t *counts, float *sums, bool finish = true);
// Σ's fixed-point exponent of the h16 chunk partials for threshold thr
int h16_fixed_point(float thr);

// Matrix-core prefilter scorer of essential matrices (kernels_e16.hip, DESIGN.md §6 "e16"): fp16
// features of the h16 layout divided by each point's rho (once per context), per batch each listed
// model's fp16 coefficient rows (hi / lo, 64 B) and rejection bound (e16_row_bytes(kmax), kmax floats), then the
// scorer over `chunks` point chunks (part = e16_part_bytes(kmax, chunks)); counts exact, Σ from
// fixed-point guarded terms, written at the listed slots
// self-test hooks (usac_selftest_*): the 5-point root step alone on B given polynomials (11 ascending
// coefficients each) -> roots (10 x B doubles, root r of polynomial h at [r B + h]) and their numbers;
// workspace = e5_workspace_bytes(B).  The root step's correctly rounded log / exp on n arguments.
hipError_t launch_e5_roots_selftest(hipStream_t st, const double *coef, uint32_t B, double *roots, int32_t *nroots,
                                    void *workspace);
hipError_t launch_jt_logexp_selftest(hipStream_t st, const double *x, uint32_t n, double *lg, double *ex);

size_t e16_feature_bytes(uint32_t n);
hipError_t launch_e16_points(hipStream_t st, const float4 *pts, uint32_t n, const H16Consts *k, void *feat);
size_t e16_row_bytes(uint32_t kmax);
hipError_t launch_e16_rows(hipStream_t st, const float *models, size_t stride, const uint32_t *list,
                           const uint32_t *list_n, uint32_t kmax, const H16Consts *k, float thr, void *rows,
                           float *cm);
size_t e16_part_bytes(uint32_t kmax, int chunks);
hipError_t launch_score_e16(hipStream_t st, const void *feat, const float4 *pts, uint32_t n, const void *rows,
                            const float *cm, const float *models, size_t stride, const uint32_t *list,
                            const uint32_t *list_n, uint32_t kmax, float thr, int chunks, void *part,
                            int32_t *counts, float *sums);

hipError_t launch_solve_line(hipStream_t st, const float2 *pts, uint32_t n, const int32_t *samples_in,
                             int32_t *samples_out, uint32_t B, DevSampler ds, uint64_t first_hyp, float *models);
hipError_t launch_prepare_line(hipStream_t st, const float *in, uint32_t B, float *models);
hipError_t launch_score_line(hipStream_t st, int chunks, const float2 *pts, uint32_t n, const float *models,
                             uint32_t B, float thr, int32_t *counts, float *sums);

// B = number of model slots; hyp_index = first_hyp + slot / spk (spk = slots per hypothesis)
// launch_argmax over the h16 scorer's chunk partials (launch_score_h16 with finish = false): the
// first pass also adds every hypothesis' chunks in chunk order and writes counts / sums, exactly as
// k_h16_finish does -- one launch fewer per batch
hipError_t launch_argmax_h16(hipStream_t st, const void *part, uint32_t B, int chunks, float thr, int32_t *counts,
                             float *sums, const float *models, int ncomp, uint64_t first_hyp, uint32_t spk,
                             void *scratch, usac_record *out);
hipError_t launch_argmax(hipStream_t st, const int32_t *counts, const float *sums, uint32_t B, const float *models,
                         int ncomp, uint64_t first_hyp, uint32_t spk, void *scratch /* 12 B x ceil(B/2048) */,
                         usac_record *out);

// One rank's slice of a sharded batch packed for the all-gather (device to device): word 0 =
// the rank's status, then counts (S of P slots, -1 on padding) and ncomp model words per slot
// (component k of slot i at models[k * S + i], zero on padding): 1 + (1 + ncomp) * P words.
hipError_t launch_pack_slice(hipStream_t st, const int32_t *counts, const float *models, uint32_t S, uint32_t P,
                             int ncomp, int32_t status, int32_t *out);

// fundamental (kernels_fund.hip): slots 3*b + j, counts -1 on empty slots, list/list_n =
// occupied slots (list_n zeroed by the launcher)
hipError_t launch_solve_f7(hipStream_t st, const float4 *pts, uint32_t n, const int32_t *samples_in,
                           int32_t *samples_out, uint32_t B, DevSampler ds, uint64_t first_hyp, float *models,
                           int32_t *counts, uint32_t *list, uint32_t *list_n);
hipError_t launch_prepare_f(hipStream_t st, const float *in, uint32_t K, float *models);
// list == nullptr: lanes = slots 0..kmax-1; else lanes walk list[0 .. *list_n) (<= kmax);
// estimator = USAC_FUNDAMENTAL (Sampson) or USAC_ESSENTIAL
hipError_t launch_score_f(hipStream_t st, int estimator, int chunks, const float4 *pts, uint32_t n,
                          const float *models, size_t stride, const uint32_t *list, const uint32_t *list_n,
                          uint32_t kmax, float thr, int32_t *counts, float *sums);
// fast two-view scorer over the k_prepare_rec records: same results as launch_score_f
// (chunks 1..128; scratch = tv_scratch_bytes(kmax, chunks): pre-sort permutation + chunk
// partials)
hipError_t launch_score_f2(hipStream_t st, int estimator, int chunks, const float4 *rec, const float4 *pts,
                           uint32_t n, float4 ext, const float *models, size_t stride, const uint32_t *list,
                           const uint32_t *list_n, uint32_t kmax, float thr, int32_t *counts, float *sums,
                           void *scratch);
size_t tv_scratch_bytes(uint32_t kmax, int chunks);
// essential 5-point (kernels_ess.hip): one slot per sample (models [9][B], counts 0 / -1,
// list / list_n); workspace = e5_workspace_bytes(B)
// thin (nullable): a CU-masked stream for the root-order kernels (k_e5_order / k_e5_order_tail: one
// register-heavy wave per SIMD for long), ordered against st by ev_in / ev_out
hipError_t launch_solve_e5(hipStream_t st, const float4 *pts, uint32_t n, const int32_t *samples_in,
                           int32_t *samples_out, uint32_t B, DevSampler ds, uint64_t first_hyp, float *models,
                           int32_t *counts, uint32_t *list, uint32_t *list_n, void *workspace,
                           hipStream_t thin = nullptr, hipEvent_t ev_in = nullptr, hipEvent_t ev_out = nullptr);
size_t e5_workspace_bytes(uint32_t B);

// SPRT parity support (kernels_sprt.hip): points permuted into pool order, and per-model
// pool-order inlier words (words[w * row_stride + row], bit b = position 32 w + b)
hipError_t launch_gather_points(hipStream_t st, const void *pts, uint32_t cols, const uint32_t *idx, uint32_t n,
                                void *out);
// tail (optional): the batch's slot counts [S], list count [1], list [S] and models [nmod] copied
// by the same launch into dst, so the host fetches a batch's results with one copy
struct PoolTail {
    const uint32_t *counts, *list_n, *list, *models;
    uint32_t S, nmod;
    uint32_t *dst;
};
hipError_t launch_pool_mask(hipStream_t st, int estimator, const void *pool_pts, uint32_t n, const float *models,
                            size_t stride, const uint32_t *list, const uint32_t *list_n, uint32_t kmax, float thr,
                            uint32_t *words, uint32_t row_stride, const PoolTail *tail = nullptr);

// throughput SPRT (batch-fixed test, decisions = the reference's fp64 product walk from each
// model's start, kernels_sprt.hip): counts -1 for rejected models, tested_total (nullable)
// accumulates the pool points tested; starts (nullable, one per slot) receives each model's
// first pool position.  surv: kmax * sprt_survivor_bytes() scratch, surv_n: one uint32 (zeroed by
// the launcher)
struct SprtConsts {
    double up, down, A;    // delta / epsilon, (1 - delta) / (1 - epsilon), A (the reference's doubles)
    double lu, ld, lA;     // their natural logarithms
    double margin, climb;  // the certificate: |P - log A| > margin, climbs < climb (1e-7, 700)
};
hipError_t launch_score_sprt(hipStream_t st, int estimator, const void *pool_pts, uint32_t n, const float *models,
                             size_t stride, const uint32_t *list, const uint32_t *list_n, uint32_t kmax, float thr,
                             const SprtConsts &kc, int32_t *counts, float *sums, uint32_t *tested_total, void *surv,
                             uint32_t *surv_n, uint32_t *starts = nullptr);
size_t sprt_survivor_bytes();

// exact inliers of one model (kernels_inliers.hip): ascending idx, count, sequential Σ;
// scratch = inliers_scratch_bytes(n, 1)
hipError_t launch_inliers(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *model, float thr,
                          int32_t *idx, int32_t *count, float *sum, void *scratch);
// the same for W models at once (models slot w at models + 9 w, row-major; thrs[w], or thr
// when thrs is null; list at idx + w * idx_stride, idx nullable = counts and sums only;
// counts[w], sums[w]).  slots (nullable): the W launched rows are slots[0..W) of a larger
// set, every other slot is left untouched.  ok (nullable): slots with ok[w] == 0 keep their
// index list (their counts / sums are undefined).  sums nullable: no Σ pass, which
// launch_inliers_sums then runs from the same scratch (e.g. on another stream, ordered after
// this launch, before the scratch is reused).  scratch = inliers_scratch_bytes(n, max slot + 1)
hipError_t launch_inliers_batch(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *models,
                                uint32_t W, float thr, const float *thrs, const uint32_t *slots, int32_t *idx,
                                size_t idx_stride, int32_t *counts, float *sums, void *scratch,
                                const int32_t *ok = nullptr);
hipError_t launch_inliers_sums(hipStream_t st, uint32_t n, uint32_t W, const uint32_t *slots, const int32_t *counts,
                               float *sums, void *scratch);
// one model's list, count and sum in one workgroup (kernels_nonmin.hip k_inliers_small): H, F, E
// on n <= kPolPtsMax points; launch_inliers_batch takes it for W = 1 with sums
hipError_t launch_inliers_small(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *model,
                                float thr, const int32_t *ok, int32_t *idx, int32_t *count, float *sum);
size_t inliers_scratch_bytes(uint32_t n, uint32_t W);
// the polish result block, int32 / float words: pass k's model[9], ok, count, sum at
// kPolPass * k (pass 0's slots 12-13: the initial getInliers' count, sum), the fitted point
// counts of passes 1..3 at kPolNs + k, the device's (best, prev) at kPolState
constexpr int kPolPass = 16, kPolNs = 64, kPolState = 68, kPolStop = 70, kPolWords = 72;
hipError_t launch_polish_prep(hipStream_t st, int32_t *res, int k, int32_t best0);
// The whole polish in one workgroup (kernels_nonmin.hip k_polish_fused): the initial
// getInliers(model0) into lists[0] and slots 12-13, then passes 0..3 exactly as the multi-launch
// passes + k_polish_prep write them (fit lists[k], score into lists[k + 1]), while a pass's
// point count is <= fit_max (<= kPolFitMax); res[kPolStop] = the passes it ran (4: all; the host runs the
// rest the multi-launch way).  H, F, E on <= kPolPtsMax points; else hipErrorInvalidValue.
constexpr uint32_t kPolFitMax = 4096, kPolPtsMax = 16384;
constexpr uint32_t kSmallFitMax = 256;  // kernels_nonmin.hip kSmallFit: fits of at most this many points take k_fit_small
struct PolLists {
    int32_t *l[5];
};
// One polish pass's tail in one workgroup (kernels_nonmin.hip k_finish_score): the fit's finish
// (as k_dlt_finish, from b's partials / q / ws, after launch_nonminimal_batch with skip_finish),
// the fitted model's getInliers over N <= kPolPtsMax points (as k_inliers_small, gated on the
// fit's ok) into idx / count / sum, and, when prep_k >= 0, k_polish_prep(res, prep_k, best0).
// Fundamental / essential / homography fits of more than kSmallFit points (W = 1).
struct NmBatch;
hipError_t launch_finish_score(hipStream_t st, int estimator, const NmBatch &b, const void *pts, uint32_t N,
                               float thr, int32_t *idx, int32_t *count, float *sum, int32_t *res, int prep_k,
                               int32_t best0);
hipError_t launch_polish_fused(hipStream_t st, int estimator, const void *pts, uint32_t N, const float *model0,
                               float thr, int32_t best0, PolLists lists, int32_t *res,
                               uint32_t fit_max = kPolFitMax, uint64_t *dbg = nullptr);
// every point's exact residual under one model (n floats)
hipError_t launch_point_errors(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *model,
                               float *errors);

// the reference's sequential fp32 sums, in parallel and bit-exact (kernels_seqsum.hip): for
// rows b < W (fit w = slots ? slots[b] : b), chains q < nch over the elements k < n_w
// (ns ? ns[w] : n1) at vals[w * vstride + k * nch + q]; out[w * nch + q] = the left-to-right
// sum from +0 -- op(s, x) = s + x (float vals) or (float)((double)s + y) (f64: double vals).
// (nch, f64) in {(1, false), (4, false), (2, true)}.  scratch: fit w at scratch + w * sstride
// (>= seqsum_scratch_bytes(nch), 8-byte aligned); have_psum: its fp64 segment sums are already
// there (a producer kernel wrote them, layout in kernels_seqsum.hip).
size_t seqsum_scratch_bytes(int nch);
hipError_t launch_seqsum(hipStream_t st, int nch, bool f64, const void *vals, size_t vstride, const uint32_t *ns,
                         uint32_t n1, uint32_t W, const uint32_t *slots, void *scratch, size_t sstride,
                         bool have_psum, float *out);

// W independent non-minimal fits (kernels_nonmin.hip).  Fit w: index list base + w *
// base_stride, read through pos + w * pos_stride when pos != nullptr; ns[w] points (device;
// ns == nullptr: every fit has n1 points);
// q: W x q_stride points (float4, float2 for line); partial: W x p_stride doubles
// (p_stride >= nonminimal_partial_stride(ns[w])); ws: W x 18; model_out: W x 9; ok: W.
struct NmBatch {
    const int32_t *base;
    size_t base_stride;
    const int32_t *pos;
    size_t pos_stride;
    const uint32_t *ns;
    uint32_t n1, W, nmax;
    void *q;
    size_t q_stride;
    double *partial;
    size_t p_stride;
    float *ws, *model_out;
    int32_t *ok;
    void *seq;  // normalisation scratch, nonminimal_seq_bytes(nmax, W) (not used by line fits)
    // weighted normalisation (homography / fundamental only; nullable): weights[point index],
    // qw = W x q_stride float4 scratch for the weighted points
    const float *weights;
    void *qw;
    // nmax is only a bound on ns (e.g. counts known on the device alone): take the fused
    // gather + segment-sum path whatever its size (the results do not depend on the path)
    bool fused_any;
    // LO pipelined stages (usac_api.cpp LoRansac; nullable, implies fused_any): the fits' point
    // counts and the stage's thresholds from the previous stage's outputs, computed by the
    // gather itself (see LoPrep) and written to ns (then read by every later kernel) / thr
    const struct LoPrep *prep;
    // the multi-launch path stops after the A^T A partials: launch_finish_score takes the finish
    bool skip_finish;
};
// ns[w] = cnt[w] while chain w may continue -- it was fitted (ns_prev > 0), its fit
// succeeded, it kept more than m inliers and (compare: after an iterative step) not fewer
// than the best's count -- else 0 (the chain's fit and scoring become no-ops that leave its
// list alone); thr[w] = thr_prev[w] - step
struct LoPrep {
    const uint32_t *ns_prev;
    const int32_t *ok_prev, *cnt_prev;
    const float *thr_prev;
    uint32_t *ns;
    float *thr;
    int32_t m, best_cnt, compare;
    float step;
    const int32_t *best_dev;  // nullable: the best count read from device memory instead of best_cnt
                              // (a captured stage graph keeps its arguments across rounds)
};
hipError_t launch_nonminimal_batch(hipStream_t st, int estimator, const void *pts, const NmBatch &b);
size_t nonminimal_partial_stride(uint32_t nmax);
size_t nonminimal_seq_bytes(uint32_t nmax, uint32_t W);

// k nearest neighbours of every point (kernels_knn.hip, nearest_neighbors.cpp:69-128):
// idx / d2 (nullable) n x k, self excluded, ascending distance, ties by index; 1 <= k <= 32
constexpr uint32_t kKnnMax = 32;
hipError_t launch_knn(hipStream_t st, const float *pts, uint32_t n, uint32_t cols, uint32_t k, int32_t *idx,
                      float *d2);

}  // namespace usac
