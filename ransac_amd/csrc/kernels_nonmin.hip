// kernels_nonmin.hip -- non-minimal (least-squares) model fits on the device, used by the
// post-loop polish (ransac.cpp:157-207):
//   homography: DLt::NormalizedDLT (normalized_dlt.cpp:7-23) with
//               GetNormalizingTransformation (normalizing_transformation.cpp:7-113);
//   line2d    : Line2DEstimator::EstimateModelNonMinimalSample PCA (line2d_estimator.hpp:59-107).
// The reference's fp32 moment sums are sequential in sample order and stay sequential
// here (one lane per accumulator).  The DLT normal matrix A^T A (fp64) has no reference
// order (OpenCV's SVD hides it); its order is fixed by this build's spec: 16-point
// blocks summed in order, 64 block partials per superblock in block order, superblocks in
// order -- shared with the oracle.
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_device_e5.hpp"
#include "usac_kernels.h"
#include "usac_seqsum.hpp"

namespace usac {

constexpr uint32_t kAtaBlock = 16;  // A^T A spec block (oracle ORC_ATA_BLOCK); 64 blocks per superblock

// round-robin Jacobi schedule: 9 rounds of 4 disjoint planes (oracle kJacobiRounds)
__constant__ signed char kJacobiRounds[9][4][2] = {
    {{1, 8}, {2, 7}, {3, 6}, {4, 5}}, {{0, 8}, {1, 6}, {2, 5}, {3, 4}}, {{0, 7}, {1, 4}, {2, 3}, {6, 8}},
    {{0, 6}, {1, 2}, {4, 8}, {5, 7}}, {{0, 5}, {2, 8}, {3, 7}, {4, 6}}, {{0, 4}, {1, 7}, {2, 6}, {3, 5}},
    {{0, 3}, {1, 5}, {2, 4}, {7, 8}}, {{0, 2}, {1, 3}, {5, 8}, {6, 7}}, {{0, 1}, {3, 8}, {4, 7}, {5, 6}}};

// Every kernel below is batched over W independent fits (blockIdx.y, or blockIdx.x for the
// one-workgroup stages): fit w uses the index list base + w * base_stride (through the
// positions pos + w * pos_stride when pos is given: idx_i = list[pos_i]), ns[w] points, and
// its own slices of q / partial / ws / model_out / ok.  A fit never reads another fit's
// data, so each result is exactly the single-fit one.

// gather q[i] = pts[idx[i]] so the sequential passes read contiguous memory
template <class P>
__global__ __launch_bounds__(256) void k_gather(const P *__restrict__ pts, const int32_t *__restrict__ base,
                                                size_t base_stride, const int32_t *__restrict__ pos,
                                                size_t pos_stride, const uint32_t *__restrict__ ns, uint32_t n1,
                                                P *__restrict__ q, size_t q_stride) {
    const uint32_t w = blockIdx.y;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= (ns ? ns[w] : n1)) return;
    const int32_t *list = base + w * base_stride;
    const int32_t j = pos ? pos[w * pos_stride + i] : (int32_t)i;
    q[w * q_stride + i] = pts[list[j]];
}

// the gather fused with the coordinate chains' fp64 segment sums (seqsum psum layout, 4 chains):
// workgroup (segment j, fit w) gathers its segment, four points per thread in flight
__global__ __launch_bounds__(256) void k_gather_psum4(const float4 *__restrict__ pts, const int32_t *__restrict__ base,
                                                      size_t base_stride, const int32_t *__restrict__ pos,
                                                      size_t pos_stride, const uint32_t *__restrict__ ns, uint32_t n1,
                                                      float4 *__restrict__ q_all, size_t q_stride, char *seq_all,
                                                      size_t sstride, LoPrep prep, int has_prep) {
    __shared__ double red[4][256];
    const uint32_t j = blockIdx.x, w = blockIdx.y;
    uint32_t n;
    if (has_prep) {  // every segment of fit w derives the same n; segment 0 publishes it
        const int32_t c = prep.cnt_prev[w];
        const int32_t best = prep.best_dev ? *prep.best_dev : prep.best_cnt;
        const bool go = prep.ns_prev[w] > 0 && prep.ok_prev[w] && c > prep.m && (!prep.compare || c >= best);
        n = go ? (uint32_t)c : 0u;
        if (j == 0 && threadIdx.x == 0) {
            prep.ns[w] = n;
            prep.thr[w] = prep.thr_prev[w] - prep.step;  // the host's `thr -= step` (fp32)
        }
    } else {
        n = ns ? ns[w] : n1;
    }
    const uint32_t L = seq::seg_len(n);
    if (j * L >= n) return;
    const uint32_t e = (j + 1) * L < n ? (j + 1) * L : n;
    const int32_t *list = base + w * base_stride;
    float4 *q = q_all + w * q_stride;
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    for (uint32_t i0 = j * L + threadIdx.x; i0 < e; i0 += 4 * 256) {
        float4 p[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + 256 * u;
            if (i < e) p[u] = pts[list[pos ? pos[w * pos_stride + i] : (int32_t)i]];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + 256 * u;
            if (i < e) {
                q[i] = p[u];
                a[0] += (double)p[u].x;
                a[1] += (double)p[u].y;
                a[2] += (double)p[u].z;
                a[3] += (double)p[u].w;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) red[k][threadIdx.x] = a[k];
    __syncthreads();
    for (uint32_t h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h)
#pragma unroll
            for (int k = 0; k < 4; k++) red[k][threadIdx.x] += red[k][threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x < 4) reinterpret_cast<double *>(seq_all + w * sstride)[j * 4 + threadIdx.x] = red[threadIdx.x][0];
}
constexpr uint32_t kFusedGatherMax = 64 * 1024;  // up to 8 points per thread and segment

// the pipelined LO stages' count / threshold derivation (LoPrep) on its own, for the fit paths
// without the fused gather
__global__ __launch_bounds__(64) void k_lo_prep(LoPrep p, uint32_t W) {
    for (uint32_t w = threadIdx.x; w < W; w += 64) {
        const int32_t c = p.cnt_prev[w];
        const int32_t best = p.best_dev ? *p.best_dev : p.best_cnt;
        const bool go = p.ns_prev[w] > 0 && p.ok_prev[w] && c > p.m && (!p.compare || c >= best);
        p.ns[w] = go ? (uint32_t)c : 0u;
        p.thr[w] = p.thr_prev[w] - p.step;
    }
}

// normalizing transformation (GetNormalizingTransformation, normalizing_transformation.cpp:
// 7-113): the four coordinate means and the two average distances are the reference's
// sequential fp32 sums in point order, evaluated bit-exactly in parallel by launch_seqsum
// (kernels_seqsum.hip); the kernels here produce the distance terms and apply the transforms.
// Per-fit seq scratch (nonminimal_seq_stride): [0, kSeqA) the seqsum scratch of the 4 mean
// chains (reused by the 2 distance chains), then the distance terms, double2 per point; after
// the W slices, sums4[W][4] (coordinate sums) and dsum2[W][2] (distance sums).
constexpr size_t kSeqA = seq::scratch_bytes(4);

__host__ __device__ __forceinline__ size_t seq_stride(uint32_t nmax) {
    return (kSeqA + 16 * (size_t)nmax + 255) & ~(size_t)255;
}

// distance terms sqrt((double)(xm * xm + ym * ym)) of both images (the reference's unqualified
// sqrt of a float is C's double sqrt) and their fp64 segment sums (seqsum psum layout, 2 chains)
__global__ __launch_bounds__(256) void k_norm_dist(const float4 *__restrict__ q_all, size_t q_stride,
                                                   const uint32_t *__restrict__ ns, uint32_t n1, char *seq_all,
                                                   size_t sstride, const float *__restrict__ sums4) {
    __shared__ double red[2][256];
    const uint32_t j = blockIdx.x, w = blockIdx.y;
    const uint32_t n = ns ? ns[w] : n1, L = seq::seg_len(n);
    if (j * L >= n) return;
    const uint32_t e = (j + 1) * L < n ? (j + 1) * L : n;
    const float4 *q = q_all + w * q_stride;
    char *seq = seq_all + w * sstride;
    double2 *sq = reinterpret_cast<double2 *>(seq + kSeqA);
    const float mx1 = sums4[4 * w + 0] / (float)n, my1 = sums4[4 * w + 1] / (float)n;
    const float mx2 = sums4[4 * w + 2] / (float)n, my2 = sums4[4 * w + 3] / (float)n;
    double a0 = 0.0, a1 = 0.0;
    for (uint32_t i0 = j * L + threadIdx.x; i0 < e; i0 += 4 * 256) {  // four points' loads in flight
        float4 pv[4];
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (i0 + 256 * u < e) pv[u] = q[i0 + 256 * u];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t i = i0 + 256 * u;
            if (i >= e) break;
            const float4 p = pv[u];
            const float xm1 = p.x - mx1, ym1 = p.y - my1;
            const float xm2 = p.z - mx2, ym2 = p.w - my2;
            const double d1 = sqrt((double)(xm1 * xm1 + ym1 * ym1)), d2 = sqrt((double)(xm2 * xm2 + ym2 * ym2));
            sq[i] = make_double2(d1, d2);
            a0 += d1;
            a1 += d2;
        }
    }
    red[0][threadIdx.x] = a0;
    red[1][threadIdx.x] = a1;
    __syncthreads();
    for (uint32_t h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) {
            red[0][threadIdx.x] += red[0][threadIdx.x + h];
            red[1][threadIdx.x] += red[1][threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x < 2) reinterpret_cast<double *>(seq)[j * 2 + threadIdx.x] = red[threadIdx.x][0];
}

// the weighted overload's inputs (normalizing_transformation.cpp:117-146): q[i] = the point,
// qw[i] = its weighted coordinates w*x (the mean chains' addends) and the distance terms
// sqrt((double)(x*x + y*y)) of the weighted points from the origin (not from the mean)
__global__ __launch_bounds__(256) void k_gather_weighted(const float4 *__restrict__ pts, const float *__restrict__ wts,
                                                         const int32_t *__restrict__ base, size_t base_stride,
                                                         const int32_t *__restrict__ pos, size_t pos_stride,
                                                         const uint32_t *__restrict__ ns, uint32_t n1,
                                                         float4 *__restrict__ q_all, float4 *__restrict__ qw_all,
                                                         size_t q_stride, char *seq_all, size_t sstride) {
    const uint32_t w = blockIdx.y;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= (ns ? ns[w] : n1)) return;
    const int32_t *list = base + w * base_stride;
    const int32_t k = list[pos ? pos[w * pos_stride + i] : (int32_t)i];
    const float4 p = pts[k];
    const float g = wts[k];
    const float x1 = g * p.x, y1 = g * p.y, x2 = g * p.z, y2 = g * p.w;
    q_all[w * q_stride + i] = p;
    qw_all[w * q_stride + i] = make_float4(x1, y1, x2, y2);
    reinterpret_cast<double2 *>(seq_all + w * sstride + kSeqA)[i] =
        make_double2(sqrt((double)(x1 * x1 + y1 * y1)), sqrt((double)(x2 * x2 + y2 * y2)));
}

// T1, T2 from the sums (the reference's expressions; ws layout (floats): [0..8] T1, [9..17]
// T2).  The normalised points are never stored: the A^T A pass (and the thin solve) apply
// x' = T[0] x + T[2], y' = T[4] y + T[5] on the fly -- the same float operations.
__device__ __forceinline__ void norm_transforms(const float *__restrict__ sums4, const float *__restrict__ dsum2,
                                                uint32_t w, uint32_t n, float *t1, float *t2) {
    float mean[4];
#pragma unroll
    for (int k = 0; k < 4; k++) mean[k] = sums4[4 * w + k] / (float)n;
    const float s1 = (float)(M_SQRT2 / (double)(dsum2[2 * w + 0] / (float)n));
    const float s2 = (float)(M_SQRT2 / (double)(dsum2[2 * w + 1] / (float)n));
    const float a[9] = {s1, 0.f, -mean[0] * s1, 0.f, s1, -mean[1] * s1, 0.f, 0.f, 1.f};
    const float c[9] = {s2, 0.f, -mean[2] * s2, 0.f, s2, -mean[3] * s2, 0.f, 0.f, 1.f};
#pragma unroll
    for (int k = 0; k < 9; k++) {
        t1[k] = a[k];
        t2[k] = c[k];
    }
}

struct NormXf {
    float ax, bx, ay, by, az, bz, aw, bw;
    __device__ __forceinline__ float4 operator()(const float4 p) const {
        float4 o;
        o.x = ax * p.x + bx;
        o.y = ay * p.y + by;
        o.z = az * p.z + bz;
        o.w = aw * p.w + bw;
        return o;
    }
};
__device__ __forceinline__ NormXf norm_xf(const float *t1, const float *t2) {
    return NormXf{t1[0], t1[2], t1[4], t1[5], t2[0], t2[2], t2[4], t2[5]};
}

// partials of A^T A: one lane per (16-point block, group of 9 of the 45 upper-triangle
// entries, row-major j <= k) -- five lanes per block, the group wave-uniform (blockIdx.y) and
// a compile-time constant in the body; each entry accumulated in registers over the block's
// points in order; then the workgroup's 64 blocks (a 1024-point superblock) summed in block
// order by one lane per entry, one partial per superblock (the spec's units and order; the
// grouping only spreads the entries over lanes).  FUND: one 8-point row per correspondence
// (eight_points.cpp:26-45), else two DLT rows.
constexpr int kAtaGroups = 5;                  // 45 = 5 x 9 entries
constexpr uint32_t kAtaGridBound = 32;         // superblock workgroups per fit at most, for a bound nmax
constexpr int kAtaPer = 45 / kAtaGroups;

template <bool FUND, int G>
__device__ __forceinline__ void ata_group(const float4 *q, const NormXf xf, uint32_t b0, uint32_t b1, double *acc_out) {
    double acc[kAtaPer];
#pragma unroll
    for (int e = 0; e < kAtaPer; e++) acc[e] = 0.0;
    // the block's points in batches of 8, the next batch's loads in flight while the current
    // one is accumulated (one point at a time would wait a memory latency per point)
    constexpr uint32_t kB = 8;
    float4 cur[kB], nxt[kB];
    auto load = [&](float4 (&x)[kB], uint32_t i0) {
#pragma unroll
        for (uint32_t u = 0; u < kB; u++) x[u] = i0 + u < b1 ? q[i0 + u] : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    load(cur, b0);
    for (uint32_t i0 = b0; i0 < b1; i0 += kB) {
        if (i0 + kB < b1) load(nxt, i0 + kB);
#pragma unroll
        for (uint32_t u = 0; u < kB; u++) {
            if (i0 + u >= b1) break;
            const float4 p = xf(cur[u]);
            double r0[9], r1[9];
            if (FUND) fund_row(p.x, p.y, p.z, p.w, r0);
            else dlt_rows(p.x, p.y, p.z, p.w, r0, r1);
            int e = 0;
#pragma unroll
            for (int j = 0; j < 9; j++)
#pragma unroll
                for (int k = j; k < 9; k++, e++) {
                    if (e < kAtaPer * G || e >= kAtaPer * (G + 1)) continue;
                    if (FUND) acc[e - kAtaPer * G] += r0[j] * r0[k];
                    else acc[e - kAtaPer * G] += r0[j] * r0[k] + r1[j] * r1[k];
                }
        }
#pragma unroll
        for (uint32_t u = 0; u < kB; u++) cur[u] = nxt[u];
    }
#pragma unroll
    for (int e = 0; e < kAtaPer; e++) acc_out[e] = acc[e];
}

// group g (wave-uniform) to its compile-time instance
template <bool FUND, int G = 0>
__device__ __forceinline__ void ata_dispatch(int g, const float4 *q, const NormXf xf, uint32_t b0, uint32_t b1,
                                             double *acc) {
    if constexpr (G + 1 < kAtaGroups) {
        if (g != G) return ata_dispatch<FUND, G + 1>(g, q, xf, b0, b1, acc);
    }
    ata_group<FUND, G>(q, xf, b0, b1, acc);
}

template <bool FUND>
__global__ __launch_bounds__(64) void k_ata_partial(const float4 *__restrict__ q_all, size_t q_stride,
                                                    const uint32_t *__restrict__ ns, uint32_t n1,
                                                    double *__restrict__ partial_all, size_t p_stride,
                                                    const float *__restrict__ sums4, const float *__restrict__ dsum2,
                                                    float *__restrict__ ws_all) {
    const uint32_t w = blockIdx.z;
    const uint32_t n = ns ? ns[w] : n1;
    // workgroup-uniform: no superblock of this workgroup within the fit's points (the grid is
    // sized for a bound on n; workgroup x takes superblocks x, x + gridDim.x, ...), or a
    // system the finish solves from the points themselves; workgroup (0, 0) still writes the
    // fit's transforms
    const bool idle = (FUND ? n <= 8 : 2 * n <= 9) || blockIdx.x * 64 * kAtaBlock >= n;
    const bool writer = blockIdx.x == 0 && blockIdx.y == 0;
    if (idle && !writer) return;
    float t1[9], t2[9];
    norm_transforms(sums4, dsum2, w, n, t1, t2);
    if (writer && threadIdx.x < 9) {
        ws_all[18 * w + threadIdx.x] = t1[threadIdx.x];
        ws_all[18 * w + 9 + threadIdx.x] = t2[threadIdx.x];
    }
    if (idle) return;
    __shared__ double red[64][kAtaPer + 1];
    const NormXf xf = norm_xf(t1, t2);
    const float4 *q = q_all + w * q_stride;
    const uint32_t nblocks = (n + kAtaBlock - 1) / kAtaBlock;
    for (uint32_t sb = blockIdx.x; sb * 64 * kAtaBlock < n; sb += gridDim.x) {
        const uint32_t blk = sb * 64 + threadIdx.x;
        double acc[kAtaPer];
        if (blk * kAtaBlock < n) {
            const uint32_t b0 = blk * kAtaBlock;
            const uint32_t b1 = b0 + kAtaBlock < n ? b0 + kAtaBlock : n;
            ata_dispatch<FUND>((int)blockIdx.y, q, xf, b0, b1, acc);
#pragma unroll
            for (int e = 0; e < kAtaPer; e++) red[threadIdx.x][e] = acc[e];
        }
        __syncthreads();
        if (threadIdx.x < kAtaPer) {  // superblock sum, blocks in order
            const uint32_t first = sb * 64;
            const uint32_t nb = nblocks - first < 64 ? nblocks - first : 64;
            double sum = 0.0;
            for (uint32_t b = 0; b < nb; b++) sum += red[b][threadIdx.x];
            partial_all[w * p_stride + (size_t)sb * 45 + kAtaPer * blockIdx.y + threadIdx.x] = sum;
        }
        __syncthreads();  // red is reused by the next superblock
    }
}

// Final solve, one wave: A^T A from the partials (lane e), round-robin Jacobi eigen over
// 36 lanes (LDS), smallest-eigenvalue vector; or the thin row-Jacobi when the system has
// <= 8 rows (homography 2n <= 8, fundamental n <= 8: SURVEY Q1/Q2); then
//   homography : H = T2^-1 * Hn * T1 (fp64), H /= H33 (normalized_dlt.cpp:18-22);
//   fundamental: F = T2^T * Fn * T1 (fp64), F /= F33 when |F33| > FLT_EPSILON
//                (eight_points.cpp:76-99);
// cast to float.
template <int R, bool FUND>
__device__ void thin_solve(const float4 *q, const NormXf xf, double *v) {
    double W[R][9];
    if (FUND) {
#pragma unroll
        for (int i = 0; i < R; i++) {
            const float4 p = xf(q[i]);
            fund_row(p.x, p.y, p.z, p.w, W[i]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < R / 2; i++) {
            const float4 p = xf(q[i]);
            dlt_rows(p.x, p.y, p.z, p.w, W[2 * i], W[2 * i + 1]);
        }
    }
    row_jacobi<R>(W);
    pick_vector<R>(W, 0, v);
}

// Smallest-eigenvalue eigenvector of the symmetric 9x9 A (LDS, both triangles): inverse
// iteration on A + 1e-12 tr(A) I through its Cholesky factor, in one lane with the factor in
// registers -- the oracle's eig_min_invit spec operation for operation (usac_oracle.c).
// Returns false when the spec falls back to the Jacobi (not positive definite, non-finite, or
// the two smallest eigenvalues too close for fast convergence).
__device__ bool eig_min_invit(const double (*A)[9], double *v) {
    double tr = 0.0;
#pragma unroll
    for (int k = 0; k < 9; k++) tr += A[k][k];
    if (!(tr > 0.0) || !isfinite(tr)) return false;
    const double mu = tr * 1e-12;
    double L[9][9], inv[9];
#pragma unroll
    for (int j = 0; j < 9; j++) {
        double d = A[j][j] + mu;
#pragma unroll
        for (int k = 0; k < j; k++) d -= L[j][k] * L[j][k];
        if (!(d > 0.0)) return false;
        L[j][j] = sqrt(d);
        inv[j] = 1.0 / L[j][j];
#pragma unroll
        for (int i = j + 1; i < 9; i++) {
            double s = A[i][j];
#pragma unroll
            for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k];
            L[i][j] = s * inv[j];
        }
    }
    double x[9], dprev = 0.0;
#pragma unroll
    for (int k = 0; k < 9; k++) x[k] = 1.0 / 3.0;
    for (int it = 0; it < 30; it++) {
        double y[9], z[9];
#pragma unroll
        for (int i = 0; i < 9; i++) {
            double s = x[i];
#pragma unroll
            for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
            y[i] = s * inv[i];
        }
#pragma unroll
        for (int i = 8; i >= 0; i--) {
            double s = y[i];
#pragma unroll
            for (int k = i + 1; k < 9; k++) s -= L[k][i] * z[k];
            z[i] = s * inv[i];
        }
        double nn = 0.0;
#pragma unroll
        for (int k = 0; k < 9; k++) nn += z[k] * z[k];
        if (!(nn > 0.0) || !isfinite(nn)) return false;
        const double r = 1.0 / sqrt(nn);
        double d = 0.0;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            const double xn = z[k] * r;
            const double e = fabs(xn - x[k]);
            if (e > d) d = e;
            x[k] = xn;
        }
        if (d <= 1e-13) {
#pragma unroll
            for (int k = 0; k < 9; k++) v[k] = x[k];
            return true;
        }
        if (it >= 2 && d > 0.25 * dprev) return false;
        dprev = d;
    }
    return false;
}

// The end of a fit, one wave: the thin row-Jacobi when the system has <= 8 rows (homography
// 2n <= 8, fundamental n <= 8: SURVEY Q1/Q2), else the smallest eigenvector of the normal
// matrix A (LDS, both triangles, filled by the caller before the call) by the spec's inverse
// iteration (lane 0) with the round-robin Jacobi as its fall-back; then the transform back and
// the cast.  q: the fit's points (global or LDS), ws: T1, T2.
template <bool FUND>
__device__ __forceinline__ void fit_finish(const float4 *q, uint32_t n, const float *ws, double (*A)[9], double (*V)[9],
                           double *s_v, float *model_out, int32_t *ok) {
    const uint32_t t = threadIdx.x;
    if (n == 0) {  // EstimateModelNonMinimalSample of no points fails
        if (t == 0) *ok = 0;
        return;
    }
    if (FUND ? n <= 8 : 2 * n <= 9) {
        if (t == 0) {
            const NormXf xf = norm_xf(ws, ws + 9);
            double v[9];
            if (FUND) {
                switch (n) {
                    case 1: thin_solve<1, true>(q, xf, v); break;
                    case 2: thin_solve<2, true>(q, xf, v); break;
                    case 3: thin_solve<3, true>(q, xf, v); break;
                    case 4: thin_solve<4, true>(q, xf, v); break;
                    case 5: thin_solve<5, true>(q, xf, v); break;
                    case 6: thin_solve<6, true>(q, xf, v); break;
                    case 7: thin_solve<7, true>(q, xf, v); break;
                    default: thin_solve<8, true>(q, xf, v); break;
                }
            } else {
                if (n == 1) thin_solve<2, false>(q, xf, v);
                else if (n == 2) thin_solve<4, false>(q, xf, v);
                else if (n == 3) thin_solve<6, false>(q, xf, v);
                else thin_solve<8, false>(q, xf, v);
            }
            for (int k = 0; k < 9; k++) s_v[k] = v[k];
        }
        __syncthreads();
    } else {
        if (t < 9)
            for (int j = 0; j < 9; j++) V[j][t] = (j == (int)t) ? 1.0 : 0.0;
        __syncthreads();
        // the spec's inverse iteration (lane 0); the Jacobi below only when it falls back
        __shared__ int s_done;
        if (t == 0) {
            double v[9];
            s_done = eig_min_invit(A, v) ? 1 : 0;
            if (s_done)
                for (int k = 0; k < 9; k++) s_v[k] = v[k];
        }
        __syncthreads();
        if (!s_done) {
        // round-robin Jacobi (the oracle's sym_eig_min_jacobi spec): per round the rotations of 4
        // disjoint planes from the matrix at the round's start, then all column updates (lane =
        // (row, plane), V alongside), then all row updates (lane = (plane, column)) -- every
        // lane owns disjoint element pairs, 3 barriers per round
        __shared__ signed char s_rounds[9][4][2];  // the schedule in LDS (not a global load per use)
        for (uint32_t i = t; i < 72; i += 64) (&s_rounds[0][0][0])[i] = (&kJacobiRounds[0][0][0])[i];
        __syncthreads();
        // lanes (plane k, row / column e), 36 of them; each lane's plane of every round in
        // registers (the round loop unrolls), so a round starts with one LDS read, not two
        const int k = (int)t / 9, e = (int)t - 9 * k;
        int rp[9], rq[9];
#pragma unroll
        for (int r = 0; r < 9; r++) {
            rp[r] = t < 36 ? s_rounds[r][k][0] : 0;
            rq[r] = t < 36 ? s_rounds[r][k][1] : 0;
        }
        for (int sweep = 0; sweep < 50; sweep++) {
            double off = 0.0, diag = 0.0;
            for (int p = 0; p < 9; p++) {
                diag += A[p][p] * A[p][p];
                for (int qq = p + 1; qq < 9; qq++) off += A[p][qq] * A[p][qq];
            }
            if (off <= 1e-30 * diag || off == 0.0) break;
#pragma unroll
            for (int r = 0; r < 9; r++) {
                // each lane computes its plane's rotation itself (the same expressions, so the
                // same bits in the 9 lanes of a plane: no LDS exchange of (c, s)); the column
                // update's operands are the round-start values, so they are read here too and
                // their LDS latency overlaps the rotation's fp64 chain
                const int p = rp[r], qq = rq[r];
                bool act = false;
                double c = 0.0, sn = 0.0, aip = 0.0, aiq = 0.0, vip = 0.0, viq = 0.0;
                if (t < 36) {
                    const double apq = A[p][qq];
                    aip = A[e][p];
                    aiq = A[e][qq];
                    vip = V[e][p];
                    viq = V[e][qq];
                    act = apq != 0.0;
                    if (act) {
                        const double theta = (A[qq][qq] - A[p][p]) / (2.0 * apq);
                        const double tt = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                        c = 1.0 / sqrt(tt * tt + 1.0);
                        sn = tt * c;
                    }
                }
                __syncthreads();  // every lane read its entries before any update
                if (act) {  // columns p, q of row e; V likewise
                    A[e][p] = c * aip - sn * aiq;
                    A[e][qq] = sn * aip + c * aiq;
                    V[e][p] = c * vip - sn * viq;
                    V[e][qq] = sn * vip + c * viq;
                }
                __syncthreads();
                if (act) {  // rows p, q at column e
                    const double apj = A[p][e], aqj = A[qq][e];
                    A[p][e] = c * apj - sn * aqj;
                    A[qq][e] = sn * apj + c * aqj;
                }
                __syncthreads();
            }
        }
        if (t == 0) {
            int m = 0;
            for (int i = 1; i < 9; i++)
                if (A[i][i] < A[m][m]) m = i;
            for (int k = 0; k < 9; k++) s_v[k] = V[k][m];
        }
        __syncthreads();
        }  // fall-back Jacobi
    }
    if (t == 0 && FUND) {
        double T1[9], tmp[9], Fd[9];
        for (int k = 0; k < 9; k++) T1[k] = (double)ws[k];
        const double T2t[9] = {(double)ws[9], 0.0, 0.0, 0.0, (double)ws[13], 0.0, (double)ws[11], (double)ws[14], 1.0};
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                double s = 0.0;
                for (int k = 0; k < 3; k++) s += s_v[3 * r + k] * T1[3 * k + c];
                tmp[3 * r + c] = s;
            }
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                double s = 0.0;
                for (int k = 0; k < 3; k++) s += T2t[3 * r + k] * tmp[3 * k + c];
                Fd[3 * r + c] = s;
            }
        if (fabs(Fd[8]) > (double)1.1920928955078125e-07f) {
            for (int k = 0; k < 9; k++) model_out[k] = (float)(Fd[k] / Fd[8]);
        } else {
            for (int k = 0; k < 9; k++) model_out[k] = (float)Fd[k];
        }
        *ok = 1;
    } else if (t == 0) {
        float T1[9], T2[9], T2i[9];
        for (int k = 0; k < 9; k++) {
            T1[k] = ws[k];
            T2[k] = ws[9 + k];
        }
        inv3x3(T2, T2i);
        double tmp[9], Hd[9];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                double s = 0.0;
                for (int k = 0; k < 3; k++) s += s_v[3 * r + k] * (double)T1[3 * k + c];
                tmp[3 * r + c] = s;
            }
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                double s = 0.0;
                for (int k = 0; k < 3; k++) s += (double)T2i[3 * r + k] * tmp[3 * k + c];
                Hd[3 * r + c] = s;
            }
        for (int k = 0; k < 9; k++) model_out[k] = (float)(Hd[k] / Hd[8]);
        *ok = 1;
    }
}


// the entry (j, k), j <= k, of lane t < 45 of the upper triangle, row-major
__device__ __forceinline__ void ata_entry(uint32_t t, int &j, int &k) {
    int rem = (int)t;
    j = 0;
    k = (int)t;
    for (int r = 0; r < 9; r++) {
        if (rem < 9 - r) {
            j = r;
            k = r + rem;
            return;
        }
        rem -= 9 - r;
    }
}

template <bool FUND>
__global__ __launch_bounds__(64) void k_dlt_finish(const float4 *__restrict__ q_all, size_t q_stride,
                                                   const uint32_t *__restrict__ ns, uint32_t n1,
                                                   const double *__restrict__ partial_all, size_t p_stride,
                                                   const float *ws_all, float *model_all, int32_t *ok_all) {
    __shared__ double A[9][9];
    __shared__ double V[9][9];
    __shared__ double s_v[9];
    const uint32_t t = threadIdx.x;
    const uint32_t w = blockIdx.x;
    const uint32_t n = ns ? ns[w] : n1;
    const double *partial = partial_all + w * p_stride;
    const uint32_t nblocks = (n + kAtaBlock * 64 - 1) / (kAtaBlock * 64);  // superblock partials
    if (n > 0 && !(FUND ? n <= 8 : 2 * n <= 9) && t < 45) {
        int j, k;
        ata_entry(t, j, k);
        // the superblock partials in order (spec), sixteen loads in flight per sixteen adds
        double acc = 0.0;
        uint32_t c = 0;
        for (; c + 16 <= nblocks; c += 16) {
            double x[16];
#pragma unroll
            for (int u = 0; u < 16; u++) x[u] = partial[(size_t)(c + u) * 45 + t];
#pragma unroll
            for (int u = 0; u < 16; u++) acc += x[u];
        }
        for (; c < nblocks; c++) acc += partial[(size_t)c * 45 + t];
        A[j][k] = acc;
        A[k][j] = acc;
    }
    fit_finish<FUND>(q_all + w * q_stride, n, ws_all + 18 * w, A, V, s_v, model_all + 9 * w, ok_all + w);
}

// A whole fit of <= kSmallFit points in one workgroup (the LO inner fits of lo_sample_size
// points, small polish lists): the points gathered into LDS; the four coordinate sums and the
// two distance sums as the reference's sequential chains, one lane each (they are short);
// T1, T2; the normal matrix in the spec's order (16-point blocks in point order, blocks in
// order: one superblock), lane = entry; fit_finish.  Bit-identical to the multi-launch path.
constexpr uint32_t kSmallFit = kSmallFitMax;
static_assert(kSmallFit <= 64 * kAtaBlock, "k_fit_small sums one A^T A superblock");

template <bool FUND>
__global__ __launch_bounds__(64) void k_fit_small(const float4 *__restrict__ pts, const int32_t *__restrict__ base,
                                                  size_t base_stride, const int32_t *__restrict__ pos,
                                                  size_t pos_stride, const uint32_t *__restrict__ ns, uint32_t n1,
                                                  float *__restrict__ ws_all, float *__restrict__ model_all,
                                                  int32_t *__restrict__ ok_all) {
    __shared__ float4 q[kSmallFit];
    __shared__ double A[9][9];
    __shared__ double V[9][9];
    __shared__ double s_v[9];
    __shared__ float s_sums[6];
    __shared__ float s_ws[18];
    const uint32_t t = threadIdx.x;
    const uint32_t w = blockIdx.x;
    const uint32_t n = ns ? ns[w] : n1;
    if (n == 0) {  // EstimateModelNonMinimalSample of no points fails
        if (t == 0) ok_all[w] = 0;
        return;
    }
    const int32_t *list = base + w * base_stride;
    for (uint32_t i = t; i < n; i += 64) q[i] = pts[list[pos ? pos[w * pos_stride + i] : (int32_t)i]];
    __syncthreads();
    if (t < 4) {  // mean chains (normalizing_transformation.cpp:13-20)
        float s = 0.f;
        for (uint32_t i = 0; i < n; i++) s += (&q[i].x)[t];
        s_sums[t] = s;
    }
    __syncthreads();
    if (t < 2) {  // distance chains (:28-47): float += double sqrt of the float expression
        const float mx = s_sums[2 * t] / (float)n, my = s_sums[2 * t + 1] / (float)n;
        float d = 0.f;
        for (uint32_t i = 0; i < n; i++) {
            const float xm = (&q[i].x)[2 * t] - mx, ym = (&q[i].x)[2 * t + 1] - my;
            d = (float)((double)d + sqrt((double)(xm * xm + ym * ym)));
        }
        s_sums[4 + t] = d;
    }
    __syncthreads();
    float t1[9], t2[9];
    norm_transforms(s_sums, s_sums + 4, 0, n, t1, t2);
    if (t < 9) {
        s_ws[t] = t1[t];
        s_ws[9 + t] = t2[t];
        ws_all[18 * w + t] = t1[t];
        ws_all[18 * w + 9 + t] = t2[t];
    }
    if (!(FUND ? n <= 8 : 2 * n <= 9) && t < 45) {
        int j, k;
        ata_entry(t, j, k);
        const NormXf xf = norm_xf(t1, t2);
        double sb = 0.0;  // the superblock (n <= kSmallFit <= 64 kAtaBlock): blocks summed in order
        for (uint32_t b0 = 0; b0 < n; b0 += kAtaBlock) {
            const uint32_t b1 = b0 + kAtaBlock < n ? b0 + kAtaBlock : n;
            double acc = 0.0;
            for (uint32_t i = b0; i < b1; i++) {
                const float4 p = xf(q[i]);
                double r0[9], r1[9];
                if (FUND) {
                    fund_row(p.x, p.y, p.z, p.w, r0);
                    acc += r0[j] * r0[k];
                } else {
                    dlt_rows(p.x, p.y, p.z, p.w, r0, r1);
                    acc += r0[j] * r0[k] + r1[j] * r1[k];
                }
            }
            sb += acc;
        }
        const double a = 0.0 + sb;  // the finish's sum over the (one) superblock partial
        A[j][k] = a;
        A[k][j] = a;
    }
    __syncthreads();
    fit_finish<FUND>(q, n, s_ws, A, V, s_v, model_all + 9 * w, ok_all + w);
}

// Line PCA: one lane, sequential fp32 moments (sum_xy = 0 initialised),
// closed-form eigenvector of the smaller eigenvalue of the 2x2 covariance (fp64).
__global__ __launch_bounds__(64) void k_line_pca(const float2 *__restrict__ q_all, size_t q_stride,
                                                 const uint32_t *__restrict__ ns, uint32_t n1, float *model_all,
                                                 int32_t *ok_all) {
    if (threadIdx.x != 0) return;
    const float2 *q = q_all + blockIdx.x * q_stride;
    const uint32_t n = ns ? ns[blockIdx.x] : n1;
    float *model_out = model_all + 9 * blockIdx.x;
    int32_t *ok = ok_all + blockIdx.x;
    if (n == 0) {
        *ok = 0;
        return;
    }
    float sx = 0, sy = 0, sxy = 0, sx2 = 0, sy2 = 0;
    for (uint32_t i = 0; i < n; i++) {
        const float2 p = q[i];
        sx += p.x;
        sy += p.y;
        sxy += p.x * p.y;
        sx2 += p.x * p.x;
        sy2 += p.y * p.y;
    }
    const float fn = (float)n;
    const float mx = sx / fn, my = sy / fn;
    const float c00 = sx2 - 2.f * sx * mx + fn * mx * mx;
    const float c01 = sxy - sx * my - sy * mx + fn * mx * my;
    const float c11 = sy2 - 2.f * sy * my + fn * my * my;
    const double p = c00, qq = c11, r = c01;
    const double half = 0.5 * (p - qq);
    const double rad = sqrt(half * half + r * r);
    const double lmin = 0.5 * (p + qq) - rad;
    double vx, vy;
    if (r == 0.0) {
        if (p <= qq) { vx = 1.0; vy = 0.0; } else { vx = 0.0; vy = 1.0; }
    } else if (fabs(lmin - p) > fabs(lmin - qq)) {
        vx = r; vy = lmin - p;
    } else {
        vx = lmin - qq; vy = r;
    }
    const double nrm = sqrt(vx * vx + vy * vy);
    const float a = (float)(vx / nrm), b = (float)(vy / nrm);
    model_out[0] = a;
    model_out[1] = b;
    model_out[2] = -a * mx - b * my;
    for (int k = 3; k < 9; k++) model_out[k] = 0.f;
    *ok = 1;
}

// EstimateModelNonMinimalSample for W fits: homography (normalized_dlt.cpp:7-23), F and E
// (EightPointsAlgorithm, fundamental_estimator.hpp:65-76, essential_estimator.hpp:64-74,
// eight_points.cpp:4-100), line (line2d_estimator.hpp:59-107).  nmax >= every ns[w].
// With b.weights: the weighted overload (normalized_dlt.cpp:25-36, eight_points.cpp:176-228),
// which differs only in the normalising transformation.
hipError_t launch_nonminimal_batch(hipStream_t st, int estimator, const void *pts, const NmBatch &b) {
    if (b.W == 0) return hipSuccess;
    // pipelined LO stages: the fused gather derives the counts; the other paths first run the
    // derivation on its own (line fits; b.ns is the prep's output)
    if (b.prep && (estimator == USAC_LINE2D || b.weights)) {
        hipLaunchKernelGGL(k_lo_prep, dim3(1), dim3(64), 0, st, *b.prep, b.W);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const dim3 gg((b.nmax + 255) / 256 ? (b.nmax + 255) / 256 : 1, b.W);
    if (estimator == USAC_LINE2D) {
        if (b.weights) return hipErrorInvalidValue;  // the reference has no weighted line fit
        float2 *q = static_cast<float2 *>(b.q);
        hipLaunchKernelGGL(k_gather<float2>, gg, dim3(256), 0, st, static_cast<const float2 *>(pts), b.base,
                           b.base_stride, b.pos, b.pos_stride, b.ns, b.n1, q, b.q_stride);
        hipLaunchKernelGGL(k_line_pca, dim3(b.W), dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.model_out, b.ok);
        return hipGetLastError();
    }
    float4 *q = static_cast<float4 *>(b.q);
    if (b.skip_finish && (b.W != 1 || b.nmax <= kSmallFit || b.weights || b.prep)) return hipErrorInvalidValue;
    if (b.nmax <= kSmallFit && !b.weights && !b.prep) {  // every fit in one workgroup, one launch
        if (estimator == USAC_HOMOGRAPHY)
            hipLaunchKernelGGL(k_fit_small<false>, dim3(b.W), dim3(64), 0, st, static_cast<const float4 *>(pts), b.base,
                               b.base_stride, b.pos, b.pos_stride, b.ns, b.n1, b.ws, b.model_out, b.ok);
        else
            hipLaunchKernelGGL(k_fit_small<true>, dim3(b.W), dim3(64), 0, st, static_cast<const float4 *>(pts), b.base,
                               b.base_stride, b.pos, b.pos_stride, b.ns, b.n1, b.ws, b.model_out, b.ok);
        return hipGetLastError();
    }
    if (b.weights) {  // the weighted overload: six independent sequential chains, then as below
        if (!b.qw) return hipErrorInvalidValue;
        char *seq = static_cast<char *>(b.seq);
        const size_t ss = seq_stride(b.nmax);
        float *sums4 = reinterpret_cast<float *>(seq + b.W * ss), *dsum2 = sums4 + 4 * b.W;
        float4 *qw = static_cast<float4 *>(b.qw);
        hipLaunchKernelGGL(k_gather_weighted, gg, dim3(256), 0, st, static_cast<const float4 *>(pts), b.weights, b.base,
                           b.base_stride, b.pos, b.pos_stride, b.ns, b.n1, q, qw, b.q_stride, seq, ss);
        hipError_t e = launch_seqsum(st, 4, false, qw, 4 * b.q_stride, b.ns, b.n1, b.W, nullptr, seq, ss, false, sums4);
        if (e != hipSuccess) return e;
        e = launch_seqsum(st, 2, true, reinterpret_cast<const double *>(seq + kSeqA), ss / sizeof(double), b.ns, b.n1,
                          b.W, nullptr, seq, ss, false, dsum2);
        if (e != hipSuccess) return e;
    } else {  // gather; normalising transforms: sequential sums (seqsum), distance terms
        char *seq = static_cast<char *>(b.seq);
        const size_t ss = seq_stride(b.nmax);
        float *sums4 = reinterpret_cast<float *>(seq + b.W * ss), *dsum2 = sums4 + 4 * b.W;
        const bool fused = b.fused_any || b.prep || b.nmax <= kFusedGatherMax;
        if (fused)
            hipLaunchKernelGGL(k_gather_psum4, dim3(seq::kSegMax, b.W), dim3(256), 0, st,
                               static_cast<const float4 *>(pts), b.base, b.base_stride, b.pos, b.pos_stride, b.ns,
                               b.n1, q, b.q_stride, seq, ss, b.prep ? *b.prep : LoPrep{}, b.prep ? 1 : 0);
        else
            hipLaunchKernelGGL(k_gather<float4>, gg, dim3(256), 0, st, static_cast<const float4 *>(pts), b.base,
                               b.base_stride, b.pos, b.pos_stride, b.ns, b.n1, q, b.q_stride);
        hipError_t e = launch_seqsum(st, 4, false, q, 4 * b.q_stride, b.ns, b.n1, b.W, nullptr, seq, ss, fused, sums4);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_norm_dist, dim3(seq::kSegMax, b.W), dim3(256), 0, st, q, b.q_stride, b.ns, b.n1, seq, ss,
                           sums4);
        e = launch_seqsum(st, 2, true, reinterpret_cast<const double *>(seq + kSeqA), ss / sizeof(double), b.ns, b.n1,
                          b.W, nullptr, seq, ss, true, dsum2);
        if (e != hipSuccess) return e;
    }
    const char *seq = static_cast<const char *>(b.seq);
    const float *sums4 = reinterpret_cast<const float *>(seq + b.W * seq_stride(b.nmax)), *dsum2 = sums4 + 4 * b.W;
    const uint32_t nblk = (b.nmax + kAtaBlock - 1) / kAtaBlock;
    // one workgroup per 64-block superblock; when nmax is only a bound (pipelined LO stages)
    // at most kAtaGridBound of them per fit, each looping over superblocks
    uint32_t gx = nblk ? (nblk + 63) / 64 : 1;
    if (b.prep && gx > kAtaGridBound) gx = kAtaGridBound;
    const dim3 ga(gx, kAtaGroups, b.W);
    if (estimator == USAC_HOMOGRAPHY) {
        hipLaunchKernelGGL(k_ata_partial<false>, ga, dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.partial, b.p_stride,
                           sums4, dsum2, b.ws);
        if (!b.skip_finish)
            hipLaunchKernelGGL(k_dlt_finish<false>, dim3(b.W), dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.partial,
                               b.p_stride, b.ws, b.model_out, b.ok);
    } else {
        hipLaunchKernelGGL(k_ata_partial<true>, ga, dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.partial, b.p_stride,
                           sums4, dsum2, b.ws);
        if (!b.skip_finish)
            hipLaunchKernelGGL(k_dlt_finish<true>, dim3(b.W), dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.partial,
                               b.p_stride, b.ws, b.model_out, b.ok);
    }
    return hipGetLastError();
}

size_t nonminimal_partial_stride(uint32_t nmax) { return 45 * ((size_t)nmax / (64 * kAtaBlock) + 2); }

size_t nonminimal_seq_bytes(uint32_t nmax, uint32_t W) {
    return seq_stride(nmax) * W + sizeof(float) * 6 * W;
}

// ---------------------------------------------------------------------------------------------
// The post-loop polish (ransac.cpp:157-207) in ONE workgroup: 4 passes of fit + score + accept
// were ~56 launches of a few microseconds each (cfg3 exact: 0.28 ms of a 0.72 ms run, round 5),
// for lists of a few thousand points.  Every value is produced by the same operations in the same
// order as the multi-launch path (which the oracle pins), so the results are bit-identical:
//   gather      q[i] = pts[list[i]] into LDS
//   seq chains  the reference's sequential fp32 sums (4 coordinate means, 2 average distances,
//               Σerr) by the same speculation as kernels_seqsum.hip, workgroup-sized: a wave per
//               (chain, segment), a lane per candidate start (64, centred on the fp64 prefix),
//               a link walk that takes the candidate whose start has the running value's exact
//               bits, or walks the segment itself
//   A^T A       the spec's 16-point blocks (ata_group, a wave per group of 9 entries), block
//               partials summed in order per 1024-point superblock, superblocks in order
//   fit_finish  as k_dlt_finish / k_fit_small
//   score       the residuals of all N points in point order (ballot compaction), the list and
//               the residuals of the inliers, then the Σerr chain
//   accept      k_polish_prep's decision, kept in registers (uniform over the workgroup)
// 512 threads: fit_finish's lane-0 inverse iteration needs ~236 VGPRs (2 waves per SIMD).
constexpr uint32_t kPolT = 512;
constexpr uint32_t kPolC = 64;  // candidate starts per segment (a wave; 16 left ~25% of the starts outside)
constexpr uint32_t kPolSbWin = 3;  // A^T A superblocks whose block partials are held at once

struct PolShared {
    float4 *Q;       // [kPolFitMax]
    double *D;       // [2 kPolFitMax] distance terms; then A^T A block partials [64][45]; then residuals
    float *E;        // (aliases D) the inliers' residuals [kPolPtsMax]
    double *part;    // superblock partials [kPolFitMax / 1024][45]
    double *psum;    // [8 * 64 / kPolC] fp64 segment sums
    float *R;        // [kPolT] candidate ends
    uint32_t *wc;    // [8][8] wave counts
    uint64_t *dbg;   // USAC_PROFILE: [40 + NCH] link misses, [48 + NCH] segments linked
};

__device__ __forceinline__ float pol_cand(float ctr, uint32_t c) {
    return seq::unkey((int32_t)((uint32_t)seq::key(ctr) + c - kPolC / 2));
}

// the sequential chains s = op(s, v[q * cstride + k]), k = 0 .. n-1, of NCH chains -> out[q]
// (LDS; chain-major values, 16-byte aligned rows).  Wave w runs chain w % NCH; its lanes form
// 64 / kPolC groups, a group per segment and a lane per candidate start (kPolC of them, centred
// on the segment's fp64 prefix: the fp32 chain stayed within a few ulps of it in every cfg3
// polish measured, round 5); each lane reads a group of its segment's next elements by 16-byte
// reads issued a group ahead.  A start outside the window is walked by the link (exact either way).
template <int NCH, bool F64>
__device__ __forceinline__ void pol_seq(const typename seq::Op<F64>::V *vals, uint32_t cstride, uint32_t n,
                                        const PolShared &sh, float *out) {
    typedef seq::Op<F64> Op;
    typedef typename Op::V V;
    constexpr uint32_t GPW = 64 / kPolC, S = kPolT / (64 * NCH) * GPW;  // segments per chain
    constexpr uint32_t kVec = 16 / sizeof(V), G = 8, NV = G / kVec;
    typedef V Vv __attribute__((ext_vector_type(kVec)));
    const uint32_t t = threadIdx.x, wave = t / 64, lane = t % 64, grp = lane / kPolC, c = lane % kPolC;
    const uint32_t q = __builtin_amdgcn_readfirstlane(wave % NCH), jw = __builtin_amdgcn_readfirstlane(wave / NCH);
    const uint32_t j = jw * GPW + grp;
    const uint32_t L = ((n + S - 1) / S + G - 1) / G * G;  // a multiple of the group: aligned reads
    const uint32_t b = j * L < n ? j * L : n, e = b + L < n ? b + L : n;
    const V *v = vals + (size_t)q * cstride;
    double a = 0.0;  // the segment's fp64 sum: only places the centres
    for (uint32_t k = b + c; k < e; k += kPolC) a += Op::wide(v[k]);
    for (uint32_t o = kPolC / 2; o > 0; o >>= 1) a += __shfl_xor(a, (int)o);
    if (c == 0) sh.psum[j * NCH + q] = a;
    __syncthreads();
    double pre = 0.0;
    for (uint32_t i = 0; i < j; i++) pre += sh.psum[i * NCH + q];
    float s = pol_cand((float)pre, c);
    uint32_t k = b;
    auto load = [&](Vv (&x)[NV], uint32_t k0) {
#pragma unroll
        for (uint32_t u = 0; u < NV; u++) x[u] = *reinterpret_cast<const Vv *>(v + k0 + kVec * u);
    };
    if (k + G <= e) {
        Vv x[NV];
        load(x, k);
        for (; k + 2 * G <= e; k += G) {
            Vv y[NV];
            load(y, k + G);
#pragma unroll
            for (uint32_t u = 0; u < NV; u++)
#pragma unroll
                for (uint32_t z = 0; z < kVec; z++) s = Op::step(s, x[u][z]);
#pragma unroll
            for (uint32_t u = 0; u < NV; u++) x[u] = y[u];
        }
#pragma unroll
        for (uint32_t u = 0; u < NV; u++)
#pragma unroll
            for (uint32_t z = 0; z < kVec; z++) s = Op::step(s, x[u][z]);
        k += G;
    }
    for (; k < e; k++) s = Op::step(s, v[k]);
    sh.R[(j * NCH + q) * kPolC + c] = s;
    __syncthreads();
    if (wave < NCH) {  // link: wave q walks chain q's segments (every lane the same value)
        const V *w = vals + (size_t)wave * cstride;
        float r = 0.f;
        double p2 = 0.0;
        uint32_t miss = 0;
        for (uint32_t jj = 0; jj < S; jj++) {
            if (jj) p2 += sh.psum[(jj - 1) * NCH + wave];
            const uint32_t bb = jj * L < n ? jj * L : n, ee = bb + L < n ? bb + L : n;
            if (bb >= ee) break;
            const float ctr = (float)p2;
            const int64_t idx = (int64_t)seq::key(r) - (int64_t)seq::key(ctr) + (int64_t)(kPolC / 2);
            bool hit = false;
            if (idx >= 0 && idx < (int64_t)kPolC && __float_as_uint(pol_cand(ctr, (uint32_t)idx)) == __float_as_uint(r)) {
                r = sh.R[(jj * NCH + wave) * kPolC + (uint32_t)idx];
                hit = true;
            }
            if (!hit) {
                miss++;
                for (uint32_t kk = bb; kk < ee; kk++) r = Op::step(r, w[kk]);
            }
        }
        if (lane == 0) out[wave] = r;
        if (sh.dbg && lane == 0 && miss)  // USAC_PROFILE: walked segments
            atomicAdd(reinterpret_cast<unsigned long long *>(sh.dbg + 40 + NCH), (unsigned long long)miss);
    }
    __syncthreads();
}

template <int EST>
__device__ __forceinline__ float pol_error(const float *m, const float4 p) {
    if constexpr (EST == USAC_HOMOGRAPHY) return homography_error(m, m + 9, p.x, p.y, p.z, p.w);
    else if constexpr (EST == USAC_FUNDAMENTAL) return fundamental_error(m, p.x, p.y, p.z, p.w);
    else return essential_error(m, p.x, p.y, p.z, p.w);
}

// getInliers of the model in sm_model (H: with its inverse) over all N points: list (global),
// the residuals (sh.E) in point order; returns the count (uniform)
template <int EST>
__device__ __forceinline__ uint32_t pol_score(const float4 *__restrict__ pts, uint32_t N, const float *sm_model, float thr,
                              int32_t *__restrict__ list, const PolShared &sh) {
    const uint32_t t = threadIdx.x, wave = t / 64, lane = t % 64;
    float m[18];
#pragma unroll
    for (int k = 0; k < 18; k++) m[k] = sm_model[k];
    constexpr uint32_t U = 8, W = kPolT / 64;
    uint32_t base = 0;
    for (uint32_t c0 = 0; c0 < N; c0 += U * kPolT) {
        float4 pv[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t i = c0 + u * kPolT + t;
            pv[u] = i < N ? pts[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        float ev[U];
        uint64_t bal[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t i = c0 + u * kPolT + t;
            ev[u] = i < N ? pol_error<EST>(m, pv[u]) : 0.f;
            bal[u] = __ballot(i < N && ev[u] < thr);
            if (lane == 0) sh.wc[u * W + wave] = (uint32_t)__popcll(bal[u]);
        }
        __syncthreads();
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            uint32_t r = base, tot = 0;
            for (uint32_t v = 0; v < W; v++) {
                const uint32_t cv = sh.wc[u * W + v];
                if (v < wave) r += cv;
                tot += cv;
            }
            if ((bal[u] >> lane) & 1ull) {
                r += (uint32_t)__popcll(bal[u] & ((1ull << lane) - 1));
                list[r] = (int32_t)(c0 + u * kPolT + t);
                sh.E[r] = ev[u];
            }
            base += tot;
        }
        __syncthreads();
    }
    return base;
}

// EstimateModelNonMinimalSample of the n points of list -> sm_model[0..8], *sm_ok (n <= kPolFitMax)
template <bool FUND>
__device__ __forceinline__ void pol_fit(const float4 *__restrict__ pts, const int32_t *__restrict__ list, uint32_t n,
                        const PolShared &sh, float *sm_sums, float *sm_ws, double (*A)[9], double (*V)[9],
                        double *s_v, float *sm_model, int32_t *sm_ok, uint64_t *st) {
    const uint32_t t = threadIdx.x;
    auto stamp = [&](int i) {
        if (st && t == 0) st[i] = wall_clock64();
    };
    float *T = reinterpret_cast<float *>(sh.D);  // the coordinates chain-major [4][kPolFitMax]
    for (uint32_t i0 = t; i0 < n; i0 += 8 * kPolT) {  // eight dependent loads in flight per thread
        int32_t ix[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) ix[u] = i0 + u * kPolT < n ? list[i0 + u * kPolT] : 0;
        float4 p[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) p[u] = i0 + u * kPolT < n ? pts[ix[u]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) {
            const uint32_t i = i0 + u * kPolT;
            if (i < n) {
                sh.Q[i] = p[u];
                T[i] = p[u].x;
                T[kPolFitMax + i] = p[u].y;
                T[2 * kPolFitMax + i] = p[u].z;
                T[3 * kPolFitMax + i] = p[u].w;
            }
        }
    }
    __syncthreads();
    stamp(0);
    if (n == 0) {
        fit_finish<FUND>(sh.Q, 0, sm_ws, A, V, s_v, sm_model, sm_ok);
        __syncthreads();
        return;
    }
    const float4 *Q = sh.Q;
    pol_seq<4, false>(T, kPolFitMax, n, sh, sm_sums);
    stamp(1);
    const float mx1 = sm_sums[0] / (float)n, my1 = sm_sums[1] / (float)n;
    const float mx2 = sm_sums[2] / (float)n, my2 = sm_sums[3] / (float)n;
    for (uint32_t i = t; i < n; i += kPolT) {  // k_norm_dist's terms
        const float4 p = Q[i];
        const float xm1 = p.x - mx1, ym1 = p.y - my1;
        const float xm2 = p.z - mx2, ym2 = p.w - my2;
        sh.D[i] = sqrt((double)(xm1 * xm1 + ym1 * ym1));  // chain-major [2][kPolFitMax]
        sh.D[kPolFitMax + i] = sqrt((double)(xm2 * xm2 + ym2 * ym2));
    }
    __syncthreads();
    stamp(2);
    pol_seq<2, true>(sh.D, kPolFitMax, n, sh, sm_sums + 4);
    stamp(3);
    float t1[9], t2[9];
    norm_transforms(sm_sums, sm_sums + 4, 0, n, t1, t2);
    if (t < 9) {
        sm_ws[t] = t1[t];
        sm_ws[9 + t] = t2[t];
    }
    if (!(FUND ? n <= 8 : 2 * n <= 9)) {
        const NormXf xf = norm_xf(t1, t2);
        const uint32_t nblocks = (n + kAtaBlock - 1) / kAtaBlock, nsb = (nblocks + 63) / 64;
        double *red = sh.D;  // [kPolSbWin][64][45] (the distance terms are consumed)
        const uint32_t wave = __builtin_amdgcn_readfirstlane(t / 64), bl = t % 64;
        for (uint32_t w0 = 0; w0 < nsb; w0 += kPolSbWin) {  // a window of superblocks: jobs (sb, group)
            const uint32_t nwin = nsb - w0 < kPolSbWin ? nsb - w0 : kPolSbWin, jobs = kAtaGroups * nwin;
            for (uint32_t jb = wave; jb < jobs; jb += kPolT / 64) {  // a wave per job, a lane per block
                const uint32_t sbl = jb / kAtaGroups, g = jb % kAtaGroups, blk = (w0 + sbl) * 64 + bl;
                if (blk < nblocks) {
                    double acc[kAtaPer];
                    const uint32_t b0 = blk * kAtaBlock, b1 = b0 + kAtaBlock < n ? b0 + kAtaBlock : n;
                    ata_dispatch<FUND>((int)g, Q, xf, b0, b1, acc);
#pragma unroll
                    for (int e = 0; e < kAtaPer; e++) red[(sbl * 64 + bl) * 45 + kAtaPer * g + e] = acc[e];
                }
            }
            __syncthreads();
            if (t < 45 * nwin) {  // each superblock's blocks in order
                const uint32_t sbl = t / 45, e = t % 45, sb = w0 + sbl;
                const uint32_t nb = nblocks - sb * 64 < 64 ? nblocks - sb * 64 : 64;
                double sum = 0.0;
                for (uint32_t b = 0; b < nb; b++) sum += red[(sbl * 64 + b) * 45 + e];
                sh.part[sb * 45 + e] = sum;
            }
            __syncthreads();
        }
        if (t < 45) {  // k_dlt_finish: the superblock partials in order
            double acc = 0.0;
            for (uint32_t c = 0; c < nsb; c++) acc += sh.part[c * 45 + t];
            int j, k;
            ata_entry(t, j, k);
            A[j][k] = acc;
            A[k][j] = acc;
        }
    }
    __syncthreads();
    stamp(4);
    fit_finish<FUND>(Q, n, sm_ws, A, V, s_v, sm_model, sm_ok);
    __syncthreads();
    stamp(5);
}

template <int EST>
__global__ __launch_bounds__(kPolT) void k_polish_fused(const float4 *__restrict__ pts, uint32_t N,
                                                        const float *__restrict__ model0, float thr, int32_t best0,
                                                        uint32_t fit_max, PolLists lists, int32_t *__restrict__ res,
                                                        uint64_t *__restrict__ dbg) {
    constexpr bool FUND = EST != USAC_HOMOGRAPHY;
    __shared__ __attribute__((aligned(16))) float4 s_q[kPolFitMax];
    __shared__ __attribute__((aligned(16))) double s_d[kPolSbWin * 64 * 45 > 2 * kPolFitMax ? kPolSbWin * 64 * 45
                                                                                            : 2 * kPolFitMax];
    __shared__ double s_part[(kPolFitMax / 1024) * 45];
    __shared__ double A[9][9], V[9][9], s_v[9], s_psum[8 * 64 / kPolC];
    __shared__ float s_R[kPolT], s_sums[8], s_ws[18], s_model[18], s_sum[1];
    __shared__ uint32_t s_wc[8 * (kPolT / 64)];
    __shared__ int32_t s_ok;
    PolShared sh;  // (not a const aggregate: LDS addresses are no static initializer)
    sh.Q = s_q;
    sh.D = s_d;
    sh.E = reinterpret_cast<float *>(s_d);
    sh.part = s_part;
    sh.psum = s_psum;
    sh.R = s_R;
    sh.wc = s_wc;
    sh.dbg = dbg;
    static_assert(sizeof(double) * 2 * kPolFitMax >= sizeof(float) * kPolPtsMax, "residuals alias the distance terms");
    const uint32_t t = threadIdx.x;
    float *resf = reinterpret_cast<float *>(res);
    auto load_model = [&](const float *mdl) {  // inl_model: the model, H^-1 for H
        if (t == 0) {
            for (int k = 0; k < 9; k++) s_model[k] = mdl[k];
            if (EST == USAC_HOMOGRAPHY) inv3x3(s_model, s_model + 9);
        }
        __syncthreads();
    };
    auto score = [&](int32_t *list, uint64_t *st) -> uint32_t {
        const uint32_t cnt = pol_score<EST>(pts, N, s_model, thr, list, sh);
        if (st && t == 0) st[0] = wall_clock64();
        pol_seq<1, false>(sh.E, 0, cnt, sh, s_sum);
        if (st && t == 0) st[1] = wall_clock64();
        return cnt;
    };
    // USAC_PROFILE: wall-clock stamps (dbg[0] start, [1..2] the first getInliers, 8 per pass)
    if (dbg && t == 0) dbg[0] = wall_clock64();
    // quality->getInliers(best_model): lists[0], slots 12-13
    load_model(model0);
    {
        const uint32_t c0 = score(lists.l[0], dbg ? dbg + 1 : nullptr);
        if (t == 0) {
            res[12] = (int32_t)c0;
            resf[13] = s_sum[0];
        }
    }
    int32_t best = best0, prev = 0;
    uint32_t n = (uint32_t)best0;
    constexpr int kPasses = 4;
    for (int k = 0; k < kPasses; k++) {
        if (n > fit_max) {  // workgroup-uniform: the host runs passes k.. the multi-launch way
            if (t == 0) res[kPolStop] = k;
            return;
        }
        float *pres = resf + kPolPass * k;
        uint64_t *st = dbg ? dbg + 3 + 8 * k : nullptr;
        pol_fit<FUND>(pts, lists.l[k], n, sh, s_sums, s_ws, A, V, s_v, s_model, &s_ok, st);
        const int32_t ok = s_ok;
        if (t == 0) {
            if (n > 0)
                for (int j = 0; j < 9; j++) pres[j] = s_model[j];
            res[kPolPass * k + 9] = ok;
        }
        uint32_t cnt = 0;
        float sum = 0.f;
        if (ok) {
            if (EST == USAC_HOMOGRAPHY && t == 0) inv3x3(s_model, s_model + 9);
            __syncthreads();
            cnt = score(lists.l[k + 1], st ? st + 6 : nullptr);
            sum = s_sum[0];
        }
        if (t == 0) {
            res[kPolPass * k + 10] = (int32_t)cnt;
            pres[11] = sum;
        }
        if (k + 1 < kPasses) {  // k_polish_prep
            const bool accept = ok && !((double)((float)(int32_t)cnt / (float)best) < 0.8) && (int32_t)cnt > prev;
            if (t == 0) reinterpret_cast<uint32_t *>(res)[kPolNs + k + 1] = accept ? cnt : 0u;
            best = accept ? (int32_t)cnt : best;
            prev = accept ? (int32_t)cnt : prev;
            if (t == 0) {
                res[kPolState] = best;
                res[kPolState + 1] = prev;
            }
            n = accept ? cnt : 0u;
        }
        __syncthreads();
    }
    if (t == 0) res[kPolStop] = kPasses;
}

hipError_t launch_polish_fused(hipStream_t st, int estimator, const void *pts, uint32_t N, const float *model0,
                               float thr, int32_t best0, PolLists lists, int32_t *res, uint32_t fit_max,
                               uint64_t *dbg) {
    if (fit_max > kPolFitMax) fit_max = kPolFitMax;
    if (N > kPolPtsMax || best0 < 0 || (uint32_t)best0 > fit_max) return hipErrorInvalidValue;
    const float4 *p = static_cast<const float4 *>(pts);
    switch (estimator) {
        case USAC_HOMOGRAPHY:
            hipLaunchKernelGGL(k_polish_fused<USAC_HOMOGRAPHY>, dim3(1), dim3(kPolT), 0, st, p, N, model0, thr, best0, fit_max, lists, res, dbg);
            break;
        case USAC_FUNDAMENTAL:
            hipLaunchKernelGGL(k_polish_fused<USAC_FUNDAMENTAL>, dim3(1), dim3(kPolT), 0, st, p, N, model0, thr, best0, fit_max, lists, res, dbg);
            break;
        case USAC_ESSENTIAL:
            hipLaunchKernelGGL(k_polish_fused<USAC_ESSENTIAL>, dim3(1), dim3(kPolT), 0, st, p, N, model0, thr, best0, fit_max, lists, res, dbg);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// getInliers of ONE model over N <= kPolPtsMax points in one workgroup (pol_score + the Σerr
// chain), for launch_inliers_batch's single-model calls with sums: one launch instead of five
// (flags, compact, and the three launches of the Σ chain), the same list, count and sum bits.
// ok (nullable): a failed fit's slot gets count 0 and sum 0 and its list is left alone.
template <int EST>
__global__ __launch_bounds__(kPolT) void k_inliers_small(const float4 *__restrict__ pts, uint32_t N,
                                                         const float *__restrict__ model, float thr,
                                                         const int32_t *__restrict__ ok, int32_t *__restrict__ idx,
                                                         int32_t *__restrict__ count, float *__restrict__ sum) {
    __shared__ __attribute__((aligned(16))) float s_e[kPolPtsMax];
    __shared__ double s_psum[8 * 64 / kPolC];
    __shared__ float s_R[kPolT], s_model[18], s_sum[1];
    __shared__ uint32_t s_wc[8 * (kPolT / 64)];
    const uint32_t t = threadIdx.x;
    if (ok && !*ok) {
        if (t == 0) {
            *count = 0;
            *sum = 0.f;
        }
        return;
    }
    PolShared sh;
    sh.Q = nullptr;
    sh.D = nullptr;
    sh.E = s_e;
    sh.part = nullptr;
    sh.psum = s_psum;
    sh.R = s_R;
    sh.wc = s_wc;
    sh.dbg = nullptr;
    if (t == 0) {  // inl_model: the model, H^-1 for H
        for (int k = 0; k < 9; k++) s_model[k] = model[k];
        if (EST == USAC_HOMOGRAPHY) inv3x3(s_model, s_model + 9);
    }
    __syncthreads();
    const uint32_t cnt = pol_score<EST>(pts, N, s_model, thr, idx, sh);
    pol_seq<1, false>(s_e, 0, cnt, sh, s_sum);
    if (t == 0) {
        *count = (int32_t)cnt;
        *sum = s_sum[0];
    }
}

hipError_t launch_inliers_small(hipStream_t st, int estimator, const void *pts, uint32_t N, const float *model,
                                float thr, const int32_t *ok, int32_t *idx, int32_t *count, float *sum) {
    if (N > kPolPtsMax) return hipErrorInvalidValue;
    const float4 *p = static_cast<const float4 *>(pts);
    switch (estimator) {
        case USAC_HOMOGRAPHY:
            hipLaunchKernelGGL(k_inliers_small<USAC_HOMOGRAPHY>, dim3(1), dim3(kPolT), 0, st, p, N, model, thr, ok, idx, count, sum);
            break;
        case USAC_FUNDAMENTAL:
            hipLaunchKernelGGL(k_inliers_small<USAC_FUNDAMENTAL>, dim3(1), dim3(kPolT), 0, st, p, N, model, thr, ok, idx, count, sum);
            break;
        case USAC_ESSENTIAL:
            hipLaunchKernelGGL(k_inliers_small<USAC_ESSENTIAL>, dim3(1), dim3(kPolT), 0, st, p, N, model, thr, ok, idx, count, sum);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// k_dlt_finish + k_inliers_small + k_polish_prep of one polish pass in one workgroup (the three
// launches' operations in their order, the model kept in LDS between them)
template <int EST>
__global__ __launch_bounds__(kPolT) void k_finish_score(const float4 *__restrict__ q, const uint32_t *__restrict__ ns,
                                                        uint32_t n1, const double *__restrict__ partial,
                                                        const float *__restrict__ ws, float *__restrict__ model_out,
                                                        int32_t *__restrict__ ok_out, const float4 *__restrict__ pts,
                                                        uint32_t N, float thr, int32_t *__restrict__ idx,
                                                        int32_t *__restrict__ count, float *__restrict__ sum,
                                                        int32_t *__restrict__ res, int prep_k, int32_t best0) {
    constexpr bool FUND = EST != USAC_HOMOGRAPHY;
    __shared__ __attribute__((aligned(16))) float s_e[kPolPtsMax];
    __shared__ double A[9][9], V[9][9], s_v[9], s_psum[8 * 64 / kPolC];
    __shared__ float s_R[kPolT], s_model[18], s_sum[1], s_ws[18];
    __shared__ uint32_t s_wc[8 * (kPolT / 64)];
    __shared__ int32_t s_ok;
    const uint32_t t = threadIdx.x;
    const uint32_t n = ns ? ns[0] : n1;
    if (t < 18) s_ws[t] = ws[t];
    if (n > 0 && !(FUND ? n <= 8 : 2 * n <= 9) && t < 45) {  // k_dlt_finish: the superblock partials in order
        int j, k;
        ata_entry(t, j, k);
        const uint32_t nblocks = (n + kAtaBlock * 64 - 1) / (kAtaBlock * 64);
        double acc = 0.0;
        for (uint32_t c = 0; c < nblocks; c++) acc += partial[(size_t)c * 45 + t];
        A[j][k] = acc;
        A[k][j] = acc;
    }
    __syncthreads();
    fit_finish<FUND>(q, n, s_ws, A, V, s_v, s_model, &s_ok);
    __syncthreads();
    const int32_t ok = s_ok;
    if (t == 0) {
        if (n > 0)
            for (int j = 0; j < 9; j++) model_out[j] = s_model[j];
        *ok_out = ok;
    }
    uint32_t cnt = 0;
    float sm = 0.f;
    if (ok) {  // k_inliers_small
        PolShared sh;
        sh.Q = nullptr;
        sh.D = nullptr;
        sh.E = s_e;
        sh.part = nullptr;
        sh.psum = s_psum;
        sh.R = s_R;
        sh.wc = s_wc;
        sh.dbg = nullptr;
        if (EST == USAC_HOMOGRAPHY && t == 0) inv3x3(s_model, s_model + 9);
        __syncthreads();
        cnt = pol_score<EST>(pts, N, s_model, thr, idx, sh);
        pol_seq<1, false>(s_e, 0, cnt, sh, s_sum);
        sm = s_sum[0];
    }
    if (t == 0) {
        *count = (int32_t)cnt;
        *sum = sm;
        if (prep_k >= 0) {  // k_polish_prep
            const int32_t best = prep_k == 0 ? best0 : res[kPolState];
            const int32_t prev = prep_k == 0 ? 0 : res[kPolState + 1];
            const int32_t c = (int32_t)cnt;
            const bool accept = ok && !((double)((float)c / (float)best) < 0.8) && c > prev;
            reinterpret_cast<uint32_t *>(res)[kPolNs + prep_k + 1] = accept ? (uint32_t)c : 0u;
            res[kPolState] = accept ? c : best;
            res[kPolState + 1] = accept ? c : prev;
        }
    }
}

hipError_t launch_finish_score(hipStream_t st, int estimator, const NmBatch &b, const void *pts, uint32_t N,
                               float thr, int32_t *idx, int32_t *count, float *sum, int32_t *res, int prep_k,
                               int32_t best0) {
    if (N > kPolPtsMax || b.W != 1 || !b.skip_finish) return hipErrorInvalidValue;
    const float4 *q = static_cast<const float4 *>(b.q), *p = static_cast<const float4 *>(pts);
#define FS(E)                                                                                                       \
    hipLaunchKernelGGL(k_finish_score<E>, dim3(1), dim3(kPolT), 0, st, q, b.ns, b.n1, b.partial, b.ws, b.model_out, \
                       b.ok, p, N, thr, idx, count, sum, res, prep_k, best0)
    switch (estimator) {
        case USAC_HOMOGRAPHY: FS(USAC_HOMOGRAPHY); break;
        case USAC_FUNDAMENTAL: FS(USAC_FUNDAMENTAL); break;
        case USAC_ESSENTIAL: FS(USAC_ESSENTIAL); break;
        default: return hipErrorInvalidValue;
    }
#undef FS
    return hipGetLastError();
}

}  // namespace usac
