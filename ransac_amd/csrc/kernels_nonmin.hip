// kernels_nonmin.hip -- non-minimal (least-squares) model fits on the device, used by the
// post-loop polish (ransac.cpp:157-207):
//   homography: DLt::NormalizedDLT (normalized_dlt.cpp:7-23) with
//               GetNormalizingTransformation (normalizing_transformation.cpp:7-113);
//   line2d    : Line2DEstimator::EstimateModelNonMinimalSample PCA (line2d_estimator.hpp:59-107).
// The reference's fp32 moment sums are sequential in sample order and stay sequential
// here (one lane per accumulator).  The DLT normal matrix A^T A (fp64) has no reference
// order (OpenCV's SVD hides it); its order is fixed by this build's spec: 64-point
// blocks summed in order, block partials summed in block order -- shared with the oracle.
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_kernels.h"

namespace usac {

constexpr uint32_t kAtaBlock = 64;

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

// normalizing transformation: lanes 0..3 = the four coordinate means, lanes 0..1 = the
// two distance sums (each a sequential fp32 chain in point order, as the reference sums);
// then every lane normalises a strided share of the points.  The chains are latency-bound:
// waves 1-3 stage the NEXT 1024-point chunk into LDS (coalesced loads; for the distance pass
// they also compute its sqrt terms) while lanes of wave 0 add the current chunk from the
// other buffer -- one barrier per chunk, the staging hidden behind the chain.
// ws layout (floats): [0..8] T1, [9..17] T2.
constexpr uint32_t kNormChunk = 1024;

__device__ __forceinline__ float chain_add_f32(float acc, const float *f, uint32_t m) {
    // 16 values in registers, the next 16 in flight from LDS (stride 4 floats)
    uint32_t k = 0;
    if (m >= 16) {
        float c[16];
#pragma unroll
        for (int u = 0; u < 16; u++) c[u] = f[4 * u];
        for (; k + 32 <= m; k += 16) {
            float nx[16];
#pragma unroll
            for (int u = 0; u < 16; u++) nx[u] = f[4 * (k + 16 + u)];
#pragma unroll
            for (int u = 0; u < 16; u++) acc += c[u];
#pragma unroll
            for (int u = 0; u < 16; u++) c[u] = nx[u];
        }
#pragma unroll
        for (int u = 0; u < 16; u++) acc += c[u];
        k += 16;
    }
    for (; k < m; k++) acc += f[4 * k];
    return acc;
}

// d = (float)((double)d + s_k): the reference's float += double (sqrt of a float in C)
__device__ __forceinline__ float chain_add_f64(float d, const double *sq, uint32_t m) {
    uint32_t k = 0;
    if (m >= 16) {
        double c[16];
#pragma unroll
        for (int u = 0; u < 16; u++) c[u] = sq[u];
        for (; k + 32 <= m; k += 16) {
            double nx[16];
#pragma unroll
            for (int u = 0; u < 16; u++) nx[u] = sq[k + 16 + u];
#pragma unroll
            for (int u = 0; u < 16; u++) d = (float)((double)d + c[u]);
#pragma unroll
            for (int u = 0; u < 16; u++) c[u] = nx[u];
        }
#pragma unroll
        for (int u = 0; u < 16; u++) d = (float)((double)d + c[u]);
        k += 16;
    }
    for (; k < m; k++) d = (float)((double)d + sq[k]);
    return d;
}

__global__ __launch_bounds__(256) void k_normalize(float4 *__restrict__ q_all, size_t q_stride,
                                                   const uint32_t *__restrict__ ns, uint32_t n1, float *ws_all) {
    __shared__ float4 s_pts[2][kNormChunk];
    __shared__ double s_sq[2][2][kNormChunk];
    __shared__ float s_mean[4];
    __shared__ float s_scale[2];
    float4 *q = q_all + blockIdx.x * q_stride;
    const uint32_t n = ns ? ns[blockIdx.x] : n1;
    float *ws = ws_all + 18 * blockIdx.x;
    const uint32_t t = threadIdx.x;
    const bool loader = t >= 64;
    const uint32_t lt = t - 64;  // loader index, 192 loaders
    const uint32_t nch = (n + kNormChunk - 1) / kNormChunk;
    auto chunk_len = [&](uint32_t c) { return n - c * kNormChunk < kNormChunk ? n - c * kNormChunk : kNormChunk; };
    // means
    if (loader && nch > 0)
        for (uint32_t i = lt; i < chunk_len(0); i += 192) s_pts[0][i] = q[i];
    __syncthreads();
    float acc = 0.f;
    for (uint32_t c = 0; c < nch; c++) {
        if (loader && c + 1 < nch) {
            const uint32_t m1 = chunk_len(c + 1), base = (c + 1) * kNormChunk;
            for (uint32_t i = lt; i < m1; i += 192) s_pts[(c + 1) & 1][i] = q[base + i];
        }
        if (t < 4) acc = chain_add_f32(acc, reinterpret_cast<const float *>(s_pts[c & 1]) + t, chunk_len(c));
        __syncthreads();
    }
    if (t < 4) s_mean[t] = acc / (float)n;
    __syncthreads();
    const float mx1 = s_mean[0], my1 = s_mean[1], mx2 = s_mean[2], my2 = s_mean[3];
    // average distances
    auto stage_sq = [&](uint32_t c) {
        const uint32_t m = chunk_len(c), base = c * kNormChunk;
        for (uint32_t i = lt; i < m; i += 192) {
            const float4 p = q[base + i];
            const float xm1 = p.x - mx1, ym1 = p.y - my1;
            const float xm2 = p.z - mx2, ym2 = p.w - my2;
            s_sq[c & 1][0][i] = sqrt((double)(xm1 * xm1 + ym1 * ym1));
            s_sq[c & 1][1][i] = sqrt((double)(xm2 * xm2 + ym2 * ym2));
        }
    };
    if (loader && nch > 0) stage_sq(0);
    __syncthreads();
    float d = 0.f;
    for (uint32_t c = 0; c < nch; c++) {
        if (loader && c + 1 < nch) stage_sq(c + 1);
        if (t < 2) d = chain_add_f64(d, s_sq[c & 1][t], chunk_len(c));
        __syncthreads();
    }
    if (t < 2) s_scale[t] = (float)(M_SQRT2 / (double)(d / (float)n));
    __syncthreads();
    const float s1 = s_scale[0], s2 = s_scale[1];
    const float t1[9] = {s1, 0.f, -s_mean[0] * s1, 0.f, s1, -s_mean[1] * s1, 0.f, 0.f, 1.f};
    const float t2[9] = {s2, 0.f, -s_mean[2] * s2, 0.f, s2, -s_mean[3] * s2, 0.f, 0.f, 1.f};
    if (t < 9) {
        ws[t] = t1[t];
        ws[9 + t] = t2[t];
    }
    __syncthreads();
    for (uint32_t i = t; i < n; i += 256) {
        float4 p = q[i];
        float4 o;
        o.x = t1[0] * p.x + t1[2];
        o.y = t1[4] * p.y + t1[5];
        o.z = t2[0] * p.z + t2[2];
        o.w = t2[4] * p.w + t2[5];
        q[i] = o;
    }
}

// block partials of A^T A: one lane per 64-point block (the spec's unit), its 45
// upper-triangle entries (row-major j <= k) accumulated in registers over the block's points
// in order -- each point's rows are built once per lane, not once per entry.
// FUND: one 8-point row per correspondence (eight_points.cpp:26-45), else two DLT rows.
template <bool FUND>
__global__ __launch_bounds__(64) void k_ata_partial(const float4 *__restrict__ q_all, size_t q_stride,
                                                    const uint32_t *__restrict__ ns, uint32_t n1,
                                                    double *__restrict__ partial_all, size_t p_stride) {
    const uint32_t w = blockIdx.y;
    const uint32_t n = ns ? ns[w] : n1;
    const uint32_t blk = blockIdx.x * 64 + threadIdx.x;
    if ((FUND ? n <= 8 : 2 * n <= 9) || blk * kAtaBlock >= n) return;
    const float4 *q = q_all + w * q_stride;
    const uint32_t b0 = blk * kAtaBlock;
    const uint32_t b1 = b0 + kAtaBlock < n ? b0 + kAtaBlock : n;
    double acc[45];
#pragma unroll
    for (int e = 0; e < 45; e++) acc[e] = 0.0;
    for (uint32_t i = b0; i < b1; i++) {
        const float4 p = q[i];
        if (FUND) {
            double r[9];
            fund_row(p.x, p.y, p.z, p.w, r);
            int e = 0;
#pragma unroll
            for (int j = 0; j < 9; j++)
#pragma unroll
                for (int k = j; k < 9; k++) acc[e++] += r[j] * r[k];
        } else {
            double r0[9], r1[9];
            dlt_rows(p.x, p.y, p.z, p.w, r0, r1);
            int e = 0;
#pragma unroll
            for (int j = 0; j < 9; j++)
#pragma unroll
                for (int k = j; k < 9; k++) acc[e++] += r0[j] * r0[k] + r1[j] * r1[k];
        }
    }
    double *out = partial_all + w * p_stride + (size_t)blk * 45;
#pragma unroll
    for (int e = 0; e < 45; e++) out[e] = acc[e];
}

// Final solve, one wave: A^T A from the partials (lane e), round-robin Jacobi eigen over
// 36 lanes (LDS), smallest-eigenvalue vector; or the thin row-Jacobi when the system has
// <= 8 rows (homography 2n <= 8, fundamental n <= 8: SURVEY Q1/Q2); then
//   homography : H = T2^-1 * Hn * T1 (fp64), H /= H33 (normalized_dlt.cpp:18-22);
//   fundamental: F = T2^T * Fn * T1 (fp64), F /= F33 when |F33| > FLT_EPSILON
//                (eight_points.cpp:76-99);
// cast to float.
template <int R, bool FUND>
__device__ void thin_solve(const float4 *q, double *v) {
    double W[R][9];
    if (FUND) {
#pragma unroll
        for (int i = 0; i < R; i++) {
            const float4 p = q[i];
            fund_row(p.x, p.y, p.z, p.w, W[i]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < R / 2; i++) {
            const float4 p = q[i];
            dlt_rows(p.x, p.y, p.z, p.w, W[2 * i], W[2 * i + 1]);
        }
    }
    row_jacobi<R>(W);
    pick_vector<R>(W, 0, v);
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
    const float4 *q = q_all + w * q_stride;
    const double *partial = partial_all + w * p_stride;
    const uint32_t nblocks = (n + kAtaBlock - 1) / kAtaBlock;
    const float *ws = ws_all + 18 * w;
    float *model_out = model_all + 9 * w;
    int32_t *ok = ok_all + w;
    if (n == 0) {  // EstimateModelNonMinimalSample of no points fails
        if (t == 0) *ok = 0;
        return;
    }
    if (FUND ? n <= 8 : 2 * n <= 9) {
        if (t == 0) {
            double v[9];
            if (FUND) {
                switch (n) {
                    case 1: thin_solve<1, true>(q, v); break;
                    case 2: thin_solve<2, true>(q, v); break;
                    case 3: thin_solve<3, true>(q, v); break;
                    case 4: thin_solve<4, true>(q, v); break;
                    case 5: thin_solve<5, true>(q, v); break;
                    case 6: thin_solve<6, true>(q, v); break;
                    case 7: thin_solve<7, true>(q, v); break;
                    default: thin_solve<8, true>(q, v); break;
                }
            } else {
                if (n == 1) thin_solve<2, false>(q, v);
                else if (n == 2) thin_solve<4, false>(q, v);
                else if (n == 3) thin_solve<6, false>(q, v);
                else thin_solve<8, false>(q, v);
            }
            for (int k = 0; k < 9; k++) s_v[k] = v[k];
        }
        __syncthreads();
    } else {
        if (t < 45) {
            int j = 0, k = t, rem = (int)t;
            for (int r = 0; r < 9; r++) {
                if (rem < 9 - r) {
                    j = r;
                    k = r + rem;
                    break;
                }
                rem -= 9 - r;
            }
            double acc = 0.0;
            for (uint32_t c = 0; c < nblocks; c++) acc += partial[(size_t)c * 45 + t];
            A[j][k] = acc;
            A[k][j] = acc;
        }
        if (t < 9)
            for (int j = 0; j < 9; j++) V[j][t] = (j == (int)t) ? 1.0 : 0.0;
        __syncthreads();
        // round-robin Jacobi (the oracle's sym_eig_min spec): per round the rotations of 4
        // disjoint planes from the matrix at the round's start (lanes 0-3), then all column
        // updates (lane = (row, plane), V alongside), then all row updates (lane = (plane,
        // column)) -- every lane owns disjoint element pairs, 3 barriers per round
        __shared__ double s_cs[4][2];
        __shared__ int s_on[4];
        for (int sweep = 0; sweep < 50; sweep++) {
            double off = 0.0, diag = 0.0;
            for (int p = 0; p < 9; p++) {
                diag += A[p][p] * A[p][p];
                for (int qq = p + 1; qq < 9; qq++) off += A[p][qq] * A[p][qq];
            }
            if (off <= 1e-30 * diag || off == 0.0) break;
            for (int r = 0; r < 9; r++) {
                if (t < 4) {
                    const int p = kJacobiRounds[r][t][0], qq = kJacobiRounds[r][t][1];
                    const double apq = A[p][qq];
                    s_on[t] = apq != 0.0;
                    if (apq != 0.0) {
                        const double theta = (A[qq][qq] - A[p][p]) / (2.0 * apq);
                        const double tt = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                        const double c = 1.0 / sqrt(tt * tt + 1.0);
                        s_cs[t][0] = c;
                        s_cs[t][1] = tt * c;
                    }
                }
                __syncthreads();
                const int k = (int)t / 9, e = (int)t - 9 * k;  // 36 lanes: plane k, row / column e
                const bool act = t < 36 && s_on[k < 4 ? k : 0];
                int p = 0, qq = 0;
                double c = 0.0, sn = 0.0;
                if (t < 36) {
                    p = kJacobiRounds[r][k][0];
                    qq = kJacobiRounds[r][k][1];
                    c = s_cs[k][0];
                    sn = s_cs[k][1];
                }
                if (act) {  // columns p, q of row e; V likewise
                    const double aip = A[e][p], aiq = A[e][qq];
                    A[e][p] = c * aip - sn * aiq;
                    A[e][qq] = sn * aip + c * aiq;
                    const double vip = V[e][p], viq = V[e][qq];
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
hipError_t launch_nonminimal_batch(hipStream_t st, int estimator, const void *pts, const NmBatch &b) {
    if (b.W == 0) return hipSuccess;
    const dim3 gg((b.nmax + 255) / 256 ? (b.nmax + 255) / 256 : 1, b.W);
    if (estimator == USAC_LINE2D) {
        float2 *q = static_cast<float2 *>(b.q);
        hipLaunchKernelGGL(k_gather<float2>, gg, dim3(256), 0, st, static_cast<const float2 *>(pts), b.base,
                           b.base_stride, b.pos, b.pos_stride, b.ns, b.n1, q, b.q_stride);
        hipLaunchKernelGGL(k_line_pca, dim3(b.W), dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.model_out, b.ok);
        return hipGetLastError();
    }
    float4 *q = static_cast<float4 *>(b.q);
    hipLaunchKernelGGL(k_gather<float4>, gg, dim3(256), 0, st, static_cast<const float4 *>(pts), b.base,
                       b.base_stride, b.pos, b.pos_stride, b.ns, b.n1, q, b.q_stride);
    hipLaunchKernelGGL(k_normalize, dim3(b.W), dim3(256), 0, st, q, b.q_stride, b.ns, b.n1, b.ws);
    const uint32_t nblk = (b.nmax + kAtaBlock - 1) / kAtaBlock;
    const dim3 ga(nblk ? (nblk + 63) / 64 : 1, b.W);
    if (estimator == USAC_HOMOGRAPHY) {
        hipLaunchKernelGGL(k_ata_partial<false>, ga, dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.partial, b.p_stride);
        hipLaunchKernelGGL(k_dlt_finish<false>, dim3(b.W), dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.partial,
                           b.p_stride, b.ws, b.model_out, b.ok);
    } else {
        hipLaunchKernelGGL(k_ata_partial<true>, ga, dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.partial, b.p_stride);
        hipLaunchKernelGGL(k_dlt_finish<true>, dim3(b.W), dim3(64), 0, st, q, b.q_stride, b.ns, b.n1, b.partial,
                           b.p_stride, b.ws, b.model_out, b.ok);
    }
    return hipGetLastError();
}

size_t nonminimal_partial_stride(uint32_t nmax) { return 45 * ((size_t)nmax / kAtaBlock + 2); }

}  // namespace usac
