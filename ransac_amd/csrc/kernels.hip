// kernels.hip -- HIP kernels of the hypothesize-and-verify hot path (gfx950 / CDNA4).
//
// Data layout in HBM (DESIGN.md "Layout"):
//   points   : N x float4 {x1,y1,x2,y2} (two-view) or N x float2 {x,y} (line), read-only,
//              L2/LDS resident (160 KB at N = 10k);
//   samples  : B x m int32;
//   models   : SoA [18][B] fp32 -- H (9) then H^-1 (9) per hypothesis, so lane h reads
//              component c at models[c*B + h] (coalesced);
//   scores   : counts int32[B], sums fp32[B].
//
// Scoring maps LANES TO HYPOTHESES: each wave owns 64 hypotheses and walks the points in
// order; a point is wave-uniform, so it arrives by scalar loads into SGPRs and feeds the
// VALU as a scalar operand (no LDS, no VGPR staging, one 16 B load shared by 64
// hypotheses).  Each lane's inlier count and Σerr are accumulated in point order, so with
// one chunk per hypothesis the sum is bit-identical to the reference's sequential fp32 sum
// (quality.hpp:89-96).  `CHUNKS` waves of a workgroup split the point range of the same 64
// hypotheses for occupancy; their partial sums are then combined in chunk order.
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_kernels.h"

namespace usac {

// ------------------------------------------------------------------------ solve (H, 4-pt)
__global__ __launch_bounds__(64) void k_solve_h4(const float4 *__restrict__ pts, uint32_t n,
                                                 const int32_t *__restrict__ samples_in, int32_t *samples_out,
                                                 uint32_t B, uint64_t seed, uint64_t first_hyp, int nullspace,
                                                 float *__restrict__ models) {
    const uint32_t h = blockIdx.x * 64 + threadIdx.x;
    if (h >= B) return;
    int32_t s[4];
    if (samples_in) {
#pragma unroll
        for (int i = 0; i < 4; i++) s[i] = samples_in[4 * (size_t)h + i];
    } else {
        draw_sample<4>(seed, first_hyp + h, n, s);
        if (samples_out) {
#pragma unroll
            for (int i = 0; i < 4; i++) samples_out[4 * (size_t)h + i] = s[i];
        }
    }
    double W[8][9];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float4 p = pts[s[i]];
        dlt_rows(p.x, p.y, p.z, p.w, W[2 * i], W[2 * i + 1]);
    }
    row_jacobi<8>(W);
    double v[9];
    pick_vector<8>(W, nullspace, v);
    float H[9], Hi[9];
#pragma unroll
    for (int k = 0; k < 9; k++) H[k] = (float)(v[k] / v[8]);
    inv3x3(H, Hi);
#pragma unroll
    for (int k = 0; k < 9; k++) {
        models[(size_t)k * B + h] = H[k];
        models[(size_t)(9 + k) * B + h] = Hi[k];
    }
}

// Host-provided models (B x 9, row-major) -> SoA H / H^-1.
__global__ __launch_bounds__(256) void k_prepare_h(const float *__restrict__ in, uint32_t B,
                                                   float *__restrict__ models) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
    float H[9], Hi[9];
#pragma unroll
    for (int k = 0; k < 9; k++) H[k] = in[9 * (size_t)h + k];
    inv3x3(H, Hi);
#pragma unroll
    for (int k = 0; k < 9; k++) {
        models[(size_t)k * B + h] = H[k];
        models[(size_t)(9 + k) * B + h] = Hi[k];
    }
}

// ------------------------------------------------------------------------ score (H)
template <int CHUNKS>
__global__ __launch_bounds__(64 * CHUNKS) void k_score_h(const float4 *__restrict__ pts, uint32_t n,
                                                         const float *__restrict__ models, uint32_t B, float thr,
                                                         int32_t *__restrict__ counts, float *__restrict__ sums) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t h = blockIdx.x * 64 + lane;
    const uint32_t hc = h < B ? h : B - 1;
    float H[9], Hi[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
        H[k] = models[(size_t)k * B + hc];
        Hi[k] = models[(size_t)(9 + k) * B + hc];
    }
    const uint32_t per = (n + CHUNKS - 1) / CHUNKS;
    const uint32_t begin = wave * per;
    const uint32_t end = begin + per < n ? begin + per : n;
    int cnt = 0;
    float sum = 0.f;
    for (uint32_t i = begin; i < end; ++i) {
        const float4 p = pts[i];
        const float err = homography_error(H, Hi, p.x, p.y, p.z, p.w);
        if (err < thr) {
            cnt++;
            sum += err;
        }
    }
    if constexpr (CHUNKS == 1) {
        if (h < B) {
            counts[h] = cnt;
            sums[h] = sum;
        }
    } else {
        __shared__ int s_cnt[CHUNKS][64];
        __shared__ float s_sum[CHUNKS][64];
        s_cnt[wave][lane] = cnt;
        s_sum[wave][lane] = sum;
        __syncthreads();
        if (wave == 0 && h < B) {
            int c = s_cnt[0][lane];
            float s = s_sum[0][lane];
#pragma unroll
            for (int w = 1; w < CHUNKS; w++) {
                c += s_cnt[w][lane];
                s += s_sum[w][lane];
            }
            counts[h] = c;
            sums[h] = s;
        }
    }
}

// ------------------------------------------------------------------------ score (H), fast path
// Point records for the fast kernel: 32 B per point, rec[2i] = {x1, x2, y1, y2} (pairs
// the two directions' coordinates for packed fp32 math), rec[2i+1].x = guard band for the
// current threshold.  Built once per context (+ once per new threshold).
__global__ __launch_bounds__(256) void k_prepare_rec(const float4 *__restrict__ pts, uint32_t n, float T,
                                                     float4 *__restrict__ rec) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 p = pts[i];
    const float mp = fabsf(p.x) + fabsf(p.y) + fabsf(p.z) + fabsf(p.w);
    rec[2 * i] = make_float4(p.x, p.z, p.y, p.w);
    rec[2 * i + 1] = make_float4(kBandMp * mp + kBandT * T, 0.f, 0.f, 0.f);
}

typedef float f2 __attribute__((ext_vector_type(2)));

// Lanes = hypotheses, points wave-uniform (scalar loads).  Per point and wave: the six
// projections as three packed fp32 pairs (forward, backward), two v_rcp, two packed
// quotient products, packed differences, two v_sqrt -- ~30 VALU issue slots for 64
// (hypothesis, point) pairs -- then the guard-band test; lanes inside the band (or with
// a non-finite fast value) re-evaluate the exact reference expression.  EXACT_SUM also
// routes every inlier through the exact expression so Σerr is the reference's
// sequential fp32 sum (parity mode); otherwise Σerr accumulates the fast values
// (throughput mode; counts are exact either way).
template <int CHUNKS, bool EXACT_SUM>
__global__ __launch_bounds__(64 * CHUNKS) void k_score_hf(const float4 *__restrict__ rec, uint32_t n,
                                                          const float *__restrict__ models, uint32_t B, float thr,
                                                          int32_t *__restrict__ counts, float *__restrict__ sums) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t h = blockIdx.x * 64 + lane;
    const uint32_t hc = h < B ? h : B - 1;
    f2 P[9];
#pragma unroll
    for (int k = 0; k < 9; k++) P[k] = f2{models[(size_t)k * B + hc], models[(size_t)(9 + k) * B + hc]};
    const float T = 2.0f * thr;
    const uint32_t per = (n + CHUNKS - 1) / CHUNKS;
    const uint32_t begin = wave * per;
    const uint32_t end = begin + per < n ? begin + per : n;
    int cnt = 0;
    float sum = 0.f;
#pragma unroll 2
    for (uint32_t i = begin; i < end; ++i) {
        const float4 a = rec[2 * i];
        const float band = rec[2 * i + 1].x;
        const f2 X = f2{a.x, a.y};   // (x1, x2)
        const f2 Y = f2{a.z, a.w};   // (y1, y2)
        // (forward, backward) projections, reference operation order, no contraction
        const f2 NX = (P[0] * X + P[1] * Y) + P[2];
        const f2 NY = (P[3] * X + P[4] * Y) + P[5];
        const f2 NZ = (P[6] * X + P[7] * Y) + P[8];
        const f2 R = f2{__builtin_amdgcn_rcpf(NZ.x), __builtin_amdgcn_rcpf(NZ.y)};
        const f2 DX = X.yx - NX * R;  // (x2 - q2x, x1 - q1x)
        const f2 DY = Y.yx - NY * R;
        const f2 D = DX * DX + DY * DY;
        const float S = __builtin_amdgcn_sqrtf(D.x) + __builtin_amdgcn_sqrtf(D.y);
        const float diff = S - T;
        const bool sure = (fabsf(diff) > band) & (S < INFINITY);
        bool inl = sure & (diff < 0.f);
        float add = S;
        const bool need = EXACT_SUM ? (!sure || inl) : !sure;
        if (need) {
            float Hh[9], Hi[9];
#pragma unroll
            for (int k = 0; k < 9; k++) {
                Hh[k] = P[k].x;
                Hi[k] = P[k].y;
            }
            const float e = homography_error(Hh, Hi, a.x, a.z, a.y, a.w);
            inl = e < thr;
            add = EXACT_SUM ? e : e + e;
        }
        if (inl) {
            cnt++;
            sum += add;
        }
    }
    if (!EXACT_SUM) sum *= 0.5f;
    if constexpr (CHUNKS == 1) {
        if (h < B) {
            counts[h] = cnt;
            sums[h] = sum;
        }
    } else {
        __shared__ int s_cnt[CHUNKS][64];
        __shared__ float s_sum[CHUNKS][64];
        s_cnt[wave][lane] = cnt;
        s_sum[wave][lane] = sum;
        __syncthreads();
        if (wave == 0 && h < B) {
            int c = s_cnt[0][lane];
            float s = s_sum[0][lane];
#pragma unroll
            for (int w = 1; w < CHUNKS; w++) {
                c += s_cnt[w][lane];
                s += s_sum[w][lane];
            }
            counts[h] = c;
            sums[h] = s;
        }
    }
}

// ------------------------------------------------------------------------ line2d
__global__ __launch_bounds__(256) void k_solve_line(const float2 *__restrict__ pts, uint32_t n,
                                                    const int32_t *__restrict__ samples_in, int32_t *samples_out,
                                                    uint32_t B, uint64_t seed, uint64_t first_hyp,
                                                    float *__restrict__ models) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
    int32_t s[2];
    if (samples_in) {
        s[0] = samples_in[2 * (size_t)h];
        s[1] = samples_in[2 * (size_t)h + 1];
    } else {
        draw_sample<2>(seed, first_hyp + h, n, s);
        if (samples_out) {
            samples_out[2 * (size_t)h] = s[0];
            samples_out[2 * (size_t)h + 1] = s[1];
        }
    }
    const float2 p1 = pts[s[0]], p2 = pts[s[1]];
    float m[3];
    line2d_estimate(p1.x, p1.y, p2.x, p2.y, m);
#pragma unroll
    for (int k = 0; k < 3; k++) models[(size_t)k * B + h] = m[k];
}

__global__ __launch_bounds__(256) void k_prepare_line(const float *__restrict__ in, uint32_t B,
                                                      float *__restrict__ models) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
#pragma unroll
    for (int k = 0; k < 3; k++) models[(size_t)k * B + h] = in[9 * (size_t)h + k];
}

template <int CHUNKS>
__global__ __launch_bounds__(64 * CHUNKS) void k_score_line(const float2 *__restrict__ pts, uint32_t n,
                                                            const float *__restrict__ models, uint32_t B, float thr,
                                                            int32_t *__restrict__ counts, float *__restrict__ sums) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t h = blockIdx.x * 64 + lane;
    const uint32_t hc = h < B ? h : B - 1;
    const float a = models[hc], b = models[(size_t)B + hc], c = models[2 * (size_t)B + hc];
    const uint32_t per = (n + CHUNKS - 1) / CHUNKS;
    const uint32_t begin = wave * per;
    const uint32_t end = begin + per < n ? begin + per : n;
    int cnt = 0;
    float sum = 0.f;
    for (uint32_t i = begin; i < end; ++i) {
        const float2 p = pts[i];
        const float err = line2d_error(a, b, c, p.x, p.y);
        if (err < thr) {
            cnt++;
            sum += err;
        }
    }
    if constexpr (CHUNKS == 1) {
        if (h < B) {
            counts[h] = cnt;
            sums[h] = sum;
        }
    } else {
        __shared__ int s_cnt[CHUNKS][64];
        __shared__ float s_sum[CHUNKS][64];
        s_cnt[wave][lane] = cnt;
        s_sum[wave][lane] = sum;
        __syncthreads();
        if (wave == 0 && h < B) {
            int cc = s_cnt[0][lane];
            float ss = s_sum[0][lane];
#pragma unroll
            for (int w = 1; w < CHUNKS; w++) {
                cc += s_cnt[w][lane];
                ss += s_sum[w][lane];
            }
            counts[h] = cc;
            sums[h] = ss;
        }
    }
}

// ------------------------------------------------------------------------ batch argmax
// One workgroup: strided scan + LDS tree under record_better (a strict total order, so
// the reduction order does not change the result).
__global__ __launch_bounds__(1024) void k_argmax(const int32_t *__restrict__ counts, const float *__restrict__ sums,
                                                 uint32_t B, const float *__restrict__ models, int ncomp,
                                                 uint64_t first_hyp, usac_record *out) {
    __shared__ int s_c[1024];
    __shared__ float s_s[1024];
    __shared__ uint32_t s_i[1024];
    const uint32_t t = threadIdx.x;
    int bc = -1;
    float bs = 0.f;
    uint32_t bi = 0xFFFFFFFFu;
    for (uint32_t i = t; i < B; i += 1024) {
        int c = counts[i];
        float s = sums[i];
        if (bc < 0 || record_better(c, s, i, bc, bs, bi)) {
            bc = c;
            bs = s;
            bi = i;
        }
    }
    s_c[t] = bc;
    s_s[t] = bs;
    s_i[t] = bi;
    __syncthreads();
    for (uint32_t w = 512; w > 0; w >>= 1) {
        if (t < w) {
            int c2 = s_c[t + w];
            if (c2 >= 0 && (s_c[t] < 0 || record_better(c2, s_s[t + w], s_i[t + w], s_c[t], s_s[t], s_i[t]))) {
                s_c[t] = c2;
                s_s[t] = s_s[t + w];
                s_i[t] = s_i[t + w];
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        usac_record r;
        const uint32_t i = s_i[0];
        r.valid = s_c[0] >= 0 ? 1 : 0;
        r.inliers = s_c[0] < 0 ? 0 : s_c[0];
        r.score = s_s[0];
        r.hyp_index = first_hyp + (i == 0xFFFFFFFFu ? 0 : i);
        for (int k = 0; k < 9; k++) r.model[k] = (k < ncomp && r.valid) ? models[(size_t)k * B + i] : 0.f;
        *out = r;
    }
}

// ------------------------------------------------------------------------ inliers (exact)
// Quality::getNumberInliers(get_inliers=true) for one model: 256 lanes evaluate a tile of
// points, then lane 0 walks the tile in point order -- ascending inlier list and the
// sequential fp32 sum of quality.hpp:80-87.
__global__ __launch_bounds__(256) void k_inliers_h(const float4 *__restrict__ pts, uint32_t n, const float *model,
                                                   float thr, int32_t *idx, int32_t *count, float *sum) {
    __shared__ float s_err[256];
    __shared__ float m[18];
    if (threadIdx.x == 0) {
        for (int k = 0; k < 9; k++) m[k] = model[k];
        inv3x3(m, m + 9);
    }
    __syncthreads();
    float H[9], Hi[9];
    for (int k = 0; k < 9; k++) {
        H[k] = m[k];
        Hi[k] = m[9 + k];
    }
    int cnt = 0;
    float s = 0.f;
    for (uint32_t base = 0; base < n; base += 256) {
        const uint32_t i = base + threadIdx.x;
        float e = 0.f;
        if (i < n) {
            float4 p = pts[i];
            e = homography_error(H, Hi, p.x, p.y, p.z, p.w);
        }
        s_err[threadIdx.x] = e;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t lim = n - base < 256 ? n - base : 256;
            for (uint32_t j = 0; j < lim; j++) {
                const float e2 = s_err[j];
                if (e2 < thr) {
                    idx[cnt++] = (int32_t)(base + j);
                    s += e2;
                }
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *count = cnt;
        *sum = s;
    }
}

__global__ __launch_bounds__(256) void k_inliers_line(const float2 *__restrict__ pts, uint32_t n, const float *model,
                                                      float thr, int32_t *idx, int32_t *count, float *sum) {
    __shared__ float s_err[256];
    const float a = model[0], b = model[1], c = model[2];
    int cnt = 0;
    float s = 0.f;
    for (uint32_t base = 0; base < n; base += 256) {
        const uint32_t i = base + threadIdx.x;
        float e = 0.f;
        if (i < n) {
            float2 p = pts[i];
            e = line2d_error(a, b, c, p.x, p.y);
        }
        s_err[threadIdx.x] = e;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t lim = n - base < 256 ? n - base : 256;
            for (uint32_t j = 0; j < lim; j++) {
                const float e2 = s_err[j];
                if (e2 < thr) {
                    idx[cnt++] = (int32_t)(base + j);
                    s += e2;
                }
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *count = cnt;
        *sum = s;
    }
}

// ------------------------------------------------------------------------ launchers
#define LAUNCH_CHECK() hipGetLastError()

hipError_t launch_solve_h4(hipStream_t st, const float4 *pts, uint32_t n, const int32_t *samples_in,
                           int32_t *samples_out, uint32_t B, uint64_t seed, uint64_t first_hyp, int nullspace,
                           float *models) {
    hipLaunchKernelGGL(k_solve_h4, dim3((B + 63) / 64), dim3(64), 0, st, pts, n, samples_in, samples_out, B, seed,
                       first_hyp, nullspace, models);
    return LAUNCH_CHECK();
}

hipError_t launch_prepare_h(hipStream_t st, const float *in, uint32_t B, float *models) {
    hipLaunchKernelGGL(k_prepare_h, dim3((B + 255) / 256), dim3(256), 0, st, in, B, models);
    return LAUNCH_CHECK();
}

hipError_t launch_score_h(hipStream_t st, int chunks, const float4 *pts, uint32_t n, const float *models, uint32_t B,
                          float thr, int32_t *counts, float *sums) {
    dim3 grid((B + 63) / 64);
    switch (chunks) {
        case 1: hipLaunchKernelGGL(k_score_h<1>, grid, dim3(64), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 2: hipLaunchKernelGGL(k_score_h<2>, grid, dim3(128), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 4: hipLaunchKernelGGL(k_score_h<4>, grid, dim3(256), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 8: hipLaunchKernelGGL(k_score_h<8>, grid, dim3(512), 0, st, pts, n, models, B, thr, counts, sums); break;
        default: return hipErrorInvalidValue;
    }
    return LAUNCH_CHECK();
}

hipError_t launch_prepare_rec(hipStream_t st, const float4 *pts, uint32_t n, float thr, float4 *rec) {
    hipLaunchKernelGGL(k_prepare_rec, dim3((n + 255) / 256), dim3(256), 0, st, pts, n, 2.0f * thr, rec);
    return LAUNCH_CHECK();
}

hipError_t launch_score_hf(hipStream_t st, int chunks, bool exact_sum, const float4 *rec, uint32_t n,
                           const float *models, uint32_t B, float thr, int32_t *counts, float *sums) {
    dim3 grid((B + 63) / 64);
#define SHF(C, E) hipLaunchKernelGGL((k_score_hf<C, E>), grid, dim3(64 * C), 0, st, rec, n, models, B, thr, counts, sums)
    if (exact_sum) {
        switch (chunks) {
            case 1: SHF(1, true); break;
            case 2: SHF(2, true); break;
            case 4: SHF(4, true); break;
            case 8: SHF(8, true); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (chunks) {
            case 1: SHF(1, false); break;
            case 2: SHF(2, false); break;
            case 4: SHF(4, false); break;
            case 8: SHF(8, false); break;
            default: return hipErrorInvalidValue;
        }
    }
#undef SHF
    return LAUNCH_CHECK();
}

hipError_t launch_solve_line(hipStream_t st, const float2 *pts, uint32_t n, const int32_t *samples_in,
                             int32_t *samples_out, uint32_t B, uint64_t seed, uint64_t first_hyp, float *models) {
    hipLaunchKernelGGL(k_solve_line, dim3((B + 255) / 256), dim3(256), 0, st, pts, n, samples_in, samples_out, B, seed,
                       first_hyp, models);
    return LAUNCH_CHECK();
}

hipError_t launch_prepare_line(hipStream_t st, const float *in, uint32_t B, float *models) {
    hipLaunchKernelGGL(k_prepare_line, dim3((B + 255) / 256), dim3(256), 0, st, in, B, models);
    return LAUNCH_CHECK();
}

hipError_t launch_score_line(hipStream_t st, int chunks, const float2 *pts, uint32_t n, const float *models,
                             uint32_t B, float thr, int32_t *counts, float *sums) {
    dim3 grid((B + 63) / 64);
    switch (chunks) {
        case 1: hipLaunchKernelGGL(k_score_line<1>, grid, dim3(64), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 2: hipLaunchKernelGGL(k_score_line<2>, grid, dim3(128), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 4: hipLaunchKernelGGL(k_score_line<4>, grid, dim3(256), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 8: hipLaunchKernelGGL(k_score_line<8>, grid, dim3(512), 0, st, pts, n, models, B, thr, counts, sums); break;
        default: return hipErrorInvalidValue;
    }
    return LAUNCH_CHECK();
}

hipError_t launch_argmax(hipStream_t st, const int32_t *counts, const float *sums, uint32_t B, const float *models,
                         int ncomp, uint64_t first_hyp, usac_record *out) {
    hipLaunchKernelGGL(k_argmax, dim3(1), dim3(1024), 0, st, counts, sums, B, models, ncomp, first_hyp, out);
    return LAUNCH_CHECK();
}

hipError_t launch_inliers_h(hipStream_t st, const float4 *pts, uint32_t n, const float *model, float thr,
                            int32_t *idx, int32_t *count, float *sum) {
    hipLaunchKernelGGL(k_inliers_h, dim3(1), dim3(256), 0, st, pts, n, model, thr, idx, count, sum);
    return LAUNCH_CHECK();
}

hipError_t launch_inliers_line(hipStream_t st, const float2 *pts, uint32_t n, const float *model, float thr,
                               int32_t *idx, int32_t *count, float *sum) {
    hipLaunchKernelGGL(k_inliers_line, dim3(1), dim3(256), 0, st, pts, n, model, thr, idx, count, sum);
    return LAUNCH_CHECK();
}

}  // namespace usac
