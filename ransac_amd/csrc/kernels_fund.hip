// kernels_fund.hip -- fundamental-matrix hot path: 7-point solve
// with the oriented-constraint filter, compaction of the valid models, Sampson scoring.
//
// Layout (DESIGN.md "Layout", fundamental):
//   models : SoA [9][3B] fp32, slot = 3*b + j for the j-th VALID model of sample b
//            (seven_points.cpp root order), so slot order = the reference loop's model order;
//   counts : int32[3B] per slot, -1 for an empty slot (never a best);
//   list   : uint32[<= 3B] the occupied slots (wave-aggregated atomics, any order) and
//            list_n = their number -- the score kernel walks only these (on cfg3 data ~15 %
//            of samples yield a model that passes the oriented filter).
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_device_e5.hpp"
#include "usac_kernels.h"

namespace usac {

// SevenPointsAlgorithm + EstimateModel validity filter for one sample per lane:
// 7 x 9 fp64 rows -> row Jacobi -> null complement (f1, f2) -> fp32 cubic coefficients ->
// IEEE cubic roots -> F per root -> oriented filter -> slot write + compaction.
__global__ __launch_bounds__(64) void k_solve_f7(const float4 *__restrict__ pts, uint32_t n,
                                                 const int32_t *__restrict__ samples_in, int32_t *samples_out,
                                                 uint32_t B, uint64_t seed, uint64_t first_hyp,
                                                 float *__restrict__ models, int32_t *__restrict__ counts,
                                                 uint32_t *__restrict__ list, uint32_t *__restrict__ list_n) {
    const uint32_t lane = threadIdx.x;
    const uint32_t h = blockIdx.x * 64 + lane;
    const bool active = h < B;
    const size_t stride = 3 * (size_t)B;
    int nvalid = 0;
    if (active) {
        int32_t s[7];
        if (samples_in) {
#pragma unroll
            for (int i = 0; i < 7; i++) s[i] = samples_in[7 * (size_t)h + i];
        } else {
            draw_sample<7>(seed, first_hyp + h, n, s);
            if (samples_out) {
#pragma unroll
                for (int i = 0; i < 7; i++) samples_out[7 * (size_t)h + i] = s[i];
            }
        }
        double W[7][9];
#pragma unroll
        for (int i = 0; i < 7; i++) {
            const float4 p = pts[s[i]];
            fund_row(p.x, p.y, p.z, p.w, W[i]);
        }
        row_jacobi<7>(W);
        double N[2][9];
        null_complement7(W, N);
        float f1[9], f2[9];
#pragma unroll
        for (int k = 0; k < 9; k++) {
            f1[k] = (float)N[0][k];
            f2[k] = (float)N[1][k];
        }
        float c[4];
        fund_cubic(f1, f2, c);
        double r[3];
        const int nr = cubic_roots((double)c[0], (double)c[1], (double)c[2], (double)c[3], r);
        for (int j = 0; j < nr; j++) {
            float F[9];
            fund_from_root(f1, f2, (float)r[j], F);
            if (fund_oriented(F, pts, s)) {
                const size_t slot = 3 * (size_t)h + nvalid;
#pragma unroll
                for (int k = 0; k < 9; k++) models[(size_t)k * stride + slot] = F[k];
                nvalid++;
            }
        }
        for (int j = 0; j < 3; j++) counts[3 * (size_t)h + j] = j < nvalid ? 0 : -1;
    }
    // wave-aggregated compaction of the occupied slots
    uint32_t incl = (uint32_t)nvalid;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += v;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    uint32_t base = 0;
    if (lane == 63 && total) base = atomicAdd(list_n, total);
    base = __shfl(base, 63, 64);
    const uint32_t excl = base + incl - (uint32_t)nvalid;
    for (int j = 0; j < nvalid; j++) list[excl + j] = 3 * h + (uint32_t)j;
}

// Host-provided models (K x 9 row-major) -> SoA [9][K], identity list.
__global__ __launch_bounds__(256) void k_prepare_f(const float *__restrict__ in, uint32_t K,
                                                   float *__restrict__ models) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= K) return;
#pragma unroll
    for (int k = 0; k < 9; k++) models[(size_t)k * K + h] = in[9 * (size_t)h + k];
}

// Sampson scoring, lanes = models.  With `list` the lanes walk list[0 .. *list_n) and the
// results land at the listed slots; without it lane i is slot i < kmax.  Points are
// wave-uniform scalar loads; per lane the count and the Σerr are accumulated in point
// order (exact sequential sums with CHUNKS == 1).
// EST = USAC_FUNDAMENTAL (Sampson) or USAC_ESSENTIAL (mean epipolar distance)
template <int EST>
__device__ __forceinline__ float two_view_error(const float *f, float x1, float y1, float x2, float y2) {
    if constexpr (EST == USAC_ESSENTIAL) return essential_error(f, x1, y1, x2, y2);
    else return fundamental_error(f, x1, y1, x2, y2);
}

template <int CHUNKS, int EST>
__global__ __launch_bounds__(64 * CHUNKS) void k_score_f(const float4 *__restrict__ pts, uint32_t n,
                                                         const float *__restrict__ models, size_t stride,
                                                         const uint32_t *__restrict__ list,
                                                         const uint32_t *__restrict__ list_n, uint32_t kmax, float thr,
                                                         int32_t *__restrict__ counts, float *__restrict__ sums) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t K = list ? __builtin_amdgcn_readfirstlane(*list_n) : kmax;
    const uint32_t i0 = blockIdx.x * 64;
    if (i0 >= K) return;  // block-uniform
    const uint32_t i = i0 + lane;
    const uint32_t ic = i < K ? i : K - 1;
    const uint32_t slot = list ? list[ic] : ic;
    float f[9];
#pragma unroll
    for (int k = 0; k < 9; k++) f[k] = models[(size_t)k * stride + slot];
    const uint32_t per = (n + CHUNKS - 1) / CHUNKS;
    const uint32_t begin = wave * per < n ? wave * per : n;
    const uint32_t end = begin + per < n ? begin + per : n;
    int cnt = 0;
    float sum = 0.f;
    uint32_t p = begin;
    for (; p + 4 <= end; p += 4) {
        const float4 a0 = pts[p], a1 = pts[p + 1], a2 = pts[p + 2], a3 = pts[p + 3];
        const float e0 = two_view_error<EST>(f, a0.x, a0.y, a0.z, a0.w);
        const float e1 = two_view_error<EST>(f, a1.x, a1.y, a1.z, a1.w);
        const float e2 = two_view_error<EST>(f, a2.x, a2.y, a2.z, a2.w);
        const float e3 = two_view_error<EST>(f, a3.x, a3.y, a3.z, a3.w);
        if (e0 < thr) { cnt++; sum += e0; }
        if (e1 < thr) { cnt++; sum += e1; }
        if (e2 < thr) { cnt++; sum += e2; }
        if (e3 < thr) { cnt++; sum += e3; }
    }
    for (; p < end; p++) {
        const float4 a = pts[p];
        const float e = two_view_error<EST>(f, a.x, a.y, a.z, a.w);
        if (e < thr) { cnt++; sum += e; }
    }
    if constexpr (CHUNKS == 1) {
        if (i < K) {
            counts[slot] = cnt;
            sums[slot] = sum;
        }
    } else {
        __shared__ int s_cnt[CHUNKS][64];
        __shared__ float s_sum[CHUNKS][64];
        s_cnt[wave][lane] = cnt;
        s_sum[wave][lane] = sum;
        __syncthreads();
        if (wave == 0 && i < K) {
            int c = s_cnt[0][lane];
            float s = s_sum[0][lane];
#pragma unroll
            for (int w = 1; w < CHUNKS; w++) {
                c += s_cnt[w][lane];
                s += s_sum[w][lane];
            }
            counts[slot] = c;
            sums[slot] = s;
        }
    }
}

hipError_t launch_solve_f7(hipStream_t st, const float4 *pts, uint32_t n, const int32_t *samples_in,
                           int32_t *samples_out, uint32_t B, uint64_t seed, uint64_t first_hyp, float *models,
                           int32_t *counts, uint32_t *list, uint32_t *list_n) {
    hipError_t e = hipMemsetAsync(list_n, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_solve_f7, dim3((B + 63) / 64), dim3(64), 0, st, pts, n, samples_in, samples_out, B, seed,
                       first_hyp, models, counts, list, list_n);
    return hipGetLastError();
}

hipError_t launch_prepare_f(hipStream_t st, const float *in, uint32_t K, float *models) {
    hipLaunchKernelGGL(k_prepare_f, dim3((K + 255) / 256), dim3(256), 0, st, in, K, models);
    return hipGetLastError();
}

hipError_t launch_score_f(hipStream_t st, int estimator, int chunks, const float4 *pts, uint32_t n,
                          const float *models, size_t stride, const uint32_t *list, const uint32_t *list_n,
                          uint32_t kmax, float thr, int32_t *counts, float *sums) {
    const dim3 grid((kmax + 63) / 64);
#define SF(C, E)                                                                                                   \
    hipLaunchKernelGGL((k_score_f<C, E>), grid, dim3(64 * C), 0, st, pts, n, models, stride, list, list_n, kmax, thr, \
                       counts, sums)
    const bool ess = estimator == USAC_ESSENTIAL;
    switch (chunks) {
        case 1: if (ess) SF(1, USAC_ESSENTIAL); else SF(1, USAC_FUNDAMENTAL); break;
        case 2: if (ess) SF(2, USAC_ESSENTIAL); else SF(2, USAC_FUNDAMENTAL); break;
        case 4: if (ess) SF(4, USAC_ESSENTIAL); else SF(4, USAC_FUNDAMENTAL); break;
        case 8: if (ess) SF(8, USAC_ESSENTIAL); else SF(8, USAC_FUNDAMENTAL); break;
        default: return hipErrorInvalidValue;
    }
#undef SF
    return hipGetLastError();
}

}  // namespace usac
