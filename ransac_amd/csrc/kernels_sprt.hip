// kernels_sprt.hip -- SPRT support (sprt.hpp:191-317) on the device.
//
// Parity path: the reference's SPRT walks a random pool of the points with a rolling
// index shared by all models and an fp64 likelihood ratio whose thresholds change with
// every accepted/rejected model -- an inherently serial walk.  The device supplies what
// the walk reads: for every model of a batch, its inlier flags (exact residual < thr)
// in POOL order, packed as 32-bit words; the host walks them (usac_host.hpp Sprt).
// Points are pre-permuted into pool order once per run so a pool position is a
// contiguous, wave-uniform scalar load.
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_kernels.h"

namespace usac {

template <class P>
__global__ __launch_bounds__(256) void k_gather(const P *__restrict__ pts, const uint32_t *__restrict__ idx, uint32_t n,
                                                P *__restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = pts[idx[i]];
}

// EST: 1 line (float2 points, models [3][stride]), 2 homography (float4, [18][stride]: H, H^-1),
// 3 fundamental (float4, [9][stride]).  Lane = one model row; with `list` the rows are
// list[0 .. *list_n) (model slot list[i] -> row i), else rows are slots 0 .. kmax-1.
// words[w * row_stride + row], bit b = pool position 32 w + b.
template <int EST>
__global__ __launch_bounds__(64) void k_pool_mask(const void *__restrict__ pool_pts, uint32_t n,
                                                  const float *__restrict__ models, size_t stride,
                                                  const uint32_t *__restrict__ list, const uint32_t *__restrict__ list_n,
                                                  uint32_t kmax, float thr, uint32_t *__restrict__ words,
                                                  uint32_t row_stride) {
    constexpr int NC = EST == 1 ? 3 : EST == 2 ? 18 : 9;
    const uint32_t K = list ? __builtin_amdgcn_readfirstlane(*list_n) : kmax;
    const uint32_t i0 = blockIdx.x * 64;
    if (i0 >= K) return;
    const uint32_t row = i0 + threadIdx.x;
    const uint32_t rc = row < K ? row : K - 1;
    const uint32_t slot = list ? list[rc] : rc;
    float m[NC];
#pragma unroll
    for (int k = 0; k < NC; k++) m[k] = models[(size_t)k * stride + slot];
    const uint32_t nw = (n + 31) / 32;
    for (uint32_t w = 0; w < nw; w++) {
        uint32_t bits = 0;
        const uint32_t p0 = 32 * w;
        const uint32_t lim = n - p0 < 32 ? n - p0 : 32;
        for (uint32_t b = 0; b < lim; b++) {
            float e;
            if constexpr (EST == 1) {
                const float2 p = static_cast<const float2 *>(pool_pts)[p0 + b];
                e = line2d_error(m[0], m[1], m[2], p.x, p.y);
            } else if constexpr (EST == 2) {
                const float4 p = static_cast<const float4 *>(pool_pts)[p0 + b];
                e = homography_error(m, m + 9, p.x, p.y, p.z, p.w);
            } else {
                const float4 p = static_cast<const float4 *>(pool_pts)[p0 + b];
                e = fundamental_error(m, p.x, p.y, p.z, p.w);
            }
            bits |= (e < thr ? 1u : 0u) << b;
        }
        if (row < K) words[(size_t)w * row_stride + row] = bits;
    }
}

hipError_t launch_gather_points(hipStream_t st, const void *pts, uint32_t cols, const uint32_t *idx, uint32_t n,
                                void *out) {
    const dim3 grid((n + 255) / 256);
    if (cols == 4)
        hipLaunchKernelGGL(k_gather<float4>, grid, dim3(256), 0, st, static_cast<const float4 *>(pts), idx, n,
                           static_cast<float4 *>(out));
    else if (cols == 2)
        hipLaunchKernelGGL(k_gather<float2>, grid, dim3(256), 0, st, static_cast<const float2 *>(pts), idx, n,
                           static_cast<float2 *>(out));
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_pool_mask(hipStream_t st, int estimator, const void *pool_pts, uint32_t n, const float *models,
                            size_t stride, const uint32_t *list, const uint32_t *list_n, uint32_t kmax, float thr,
                            uint32_t *words, uint32_t row_stride) {
    const dim3 grid((kmax + 63) / 64);
    switch (estimator) {
        case USAC_LINE2D:
            hipLaunchKernelGGL(k_pool_mask<1>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax,
                               thr, words, row_stride);
            break;
        case USAC_HOMOGRAPHY:
            hipLaunchKernelGGL(k_pool_mask<2>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax,
                               thr, words, row_stride);
            break;
        case USAC_FUNDAMENTAL:
            hipLaunchKernelGGL(k_pool_mask<3>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax,
                               thr, words, row_stride);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace usac
