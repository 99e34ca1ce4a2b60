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
#include "usac_device_e5.hpp"
#include "usac_kernels.h"

namespace usac {

template <class P>
__global__ __launch_bounds__(256) void k_gather(const P *__restrict__ pts, const uint32_t *__restrict__ idx, uint32_t n,
                                                P *__restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = pts[idx[i]];
}

// EST: 1 line (float2 points, models [3][stride]), 2 homography (float4, [18][stride]: H, H^-1),
// 3 fundamental / 4 essential (float4, [9][stride]).  Lane = one model row; with `list` the rows are
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
            } else if constexpr (EST == 3) {
                const float4 p = static_cast<const float4 *>(pool_pts)[p0 + b];
                e = fundamental_error(m, p.x, p.y, p.z, p.w);
            } else {
                const float4 p = static_cast<const float4 *>(pool_pts)[p0 + b];
                e = essential_error(m, p.x, p.y, p.z, p.w);
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
        case USAC_ESSENTIAL:
            hipLaunchKernelGGL(k_pool_mask<4>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax,
                               thr, words, row_stride);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace usac

namespace usac {

// Throughput SPRT ("batch-native"): every model of a batch is verified with
// the same test (log A, log(delta/eps), log((1-delta)/(1-eps)) fixed for the batch, from
// the host's current SPRT history), walking the pool-ordered points from a wave-uniform
// start (pool position (block * 7919) mod n, wrapping) -- the reference's rolling pool
// index places each model's test at an arbitrary pool position too.  The log-likelihood
// ratio L is accumulated in fp32; a model is rejected at the first point where L > log A
// (count -1, never a best).  A model that passes all n points is accepted: count = its
// inliers over all points (the reference's `tested_inliers`), score = (float)count
// (sprt.hpp:276-281).
//
// Two phases, because nearly every model is rejected within a few dozen points while the
// few good ones must walk all n:
//   phase 1 (lanes = models): the first kHead pool points, wave exit once all lanes
//            decided; lanes still undecided are appended to a survivor list with (L, count);
//   phase 2 (a workgroup per survivor, lanes = points): the remaining points split into
//            256 contiguous chunks; each thread reduces its chunk to (count, ΣΔL, max prefix
//            of ΔL); thread 0 combines the chunks in pool order -- rejected iff some prefix
//            exceeds log A, the sequential test re-associated (fp32).
// kHead = 64 (round 3; was 256): a wave of phase 1 runs until its last lane decides, and on
// cfg3 most waves hold one of the few good models, so the head is as long as the wave walks;
// 64 points reject nearly every bad model and the survivors' tails run in parallel
// (cfg3 883-894 -> 1065-1069 M hyp/s same-box; 32: 961-1088)
constexpr uint32_t kHead = 64;

template <int EST>
__device__ __forceinline__ float sprt_error(const float *m, const void *pts, uint32_t p) {
    if constexpr (EST == 1) {
        const float2 q = static_cast<const float2 *>(pts)[p];
        return line2d_error(m[0], m[1], m[2], q.x, q.y);
    } else if constexpr (EST == 2) {
        const float4 q = static_cast<const float4 *>(pts)[p];
        return homography_error(m, m + 9, q.x, q.y, q.z, q.w);
    } else if constexpr (EST == 3) {
        const float4 q = static_cast<const float4 *>(pts)[p];
        return fundamental_error(m, q.x, q.y, q.z, q.w);
    } else {
        const float4 q = static_cast<const float4 *>(pts)[p];
        return essential_error(m, q.x, q.y, q.z, q.w);
    }
}

struct SprtSurvivor {
    uint32_t slot, start;  // model slot, pool position where phase 2 begins
    float L;
    int cnt;
};

template <int EST>
__global__ __launch_bounds__(64) void k_sprt_head(const void *__restrict__ pool_pts, uint32_t n,
                                                  const float *__restrict__ models, size_t stride,
                                                  const uint32_t *__restrict__ list,
                                                  const uint32_t *__restrict__ list_n, uint32_t kmax, float thr,
                                                  float log_up, float log_down, float log_A,
                                                  int32_t *__restrict__ counts, float *__restrict__ sums,
                                                  uint32_t *__restrict__ tested_total, SprtSurvivor *__restrict__ surv,
                                                  uint32_t *__restrict__ surv_n) {
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
    const uint32_t start = (uint32_t)(((uint64_t)blockIdx.x * 7919u) % n);
    const uint32_t head = n < kHead ? n : kHead;
    float L = 0.f;
    int cnt = 0;
    bool live = row < K;
    uint32_t tested = 0;
    uint32_t p = start;
    for (uint32_t t = 0; t < head; t += 4) {
        // four independent residuals per step (pool positions wave-uniform: scalar loads)
        float e[4];
        uint32_t q = p;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            e[u] = t + u < head ? sprt_error<EST>(m, pool_pts, q) : __builtin_nanf("");
            if (++q == n) q = 0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (live && t + u < head) {
                const bool in = e[u] < thr;
                cnt += in ? 1 : 0;
                L += in ? log_up : log_down;
                tested++;
                if (L > log_A) live = false;
            }
        }
        p = q;
        if (!__any(live)) break;
    }
    if (row < K) {
        if (!live) {
            counts[slot] = -1;
            sums[slot] = 0.f;
        } else if (head == n) {
            counts[slot] = cnt;
            sums[slot] = (float)cnt;
        } else {
            const uint32_t k = atomicAdd(surv_n, 1u);
            surv[k] = SprtSurvivor{slot, (start + head) % n, L, cnt};
        }
    }
    uint32_t v = row < K ? tested : 0;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (threadIdx.x == 0 && tested_total) atomicAdd(tested_total, v);
}

template <int EST>
__global__ __launch_bounds__(256) void k_sprt_tail(const void *__restrict__ pool_pts, uint32_t n,
                                                   const float *__restrict__ models, size_t stride, float thr,
                                                   float log_up, float log_down, float log_A,
                                                   const SprtSurvivor *__restrict__ surv,
                                                   const uint32_t *__restrict__ surv_n, int32_t *__restrict__ counts,
                                                   float *__restrict__ sums, uint32_t *__restrict__ tested_total) {
    constexpr int NC = EST == 1 ? 3 : EST == 2 ? 18 : 9;
    __shared__ int s_cnt[256];
    __shared__ float s_sum[256], s_max[256];
    const uint32_t ns = *surv_n;
    const uint32_t rest = n - kHead;  // launched only when n > kHead
    const uint32_t per = (rest + 255) / 256;
    for (uint32_t k = blockIdx.x; k < ns; k += gridDim.x) {
        const SprtSurvivor sv = surv[k];
        float m[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) m[c] = models[(size_t)c * stride + sv.slot];
        const uint32_t b = threadIdx.x * per;
        const uint32_t e = b + per < rest ? b + per : rest;
        int cnt = 0;
        float acc = 0.f, mx = -INFINITY;
        uint32_t p = sv.start + (b < rest ? b : rest);
        if (p >= n) p -= n;
        for (uint32_t t = b; t < e; t++) {
            const bool in = sprt_error<EST>(m, pool_pts, p) < thr;
            cnt += in ? 1 : 0;
            acc += in ? log_up : log_down;
            mx = fmaxf(mx, acc);
            if (++p == n) p = 0;
        }
        s_cnt[threadIdx.x] = cnt;
        s_sum[threadIdx.x] = acc;
        s_max[threadIdx.x] = mx;
        __syncthreads();
        if (threadIdx.x < 64) {
            // the chunks combined in pool order by wave 0: lane l holds chunks 4l..4l+3 in
            // registers (one LDS round trip), and the sequential walk reads them with
            // v_readlane (wave-uniform lane index) instead of three dependent LDS reads per
            // chunk; every lane runs the same fp32 chain as a single thread did
            const uint32_t l = threadIdx.x;
            int rc[4];
            float rs[4], rm[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                rc[u] = s_cnt[4 * l + u];
                rs[u] = s_sum[4 * l + u];
                rm[u] = s_max[4 * l + u];
            }
            float L = sv.L;
            int c = sv.cnt;
            bool good = true, end = false;
            uint32_t tested = kHead;
            for (int src = 0; src < 64 && !end; src++) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t j = 4 * src + u;
                    const uint32_t cb = j * per, ce = cb + per < rest ? cb + per : rest;
                    if (cb >= ce) {
                        end = true;
                        break;
                    }
                    const float mj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rm[u]), src));
                    if (L + mj > log_A) {  // rejected inside chunk j
                        good = false;
                        tested += ce - cb;  // upper bound of the points the sequential test reads
                        end = true;
                        break;
                    }
                    L += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rs[u]), src));
                    c += __builtin_amdgcn_readlane(rc[u], src);
                    tested += ce - cb;
                }
            }
            if (l == 0) {
                counts[sv.slot] = good ? c : -1;
                sums[sv.slot] = good ? (float)c : 0.f;
                if (tested_total) atomicAdd(tested_total, tested - kHead);
            }
        }
        __syncthreads();
    }
}

hipError_t launch_score_sprt(hipStream_t st, int estimator, const void *pool_pts, uint32_t n, const float *models,
                             size_t stride, const uint32_t *list, const uint32_t *list_n, uint32_t kmax, float thr,
                             float log_up, float log_down, float log_A, int32_t *counts, float *sums,
                             uint32_t *tested_total, void *surv, uint32_t *surv_n) {
    hipError_t err = hipMemsetAsync(surv_n, 0, sizeof(uint32_t), st);
    if (err != hipSuccess) return err;
    const dim3 grid((kmax + 63) / 64);
    SprtSurvivor *sv = static_cast<SprtSurvivor *>(surv);
    const dim3 tgrid(kmax < 2048 ? (kmax ? kmax : 1) : 2048);
#define SS(E)                                                                                                         \
    do {                                                                                                              \
        hipLaunchKernelGGL(k_sprt_head<E>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax, thr, \
                           log_up, log_down, log_A, counts, sums, tested_total, sv, surv_n);                          \
        if (n > kHead)                                                                                                \
            hipLaunchKernelGGL(k_sprt_tail<E>, tgrid, dim3(256), 0, st, pool_pts, n, models, stride, thr, log_up,    \
                               log_down, log_A, sv, surv_n, counts, sums, tested_total);                             \
    } while (0)
    switch (estimator) {
        case USAC_LINE2D: SS(1); break;
        case USAC_HOMOGRAPHY: SS(2); break;
        case USAC_FUNDAMENTAL: SS(3); break;
        case USAC_ESSENTIAL: SS(4); break;
        default: return hipErrorInvalidValue;
    }
#undef SS
    return hipGetLastError();
}

size_t sprt_survivor_bytes() { return sizeof(SprtSurvivor); }

}  // namespace usac
