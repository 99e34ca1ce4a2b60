// kernels_inliers.hip -- Quality::getNumberInliers(score, model, thr, get_inliers = true,
// inliers) (quality.hpp:60-101) for ONE model over all N points, exactly: the ascending
// inlier index list, the count, and the reference's sequential fp32 Σerr (point order).
// Used by the polish (ransac.cpp:157-214), LO-RANSAC (inner_local_optimization.hpp:74-133)
// and PROSAC's termination scan.
//
//   k_inl_flags   grid over points: exact residual (kept in scratch), per-block inlier count
//   k_inl_compact grid over points: each block sums the earlier blocks' counts (its output
//                 offset; the last block writes the total), ordered compaction of indices
//                 and residuals                                                 (parallel)
//   seqsum        the sequential fp32 sum over the compacted residuals
//                 (the reference's order; evaluated in parallel, bit-exactly, by launch_seqsum)
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <type_traits>

#include "usac_device.hpp"
#include "usac_device_e5.hpp"
#include "usac_kernels.h"
#include "usac_seqsum.hpp"

namespace usac {

constexpr uint32_t kInlThreads = 256;               // threads per workgroup
constexpr uint32_t kInlPer = 4;                     // points per thread
constexpr uint32_t kInlBlock = kInlThreads * kInlPer;  // points per workgroup (block)

template <int EST>
__device__ __forceinline__ float inl_error(const float *m, const void *pts, uint32_t i) {
    if constexpr (EST == USAC_LINE2D) {
        const float2 p = static_cast<const float2 *>(pts)[i];
        return line2d_error(m[0], m[1], m[2], p.x, p.y);
    } else if constexpr (EST == USAC_HOMOGRAPHY) {
        const float4 p = static_cast<const float4 *>(pts)[i];
        return homography_error(m, m + 9, p.x, p.y, p.z, p.w);
    } else if constexpr (EST == USAC_FUNDAMENTAL) {
        const float4 p = static_cast<const float4 *>(pts)[i];
        return fundamental_error(m, p.x, p.y, p.z, p.w);
    } else {
        const float4 p = static_cast<const float4 *>(pts)[i];
        return essential_error(m, p.x, p.y, p.z, p.w);
    }
}

// the same residual of an already loaded point (k_inl_flags issues its points' loads first)
template <int EST, class P>
__device__ __forceinline__ float inl_error_p(const float *m, const P &p) {
    if constexpr (EST == USAC_LINE2D) return line2d_error(m[0], m[1], m[2], p.x, p.y);
    else if constexpr (EST == USAC_HOMOGRAPHY) return homography_error(m, m + 9, p.x, p.y, p.z, p.w);
    else if constexpr (EST == USAC_FUNDAMENTAL) return fundamental_error(m, p.x, p.y, p.z, p.w);
    else return essential_error(m, p.x, p.y, p.z, p.w);
}

// model parameters of one block (H also needs H^-1: cv::Mat::inv, homography_estimator.hpp:35)
template <int EST>
__device__ __forceinline__ void inl_model(const float *model, float *sm) {
    if (threadIdx.x == 0) {
        for (int k = 0; k < 9; k++) sm[k] = model[k];
        if (EST == USAC_HOMOGRAPHY) inv3x3(sm, sm + 9);
    }
    __syncthreads();
}

// Batched over W models: blockIdx.y = model w (model w at models + 9 w, threshold thrs[w]
// or the scalar thr).  Per model the scratch holds its block counts (nb padded to 64),
// its compacted residuals (n floats) and every point's residual (n floats): inl_stride(n) words.  Every model's
// result is exactly the single-model one (the kernels never mix models).
// The residuals are followed by the model's seqsum scratch (one chain, 8-byte aligned: every
// part of the stride is even).
constexpr size_t kInlSeqWords = seq::scratch_bytes(1) / sizeof(uint32_t);

__host__ __device__ __forceinline__ size_t inl_res_words(uint32_t n) {
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    return (size_t)((nb + 63) & ~63u) + 2 * (size_t)((n + 1) & ~1u);
}
// every point's residual (k_inl_flags writes them, k_inl_compact reads them back instead of
// evaluating the model again), after the compacted residuals
__host__ __device__ __forceinline__ size_t inl_all_offset(uint32_t n) {
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    return (size_t)((nb + 63) & ~63u) + ((n + 1) & ~1u);
}
__host__ __device__ __forceinline__ size_t inl_stride(uint32_t n) { return inl_res_words(n) + kInlSeqWords; }

// model slot of workgroup row b: slots[b] when a slot list is given (a subset of the W models)
__device__ __forceinline__ uint32_t inl_slot(const uint32_t *slots, uint32_t b) { return slots ? slots[b] : b; }

// Blocks of kInlBlock points in point order: thread t of block b takes points
// b * kInlBlock + u * kInlThreads + t, u = 0 .. kInlPer - 1, so (u, wave, lane) is point order.
template <int EST>
__global__ __launch_bounds__(kInlThreads) void k_inl_flags(const void *__restrict__ pts, uint32_t n,
                                                           const float *__restrict__ models, float thr,
                                                           const float *__restrict__ thrs,
                                                           const uint32_t *__restrict__ slots,
                                                           uint32_t *__restrict__ scratch,
                                                           const int32_t *__restrict__ ok) {
    typedef typename std::conditional<EST == USAC_LINE2D, float2, float4>::type P;
    __shared__ uint32_t wsum[kInlThreads / 64];
    // the points' loads go out first: they do not depend on the model, whose slot, ok word and
    // parameters are three dependent loads of their own
    P pv[kInlPer];
#pragma unroll
    for (uint32_t u = 0; u < kInlPer; u++) {
        const uint32_t i = blockIdx.x * kInlBlock + u * kInlThreads + threadIdx.x;
        if (i < n) pv[u] = static_cast<const P *>(pts)[i];
    }
    const uint32_t w = inl_slot(slots, blockIdx.y);
    // the model, its threshold and its ok word: independent (uniform) loads, all in flight; every
    // lane derives H^-1 itself (the same operations as one lane would: no LDS round trip, no barrier)
    float m[18];
#pragma unroll
    for (int k = 0; k < 9; k++) m[k] = models[9 * (size_t)w + k];
    const float t = thrs ? thrs[w] : thr;
    if (ok && !ok[w]) return;  // a failed fit: k_inl_compact skips the slot too
    if constexpr (EST == USAC_HOMOGRAPHY) inv3x3(m, m + 9);
    float *all_e = reinterpret_cast<float *>(scratch + w * inl_stride(n) + inl_all_offset(n));
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t u = 0; u < kInlPer; u++) {
        const uint32_t i = blockIdx.x * kInlBlock + u * kInlThreads + threadIdx.x;
        const float e = i < n ? inl_error_p<EST>(m, pv[u]) : 0.f;
        if (i < n) all_e[i] = e;
        cnt += (uint32_t)__popcll(__ballot(i < n && e < t));
    }
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (uint32_t v = 0; v < kInlThreads / 64; v++) tot += wsum[v];
        scratch[w * inl_stride(n) + blockIdx.x] = tot;
    }
}

template <int EST>
__global__ __launch_bounds__(kInlThreads) void k_inl_compact(const void *__restrict__ pts, uint32_t n,
                                                             const float *__restrict__ models, float thr,
                                                             const float *__restrict__ thrs,
                                                             const uint32_t *__restrict__ slots,
                                                             uint32_t *__restrict__ scratch, int32_t *__restrict__ idx,
                                                             size_t idx_stride, const int32_t *__restrict__ ok,
                                                             int32_t *__restrict__ totals) {
    __shared__ uint32_t wsum[kInlPer][kInlThreads / 64], wpre[kInlThreads / 64];
    const uint32_t ws = inl_slot(slots, blockIdx.y);
    const size_t stride = inl_stride(n);
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    const uint32_t *block_counts = scratch + ws * stride;
    float *errs = reinterpret_cast<float *>(scratch + ws * stride + ((nb + 63) & ~63u));
    const float *all_e = reinterpret_cast<const float *>(scratch + ws * stride + inl_all_offset(n));
    // the residual loads go out before the ok word is read (a failed fit's are never used)
    float e[kInlPer];
#pragma unroll
    for (uint32_t u = 0; u < kInlPer; u++) {
        const uint32_t i = blockIdx.x * kInlBlock + u * kInlThreads + threadIdx.x;
        e[u] = i < n ? all_e[i] : 0.f;
    }
    const float t = thrs ? thrs[ws] : thr;  // in flight with the ok word
    if (ok && !ok[ws]) {  // a failed fit: its list is left as it was (workgroup-uniform) and its
        // count reads 0, so the Σ pass over this slot (launch_seqsum) sums nothing
        if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) totals[ws] = 0;
        return;
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t bal[kInlPer];
#pragma unroll
    for (uint32_t u = 0; u < kInlPer; u++) {
        const uint32_t i = blockIdx.x * kInlBlock + u * kInlThreads + threadIdx.x;
        bal[u] = __ballot(i < n && e[u] < t);
        if (lane == 0) wsum[u][wave] = (uint32_t)__popcll(bal[u]);
    }
    // this block's output offset: the sum of the earlier blocks' counts (k_inl_flags), summed
    // here (integers: any order) -- no separate scan launch; the last block writes the total
    uint32_t pre = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += kInlThreads) pre += block_counts[b];
    for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o);
    if (lane == 0) wpre[wave] = pre;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t v = 0; v < kInlThreads / 64; v++) base += wpre[v];
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        uint32_t tot = base;
        for (uint32_t u = 0; u < kInlPer; u++)
            for (uint32_t v = 0; v < kInlThreads / 64; v++) tot += wsum[u][v];
        totals[ws] = (int32_t)tot;
    }
#pragma unroll
    for (uint32_t u = 0; u < kInlPer; u++) {
        uint32_t r = base;
        for (uint32_t v = 0; v < wave; v++) r += wsum[u][v];
        if ((bal[u] >> lane) & 1ull) {
            r += (uint32_t)__popcll(bal[u] & ((1ull << lane) - 1));
            if (idx) idx[ws * idx_stride + r] = (int32_t)(blockIdx.x * kInlBlock + u * kInlThreads + threadIdx.x);
            errs[r] = e[u];
        }
        for (uint32_t v = 0; v < kInlThreads / 64; v++) base += wsum[u][v];
    }
}

// The polish's acceptance of pass k (ransac.cpp:170-200) on the device, so the four passes go
// out in one submission: pass k+1 fits pass k's inlier list with ns[k + 1] points when pass k
// was accepted -- its fit succeeded, (double)((float)cnt / (float)best) >= 0.8 and cnt > prev
// -- else with 0 points (a no-op fit whose scoring leaves its list alone).  The host replays
// the same decisions from the results and stops at the first rejection, so the passes after it
// are never read.  res: the polish result block (polish_layout in usac_kernels.h).
__global__ void k_polish_prep(int32_t *res, int k, int32_t best0) {
    if (threadIdx.x != 0) return;
    const int32_t *r = res + kPolPass * k;
    const int32_t best = k == 0 ? best0 : res[kPolState];
    const int32_t prev = k == 0 ? 0 : res[kPolState + 1];
    const int32_t ok = r[9], cnt = r[10];
    const bool accept = ok && !((double)((float)cnt / (float)best) < 0.8) && cnt > prev;
    reinterpret_cast<uint32_t *>(res)[kPolNs + k + 1] = accept ? (uint32_t)cnt : 0u;
    res[kPolState] = accept ? cnt : best;
    res[kPolState + 1] = accept ? cnt : prev;
}

hipError_t launch_polish_prep(hipStream_t st, int32_t *res, int k, int32_t best0) {
    hipLaunchKernelGGL(k_polish_prep, dim3(1), dim3(64), 0, st, res, k, best0);
    return hipGetLastError();
}

hipError_t launch_inliers_batch(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *models,
                                uint32_t W, float thr, const float *thrs, const uint32_t *slots, int32_t *idx,
                                size_t idx_stride, int32_t *counts, float *sums, void *scratch, const int32_t *ok) {
    if (W == 0) return hipSuccess;
    // one model with its sum over a few thousand points: one workgroup, one launch (the five
    // launches below are ~5 us each at this size; USAC_INLIERS_SMALL=0 keeps them)
    static const bool small_on = [] {
        const char *e = getenv("USAC_INLIERS_SMALL");
        return !e || atoi(e) != 0;
    }();
    if (small_on && W == 1 && !thrs && !slots && idx && sums && n <= kPolPtsMax && estimator != USAC_LINE2D)
        return launch_inliers_small(st, estimator, pts, n, models, thr, ok, idx, counts, sums);
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    uint32_t *scr = static_cast<uint32_t *>(scratch);
    const dim3 grid(nb, W);
#define INL(E)                                                                                                   \
    do {                                                                                                         \
        hipLaunchKernelGGL(k_inl_flags<E>, grid, dim3(kInlThreads), 0, st, pts, n, models, thr, thrs, slots, scr, ok);  \
        hipLaunchKernelGGL(k_inl_compact<E>, grid, dim3(kInlThreads), 0, st, pts, n, models, thr, thrs, slots, scr, \
                           idx, idx_stride, ok, counts);                                                         \
    } while (0)
    switch (estimator) {
        case USAC_LINE2D: INL(USAC_LINE2D); break;
        case USAC_HOMOGRAPHY: INL(USAC_HOMOGRAPHY); break;
        case USAC_FUNDAMENTAL: INL(USAC_FUNDAMENTAL); break;
        case USAC_ESSENTIAL: INL(USAC_ESSENTIAL); break;
        default: return hipErrorInvalidValue;
    }
#undef INL
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !sums) return e;
    return launch_inliers_sums(st, n, W, slots, counts, sums, scratch);
}

// the reference's sequential fp32 Σ in point order (quality.hpp:85) over the residuals the
// compaction left in scratch
hipError_t launch_inliers_sums(hipStream_t st, uint32_t n, uint32_t W, const uint32_t *slots, const int32_t *counts,
                               float *sums, void *scratch) {
    if (W == 0) return hipSuccess;
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    uint32_t *scr = static_cast<uint32_t *>(scratch);
    const size_t stride = inl_stride(n), res0 = (nb + 63) & ~63u;
    return launch_seqsum(st, 1, false, reinterpret_cast<const float *>(scr + res0), stride,
                         reinterpret_cast<const uint32_t *>(counts), 0, W, slots, scr + inl_res_words(n),
                         sizeof(uint32_t) * stride, false, sums);
}

// every point's exact residual under one model (Estimator::GetError, e.g. for the graph-cut
// LO's energies, graphcut.cpp:17-28)
template <int EST>
__global__ __launch_bounds__(kInlThreads) void k_point_errors(const void *__restrict__ pts, uint32_t n,
                                                            const float *__restrict__ model,
                                                            float *__restrict__ errors) {
    __shared__ float sm[18];
    inl_model<EST>(model, sm);
    float m[18];
#pragma unroll
    for (int k = 0; k < 18; k++) m[k] = sm[k];
    const uint32_t i = blockIdx.x * kInlThreads + threadIdx.x;
    if (i < n) errors[i] = inl_error<EST>(m, pts, i);
}

hipError_t launch_point_errors(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *model,
                               float *errors) {
    const dim3 grid((n + kInlThreads - 1) / kInlThreads);
    switch (estimator) {
        case USAC_LINE2D: hipLaunchKernelGGL(k_point_errors<USAC_LINE2D>, grid, dim3(kInlThreads), 0, st, pts, n, model, errors); break;
        case USAC_HOMOGRAPHY: hipLaunchKernelGGL(k_point_errors<USAC_HOMOGRAPHY>, grid, dim3(kInlThreads), 0, st, pts, n, model, errors); break;
        case USAC_FUNDAMENTAL: hipLaunchKernelGGL(k_point_errors<USAC_FUNDAMENTAL>, grid, dim3(kInlThreads), 0, st, pts, n, model, errors); break;
        case USAC_ESSENTIAL: hipLaunchKernelGGL(k_point_errors<USAC_ESSENTIAL>, grid, dim3(kInlThreads), 0, st, pts, n, model, errors); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_inliers(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *model, float thr,
                          int32_t *idx, int32_t *count, float *sum, void *scratch) {
    return launch_inliers_batch(st, estimator, pts, n, model, 1, thr, nullptr, nullptr, idx, 0, count, sum, scratch);
}

size_t inliers_scratch_bytes(uint32_t n, uint32_t W) { return sizeof(uint32_t) * inl_stride(n) * W; }

}  // namespace usac
