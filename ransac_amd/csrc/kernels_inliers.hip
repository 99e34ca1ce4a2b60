// kernels_inliers.hip -- Quality::getNumberInliers(score, model, thr, get_inliers = true,
// inliers) (quality.hpp:60-101) for ONE model over all N points, exactly: the ascending
// inlier index list, the count, and the reference's sequential fp32 Σerr (point order).
// Used by the polish (ransac.cpp:157-214), LO-RANSAC (inner_local_optimization.hpp:74-133)
// and PROSAC's termination scan.
//
//   k_inl_flags   grid over points: exact residual, per-block inlier count      (parallel)
//   k_inl_scan    one workgroup: exclusive scan of the block counts -> offsets  (tiny)
//   k_inl_compact grid over points: ordered compaction of indices and residuals (parallel)
//   k_inl_sum     one workgroup: the sequential fp32 sum over the compacted residuals
//                 (the only inherently serial part: one dependent add per inlier)
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_device_e5.hpp"
#include "usac_kernels.h"

namespace usac {

constexpr uint32_t kInlBlock = 256;

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
// or the scalar thr).  Per model the scratch holds its block counts (nb padded to 64)
// followed by its compacted residuals (n floats): inl_stride(n) words.  Every model's
// result is exactly the single-model one (the kernels never mix models).
__host__ __device__ __forceinline__ size_t inl_stride(uint32_t n) {
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    return (size_t)((nb + 63) & ~63u) + n;
}

// model slot of workgroup row b: slots[b] when a slot list is given (a subset of the W models)
__device__ __forceinline__ uint32_t inl_slot(const uint32_t *slots, uint32_t b) { return slots ? slots[b] : b; }

template <int EST>
__global__ __launch_bounds__(kInlBlock) void k_inl_flags(const void *__restrict__ pts, uint32_t n,
                                                         const float *__restrict__ models, float thr,
                                                         const float *__restrict__ thrs,
                                                         const uint32_t *__restrict__ slots,
                                                         uint32_t *__restrict__ scratch) {
    __shared__ float sm[18];
    __shared__ uint32_t wsum[kInlBlock / 64];
    const uint32_t w = inl_slot(slots, blockIdx.y);
    inl_model<EST>(models + 9 * (size_t)w, sm);
    const float t = thrs ? thrs[w] : thr;
    float m[18];
#pragma unroll
    for (int k = 0; k < 18; k++) m[k] = sm[k];
    const uint32_t i = blockIdx.x * kInlBlock + threadIdx.x;
    const bool in = i < n && inl_error<EST>(m, pts, i) < t;
    const uint64_t bal = __ballot(in);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = (uint32_t)__popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (uint32_t w = 0; w < kInlBlock / 64; w++) tot += wsum[w];
        scratch[w * inl_stride(n) + blockIdx.x] = tot;
    }
}

__global__ __launch_bounds__(1024) void k_inl_scan(uint32_t *__restrict__ scratch, uint32_t n, uint32_t nblocks,
                                                   const uint32_t *__restrict__ slots, int32_t *__restrict__ totals) {
    // exclusive scan in place, 1024 threads, sequential chunks per thread
    __shared__ uint32_t part[1024];
    const uint32_t w = inl_slot(slots, blockIdx.x);
    uint32_t *block_counts = scratch + w * inl_stride(n);
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nblocks + 1023) / 1024;
    const uint32_t b0 = t * per, b1 = b0 + per < nblocks ? b0 + per : nblocks;
    uint32_t s = 0;
    for (uint32_t b = b0; b < b1; b++) s += block_counts[b];
    part[t] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - s;  // exclusive prefix of this thread's chunk
    for (uint32_t b = b0; b < b1; b++) {
        const uint32_t c = block_counts[b];
        block_counts[b] = run;
        run += c;
    }
    if (t == 1023) totals[w] = (int32_t)part[1023];
}

template <int EST>
__global__ __launch_bounds__(kInlBlock) void k_inl_compact(const void *__restrict__ pts, uint32_t n,
                                                           const float *__restrict__ models, float thr,
                                                           const float *__restrict__ thrs,
                                                           const uint32_t *__restrict__ slots,
                                                           uint32_t *__restrict__ scratch, int32_t *__restrict__ idx,
                                                           size_t idx_stride) {
    __shared__ float sm[18];
    __shared__ uint32_t wsum[kInlBlock / 64];
    const uint32_t ws = inl_slot(slots, blockIdx.y);
    inl_model<EST>(models + 9 * (size_t)ws, sm);
    const float t = thrs ? thrs[ws] : thr;
    float m[18];
#pragma unroll
    for (int k = 0; k < 18; k++) m[k] = sm[k];
    const size_t stride = inl_stride(n);
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    const uint32_t *block_offsets = scratch + ws * stride;
    float *errs = reinterpret_cast<float *>(scratch + ws * stride + ((nb + 63) & ~63u));
    const uint32_t i = blockIdx.x * kInlBlock + threadIdx.x;
    const float e = i < n ? inl_error<EST>(m, pts, i) : 0.f;
    const bool in = i < n && e < t;
    const uint64_t bal = __ballot(in);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) wsum[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t base = block_offsets[blockIdx.x];
    for (uint32_t w = 0; w < wave; w++) base += wsum[w];
    if (in) {
        const uint32_t r = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
        if (idx) idx[ws * idx_stride + r] = (int32_t)i;
        errs[r] = e;
    }
}

// the reference's sequential fp32 sum in point order (quality.hpp:85), one workgroup per
// model: lane 0 adds the residuals of one 2048-entry LDS chunk in order (one dependent add
// per inlier -- the only inherently serial part) while waves 1-3 stage the next chunk into
// the other buffer with coalesced loads; one barrier per chunk.
constexpr uint32_t kSumChunk = 2048;

__global__ __launch_bounds__(256) void k_inl_sum(const uint32_t *__restrict__ scratch, uint32_t n_pts,
                                                 const uint32_t *__restrict__ slots,
                                                 const int32_t *__restrict__ totals, float *__restrict__ sums) {
    __shared__ __attribute__((aligned(16))) float s_e[2][kSumChunk];
    const uint32_t nb = (n_pts + kInlBlock - 1) / kInlBlock;
    const uint32_t w = inl_slot(slots, blockIdx.x);
    const float *errs = reinterpret_cast<const float *>(scratch + w * inl_stride(n_pts) + ((nb + 63) & ~63u));
    const uint32_t n = (uint32_t)totals[w];
    const uint32_t t = threadIdx.x;
    const bool loader = t >= 64;
    const uint32_t lt = t - 64;
    const uint32_t nch = (n + kSumChunk - 1) / kSumChunk;
    auto len = [&](uint32_t c) { return n - c * kSumChunk < kSumChunk ? n - c * kSumChunk : kSumChunk; };
    if (loader && nch > 0)
        for (uint32_t i = lt; i < len(0); i += 192) s_e[0][i] = errs[i];
    __syncthreads();
    float s = 0.f;
    for (uint32_t c = 0; c < nch; c++) {
        if (loader && c + 1 < nch) {
            const uint32_t m1 = len(c + 1), base = (c + 1) * kSumChunk;
            for (uint32_t i = lt; i < m1; i += 192) s_e[(c + 1) & 1][i] = errs[base + i];
        }
        if (t == 0) {
            // 16 residuals in registers, the next 16 in flight from LDS
            const uint32_t m = len(c);
            const float *e = s_e[c & 1];
            const float4 *v = reinterpret_cast<const float4 *>(e);
            uint32_t k = 0;
            if (m >= 16) {
                float4 c0 = v[0], c1 = v[1], c2 = v[2], c3 = v[3];
                for (; k + 32 <= m; k += 16) {
                    const uint32_t j = (k + 16) / 4;
                    const float4 n0 = v[j], n1 = v[j + 1], n2 = v[j + 2], n3 = v[j + 3];
                    s += c0.x; s += c0.y; s += c0.z; s += c0.w;
                    s += c1.x; s += c1.y; s += c1.z; s += c1.w;
                    s += c2.x; s += c2.y; s += c2.z; s += c2.w;
                    s += c3.x; s += c3.y; s += c3.z; s += c3.w;
                    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
                }
                s += c0.x; s += c0.y; s += c0.z; s += c0.w;
                s += c1.x; s += c1.y; s += c1.z; s += c1.w;
                s += c2.x; s += c2.y; s += c2.z; s += c2.w;
                s += c3.x; s += c3.y; s += c3.z; s += c3.w;
                k += 16;
            }
            for (; k < m; k++) s += e[k];
        }
        __syncthreads();
    }
    if (t == 0) sums[w] = s;
}

hipError_t launch_inliers_batch(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *models,
                                uint32_t W, float thr, const float *thrs, const uint32_t *slots, int32_t *idx,
                                size_t idx_stride, int32_t *counts, float *sums, void *scratch) {
    if (W == 0) return hipSuccess;
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    uint32_t *scr = static_cast<uint32_t *>(scratch);
    const dim3 grid(nb, W);
#define INL(E)                                                                                                   \
    do {                                                                                                         \
        hipLaunchKernelGGL(k_inl_flags<E>, grid, dim3(kInlBlock), 0, st, pts, n, models, thr, thrs, slots, scr);        \
        hipLaunchKernelGGL(k_inl_scan, dim3(W), dim3(1024), 0, st, scr, n, nb, slots, counts);                         \
        hipLaunchKernelGGL(k_inl_compact<E>, grid, dim3(kInlBlock), 0, st, pts, n, models, thr, thrs, slots, scr, \
                           idx, idx_stride);                                                                     \
        hipLaunchKernelGGL(k_inl_sum, dim3(W), dim3(256), 0, st, scr, n, slots, counts, sums);                         \
    } while (0)
    switch (estimator) {
        case USAC_LINE2D: INL(USAC_LINE2D); break;
        case USAC_HOMOGRAPHY: INL(USAC_HOMOGRAPHY); break;
        case USAC_FUNDAMENTAL: INL(USAC_FUNDAMENTAL); break;
        case USAC_ESSENTIAL: INL(USAC_ESSENTIAL); break;
        default: return hipErrorInvalidValue;
    }
#undef INL
    return hipGetLastError();
}

// every point's exact residual under one model (Estimator::GetError, e.g. for the graph-cut
// LO's energies, graphcut.cpp:17-28)
template <int EST>
__global__ __launch_bounds__(kInlBlock) void k_point_errors(const void *__restrict__ pts, uint32_t n,
                                                            const float *__restrict__ model,
                                                            float *__restrict__ errors) {
    __shared__ float sm[18];
    inl_model<EST>(model, sm);
    float m[18];
#pragma unroll
    for (int k = 0; k < 18; k++) m[k] = sm[k];
    const uint32_t i = blockIdx.x * kInlBlock + threadIdx.x;
    if (i < n) errors[i] = inl_error<EST>(m, pts, i);
}

hipError_t launch_point_errors(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *model,
                               float *errors) {
    const dim3 grid((n + kInlBlock - 1) / kInlBlock);
    switch (estimator) {
        case USAC_LINE2D: hipLaunchKernelGGL(k_point_errors<USAC_LINE2D>, grid, dim3(kInlBlock), 0, st, pts, n, model, errors); break;
        case USAC_HOMOGRAPHY: hipLaunchKernelGGL(k_point_errors<USAC_HOMOGRAPHY>, grid, dim3(kInlBlock), 0, st, pts, n, model, errors); break;
        case USAC_FUNDAMENTAL: hipLaunchKernelGGL(k_point_errors<USAC_FUNDAMENTAL>, grid, dim3(kInlBlock), 0, st, pts, n, model, errors); break;
        case USAC_ESSENTIAL: hipLaunchKernelGGL(k_point_errors<USAC_ESSENTIAL>, grid, dim3(kInlBlock), 0, st, pts, n, model, errors); break;
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
