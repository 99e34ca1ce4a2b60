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

template <int EST>
__global__ __launch_bounds__(kInlBlock) void k_inl_flags(const void *__restrict__ pts, uint32_t n,
                                                         const float *__restrict__ model, float thr,
                                                         uint32_t *__restrict__ block_counts) {
    __shared__ float sm[18];
    __shared__ uint32_t wsum[kInlBlock / 64];
    inl_model<EST>(model, sm);
    float m[18];
#pragma unroll
    for (int k = 0; k < 18; k++) m[k] = sm[k];
    const uint32_t i = blockIdx.x * kInlBlock + threadIdx.x;
    const bool in = i < n && inl_error<EST>(m, pts, i) < thr;
    const uint64_t bal = __ballot(in);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = (uint32_t)__popcll(bal);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < kInlBlock / 64; w++) t += wsum[w];
        block_counts[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(1024) void k_inl_scan(uint32_t *__restrict__ block_counts, uint32_t nblocks,
                                                   int32_t *__restrict__ total) {
    // exclusive scan in place, 1024 threads, sequential chunks per thread
    __shared__ uint32_t part[1024];
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
    if (t == 1023) *total = (int32_t)part[1023];
}

template <int EST>
__global__ __launch_bounds__(kInlBlock) void k_inl_compact(const void *__restrict__ pts, uint32_t n,
                                                           const float *__restrict__ model, float thr,
                                                           const uint32_t *__restrict__ block_offsets,
                                                           int32_t *__restrict__ idx, float *__restrict__ errs) {
    __shared__ float sm[18];
    __shared__ uint32_t wsum[kInlBlock / 64];
    inl_model<EST>(model, sm);
    float m[18];
#pragma unroll
    for (int k = 0; k < 18; k++) m[k] = sm[k];
    const uint32_t i = blockIdx.x * kInlBlock + threadIdx.x;
    const float e = i < n ? inl_error<EST>(m, pts, i) : 0.f;
    const bool in = i < n && e < thr;
    const uint64_t bal = __ballot(in);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) wsum[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t base = block_offsets[blockIdx.x];
    for (uint32_t w = 0; w < wave; w++) base += wsum[w];
    if (in) {
        const uint32_t r = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
        idx[r] = (int32_t)i;
        errs[r] = e;
    }
}

// sequential fp32 sum in point order (quality.hpp:85), one wave: 64 residuals per step are
// loaded in parallel and added one after the other through v_readlane (no LDS round trip)
// 256 threads stage 4096-residual chunks in LDS with coalesced loads; lane 0 adds them in
// order (the reference's sequential fp32 sum, one dependent add per inlier)
constexpr uint32_t kSumChunk = 4096;

__global__ __launch_bounds__(256) void k_inl_sum(const float *__restrict__ errs, const int32_t *__restrict__ total,
                                                 float *__restrict__ sum) {
    __shared__ __attribute__((aligned(16))) float s_e[kSumChunk];
    const uint32_t n = (uint32_t)*total;
    const uint32_t t = threadIdx.x;
    float s = 0.f;
    for (uint32_t c0 = 0; c0 < n; c0 += kSumChunk) {
        const uint32_t m = n - c0 < kSumChunk ? n - c0 : kSumChunk;
        for (uint32_t i = t; i < m; i += 256) s_e[i] = errs[c0 + i];
        __syncthreads();
        if (t == 0) {
            // 16 residuals in registers, the next 16 in flight from LDS
            const float4 *v = reinterpret_cast<const float4 *>(s_e);
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
            for (; k < m; k++) s += s_e[k];
        }
        __syncthreads();
    }
    if (t == 0) *sum = s;
}

hipError_t launch_inliers(hipStream_t st, int estimator, const void *pts, uint32_t n, const float *model, float thr,
                          int32_t *idx, int32_t *count, float *sum, void *scratch) {
    // scratch: block counts (nblocks u32) followed by the compacted residuals (n floats)
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    uint32_t *bc = static_cast<uint32_t *>(scratch);
    float *errs = reinterpret_cast<float *>(bc + ((nb + 63) & ~63u));
#define INL(E)                                                                                                      \
    do {                                                                                                            \
        hipLaunchKernelGGL(k_inl_flags<E>, dim3(nb), dim3(kInlBlock), 0, st, pts, n, model, thr, bc);               \
        hipLaunchKernelGGL(k_inl_scan, dim3(1), dim3(1024), 0, st, bc, nb, count);                                 \
        hipLaunchKernelGGL(k_inl_compact<E>, dim3(nb), dim3(kInlBlock), 0, st, pts, n, model, thr, bc, idx, errs); \
        hipLaunchKernelGGL(k_inl_sum, dim3(1), dim3(256), 0, st, errs, count, sum);                                \
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

size_t inliers_scratch_bytes(uint32_t n) {
    const uint32_t nb = (n + kInlBlock - 1) / kInlBlock;
    return sizeof(uint32_t) * ((nb + 63) & ~63u) + sizeof(float) * (size_t)n;
}

}  // namespace usac
