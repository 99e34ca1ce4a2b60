// kernels_knn.hip -- NearestNeighbors::getNearestNeighbors_nanoflann
// (nearest_neighbors.cpp:69-128): the k nearest neighbours of every point, exactly, by brute
// force on the device instead of a KD-tree.
//
// Distance = nanoflann's L2_Adaptor::evalMetric in float (components in groups of four,
// result += d0*d0 + d1*d1 + d2*d2 + d3*d3, remaining components one by one; no FMA), the
// query itself excluded (the reference drops the first result), equal distances in ascending
// index (nanoflann keeps its tree's visiting order there -- unpinned), missing neighbours
// (n - 1 < k) as index -1 / +inf.  Same spec as oracle/usac_oracle.c:orc_knn.
//
// Layout: a workgroup = 64 queries (one per lane) x KNN_WAVES candidate ranges (one per
// wave).  Candidates are wave-uniform, read through the scalar cache (SGPR operands), so a
// candidate costs ~12 VALU ops for 64 queries.  Each lane keeps its K best in registers,
// right-aligned (slots below K - k hold -inf sentinels, so every index is static); the
// insertion network shifts only when a candidate beats the current k-th distance.  The
// waves' lists are merged in candidate-range order through LDS: an element is placed after
// every equal distance already present, and every earlier range holds smaller indices, so
// ties stay in ascending index order.
#include <hip/hip_runtime.h>
#include <math.h>

#include "usac_kernels.h"

namespace usac {

constexpr int kKnnWaves = 4;

template <int COLS>
__device__ __forceinline__ float knn_dist(const float *a, const float *b) {
    float r = 0.f;
    int d = 0;
#pragma unroll
    for (; d + 4 <= COLS; d += 4) {
        const float d0 = a[d] - b[d], d1 = a[d + 1] - b[d + 1], d2 = a[d + 2] - b[d + 2], d3 = a[d + 3] - b[d + 3];
        r += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
#pragma unroll
    for (; d < COLS; d++) {
        const float d0 = a[d] - b[d];
        r += d0 * d0;
    }
    return r;
}

// insert (d, j) into the ascending right-aligned list D/I[0..K); caller checked d < D[K-1]
template <int K>
__device__ __forceinline__ void knn_insert(float (&D)[K], int32_t (&I)[K], float d, int32_t j) {
    bool placed = false;
#pragma unroll
    for (int t = K - 1; t >= 1; --t) {
        const bool sh = D[t - 1] > d;
        const bool here = !sh && !placed;
        D[t] = sh ? D[t - 1] : (here ? d : D[t]);
        I[t] = sh ? I[t - 1] : (here ? j : I[t]);
        placed |= !sh;
    }
    if (!placed) {
        D[0] = d;
        I[0] = j;
    }
}

template <int COLS, int K>
__global__ __launch_bounds__(64 * kKnnWaves) void k_knn(const float *__restrict__ pts, uint32_t n, uint32_t k,
                                                        int32_t *__restrict__ idx_out, float *__restrict__ d2_out) {
    __shared__ float s_d[kKnnWaves][K][64];
    __shared__ int32_t s_i[kKnnWaves][K][64];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t p = blockIdx.x * 64 + lane;
    const uint32_t pc = p < n ? p : n - 1;
    float q[COLS];
#pragma unroll
    for (int c = 0; c < COLS; c++) q[c] = pts[(size_t)pc * COLS + c];
    float D[K];
    int32_t I[K];
#pragma unroll
    for (int t = 0; t < K; t++) {
        D[t] = t < K - (int)k ? -INFINITY : INFINITY;
        I[t] = -1;
    }
    const uint32_t per = (n + kKnnWaves - 1) / kKnnWaves;
    const uint32_t j0 = wave * per;
    const uint32_t j1 = j0 + per < n ? j0 + per : n;
    uint32_t j = j0;
    for (; j + 4 <= j1; j += 4) {  // four candidates per scalar load batch
        float b[4][COLS];
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int c = 0; c < COLS; c++) b[u][c] = pts[(size_t)(j + u) * COLS + c];  // uniform: scalar loads
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float d = knn_dist<COLS>(q, b[u]);
            if (d < D[K - 1] && j + u != p) knn_insert<K>(D, I, d, (int32_t)(j + u));
        }
    }
    for (; j < j1; j++) {
        float b[COLS];
#pragma unroll
        for (int c = 0; c < COLS; c++) b[c] = pts[(size_t)j * COLS + c];
        const float d = knn_dist<COLS>(q, b);
        if (d < D[K - 1] && j != p) knn_insert<K>(D, I, d, (int32_t)j);
    }
#pragma unroll
    for (int t = 0; t < K; t++) {
        s_d[wave][t][lane] = D[t];
        s_i[wave][t][lane] = I[t];
    }
    __syncthreads();
    if (wave != 0) return;
    for (int w = 1; w < kKnnWaves; w++)
        for (int t = K - (int)k; t < K; t++) {
            const float d = s_d[w][t][lane];
            if (d < D[K - 1]) knn_insert<K>(D, I, d, s_i[w][t][lane]);
        }
    if (p >= n) return;
    for (uint32_t t = 0; t < k; t++) {
        idx_out[(size_t)p * k + t] = I[K - k + t];
        if (d2_out) d2_out[(size_t)p * k + t] = D[K - k + t];
    }
}

template <int COLS>
hipError_t knn_cols(hipStream_t st, const float *pts, uint32_t n, uint32_t k, int32_t *idx, float *d2) {
    const dim3 grid((n + 63) / 64), block(64 * kKnnWaves);
    if (k <= 4) hipLaunchKernelGGL((k_knn<COLS, 4>), grid, block, 0, st, pts, n, k, idx, d2);
    else if (k <= 8) hipLaunchKernelGGL((k_knn<COLS, 8>), grid, block, 0, st, pts, n, k, idx, d2);
    else if (k <= 16) hipLaunchKernelGGL((k_knn<COLS, 16>), grid, block, 0, st, pts, n, k, idx, d2);
    else hipLaunchKernelGGL((k_knn<COLS, 32>), grid, block, 0, st, pts, n, k, idx, d2);
    return hipGetLastError();
}

hipError_t launch_knn(hipStream_t st, const float *pts, uint32_t n, uint32_t cols, uint32_t k, int32_t *idx,
                      float *d2) {
    if (k == 0 || k > kKnnMax || n == 0) return hipErrorInvalidValue;
    return cols == 2 ? knn_cols<2>(st, pts, n, k, idx, d2) : knn_cols<4>(st, pts, n, k, idx, d2);
}

}  // namespace usac
