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
// words[w * row_stride + row], bit b = pool position 32 w + b; row_stride 0: the row count itself
// (the listed rows' words packed [nw][*list_n], one plain copy for the host).
constexpr uint32_t kMaskWords = 8;  // pool words (256 points) per k_pool_mask lane, at most

template <int EST>
__global__ __launch_bounds__(64) void k_pool_mask(const void *__restrict__ pool_pts, uint32_t n,
                                                  const float *__restrict__ models, size_t stride,
                                                  const uint32_t *__restrict__ list, const uint32_t *__restrict__ list_n,
                                                  uint32_t kmax, float thr, uint32_t *__restrict__ words,
                                                  uint32_t row_stride, uint32_t wpl, PoolTail tail) {
    constexpr int NC = EST == 1 ? 3 : EST == 2 ? 18 : 9;
    if (tail.dst && blockIdx.y == 0) {  // the batch's other results next to the words (PoolTail)
        const uint32_t S = tail.S, T = 2 * S + 1 + tail.nmod;
        for (uint32_t w = blockIdx.x * 64 + threadIdx.x; w < T; w += gridDim.x * 64)
            tail.dst[w] = w < S ? tail.counts[w] : w == S ? *tail.list_n : w <= 2 * S ? tail.list[w - S - 1]
                                                                                   : tail.models[w - 2 * S - 1];
    }
    const uint32_t K = list ? __builtin_amdgcn_readfirstlane(*list_n) : kmax;
    const uint32_t i0 = blockIdx.x * 64;
    if (i0 >= K) return;
    const uint32_t row = i0 + threadIdx.x;
    const size_t rs = row_stride ? row_stride : K;
    const uint32_t rc = row < K ? row : K - 1;
    const uint32_t slot = list ? list[rc] : rc;
    float m[NC];
#pragma unroll
    for (int k = 0; k < NC; k++) m[k] = models[(size_t)k * stride + slot];
    // this block's word ranges (blockIdx.y, then every gridDim.y-th range: the y grid is capped at
    // 65535 blocks, reached above 16.7 M points): a lane walks wpl words at a time, not all n / 32 --
    // the loop's batches hold a few hundred models, so lanes = models alone is a handful of waves
    const uint32_t nw = (n + 31) / 32;
    for (uint32_t w0 = blockIdx.y * wpl; w0 < nw; w0 += gridDim.y * wpl)
    for (uint32_t w = w0, w1 = w0 + wpl < nw ? w0 + wpl : nw; w < w1; w++) {
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
        if (row < K) words[(size_t)w * rs + row] = bits;
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
                            uint32_t *words, uint32_t row_stride, const PoolTail *tail) {
    const PoolTail tl = tail ? *tail : PoolTail{nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr};
    // words per lane: kMaskWords, fewer while the grid would hold under ~2048 workgroups (PROSAC's
    // first batches: a few dozen samples, ~100 models -- round 5: all the pool's words at 8 per lane
    // made two workgroup columns of 40 ranges, latency-bound)
    const uint32_t nw = (n + 31) / 32, bx = (kmax + 63) / 64;
    uint32_t wpl = kMaskWords;
    while (wpl > 1 && (size_t)bx * ((nw + wpl - 1) / wpl) < 2048) wpl >>= 1;
    const uint32_t ranges = (nw + wpl - 1) / wpl;
    const dim3 grid(bx, ranges < 65535u ? ranges : 65535u);
    switch (estimator) {
        case USAC_LINE2D:
            hipLaunchKernelGGL(k_pool_mask<1>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax,
                               thr, words, row_stride, wpl, tl);
            break;
        case USAC_HOMOGRAPHY:
            hipLaunchKernelGGL(k_pool_mask<2>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax,
                               thr, words, row_stride, wpl, tl);
            break;
        case USAC_FUNDAMENTAL:
            hipLaunchKernelGGL(k_pool_mask<3>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax,
                               thr, words, row_stride, wpl, tl);
            break;
        case USAC_ESSENTIAL:
            hipLaunchKernelGGL(k_pool_mask<4>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax,
                               thr, words, row_stride, wpl, tl);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace usac

namespace usac {

// Throughput SPRT ("batch-native"): every model of a batch is verified with
// the same test -- (epsilon, delta, A) fixed for the batch -- walking the pool-ordered points from
// a wave-uniform start (pool position (block * 7919) mod n, wrapping; the reference's rolling pool
// index places each model's test at an arbitrary pool position too).  A model is rejected at the
// first point where the reference's fp64 product lambda = prod (in ? up : down), up = delta /
// epsilon, down = (1 - delta) / (1 - epsilon) (sprt.hpp:209-234), exceeds A; rejected models get
// count -1 (never a best), a model that passes all n points count = its inliers over all points
// and score = (float)count (sprt.hpp:276-281).
//
// Decisions equal the reference's fp64 product walk from the same start, certified (round 4):
// after a inliers and b outliers, log lambda = P = a log(up) + b log(down) exactly (for the fp64
// up / down), and the fp64 product stays within a relative t 2^-53 of it while it is a normal
// number.  The kernels evaluate P in fp64 from exact counts and decide "rejected at the first P >
// log A" wherever that is certain: every prefix's |P - log A| > margin, and no climb P_t -
// min_{s<=t} P_s reaches climb = 700 (so a walk that crosses log A > 0 never passed through
// subnormal lambda, and an accepted walk's rounding inflation stays below 2^-1074 n e^700 << 1 <= A).
// The margin is set per context from n (usac_set_sprt, sprt_margin): with L = max(|lu|, |ld|, 1),
// the logs' roundings over n terms and the product's drift are <= n L 2^-51, P from the counts
// (two products and a sum) <= n L 2^-51, a tail chunk's running sum over `per` = ceil((n - 64) /
// 256) adds <= per^2 L 2^-53 (the head's 64 adds likewise), log A's rounding <= |lA| 2^-53; the
// margin is 8x their sum and never below 1e-7 (1.3e-10 at cfg3's n = 10 k, so 1e-7 there; the
// budget grows with n -- 2^26 points give ~4e-4 -- and more walks then take the sequential path,
// which is exact for any n).  A model whose walk is not
// certified (|P - log A| <= margin at the deciding prefix, or a climb >= climb) is decided by the
// reference's own sequential fp64 product from its start (one lane; rare by construction).
//
// Two phases, because nearly every model is rejected within a few dozen points while the
// few good ones must walk all n:
//   phase 1 (lanes = models): the first kHead pool points, wave exit once all lanes
//            decided; lanes still undecided are appended to a survivor list (counts, min P);
//   phase 2 (a workgroup per survivor, lanes = points): the remaining points split into
//            256 contiguous chunks; each thread reduces its chunk to (inliers, max / min prefix
//            of Delta P, largest climb inside the chunk); wave 0 scans the chunks in pool order
//            (exact count prefix, then P at every chunk start from counts, prefix minima) and the
//            first chunk that reaches log A - margin or a climb of climb decides.
// kHead = 64 (round 3; was 256): a wave of phase 1 runs until its last lane decides, and on
// cfg3 most waves hold one of the few good models, so the head is as long as the wave walks;
// 64 points reject nearly every bad model and the survivors' tails run in parallel
// (cfg3 883-894 -> 1065-1069 M hyp/s same-box; 32: 961-1088)
constexpr uint32_t kHead = 64;
// (the certificate's kc.margin = 1e-7 and kc.climb = 700 travel in SprtConsts::margin / ::climb, so a
// test can shrink the certified region and drive every walk down the sequential path)

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
    int cnt;               // inliers among the head's points
    uint32_t exact;        // 1: the head could not certify the walk -> the sequential fp64 walk
    double pmin;           // min of P over the head's prefixes (P_0 = 0 included)
};

// the reference's own walk (sprt.hpp:209-234) from pool position `start`: good, inliers, points read
template <int EST>
__device__ bool sprt_exact_walk(const float *m, const void *pool_pts, uint32_t n, float thr, uint32_t start,
                                const SprtConsts &k, int &cnt, uint32_t &tested) {
    double lambda = 1.0;
    uint32_t p = start;
    cnt = 0;
    for (uint32_t t = 0; t < n; t++) {
        const bool in = sprt_error<EST>(m, pool_pts, p) < thr;
        cnt += in ? 1 : 0;
        const double next = lambda * (in ? k.up : k.down);
        if (++p == n) p = 0;
        if (next > k.A) {
            tested = t + 1;
            return false;
        }
        lambda = next;
    }
    tested = n;
    return true;
}

template <int EST>
__global__ __launch_bounds__(64) void k_sprt_head(const void *__restrict__ pool_pts, uint32_t n,
                                                  const float *__restrict__ models, size_t stride,
                                                  const uint32_t *__restrict__ list,
                                                  const uint32_t *__restrict__ list_n, uint32_t kmax, float thr,
                                                  SprtConsts kc, int32_t *__restrict__ counts,
                                                  float *__restrict__ sums, uint32_t *__restrict__ tested_total,
                                                  SprtSurvivor *__restrict__ surv, uint32_t *__restrict__ surv_n,
                                                  uint32_t *__restrict__ starts) {
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
    double P = 0.0, pmin = 0.0;
    int cnt = 0;
    bool live = row < K, amb = false;
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
                P += in ? kc.lu : kc.ld;  // <= 64 fp64 adds: error < 1e-12
                tested++;
                if (fabs(P - kc.lA) <= kc.margin || P - pmin >= kc.climb) {
                    amb = true;  // not certified: the sequential walk decides
                    live = false;
                } else if (P > kc.lA) {
                    live = false;  // rejected
                }
                pmin = fmin(pmin, P);
            }
        }
        p = q;
        if (!__any(live)) break;
    }
    if (row < K) {
        if (starts) starts[slot] = start;
        if (amb && head == n) {  // no phase 2: walk it here
            int c2 = 0;
            uint32_t t2 = 0;
            const bool good = sprt_exact_walk<EST>(m, pool_pts, n, thr, start, kc, c2, t2);
            counts[slot] = good ? c2 : -1;
            sums[slot] = good ? (float)c2 : 0.f;
            tested = t2;
        } else if (!live && !amb) {
            counts[slot] = -1;
            sums[slot] = 0.f;
        } else if (head == n) {
            counts[slot] = cnt;
            sums[slot] = (float)cnt;
        } else {
            const uint32_t k = atomicAdd(surv_n, 1u);
            surv[k] = SprtSurvivor{slot, (start + head) % n, cnt, amb ? 1u : 0u, pmin};
        }
    }
    uint32_t v = row < K ? tested : 0;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (threadIdx.x == 0 && tested_total) atomicAdd(tested_total, v);
}

__device__ __forceinline__ double readlane_f64(double v, int src) {
    const int2 w = *reinterpret_cast<const int2 *>(&v);
    int2 r;
    r.x = __builtin_amdgcn_readlane(w.x, src);
    r.y = __builtin_amdgcn_readlane(w.y, src);
    return *reinterpret_cast<const double *>(&r);
}

template <int EST>
__global__ __launch_bounds__(256) void k_sprt_tail(const void *__restrict__ pool_pts, uint32_t n,
                                                   const float *__restrict__ models, size_t stride, float thr,
                                                   SprtConsts kc, const SprtSurvivor *__restrict__ surv,
                                                   const uint32_t *__restrict__ surv_n, int32_t *__restrict__ counts,
                                                   float *__restrict__ sums, uint32_t *__restrict__ tested_total) {
    constexpr int NC = EST == 1 ? 3 : EST == 2 ? 18 : 9;
    __shared__ int s_cnt[256];
    __shared__ double s_max[256], s_min[256], s_clb[256];
    __shared__ int s_exact;
    const uint32_t ns = *surv_n;
    const uint32_t rest = n - kHead;  // launched only when n > kHead
    const uint32_t per = (rest + 255) / 256;
    for (uint32_t k = blockIdx.x; k < ns; k += gridDim.x) {
        const SprtSurvivor sv = surv[k];
        float m[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) m[c] = models[(size_t)c * stride + sv.slot];
        if (!sv.exact) {
            const uint32_t b = threadIdx.x * per;
            const uint32_t e = b + per < rest ? b + per : rest;
            int cnt = 0;
            double d = 0.0, dmax = -INFINITY, dmin = INFINITY, rmin = 0.0, clb = 0.0;
            uint32_t p = sv.start + (b < rest ? b : rest);
            if (p >= n) p -= n;
            for (uint32_t t = b; t < e; t++) {
                const bool in = sprt_error<EST>(m, pool_pts, p) < thr;
                cnt += in ? 1 : 0;
                d += in ? kc.lu : kc.ld;  // a chunk's <= ceil(n / 256) adds
                dmax = fmax(dmax, d);
                dmin = fmin(dmin, d);
                clb = fmax(clb, d - rmin);
                rmin = fmin(rmin, d);
                if (++p == n) p = 0;
            }
            s_cnt[threadIdx.x] = cnt;
            s_max[threadIdx.x] = dmax;
            s_min[threadIdx.x] = dmin;
            s_clb[threadIdx.x] = clb;
        }
        __syncthreads();
        if (threadIdx.x < 64 && !sv.exact) {
            // wave 0: lane l holds chunks 4l .. 4l+3.  Exact inlier / point counts at every chunk
            // start by a wave scan; P there from the counts (no accumulated rounding); the prefix
            // minimum of P before each chunk by a second scan; then the first chunk (in pool
            // order) that reaches log A - kc.margin or a climb of kc.climb decides.
            const uint32_t l = threadIdx.x;
            int cc[4];
            double cmax[4], cmin[4], cclb[4];
            uint32_t clen[4];
            int lane_c = 0;
            uint32_t lane_len = 0;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t j = 4 * l + u;
                const uint32_t cb = j * per, ce = cb + per < rest ? cb + per : rest;
                clen[u] = cb < ce ? ce - cb : 0;
                cc[u] = s_cnt[j];
                cmax[u] = s_max[j];
                cmin[u] = s_min[j];
                cclb[u] = s_clb[j];
                lane_c += clen[u] ? cc[u] : 0;
                lane_len += clen[u];
            }
            // exclusive scan of (inliers, points) over lanes
            int ex_c = lane_c;
            uint32_t ex_len = lane_len;
            for (int off = 1; off < 64; off <<= 1) {
                const int vc = __shfl_up(ex_c, off, 64);
                const uint32_t vl = __shfl_up(ex_len, off, 64);
                if ((int)l >= off) {
                    ex_c += vc;
                    ex_len += vl;
                }
            }
            ex_c -= lane_c;
            ex_len -= lane_len;
            // P at each chunk start; hi = its largest prefix P; lo = its smallest
            double hi[4], lo[4];
            int a = sv.cnt + ex_c;
            uint32_t t = kHead + ex_len;
            double lane_min = INFINITY;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const double P0 = (double)a * kc.lu + (double)(int)(t - (uint32_t)a) * kc.ld;
                hi[u] = clen[u] ? P0 + cmax[u] : -INFINITY;
                lo[u] = clen[u] ? P0 + cmin[u] : INFINITY;
                lane_min = fmin(lane_min, lo[u]);
                a += clen[u] ? cc[u] : 0;
                t += clen[u];
            }
            // exclusive prefix minimum over lanes (the head's minimum included)
            double ex_min = lane_min;
            for (int off = 1; off < 64; off <<= 1) {
                const double v = __shfl_up(ex_min, off, 64);
                if ((int)l >= off) ex_min = fmin(ex_min, v);
            }
            const double prev_lane_min = __shfl_up(ex_min, 1, 64);
            double mb = fmin(sv.pmin, l ? prev_lane_min : INFINITY);
            // first deciding chunk of this lane: 0..3, or 4 = none
            int first = 4;
            bool rej = false;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (first == 4 && clen[u]) {
                    const bool climb = fmax(cclb[u], hi[u] - mb) >= kc.climb;
                    if (climb || hi[u] > kc.lA - kc.margin) {
                        first = u;
                        rej = !climb && hi[u] > kc.lA + kc.margin;
                    }
                    mb = fmin(mb, lo[u]);
                }
            }
            const uint64_t hit = __ballot(first < 4);
            int exact = 0;
            if (hit) {
                const int src = __builtin_ctzll(hit);  // the lane holding the first deciding chunk
                const int srej = __builtin_amdgcn_readlane(rej ? 1 : 0, src);
                const int sfirst = __builtin_amdgcn_readlane(first, src);
                if (!srej) {
                    exact = 1;
                } else if (l == 0) {
                    counts[sv.slot] = -1;
                    sums[sv.slot] = 0.f;
                    // points read up to the deciding chunk's end (an upper bound of the test's)
                    const uint32_t ce = (4u * (uint32_t)src + (uint32_t)sfirst + 1u) * per;
                    if (tested_total) atomicAdd(tested_total, ce < rest ? ce : rest);
                }
            } else if (l == 0) {
                const int total = sv.cnt + __builtin_amdgcn_readlane(ex_c + lane_c, 63);
                counts[sv.slot] = total;
                sums[sv.slot] = (float)total;
                if (tested_total) atomicAdd(tested_total, rest);
            }
            if (l == 0) s_exact = exact;
        }
        if (threadIdx.x == 0 && sv.exact) s_exact = 1;
        __syncthreads();
        if (s_exact && threadIdx.x == 0) {  // not certified: the reference's sequential walk
            int c2 = 0;
            uint32_t t2 = 0;
            const uint32_t start0 = (sv.start + n - kHead) % n;
            const bool good = sprt_exact_walk<EST>(m, pool_pts, n, thr, start0, kc, c2, t2);
            counts[sv.slot] = good ? c2 : -1;
            sums[sv.slot] = good ? (float)c2 : 0.f;
            if (tested_total) atomicAdd(tested_total, t2 > kHead ? t2 - kHead : 0u);
        }
        __syncthreads();
    }
}

hipError_t launch_score_sprt(hipStream_t st, int estimator, const void *pool_pts, uint32_t n, const float *models,
                             size_t stride, const uint32_t *list, const uint32_t *list_n, uint32_t kmax, float thr,
                             const SprtConsts &kc, int32_t *counts, float *sums, uint32_t *tested_total, void *surv,
                             uint32_t *surv_n, uint32_t *starts) {
    hipError_t err = hipMemsetAsync(surv_n, 0, sizeof(uint32_t), st);
    if (err != hipSuccess) return err;
    const dim3 grid((kmax + 63) / 64);
    SprtSurvivor *sv = static_cast<SprtSurvivor *>(surv);
    const dim3 tgrid(kmax < 2048 ? (kmax ? kmax : 1) : 2048);
#define SS(E)                                                                                                         \
    do {                                                                                                              \
        hipLaunchKernelGGL(k_sprt_head<E>, grid, dim3(64), 0, st, pool_pts, n, models, stride, list, list_n, kmax, thr, \
                           kc, counts, sums, tested_total, sv, surv_n, starts);                                       \
        if (n > kHead)                                                                                                \
            hipLaunchKernelGGL(k_sprt_tail<E>, tgrid, dim3(256), 0, st, pool_pts, n, models, stride, thr, kc, sv,    \
                               surv_n, counts, sums, tested_total);                                                   \
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
