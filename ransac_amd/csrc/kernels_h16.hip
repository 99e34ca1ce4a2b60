// kernels_h16.hip -- the homography score with a matrix-core prefilter (gfx950 MFMA, fp16 in,
// fp32 accumulate), exact counts (DESIGN.md §6 "h16").
//
// Every (hypothesis, point) pair of the reference's Quality::getNumberInliers scan
// (quality.hpp:60-101, homography_estimator.hpp:85-110) needs e = (x2 Z - X, y2 Z - Y) and Z of
// H p1.  Each of the three is a dot product of nine per-hypothesis coefficients with nine per-point
// features f = (u, v, 1, p u, p v, p, q u, q v, q) of the centred, power-of-two-scaled coordinates
// (x1 = cx1 + s1 u, ..., x2 = cx2 + s2 p, y2 = cy2 + s2 q):
//   ex = x2 Z - X = sum over (u, v, 1) of (cx2 Z_k - X_k) f_k + sum over (p u, p v, p) of s2 Z_k f_k,
// likewise ey with (q u, q v, q), and Z with (u, v, 1).  So a 32-row x 32-point tile of them is ONE
// v_mfma_f32_32x32x16_f16: rows = (hypothesis, {ex, ey, Z}) for ten hypotheses (30 of 32 rows),
// columns = 32 points, K = the nine features (of 16).  The fp16 coefficients and features carry a
// rounding error, so the MFMA tile is a PREFILTER with a rigorous bound: per hypothesis a slack F_m
// (k_h16_rows) such that
//   max(|ex_m|, |ey_m|) > |zr_m| + F_m   ==>   max(|ex_fma|, |ey_fma|) > trm |Z_fma| + F,
// the packed stage A of k_score_hf (usac_hscore.hpp stage_a_keep2), which proves the reference's
// error is not below thr.  zr is the Z row times trm (1 + 2^-10).  The derivation: |f~ - f| <=
// 2^-11 |f| + 2^-25 (fp16 rounding, subnormal floor), |g~ - g| likewise plus the coefficients' own
// fp32 rounding (<= 2^-21 of the sum a_k of their terms' magnitudes), the MFMA's fp32 accumulation of 16
// exact fp16 products <= 2^-19 sum |g~ f~|; |f| <= fmax (dataset constants), so per row
// D = sum_k |g~_k| (2^-10 fmax_k + 2^-25) + fmax_k (2^-10 |g_k| + 2^-25 + 2^-21 a_k) + 2^-19 |g~_k| (fmax_k
// + 2^-24), and with the FMA chains' own errors (|ex_fma - ex| <= c.z dZ + dX, |Z_fma - Z| <= dZ,
// stage_a_bounds) F_m = [F + max(D_ex + c.z dZ + dX, D_ey + c.w dZ + dY) + trm' dZ + D_zr](1 + 2^-20),
// everything in the hypothesis' power-of-two scale 2^-c.  The (1 + 2^-10) on trm dominates the
// rounding of |zr_m| + F_m.  Non-finite hypotheses get zero rows and F_m = +inf (every pair goes to
// the exact stage); padding and non-finite points get NaN features (never kept -- the reference
// never counts them: their error is NaN or infinite).
//
// A kept pair goes to the exact stage B of k_score_hf (stage_b: v_rcp / v_sqrt with the guard band,
// the reference's own expression inside it) through a per-wave LDS queue of (hypothesis, point)
// entries, drained 64 at a time so every lane of the drain works (kept pairs are ~0.1 % of all).
// Counts are exact; Σ adds stage B's terms as 2^-k fixed point (integer adds: deterministic, an
// error of one unit per term), per point chunk, the chunks summed by k_h16_finish.
#include <hip/hip_runtime.h>
#include <math.h>

#include <stdlib.h>

#include <algorithm>

#include "usac_device.hpp"
#include "usac_h16.hpp"
#include "usac_hscore.hpp"
#include "usac_kernels.h"

namespace usac {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// queue entries per wave: a ring of < 64 waiting entries plus one iteration's appends (<= 64 per row)
template <int NA, int U>
constexpr uint32_t h16_queue() { return 64u * 5u * NA * U + 64u; }

// ------------------------------------------------------------------------ dataset constants
// One workgroup (once per context, at its first h16 batch; no host pass over the points): the
// box of the finite points, centres = the box midpoints rounded to fp32 (k_h16_rows works in
// fp32 and must use the very centres the features used), scales = the smallest powers of two
// >= the half-extents (every centred coordinate in [-1, 1]), then fmax[k] >= |f_k| over the
// finite points for the nine features in fp64 -- rounded up to a float above fmax (1 + 2^-40):
// k_h16_rows reads fmax as floats and the features' own fp64 evaluation may round up.
constexpr int kConstThreads = 1024;

__device__ __forceinline__ double h16_pow2_at_least(double v) { return v > 0 ? ldexp(1.0, ilogb(v) + 1) : 1.0; }

__global__ __launch_bounds__(kConstThreads) void k_h16_consts(const float4 *__restrict__ pts, uint32_t n, float4 ext,
                                                              H16Consts *__restrict__ out) {
    __shared__ double red[kConstThreads / 64][9];
    __shared__ double sc[6];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    // pass 1: min / max of the four coordinates over the finite points (max of -x for the min)
    double m[8];
#pragma unroll
    for (int k = 0; k < 8; k++) m[k] = -INFINITY;
    for (uint32_t i = t; i < n; i += kConstThreads) {
        const float4 p = pts[i];
        if (!(isfinite(p.x) && isfinite(p.y) && isfinite(p.z) && isfinite(p.w))) continue;
        const double c[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            m[k] = fmax(m[k], c[k]);
            m[4 + k] = fmax(m[4 + k], -c[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m[k] = fmax(m[k], __shfl_xor(m[k], o));
        if (lane == 0) red[w][k] = m[k];
    }
    __syncthreads();
    if (t == 0) {
        double hi[4], lo[4];
        for (int k = 0; k < 4; k++) {
            hi[k] = lo[k] = -INFINITY;
            for (int v = 0; v < kConstThreads / 64; v++) {
                hi[k] = fmax(hi[k], red[v][k]);
                lo[k] = fmax(lo[k], red[v][4 + k]);
            }
            lo[k] = -lo[k];
        }
        const bool any = hi[0] >= lo[0];  // a finite point exists
        double cc[4];
        for (int k = 0; k < 4; k++) cc[k] = any ? (double)(float)(0.5 * (lo[k] + hi[k])) : 0.0;
        const double e1 = fmax(fmax(hi[0] - cc[0], cc[0] - lo[0]), fmax(hi[1] - cc[1], cc[1] - lo[1]));
        const double e2 = fmax(fmax(hi[2] - cc[2], cc[2] - lo[2]), fmax(hi[3] - cc[3], cc[3] - lo[3]));
        sc[0] = cc[0];
        sc[1] = cc[1];
        sc[2] = any ? h16_pow2_at_least(e1) : 1.0;
        sc[3] = cc[2];
        sc[4] = cc[3];
        sc[5] = any ? h16_pow2_at_least(e2) : 1.0;
    }
    __syncthreads();
    const double cx1 = sc[0], cy1 = sc[1], s1 = sc[2], cx2 = sc[3], cy2 = sc[4], s2 = sc[5];
    // pass 2: max |f_k| (the same fp64 expressions as k_h16_points)
    double f[9];
#pragma unroll
    for (int k = 0; k < 9; k++) f[k] = 0.0;
    for (uint32_t i = t; i < n; i += kConstThreads) {
        const float4 p = pts[i];
        if (!(isfinite(p.x) && isfinite(p.y) && isfinite(p.z) && isfinite(p.w))) continue;
        const double u = ((double)p.x - cx1) / s1, v = ((double)p.y - cy1) / s1;
        const double pp = ((double)p.z - cx2) / s2, q = ((double)p.w - cy2) / s2;
        const double g[9] = {u, v, 1.0, pp * u, pp * v, pp, q * u, q * v, q};
#pragma unroll
        for (int k = 0; k < 9; k++) f[k] = fmax(f[k], fabs(g[k]));
    }
    __syncthreads();  // red[] is reused
#pragma unroll
    for (int k = 0; k < 9; k++) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) f[k] = fmax(f[k], __shfl_xor(f[k], o));
        if (lane == 0) red[w][k] = f[k];
    }
    __syncthreads();
    if (t == 0) {
        H16Consts k;
        k.cx1 = cx1;
        k.cy1 = cy1;
        k.s1 = s1;
        k.cx2 = cx2;
        k.cy2 = cy2;
        k.s2 = s2;
        for (int q = 0; q < 9; q++) {
            double mx = 0.0;
            for (int v = 0; v < kConstThreads / 64; v++) mx = fmax(mx, red[v][q]);
            k.fmax[q] = (double)nextafterf((float)(mx * (1.0 + 0x1p-40)), INFINITY);
        }
        k.ext = ext;
        *out = k;
    }
}

hipError_t launch_h16_consts(hipStream_t st, const float4 *pts, uint32_t n, float4 ext, H16Consts *out) {
    hipLaunchKernelGGL(k_h16_consts, dim3(1), dim3(kConstThreads), 0, st, pts, n, ext, out);
    return hipGetLastError();
}

size_t h16_feature_bytes(uint32_t n) { return (size_t)((n + 31) / 32) * 1024; }

// one thread per (32-point block, lane): lane l holds B[k = 8 (l >> 5) + j][column l & 31]
__global__ __launch_bounds__(256) void k_h16_points(const float4 *__restrict__ pts, uint32_t n,
                                                    const H16Consts *__restrict__ kc, half8 *__restrict__ feat) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    const uint32_t nblk = (n + 31) / 32;
    if (t >= nblk * 64) return;
    const uint32_t blk = t >> 6, l = t & 63, i = blk * 32 + (l & 31), hf = l >> 5;
    half8 o;
    bool ok = i < n;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) {
        p = pts[i];
        ok = isfinite(p.x) && isfinite(p.y) && isfinite(p.z) && isfinite(p.w);
    }
    if (!ok) {
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = (_Float16)__builtin_nanf("");
    } else {
        const double u = ((double)p.x - kc->cx1) / kc->s1, v = ((double)p.y - kc->cy1) / kc->s1;
        const double pp = ((double)p.z - kc->cx2) / kc->s2, q = ((double)p.w - kc->cy2) / kc->s2;
        const double f[16] = {u, v, 1.0, pp * u, pp * v, pp, q * u, q * v, q, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = (_Float16)(float)f[8 * hf + j];
    }
    feat[t] = o;
}

hipError_t launch_h16_points(hipStream_t st, const float4 *pts, uint32_t n, const H16Consts *k, void *feat) {
    const uint32_t threads = (n + 31) / 32 * 64;
    hipLaunchKernelGGL(k_h16_points, dim3((threads + 255) / 256), dim3(256), 0, st, pts, n, k,
                       static_cast<half8 *>(feat));
    return hipGetLastError();
}

// ------------------------------------------------------------------------ per-hypothesis rows
// (the solvers write them themselves for usac_hypothesize* batches; this kernel serves the others)
__global__ __launch_bounds__(256) void k_h16_rows(const float *__restrict__ models, uint32_t B,
                                                  const H16Consts *__restrict__ kc, float thr,
                                                  half8 *__restrict__ rows, float *__restrict__ fm) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
    float Hm[9];
#pragma unroll
    for (int c = 0; c < 9; c++) Hm[c] = models[(size_t)c * B + h];
    h16_rows_of(Hm, kc, thr, h, rows, fm);
}

hipError_t launch_h16_rows(hipStream_t st, const float *models, uint32_t B, const H16Consts *k, float thr, void *rows,
                           float *fm) {
    hipLaunchKernelGGL(k_h16_rows, dim3((B + 255) / 256), dim3(256), 0, st, models, B, k, thr,
                       static_cast<half8 *>(rows), fm);
    return hipGetLastError();
}

// ------------------------------------------------------------------------ the scorer
// LDS ordering inside one wave (the queue, the model table, the counters): a workgroup-scope fence
// waits for the wave's LDS operations and keeps the compiler from moving them across
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// Drain `cnt` (<= 64) queue entries from `head`: lane i evaluates entry head + i exactly (stage_b,
// throughput mode: S ~ 2 err, or the exact 2 err inside the band) and adds its inlier to the
// hypothesis' LDS counters (count, Σ in 2^-fxs fixed point).
template <uint32_t Q>
__device__ __forceinline__ void h16_drain(uint32_t cnt, uint32_t head, uint32_t *q, const float (*sh)[20],
                                          uint32_t *sc, unsigned long long *ss, const float4 *__restrict__ pts,
                                          float T, float thr, double fxs) {
    const uint32_t lane = threadIdx.x & 63;
    wave_lds_sync();
    if (lane < cnt) {
        const uint32_t qi = head + lane;  // head < Q
        const uint32_t e = q[qi >= Q ? qi - Q : qi];
        const uint32_t hk = e >> 25, p = e & 0x1FFFFFFu;
        const float4 pt = pts[p];
        HModel M;
#pragma unroll
        for (int c = 0; c < 9; c++) {
            M.h[c] = sh[hk][c];
            M.hi[c] = sh[hk][9 + c];
        }
        // the point's guard band, as k_prepare_rec writes it
        const float mp = fabsf(pt.x) + fabsf(pt.y) + fabsf(pt.z) + fabsf(pt.w);
        const float band = kBandMp * mp + kBandT * T;
        int c = 0;
        float s = 0.f;
        stage_b<false>(M, pt.x, pt.y, pt.z, pt.w, band, T, thr, c, s);
        if (c) {
            atomicAdd(&sc[hk], 1u);
            atomicAdd(&ss[hk], (unsigned long long)llrint((double)s * fxs));
        }
    }
    wave_lds_sync();
}

// Workgroup = 4 waves; wave w owns hypotheses [hb, hb + 10 NA) and point chunk blockIdx.y.
// A fragments (lane l: row l & 31 of each 32-row tile, coefficients 8 (l >> 5) ..): row rho holds
// (hypothesis t, component r) with i = (rho & 3) + 4 (rho >> 3), t = 5 ((rho >> 2) & 1) + i / 3, r = i % 3
// (i < 15; row i = 15 of each lane half is spare), so that the D register q of lane half hf holds
// (hypothesis 5 hf + q / 3, component q % 3): each lane owns whole (ex, ey, zr) triples of five
// hypotheses of each tile for its point.
template <int NA, int U, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_score_h16(const half8 *__restrict__ feat, const float4 *__restrict__ pts,
                                                   uint32_t n, const half8 *__restrict__ rows,
                                                   const float *__restrict__ fm, const float *__restrict__ models,
                                                   uint32_t B, float thr, double fxs, uint32_t *__restrict__ cpart,
                                                   unsigned long long *__restrict__ spart) {
    constexpr int HW = 10 * NA;
    __shared__ float sH[4][HW][20];
    __shared__ uint32_t sC[4][HW];
    __shared__ unsigned long long sS[4][HW];
    constexpr uint32_t Q = h16_queue<NA, U>();
    __shared__ uint32_t sQ[4][Q];
    const uint32_t lane = threadIdx.x & 63, hf = lane >> 5;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t hb = (blockIdx.x * 4 + wave) * HW;
    const float T = 2.0f * thr;
    if (lane < HW) {
        const uint32_t h = hb + lane;
#pragma unroll
        for (int c = 0; c < 18; c++) sH[wave][lane][c] = h < B ? models[(size_t)c * B + h] : 0.f;
        sC[wave][lane] = 0;
        sS[wave][lane] = 0;
    }
    half8 A[NA];
    float F[NA][5];
    {
        const uint32_t rho = lane & 31, rh = (rho >> 2) & 1, i = (rho & 3) + 4 * (rho >> 3);
        const uint32_t t = 5 * rh + i / 3, r = i % 3;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            const uint32_t h = hb + 10 * a + t;
            half8 z;
#pragma unroll
            for (int j = 0; j < 8; j++) z[j] = (_Float16)0.0f;
            A[a] = (i < 15 && h < B) ? rows[((size_t)h * 3 + r) * 2 + hf] : z;
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const uint32_t hj = hb + 10 * a + 5 * hf + j;
                F[a][j] = hj < B ? fm[hj] : -1.0f;  // a missing hypothesis keeps nothing (0 <= -1 is false)
            }
        }
    }
    const uint32_t nblk = (n + 31) / 32, nch = gridDim.y, ch = blockIdx.y;
    const uint32_t per = (nblk + nch - 1) / nch;
    const uint32_t b0 = ch * per < nblk ? ch * per : nblk, b1 = b0 + per < nblk ? b0 + per : nblk;
    uint32_t qn = 0, qh = 0;
    const f32x16 zero = {};
    wave_lds_sync();
    // U 32-point blocks per iteration (their MFMAs issue back to back, then all the tests), the next
    // iteration's blocks' features loaded while this iteration's tiles are tested
    half8 bn[U];
#pragma unroll
    for (int u = 0; u < U; u++) bn[u] = b0 + u < b1 ? feat[(size_t)(b0 + u) * 64 + lane] : half8{};
    for (uint32_t blk = b0; blk < b1; blk += U) {
        half8 bf[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            bf[u] = bn[u];
            if (blk + U + u < b1) bn[u] = feat[(size_t)(blk + U + u) * 64 + lane];
        }
        f32x16 acc[U][NA];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int a = 0; a < NA; a++) acc[u][a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[a], bf[u], zero, 0, 0, 0);
        uint64_t msk[U][NA][5], any = 0;
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int a = 0; a < NA; a++)
#pragma unroll
                for (int j = 0; j < 5; j++) {
                    // keep iff |ex| <= R and |ey| <= R, R = |zr| + F: two compares with |.| source
                    // modifiers (a max would first canonicalise both operands in IEEE mode); a block
                    // past the chunk's end keeps nothing
                    const float R = fabsf(acc[u][a][3 * j + 2]) + F[a][j];
                    msk[u][a][j] = blk + u < b1 ? __builtin_amdgcn_ballot_w64(fabsf(acc[u][a][3 * j]) <= R) &
                                                      __builtin_amdgcn_ballot_w64(fabsf(acc[u][a][3 * j + 1]) <= R)
                                                : 0;
                    any |= msk[u][a][j];
                }
        if (__builtin_expect(any != 0, 0)) {  // append the kept pairs, draining full groups of 64 per block
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t point = (blk + u) * 32 + (lane & 31);
#pragma unroll
                for (int a = 0; a < NA; a++)
#pragma unroll
                    for (int j = 0; j < 5; j++) {
                        const uint64_t mk = msk[u][a][j];
                        if (mk) {
                            const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                                (uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
                            if ((mk >> lane) & 1) {
                                const uint32_t qi = qh + qn + below;  // < 2 Q
                                sQ[wave][qi >= Q ? qi - Q : qi] = ((uint32_t)(10 * a + 5 * hf + j) << 25) | point;
                            }
                            qn += (uint32_t)__builtin_popcountll(mk);
                        }
                    }
                while (qn >= 64) {
                    h16_drain<Q>(64, qh, sQ[wave], sH[wave], sC[wave], sS[wave], pts, T, thr, fxs);
                    qh = qh + 64 >= Q ? qh + 64 - Q : qh + 64;
                    qn -= 64;
                }
            }
        }
    }
    while (qn) {
        const uint32_t d = qn < 64 ? qn : 64;
        h16_drain<Q>(d, qh, sQ[wave], sH[wave], sC[wave], sS[wave], pts, T, thr, fxs);
        qh = qh + d >= Q ? qh + d - Q : qh + d;
        qn -= d;
    }
    wave_lds_sync();
    if (lane < HW && hb + lane < B) {
        cpart[(size_t)ch * B + hb + lane] = sC[wave][lane];
        spart[(size_t)ch * B + hb + lane] = sS[wave][lane];
    }
}

// counts / sums from the chunk partials (integers: any order gives the same result)
__global__ __launch_bounds__(256) void k_h16_finish(const uint32_t *__restrict__ cpart,
                                                    const unsigned long long *__restrict__ spart, uint32_t B,
                                                    uint32_t nch, double inv_fxs, int32_t *__restrict__ counts,
                                                    float *__restrict__ sums) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
    uint32_t c = 0;
    unsigned long long s = 0;
    for (uint32_t y = 0; y < nch; y++) {
        c += cpart[(size_t)y * B + h];
        s += spart[(size_t)y * B + h];
    }
    counts[h] = (int32_t)c;
    sums[h] = (float)((double)s * inv_fxs * 0.5);  // stage B adds S ~ 2 err (k_score_hf halves at the end)
}

size_t h16_part_bytes(uint32_t B, int chunks) { return (size_t)chunks * B * (sizeof(uint32_t) + sizeof(uint64_t)); }

int h16_fixed_point(float thr) {
    const double T = 2.0 * (double)thr;
    return T > 0 ? 39 - ilogb(T) : 40;
}

hipError_t launch_score_h16(hipStream_t st, const void *feat, const float4 *pts, uint32_t n, const void *rows,
                            const float *fm, const float *models, uint32_t B, float thr, int chunks, void *part,
                            int32_t *counts, float *sums, bool finish) {
    static const int na = getenv("USAC_H16_NA") ? atoi(getenv("USAC_H16_NA")) : 2;  // 10-hypothesis tiles per wave
    if (chunks < 1 || n == 0 || n > 0x2000000u) return hipErrorInvalidValue;  // 25-bit point indices in the queue
    // Σ in fixed point: a stage-B term is < 2 T (1 + 2^-15) (S ~ 2 err of an inlier, err < thr = T / 2), so
    // 2^fx with 2 T 2^fx <= 2^40 leaves 2^23 terms per hypothesis and chunk below 2^63: a chunk of more
    // than 2^23 points could wrap its partial, so such a launch is refused (h16_chunks never asks for one)
    const uint32_t nblk = (n + 31) / 32, per = (nblk + (uint32_t)chunks - 1) / (uint32_t)chunks;
    if ((uint64_t)per * 32 > (1u << 23)) return hipErrorInvalidValue;
    const int fx = h16_fixed_point(thr);
    const double fxs = ldexp(1.0, fx);
    unsigned long long *sp = static_cast<unsigned long long *>(part);  // 8-byte words first (alignment)
    uint32_t *cp = reinterpret_cast<uint32_t *>(sp + (size_t)chunks * B);
    static const int uu = getenv("USAC_H16_U") ? atoi(getenv("USAC_H16_U")) : 1;  // blocks per iteration
    // min waves per SIMD: 8 (64 VGPRs, no spills) -- same-box cfg2 559-570 vs 551-555 M hyp/s at 7
    static const int wpe = getenv("USAC_H16_WPE") ? atoi(getenv("USAC_H16_WPE")) : 8;
#define H16(NA_, U_, W_)                                                                                            \
    hipLaunchKernelGGL((k_score_h16<NA_, U_, W_>), dim3((B + 40 * NA_ - 1) / (40 * NA_), chunks), dim3(256), 0, st,   \
                       static_cast<const half8 *>(feat), pts, n, static_cast<const half8 *>(rows), fm, models, B, thr, \
                       fxs, cp, sp)
    if (na == 4)
        H16(4, 1, 1);
    else if (uu == 2)
        H16(2, 2, 1);
    else if (wpe == 8)
        H16(2, 1, 8);
    else
        H16(2, 1, 1);
#undef H16
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !finish) return e;  // !finish: the caller's launch_argmax_h16 adds the chunks
    hipLaunchKernelGGL(k_h16_finish, dim3((B + 255) / 256), dim3(256), 0, st, cp, sp, B, (uint32_t)chunks,
                       ldexp(1.0, -fx), counts, sums);
    return hipGetLastError();
}

}  // namespace usac
