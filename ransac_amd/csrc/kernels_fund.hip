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
#include "usac_pk.hpp"

namespace usac {

// SevenPointsAlgorithm + EstimateModel validity filter for one sample per lane:
// 7 x 9 fp64 rows -> QR null basis (f1, f2; row Jacobi + null complement as the fall-back) ->
// fp32 cubic coefficients ->
// IEEE cubic roots -> F per root -> oriented filter -> slot write + compaction.
__global__ __launch_bounds__(64) void k_solve_f7(const float4 *__restrict__ pts, uint32_t n,
                                                 const int32_t *__restrict__ samples_in, int32_t *samples_out,
                                                 uint32_t B, DevSampler ds, uint64_t first_hyp,
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
            draw_sample<7>(ds, first_hyp + h, n, s);
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
        double N[2][9];
        if (!qr_null<7>(W, N)) {  // a zero / non-finite column: the row-Jacobi completion
#pragma unroll
            for (int i = 0; i < 7; i++) {
                const float4 p = pts[s[i]];
                fund_row(p.x, p.y, p.z, p.w, W[i]);
            }
            row_jacobi<7>(W);
            null_complement7(W, N);
        }
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

// ---------------------------------------------------------------- fast two-view scoring
// Same results as k_score_f (counts and Σerr bit for bit):
//
//   stage A  FMA chains (two points per v_pk_fma_f32) for the quantities of the reference's
//            residual, then a division- and sqrt-free test that only rejects pairs whose
//            REFERENCE error is provably >= thr.  The fused values differ from the reference's
//            (rounded, differently associated) ones by at most per-model bounds derived from
//            the dataset box |x1| <= c.x, |y1| <= c.y, |x2| <= c.z, |y2| <= c.w (DESIGN.md
//            "Two-view stage A" has the derivation); the test absorbs them:
//              Sampson   e = S/D, s the numerator root:  reject iff ¬(s² <= D K + C)
//              essential e = (|a1/a2| + |b1/b2|)/2:      reject iff ¬(a1² <= Qa K + C)
//            with K = thr (1 + 2^-9) resp. 4 thr² (1 + 2^-9) and C = (δD K + 1026 δs²)(1 + 2^-20)
//            (δ = the per-model bounds), C >= 2^-126.  Models whose bounds are not finite and
//            <= 2^60 (overflow could otherwise hide in the fused chain) skip stage A: every
//            point of theirs goes to stage B.  A NaN point rejects (its exact error is NaN);
//   stage B  the exact expression (two_view_error) on the kept pairs only, sequential
//            accumulation per model (see the queues below).
//
// Points come from the fast-kernel records (k_prepare_rec: SoA groups of four, NaN-padded
// tail, never queued).

template <int EST>
struct TwoViewModel {
    float f[9];
    v2f f2[9];
    v2f K, C;          // stage-A test constants, duplicated for the packed halves
    uint32_t all;      // 0xFF: stage A disabled for this model (every point kept)
};

__device__ __forceinline__ float ceil_fudge(float x) { return x * 1.00000095367431640625f; }  // (1 + 2^-20)

template <int EST>
__device__ __forceinline__ void two_view_setup(TwoViewModel<EST> &M, float4 c, float thr) {
    const float *f = M.f;
#pragma unroll
    for (int k = 0; k < 9; k++) M.f2[k] = v2f{f[k], f[k]};
    float dv2, ds2, lim1, lim2;  // bound of the squared quantity's error, of the root's error^2
    float K;
    if constexpr (EST == USAC_ESSENTIAL) {
        const float L1 = ceil_fudge(fabsf(f[0]) * c.z + fabsf(f[3]) * c.w + fabsf(f[6]));
        const float L2 = ceil_fudge(fabsf(f[1]) * c.z + fabsf(f[4]) * c.w + fabsf(f[7]));
        const float L3 = ceil_fudge(fabsf(f[2]) * c.z + fabsf(f[5]) * c.w + fabsf(f[8]));
        const float Aa = ceil_fudge(L1 * c.x + L2 * c.y + L3);
        const float LQ = ceil_fudge(L1 * L1 + L2 * L2);
        const float da = ceil_fudge(Aa * 9.5367431640625e-07f);  // 2^-20 Aa
        dv2 = ceil_fudge(LQ * 1.9073486328125e-06f);             // δQ = 2^-19 LQ
        ds2 = ceil_fudge(da * da);
        lim1 = Aa;
        lim2 = LQ;
        K = ((4.0f * thr) * thr) * 1.001953125f;                  // 4 thr² (1 + 2^-9)
    } else {
        const float LFx = ceil_fudge(fabsf(f[0]) * c.x + fabsf(f[1]) * c.y + fabsf(f[2]));
        const float LFy = ceil_fudge(fabsf(f[3]) * c.x + fabsf(f[4]) * c.y + fabsf(f[5]));
        const float LGx = ceil_fudge(fabsf(f[0]) * c.z + fabsf(f[3]) * c.w + fabsf(f[6]));
        const float LGy = ceil_fudge(fabsf(f[1]) * c.z + fabsf(f[4]) * c.w + fabsf(f[7]));
        const float Ls =
            ceil_fudge(c.z * LFx + c.w * LFy + fabsf(f[6]) * c.x + fabsf(f[7]) * c.y + fabsf(f[8]));
        const float LD = ceil_fudge(LFx * LFx + LFy * LFy + LGx * LGx + LGy * LGy);
        const float ds = ceil_fudge(Ls * 1.9073486328125e-06f);  // δs = 2^-19 Ls
        dv2 = ceil_fudge(LD * 1.9073486328125e-06f);             // δD = 2^-19 LD
        ds2 = ceil_fudge(ds * ds);
        lim1 = Ls;
        lim2 = LD;
        K = thr * 1.001953125f;                                   // thr (1 + 2^-9)
    }
    float C = ceil_fudge(ceil_fudge(dv2 * K) + ceil_fudge(1026.0f * ds2));
    C = C > 1.17549435e-38f ? C : 1.17549435e-38f;                // >= 2^-126
    M.all = (lim1 <= 1.152921504606846976e18f && lim2 <= 1.329227995784915873e36f) ? 0u : 0xFFu;  // 2^60, 2^120
    M.K = v2f{K, K};
    M.C = v2f{C, C};
}

// stage A for two points: true = sure outlier
template <int EST>
__device__ __forceinline__ void two_view_reject2(const TwoViewModel<EST> &M, v2f x1, v2f y1, v2f x2, v2f y2,
                                                 bool &r0, bool &r1) {
    const v2f *f = M.f2;
    v2f A, T;
    if constexpr (EST == USAC_ESSENTIAL) {
        const v2f l1 = vfma(f[0], x2, vfma(f[3], y2, f[6]));
        const v2f l2 = vfma(f[1], x2, vfma(f[4], y2, f[7]));
        const v2f l3 = vfma(f[2], x2, vfma(f[5], y2, f[8]));
        const v2f a1 = vfma(l1, x1, vfma(l2, y1, l3));
        const v2f Qa = vfma(l1, l1, l2 * l2);
        A = a1 * a1;
        T = vfma(Qa, M.K, M.C);
    } else {
        const v2f Fx = vfma(f[0], x1, vfma(f[1], y1, f[2]));
        const v2f Fy = vfma(f[3], x1, vfma(f[4], y1, f[5]));
        const v2f Gx = vfma(f[0], x2, vfma(f[3], y2, f[6]));
        const v2f Gy = vfma(f[1], x2, vfma(f[4], y2, f[7]));
        const v2f sv = vfma(
            x2, Fx, vfma(y2, Fy, vfma(f[6], x1, vfma(f[7], y1, f[8]))));
        const v2f D = vfma(
            Fx, Fx, vfma(Fy, Fy, vfma(Gx, Gx, Gy * Gy)));
        A = sv * sv;
        T = vfma(D, M.K, M.C);
    }
#ifdef TV_EXP_NOKEEP
    r0 = !(A.x <= T.x) || true;
    r1 = !(A.y <= T.y) || true;
#else
    r0 = !(A.x <= T.x);
    r1 = !(A.y <= T.y);
#endif
}

// Stage B is deferred: per eight points (two groups) a lane appends one entry -- the group
// index and an 8-bit mask of the points its model kept -- to a private LDS queue, only when
// the mask is not empty.  When some lane's queue is full, and at the end, the wave drains
// all queues together, entry t of every lane per trip, each lane evaluating the exact
// expression on its own kept points in point order (sequential Σ, bit-exact).  Stage A keeps
// ~1 % of the (model, point) pairs on typical data, so a per-group "any lane kept a point"
// branch would run the exact path nearly always; the queues run it only for kept pairs.
constexpr int kTvQueue = 16;  // entries per lane (4 KB of LDS per wave)

// essential_error_guarded (usac_device_e5.hpp): the throughput drains' guarded essential residual

template <int EST>
__device__ __forceinline__ void two_view_drain(const TwoViewModel<EST> &M, const float4 *__restrict__ pts,
                                               const uint32_t *q, int &len, float thr, int &cnt, float &sum,
                                               bool fast = false, float lo = 0.f, float hi = 0.f) {
    // each lane walks its kept points in order, two per trip: the two loads and exact
    // evaluations of a trip are independent (latency overlap), the adds stay in order
    int t = 0;
    uint32_t m = 0, base = 0;
    for (;;) {
        if (m == 0 && t < len) {  // queue entries never have an empty mask
            const uint32_t e = q[t * 64];
            t++;
            m = e & 255u;
            base = (e >> 8) * 4;
        }
        const bool h0 = m != 0;
        const uint32_t i0 = h0 ? base + __builtin_ctz(m) : 0u;
        m &= m - 1;
        if (m == 0 && t < len) {
            const uint32_t e = q[t * 64];
            t++;
            m = e & 255u;
            base = (e >> 8) * 4;
        }
        const bool h1 = m != 0;
        const uint32_t i1 = h1 ? base + __builtin_ctz(m) : 0u;
        m &= m - 1;
        if (!__builtin_amdgcn_ballot_w64(h0)) break;
        const float4 p0 = pts[i0];
        const float4 p1 = pts[i1];
#ifdef TV_EXP_CHEAPDRAIN  // A/B hook: the drain's loads and queue walk, a trivial residual
        const float e0 = fabsf(p0.x * M.f[0] + p0.w), e1 = fabsf(p1.x * M.f[0] + p1.w);
        const bool in0 = e0 < thr, in1 = e1 < thr;
#else
        float e0, e1;
        bool in0, in1;
        if (EST == USAC_ESSENTIAL && fast) {  // wave-uniform
            e0 = essential_error_guarded(M.f, p0.x, p0.y, p0.z, p0.w, thr, lo, hi, in0);
            e1 = essential_error_guarded(M.f, p1.x, p1.y, p1.z, p1.w, thr, lo, hi, in1);
        } else {
            e0 = two_view_error<EST>(M.f, p0.x, p0.y, p0.z, p0.w);
            e1 = two_view_error<EST>(M.f, p1.x, p1.y, p1.z, p1.w);
            in0 = e0 < thr;
            in1 = e1 < thr;
        }
#endif
        if (h0 && in0) {
            cnt++;
            sum += e0;
        }
        if (h1 && in1) {
            cnt++;
            sum += e1;
        }
    }
    len = 0;
}

// stage A of four points -> 4-bit mask of the kept ones
template <int EST>
__device__ __forceinline__ uint32_t two_view_group(const TwoViewModel<EST> &M, float4 X1, float4 Y1, float4 X2,
                                                   float4 Y2) {
    bool r0, r1, r2, r3;
    two_view_reject2<EST>(M, v2f{X1.x, X1.y}, v2f{Y1.x, Y1.y}, v2f{X2.x, X2.y}, v2f{Y2.x, Y2.y}, r0, r1);
    two_view_reject2<EST>(M, v2f{X1.z, X1.w}, v2f{Y1.z, Y1.w}, v2f{X2.z, X2.w}, v2f{Y2.z, Y2.w}, r2, r3);
    return (r0 ? 0u : 1u) | (r1 ? 0u : 2u) | (r2 ? 0u : 4u) | (r3 ? 0u : 8u);
}

// append (g, mask) when the mask is not empty (the slot is written either way).  Points
// 4g .. 4g+7 past n (the NaN padding) are masked off: a model without stage A keeps all.
__device__ __forceinline__ void two_view_append(uint32_t *q, int &len, uint32_t g, uint32_t n, uint32_t mask) {
    if (4 * g + 8 > n) mask &= (1u << (n - 4 * g)) - 1u;  // wave-uniform: the last group(s) only
    q[64 * len] = (g << 8) | mask;
    len += mask ? 1 : 0;
}

// One wave per workgroup: blockIdx.x = 64 listed models, blockIdx.y = point chunk.  With
// one chunk the wave writes (count, Σ) at the slots; with C > 1 it writes its partials at
// [chunk][list position] and k_tv_combine adds them in chunk order (deterministic).  Small
// workgroups spread the few model tiles of a two-view batch evenly over the 256 CUs.
template <int EST>
__global__ __launch_bounds__(64) void k_score_f2(const float4 *__restrict__ rec, const float4 *__restrict__ pts,
                                                 uint32_t n, float4 ext, const float *__restrict__ models, size_t stride,
                                                 const uint32_t *__restrict__ list,
                                                 const uint32_t *__restrict__ list_n, uint32_t kmax, float thr,
                                                 const uint32_t *__restrict__ perm,
                                                 int32_t *__restrict__ counts, float *__restrict__ sums,
                                                 int32_t *__restrict__ part_cnt, float *__restrict__ part_sum) {
    __shared__ uint32_t s_q[kTvQueue * 64];
    const uint32_t lane = threadIdx.x;
    const uint32_t chunk = blockIdx.y, C = gridDim.y;
    const uint32_t K = list ? __builtin_amdgcn_readfirstlane(*list_n) : kmax;
    const uint32_t i0 = blockIdx.x * 64;
    if (i0 >= K) return;  // block-uniform
    const uint32_t j = i0 + lane < K ? i0 + lane : K - 1;
    const uint32_t ic = perm ? perm[j] : j;  // list position scored by this lane
    const bool live = i0 + lane < K;
    const uint32_t slot = list ? list[ic] : ic;
    TwoViewModel<EST> M;
#pragma unroll
    for (int k = 0; k < 9; k++) M.f[k] = models[(size_t)k * stride + slot];
    two_view_setup<EST>(M, ext, thr);
    const uint32_t ngroups = (n + 3) / 4;
    const uint32_t per = (ngroups + C - 1) / C;
    const uint32_t gbeg = chunk * per < ngroups ? chunk * per : ngroups;
    const uint32_t gend = gbeg + per < ngroups ? gbeg + per : ngroups;
    // throughput launches (C > 1: Σ re-associated over chunks): the essential drains take the
    // guarded residual (essential_error_guarded; counts exact, Σ terms within 2^-19 relative)
    const bool fast = EST == USAC_ESSENTIAL && C > 1 && thr >= 7.888609052210118e-31f && thr < 1.0e30f;  // 2^-100
    const float lo = thr * 0.9999847412109375f, hi = thr * 1.0000152587890625f;  // thr (1 -+ 2^-16)
    uint32_t *q = &s_q[lane];
    int len = 0, cnt = 0;
    float sum = 0.f;
    uint32_t g = gbeg;
    if (g + 2 <= gend) {
        // software-pipelined scalar loads: the next two groups are in flight while the
        // current two are evaluated
        const float4 *p = rec + 8 * (size_t)g;
        float4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
        float4 b0 = p[8], b1 = p[9], b2 = p[10], b3 = p[11];
        for (; g + 2 <= gend; g += 2) {
            const uint32_t gn = g + 4 <= gend ? g + 2 : g;
            const float4 *pn = rec + 8 * (size_t)gn;
            const float4 c0 = pn[0], c1 = pn[1], c2 = pn[2], c3 = pn[3];
            const float4 d0 = pn[8], d1 = pn[9], d2 = pn[10], d3 = pn[11];
            const uint32_t ma = two_view_group<EST>(M, a0, a1, a2, a3);
            const uint32_t mb = two_view_group<EST>(M, b0, b1, b2, b3);
#ifdef TV_EXP_NODRAIN  // A/B hook: stage A computed, nothing queued (stage-A cost alone)
            uint32_t sink = ma | (mb << 4);
            __asm__ volatile("" : "+v"(sink));
            two_view_append(q, len, g, n, sink & 0u);
#else
            two_view_append(q, len, g, n, ma | (mb << 4) | M.all);
#endif
            if (__builtin_amdgcn_ballot_w64(len == kTvQueue))
                two_view_drain<EST>(M, pts, q, len, thr, cnt, sum, fast, lo, hi);
            a0 = c0; a1 = c1; a2 = c2; a3 = c3;
            b0 = d0; b1 = d1; b2 = d2; b3 = d3;
        }
    }
    if (g < gend) {
        const float4 *p = rec + 8 * (size_t)g;
        two_view_append(q, len, g, n, (two_view_group<EST>(M, p[0], p[1], p[2], p[3]) | M.all) & 0xFu);
    }
    two_view_drain<EST>(M, pts, q, len, thr, cnt, sum, fast, lo, hi);
    if (!live) return;
    if (C == 1) {
        counts[slot] = cnt;
        sums[slot] = sum;
    } else {
        part_cnt[(size_t)chunk * kmax + ic] = cnt;
        part_sum[(size_t)chunk * kmax + ic] = sum;
    }
}

// Model pre-sort for k_score_f2: stage-A keeps of every listed model on the first
// kTvPresortGroups point groups (the exact stage-A test -- a heuristic only for WHERE a model
// is scored, never for its result).  Models with >= kTvPresortKeeps keeps (those with many
// inliers, whose queues fill fast) go to the front of perm, the rest to the back, so the
// costly drains concentrate in few waves instead of one slow lane per wave.
constexpr uint32_t kTvPresortGroups = 32;  // 128 points
constexpr int kTvPresortKeeps = 8;

template <int EST>
__global__ __launch_bounds__(64) void k_presort_tv(const float4 *__restrict__ rec, uint32_t n, float4 ext,
                                                   const float *__restrict__ models, size_t stride,
                                                   const uint32_t *__restrict__ list,
                                                   const uint32_t *__restrict__ list_n, uint32_t kmax, float thr,
                                                   uint32_t *__restrict__ perm, uint32_t *__restrict__ ends) {
    const uint32_t lane = threadIdx.x;
    const uint32_t K = list ? __builtin_amdgcn_readfirstlane(*list_n) : kmax;
    const uint32_t i0 = blockIdx.x * 64;
    if (i0 >= K) return;
    const uint32_t i = i0 + lane;
    const uint32_t ic = i < K ? i : K - 1;
    const uint32_t slot = list ? list[ic] : ic;
    TwoViewModel<EST> M;
#pragma unroll
    for (int k = 0; k < 9; k++) M.f[k] = models[(size_t)k * stride + slot];
    two_view_setup<EST>(M, ext, thr);
    const uint32_t ngroups = (n + 3) / 4;
    const uint32_t g1 = ngroups < kTvPresortGroups ? ngroups : kTvPresortGroups;
    int keeps = 0;
    for (uint32_t g = 0; g < g1; g++) {
        const float4 *p = rec + 8 * (size_t)g;
        keeps += __builtin_popcount(two_view_group<EST>(M, p[0], p[1], p[2], p[3]) | (M.all & 0xFu));
    }
    const bool valid = i < K;
    const bool heavy = valid && keeps >= kTvPresortKeeps;
    const uint64_t bh = __ballot(heavy), bl = __ballot(valid && !heavy);
    const uint64_t below_mask = (1ull << lane) - 1;
    const uint32_t below = (uint32_t)__popcll((heavy ? bh : bl) & below_mask);
    uint32_t hbase = 0, lbase = 0;
    if (lane == 0) {
        if (bh) hbase = atomicAdd(&ends[0], (uint32_t)__popcll(bh));
        if (bl) lbase = atomicAdd(&ends[1], (uint32_t)__popcll(bl));
    }
    hbase = __shfl(hbase, 0, 64);
    lbase = __shfl(lbase, 0, 64);
    if (valid) perm[heavy ? hbase + below : K - 1 - (lbase + below)] = i;
}

// (count, Σ) of listed model i = chunk partials added in chunk order
__global__ __launch_bounds__(256) void k_tv_combine(const uint32_t *__restrict__ list,
                                                    const uint32_t *__restrict__ list_n, uint32_t kmax, uint32_t C,
                                                    const int32_t *__restrict__ part_cnt,
                                                    const float *__restrict__ part_sum, int32_t *__restrict__ counts,
                                                    float *__restrict__ sums) {
    const uint32_t K = list ? *list_n : kmax;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= K) return;
    // the chunks in order, 16 chunks' loads in flight per 16 adds (one thread per model: at a
    // few hundred waves for the whole batch, a load per add would wait a memory latency each)
    int c = part_cnt[i];
    float s = part_sum[i];
    uint32_t j = 1;
    for (; j + 16 <= C; j += 16) {
        int pc[16];
        float psv[16];
#pragma unroll
        for (uint32_t u = 0; u < 16; u++) {
            pc[u] = part_cnt[(size_t)(j + u) * kmax + i];
            psv[u] = part_sum[(size_t)(j + u) * kmax + i];
        }
#pragma unroll
        for (uint32_t u = 0; u < 16; u++) {
            c += pc[u];
            s += psv[u];
        }
    }
    for (; j < C; j++) {
        c += part_cnt[(size_t)j * kmax + i];
        s += part_sum[(size_t)j * kmax + i];
    }
    const uint32_t slot = list ? list[i] : i;
    counts[slot] = c;
    sums[slot] = s;
}

size_t tv_scratch_bytes(uint32_t kmax, int chunks) {
    return 256 + sizeof(uint32_t) * (((size_t)kmax + 63) & ~(size_t)63) +
           (chunks > 1 ? (sizeof(int32_t) + sizeof(float)) * (size_t)chunks * kmax : 0);
}

hipError_t launch_solve_f7(hipStream_t st, const float4 *pts, uint32_t n, const int32_t *samples_in,
                           int32_t *samples_out, uint32_t B, DevSampler ds, uint64_t first_hyp, float *models,
                           int32_t *counts, uint32_t *list, uint32_t *list_n) {
    hipError_t e = hipMemsetAsync(list_n, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_solve_f7, dim3((B + 63) / 64), dim3(64), 0, st, pts, n, samples_in, samples_out, B, ds,
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

namespace usac {
hipError_t launch_score_f2(hipStream_t st, int estimator, int chunks, const float4 *rec, const float4 *pts,
                           uint32_t n, float4 ext, const float *models, size_t stride, const uint32_t *list,
                           const uint32_t *list_n, uint32_t kmax, float thr, int32_t *counts, float *sums,
                           void *scratch) {
    if (chunks < 1 || chunks > 128 || !scratch) return hipErrorInvalidValue;
    // scratch: ends[2] (padded to 256 B), perm[kmax], then the chunk partials
    uint32_t *ends = static_cast<uint32_t *>(scratch);
    uint32_t *perm = ends + 64;
    int32_t *pc = reinterpret_cast<int32_t *>(perm + (((size_t)kmax + 63) & ~(size_t)63));
    float *ps = reinterpret_cast<float *>(pc + (size_t)chunks * kmax);
    hipError_t e = hipMemsetAsync(ends, 0, 2 * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    const bool ess = estimator == USAC_ESSENTIAL;
    const dim3 pgrid((kmax + 63) / 64);
    if (ess)
        hipLaunchKernelGGL((k_presort_tv<USAC_ESSENTIAL>), pgrid, dim3(64), 0, st, rec, n, ext, models, stride, list,
                           list_n, kmax, thr, perm, ends);
    else
        hipLaunchKernelGGL((k_presort_tv<USAC_FUNDAMENTAL>), pgrid, dim3(64), 0, st, rec, n, ext, models, stride, list,
                           list_n, kmax, thr, perm, ends);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    const dim3 grid((kmax + 63) / 64, chunks);
    if (ess)
        hipLaunchKernelGGL((k_score_f2<USAC_ESSENTIAL>), grid, dim3(64), 0, st, rec, pts, n, ext, models, stride, list,
                           list_n, kmax, thr, perm, counts, sums, pc, ps);
    else
        hipLaunchKernelGGL((k_score_f2<USAC_FUNDAMENTAL>), grid, dim3(64), 0, st, rec, pts, n, ext, models, stride, list,
                           list_n, kmax, thr, perm, counts, sums, pc, ps);
    e = hipGetLastError();
    if (e != hipSuccess || chunks == 1) return e;
    hipLaunchKernelGGL(k_tv_combine, dim3((kmax + 255) / 256), dim3(256), 0, st, list, list_n, kmax,
                       (uint32_t)chunks, pc, ps, counts, sums);
    return hipGetLastError();
}
}  // namespace usac
