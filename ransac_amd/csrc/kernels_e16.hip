// kernels_e16.hip -- the essential score with a matrix-core prefilter (gfx950 MFMA, fp16 in, fp32
// accumulate), exact counts (DESIGN.md §6 "e16").  The two-view counterpart of kernels_h16.hip.
//
// The reference's residual (essential_estimator.hpp:76-107) of a pair is
//   err = (|a1| / ||l12|| + |b1| / ||t12||) / 2,   l = E^T p2, t = E p1, a1 ~ b1 ~ r = p2^T E p1,
// so err >= |r| / max(||l12||, ||t12||) >= |r| / (S rho): S = max(||E[:, 0:2]||_2, ||E[0:2, :]||_2) per
// hypothesis, rho = max(||(x1, y1, 1)||, ||(x2, y2, 1)||) per point.  r is bilinear in the point: a
// dot product of nine per-hypothesis coefficients G with the nine features f = (u, v, 1, p u, p v, p,
// q u, q v, q) of the centred, power-of-two-scaled coordinates of kernels_h16.hip (G = T2^T E T1,
// T the centring transforms).  With the features divided by rho per point, one MFMA tile
// (v_mfma_f32_32x32x16_f16, K = the nine features) gives r / rho for 32 hypotheses x 32 points and
// the rejection test is one compare per pair against a per-hypothesis constant:
//   keep iff |r~'| < C,   C = 2^e C0 (1 + 2^-20) + D,   C0 = delta + thr (1 + 2^-19) (S + 2^-21 M + 2^-100),
// delta = 2^-20 Mabs + 2^-120 bounds |a1 - r| and |b1 - r| of the reference's fp32 chains (Mabs = the
// dataset box's bound of sum |E_jk p2_j p1_k|), M = the box's bound of ||l12|| and ||t12|| (their fp32
// evaluation is within 2^-21 M of the exact norms), 2^e the hypothesis' power-of-two scale, and D the
// bound of the matrix cores' rounding: coefficients and features are split into fp16 hi + lo parts and
// two chained MFMAs add gh fh + gl fh + gh fl (the lo parts of seven coefficients ride in the spare K
// slots of the first, the rest in the second), so the products miss only gl fl and the parts' own
// roundings -- D = (1 + 2^-10) sum_k [2^-17 a_k fmax_k + 2^-23 (a_k + fmax_k)], a_k = |gh_k| + |gl_k| +
// 2^-24, fmax the dataset's feature maxima (k_h16_consts) -- instead of ~2^-10 of the products with one
// fp16 part each (twice the kept pairs on cfg4: the drain and the append, not the MFMA, are the cost).  A rejected pair has
// (1 - 2^-22)(|r| - delta) >= thr max(a2, b2) for the reference's own a2, b2, i.e. err >= thr: not an
// inlier.  Hypotheses whose bounds are not finite or whose box bounds reach 2^60 (fp32 overflow in
// the reference's chain) get zero rows and C = +inf (every pair to the exact stage); padding and
// non-finite points get NaN features (never kept -- the reference never counts them).
//
// The test builds each lane's 16-bit keep mask of a tile from sign bits (|r~'| - C < 0); non-empty masks
// go onto per-lane LDS stacks and their pairs to the exact stage (essential_error_guarded: counts
// exact, Σ terms within 2^-19 relative), one pair per lane per drain round; counts and Σ (2^-fx fixed point,
// integer adds, deterministic) per point chunk, added by k_e16_finish.  Models are the listed
// slots of the batch (list / list_n), as for k_score_f2.
#include <hip/hip_runtime.h>
#include <math.h>

#include "usac_device.hpp"
#include "usac_device_e5.hpp"
#include "usac_h16.hpp"
#include "usac_kernels.h"

namespace usac {

typedef float e16_f32x16 __attribute__((ext_vector_type(16)));

constexpr int kE16NA = 2;                       // 32-hypothesis tiles per wave
constexpr int kE16HW = 32 * kE16NA;             // hypotheses per wave

// ------------------------------------------------------------------------ point features / rho
// per 32-point block two B matrices of the h16 layout (lane l holds B[k = 8 (l >> 5) + j][column l & 31]),
// the features divided by the point's rho (rounded up: a larger rho only loosens the test) and split
// into fp16 hi + lo parts: B1 = (fh_0 .. fh_8, fh_0 .. fh_6), B2 = (fl_0 .. fl_8, fh_7, fh_8, 0 ..);
// feat[(2 blk + m) 64 + lane], m = 0 (B1), 1 (B2)
size_t e16_feature_bytes(uint32_t n) { return (size_t)((n + 31) / 32) * 2048; }

__global__ __launch_bounds__(256) void k_e16_points(const float4 *__restrict__ pts, uint32_t n,
                                                    const H16Consts *__restrict__ kc, half8 *__restrict__ feat) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    const uint32_t nblk = (n + 31) / 32;
    if (t >= nblk * 64) return;
    const uint32_t blk = t >> 6, l = t & 63, i = blk * 32 + (l & 31), hf = l >> 5;
    half8 o1, o2;
    bool ok = i < n;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) {
        p = pts[i];
        ok = isfinite(p.x) && isfinite(p.y) && isfinite(p.z) && isfinite(p.w);
    }
    if (!ok) {
#pragma unroll
        for (int j = 0; j < 8; j++) o1[j] = o2[j] = (_Float16)__builtin_nanf("");
    } else {
        const double x1 = p.x, y1 = p.y, x2 = p.z, y2 = p.w;
        const double rho = fmax(sqrt(x1 * x1 + y1 * y1 + 1.0), sqrt(x2 * x2 + y2 * y2 + 1.0)) * (1.0 + 0x1p-40);
        const double u = (x1 - kc->cx1) / kc->s1, v = (y1 - kc->cy1) / kc->s1;
        const double pp = (x2 - kc->cx2) / kc->s2, q = (y2 - kc->cy2) / kc->s2;
        const double f[9] = {u / rho, v / rho, 1.0 / rho, pp * u / rho, pp * v / rho, pp / rho,
                             q * u / rho, q * v / rho, q / rho};
        _Float16 fh[9], fl[9];
#pragma unroll
        for (int k = 0; k < 9; k++) {
            fh[k] = (_Float16)(float)f[k];
            fl[k] = (_Float16)(float)(f[k] - (double)(float)fh[k]);
        }
        const _Float16 z = (_Float16)0.0f;
        const _Float16 b1[16] = {fh[0], fh[1], fh[2], fh[3], fh[4], fh[5], fh[6], fh[7],
                                 fh[8], fh[0], fh[1], fh[2], fh[3], fh[4], fh[5], fh[6]};
        const _Float16 b2[16] = {fl[0], fl[1], fl[2], fl[3], fl[4], fl[5], fl[6], fl[7], fl[8], fh[7], fh[8], z, z, z, z, z};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            o1[j] = b1[8 * hf + j];
            o2[j] = b2[8 * hf + j];
        }
    }
    feat[(2 * (size_t)blk) * 64 + l] = o1;
    feat[(2 * (size_t)blk + 1) * 64 + l] = o2;
}

hipError_t launch_e16_points(hipStream_t st, const float4 *pts, uint32_t n, const H16Consts *k, void *feat) {
    const uint32_t threads = (n + 31) / 32 * 64;
    hipLaunchKernelGGL(k_e16_points, dim3((threads + 255) / 256), dim3(256), 0, st, pts, n, k,
                       static_cast<half8 *>(feat));
    return hipGetLastError();
}

// ------------------------------------------------------------------------ per-hypothesis rows
// rows[4 pos + 2 m + half]: A1 (m = 0: gh_0 .. gh_8, gl_0 .. gl_6) and A2 (m = 1: gh_0 .. gh_8, gl_7, gl_8,
// 0 ..) of listed position pos, coefficients 8 half .. 8 half + 7; cm[pos] = C
__device__ __forceinline__ double e16_up(double x) { return x * (1.0 + 0x1p-40); }

__global__ __launch_bounds__(256) void k_e16_rows(const float *__restrict__ models, size_t stride,
                                                  const uint32_t *__restrict__ list,
                                                  const uint32_t *__restrict__ list_n, uint32_t kmax,
                                                  const H16Consts *__restrict__ kc, float thr,
                                                  half8 *__restrict__ rows, float *__restrict__ cm) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t K = list ? *list_n : kmax;
    if (i >= K) return;
    const uint32_t slot = list ? list[i] : i;
    double E[9];
#pragma unroll
    for (int k = 0; k < 9; k++) E[k] = models[(size_t)k * stride + slot];
    const float4 c = kc->ext;
    const double C1[3] = {c.x, c.y, 1.0}, C2[3] = {c.z, c.w, 1.0};
    // box bounds: Mabs >= sum |E_jk| |p2_j| |p1_k|, M >= ||l12||, ||t12|| (l_k = sum_j E_jk p2_j, t_j = sum_k E_jk p1_k)
    double Mabs = 0.0, Lb[2] = {0.0, 0.0}, Tb[2] = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 3; j++)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const double a = fabs(E[3 * j + k]);
            Mabs += a * C2[j] * C1[k];
            if (k < 2) Lb[k] += a * C2[j];
            if (j < 2) Tb[j] += a * C1[k];
        }
    const double M = e16_up(fmax(sqrt(Lb[0] * Lb[0] + Lb[1] * Lb[1]), sqrt(Tb[0] * Tb[0] + Tb[1] * Tb[1])));
    // S >= the spectral norms of E[:, 0:2] (l12 = E[:, 0:2]^T p2) and E[0:2, :] (t12 = E[0:2, :] p1): the
    // larger eigenvalue of each 2 x 2 Gram matrix, (g00 + g11) / 2 + sqrt(((g00 - g11) / 2)^2 + g01^2), is
    // within ~40 ulp of the computed one relative to g00 + g11 <= 2 lambda, so (1 + 2^-40) covers it
    // (round 6: Frobenius norms before -- up to sqrt 2 larger, 23 % more kept pairs on cfg4)
    double gA[3] = {0.0, 0.0, 0.0}, gB[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 3; j++) {
        gA[0] += E[3 * j] * E[3 * j];
        gA[1] += E[3 * j + 1] * E[3 * j + 1];
        gA[2] += E[3 * j] * E[3 * j + 1];
        gB[0] += E[j] * E[j];
        gB[1] += E[3 + j] * E[3 + j];
        gB[2] += E[j] * E[3 + j];
    }
    auto lmax = [](const double (&g)[3]) {
        const double h = 0.5 * (g[0] - g[1]);
        return e16_up(e16_up(0.5 * (g[0] + g[1]) + sqrt(h * h + g[2] * g[2])));
    };
    const double S = e16_up(sqrt(fmax(lmax(gA), lmax(gB))));
    const double delta = e16_up(0x1p-20 * e16_up(Mabs)) + 0x1p-120;
    const double C0 = e16_up(delta + e16_up((double)thr * (1.0 + 0x1p-19) * (S + 0x1p-21 * M + 0x1p-100)));
    // G = T2^T E T1 in the feature order (u, v, 1 | p u, p v, p | q u, q v, q): row 2, row 0, row 1
    const double s1 = kc->s1, s2 = kc->s2, cx1 = kc->cx1, cy1 = kc->cy1, cx2 = kc->cx2, cy2 = kc->cy2;
    double X[3][3], aX[3][3];  // E T1 and its terms' magnitudes
#pragma unroll
    for (int j = 0; j < 3; j++) {
        X[j][0] = E[3 * j] * s1;
        X[j][1] = E[3 * j + 1] * s1;
        X[j][2] = E[3 * j] * cx1 + E[3 * j + 1] * cy1 + E[3 * j + 2];
        aX[j][0] = fabs(X[j][0]);
        aX[j][1] = fabs(X[j][1]);
        aX[j][2] = fabs(E[3 * j] * cx1) + fabs(E[3 * j + 1] * cy1) + fabs(E[3 * j + 2]);
    }
    double g[9], a[9];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        g[k] = cx2 * X[0][k] + cy2 * X[1][k] + X[2][k];
        a[k] = fabs(cx2) * aX[0][k] + fabs(cy2) * aX[1][k] + aX[2][k];
        g[3 + k] = s2 * X[0][k];
        a[3 + k] = s2 * aX[0][k];
        g[6 + k] = s2 * X[1][k];
        a[6 + k] = s2 * aX[1][k];
    }
    double mx = 0.0;
    bool fin = isfinite(C0) && isfinite(M) && M < 0x1p60 && Mabs < 0x1p60;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        fin = fin && isfinite(a[k]);
        mx = fmax(mx, fabs(g[k]));
    }
    fin = fin && mx > 0x1p-100 && mx < 0x1p100;
    half8 out[4];
    float cv = INFINITY;
    if (!fin) {
#pragma unroll
        for (int m = 0; m < 4; m++)
#pragma unroll
            for (int j = 0; j < 8; j++) out[m][j] = (_Float16)0.0f;
    } else {
        const int e = -(ilogb(mx) + 1);  // max |g| 2^e in [0.5, 1)
        _Float16 gh[9], gl[9];
        double D = 0x1p-100;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            const double gs = ldexp(g[k], e);
            gh[k] = (_Float16)(float)gs;
            gl[k] = (_Float16)(float)(gs - (double)(float)gh[k]);
            const double ak = fabs((double)(float)gh[k]) + fabs((double)(float)gl[k]) + 0x1p-24, fk = kc->fmax[k];
            D += 0x1p-17 * ak * fk + 0x1p-23 * (ak + fk) + 0x1p-50 * ldexp(a[k], e) * fk;
        }
        const _Float16 z = (_Float16)0.0f;
        const _Float16 a1[16] = {gh[0], gh[1], gh[2], gh[3], gh[4], gh[5], gh[6], gh[7],
                                 gh[8], gl[0], gl[1], gl[2], gl[3], gl[4], gl[5], gl[6]};
        const _Float16 a2[16] = {gh[0], gh[1], gh[2], gh[3], gh[4], gh[5], gh[6], gh[7], gh[8], gl[7], gl[8], z, z, z, z, z};
#pragma unroll
        for (int j = 0; j < 8; j++) {
            out[0][j] = a1[j];
            out[1][j] = a1[8 + j];
            out[2][j] = a2[j];
            out[3][j] = a2[8 + j];
        }
        const double Cd = e16_up(ldexp(C0, e) * (1.0 + 0x1p-20) + D * (1.0 + 0x1p-10));
        const float Cf = (float)Cd;
        cv = (double)Cf >= Cd ? Cf : nextafterf(Cf, INFINITY);
        if (!isfinite(cv)) cv = INFINITY;
    }
#pragma unroll
    for (int m = 0; m < 4; m++) rows[4 * (size_t)i + m] = out[m];
    cm[i] = cv;
}

hipError_t launch_e16_rows(hipStream_t st, const float *models, size_t stride, const uint32_t *list,
                           const uint32_t *list_n, uint32_t kmax, const H16Consts *k, float thr, void *rows,
                           float *cm) {
    hipLaunchKernelGGL(k_e16_rows, dim3((kmax + 255) / 256), dim3(256), 0, st, models, stride, list, list_n, kmax, k,
                       thr, static_cast<half8 *>(rows), cm);
    return hipGetLastError();
}

// ------------------------------------------------------------------------ the scorer
__device__ __forceinline__ void e16_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// per-lane stacks of tile masks: for each tile lane l pushes one entry -- the 16-bit mask of the
// tile's hypotheses its point kept (built one compare + one add-with-carry per hypothesis), the
// tile and the block -- if any was kept (LDS [entry][lane]: a push of all 64 lanes is one
// conflict-free ds_write_b64).  A drain round: every lane with an entry evaluates one kept pair of
// its top entry (the lowest mask bit) and clears it, popping the entry when its mask empties; rounds
// run before a tile while >= kE16Round lanes hold an entry or a stack is full (a tile pushes at most
// one).  The order of the integer count / fixed-point Σ adds does not matter.
constexpr uint32_t kE16Lane = 8u, kE16Round = 48u;

__device__ __forceinline__ void e16_drain_lane(bool has, uint32_t hk, uint32_t p, const float (*sm)[9], uint32_t *sc,
                                               unsigned long long *ss, const float4 *__restrict__ pts, float thr,
                                               float lo, float hi, double fxs) {
    if (has) {
        const float4 pt = pts[p];
        float m[9];
#pragma unroll
        for (int k = 0; k < 9; k++) m[k] = sm[hk][k];
        bool inl;
        const float val = essential_error_guarded(m, pt.x, pt.y, pt.z, pt.w, thr, lo, hi, inl);
        if (inl) {
            atomicAdd(&sc[hk], 1u);
            atomicAdd(&ss[hk], (unsigned long long)llrint((double)val * fxs));
        }
    }
}

// one drain round over the lanes' top entries (every lane calls; q = this lane's column).  No
// barrier: a lane's stack is its own (a wave's LDS operations complete in order), the models are
// read-only after the kernel's first barrier and the counters take LDS atomics
__device__ __forceinline__ void e16_round(uint32_t &d, uint2 *q, uint32_t lane, uint32_t hf, const float (*sm)[9],
                                          uint32_t *sc, unsigned long long *ss, const float4 *__restrict__ pts,
                                          float thr, float lo, float hi, double fxs) {
    const bool has = d > 0;
    uint32_t hk = 0, p = 0;
    if (has) {
        const uint2 e = q[64 * (d - 1)];
        const uint32_t m = e.x & 0xFFFFu, a = e.x >> 16;
        const uint32_t b = (uint32_t)__builtin_ctz(m), j = 15u - b;  // bit 15 - j <-> hypothesis row j
        const uint32_t rest = m & (m - 1u);
        if (rest) q[64 * (d - 1)].x = rest | (a << 16);
        else d--;
        hk = 32 * a + (j & 3) + 4 * hf + 8 * (j >> 2);
        p = e.y * 32 + (lane & 31);
    }
    e16_drain_lane(has, hk, p, sm, sc, ss, pts, thr, lo, hi, fxs);
}

// Workgroup = 4 waves; wave w owns listed positions [hb, hb + 64) and point chunk blockIdx.y.  A
// fragment of tile a: lane l holds row l & 31 (position hb + 32 a + (l & 31)), coefficients 8 (l >> 5)
// ..; the D register j of lane l holds row (j & 3) + 4 (l >> 5) + 8 (j >> 2), column l & 31.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_score_e16(
    const half8 *__restrict__ feat, const float4 *__restrict__ pts, uint32_t n, const half8 *__restrict__ rows,
    const float *__restrict__ cm, const float *__restrict__ models, size_t stride, const uint32_t *__restrict__ list,
    const uint32_t *__restrict__ list_n, uint32_t kmax, float thr, double fxs, uint32_t *__restrict__ cpart,
    unsigned long long *__restrict__ spart) {
    __shared__ float sM[4][kE16HW][9];
    __shared__ uint32_t sC[4][kE16HW];
    __shared__ unsigned long long sS[4][kE16HW];
    __shared__ uint2 sQ[4][kE16Lane][64];
    __shared__ float sCv[4][kE16NA][2][16];  // the tiles' constants C by lane half (read per tile)
    const uint32_t K = list ? __builtin_amdgcn_readfirstlane(*list_n) : kmax;
    const uint32_t lane = threadIdx.x & 63, hf = lane >> 5;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t hb = (blockIdx.x * 4 + wave) * kE16HW;
    if (hb >= K) return;  // wave-uniform; no workgroup barrier below
    {
        const uint32_t pos = hb + lane;
        const uint32_t slot = pos < K ? (list ? list[pos] : pos) : 0u;
#pragma unroll
        for (int k = 0; k < 9; k++) sM[wave][lane][k] = pos < K ? models[(size_t)k * stride + slot] : 0.f;
        sC[wave][lane] = 0;
        sS[wave][lane] = 0;
    }
    half8 A1[kE16NA], A2[kE16NA];
#pragma unroll
    for (int a = 0; a < kE16NA; a++) {
        const uint32_t pos = hb + 32 * a + (lane & 31);
        half8 z;
#pragma unroll
        for (int j = 0; j < 8; j++) z[j] = (_Float16)0.0f;
        A1[a] = pos < K ? rows[4 * (size_t)pos + hf] : z;
        A2[a] = pos < K ? rows[4 * (size_t)pos + 2 + hf] : z;
        if ((lane & 31) < 16) {
            const uint32_t j = lane & 15, pj = hb + 32 * a + (j & 3) + 4 * hf + 8 * (j >> 2);
            sCv[wave][a][hf][j] = pj < K ? cm[pj] : 0.0f;  // a missing hypothesis keeps nothing
        }
    }
    const uint32_t nblk = (n + 31) / 32, nch = gridDim.y, ch = blockIdx.y;
    const uint32_t per = (nblk + nch - 1) / nch;
    const uint32_t b0 = ch * per < nblk ? ch * per : nblk, b1 = b0 + per < nblk ? b0 + per : nblk;
    const float lo = thr * 0.9999847412109375f, hi = thr * 1.0000152587890625f;  // thr (1 -+ 2^-16)
    uint32_t d = 0;  // this lane's stack depth
    const e16_f32x16 zero = {};
    e16_wave_sync();
    half8 bn1 = b0 < b1 ? feat[(2 * (size_t)b0) * 64 + lane] : half8{};
    half8 bn2 = b0 < b1 ? feat[(2 * (size_t)b0 + 1) * 64 + lane] : half8{};
    uint2 *const q = &sQ[wave][0][lane];
    for (uint32_t blk = b0; blk < b1; blk++) {
        const half8 bf1 = bn1, bf2 = bn2;
        if (blk + 1 < b1) {
            bn1 = feat[(2 * (size_t)blk + 2) * 64 + lane];
            bn2 = feat[(2 * (size_t)blk + 3) * 64 + lane];
        }
        e16_f32x16 acc[kE16NA];
#pragma unroll
        for (int a = 0; a < kE16NA; a++) {
            acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1[a], bf1, zero, 0, 0, 0);
            acc[a] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2[a], bf2, acc[a], 0, 0, 0);
        }
#pragma unroll
        for (int a = 0; a < kE16NA; a++) {
            // drain rounds until fewer than kE16Round lanes hold an entry and no stack is full
            for (;;) {
                const uint64_t ne = __builtin_amdgcn_ballot_w64(d > 0);
                if (__builtin_popcountll(ne) < (int)kE16Round && __builtin_amdgcn_ballot_w64(d >= kE16Lane) == 0)
                    break;
                e16_round(d, q, lane, hf, sM[wave], sC[wave], sS[wave], pts, thr, lo, hi, fxs);
            }
            // the tile's keep mask (bit 15 - j: hypothesis row j), pushed when not empty; C read from LDS
            // each tile (a broadcast read: 16 registers fewer, a fifth wave per SIMD)
            __asm__ volatile("" ::: "memory");
            float Cv[16];
#pragma unroll
            for (int j = 0; j < 16; j++) Cv[j] = sCv[wave][a][hf][j];
            uint32_t m = 0;
#pragma unroll
            for (int j = 0; j < 16; j++) {
                // kept iff |r~'| < C iff |r~'| - C < 0 (exact in sign with denormals kept; a NaN feature
                // gives a positive NaN: not kept, as the compare); its sign bit shifted into m by one
                // v_alignbit: m = (m << 1) | sign
                const float t = fabsf(acc[a][j]) - Cv[j];
                m = __builtin_amdgcn_alignbit(m, __float_as_uint(t), 31);
            }
            q[64 * d] = make_uint2(m | ((uint32_t)a << 16), blk);
            d += m != 0 ? 1u : 0u;
        }
    }
    while (__builtin_amdgcn_ballot_w64(d > 0) != 0)
        e16_round(d, q, lane, hf, sM[wave], sC[wave], sS[wave], pts, thr, lo, hi, fxs);
    e16_wave_sync();
    if (hb + lane < K) {
        cpart[(size_t)ch * kmax + hb + lane] = sC[wave][lane];
        spart[(size_t)ch * kmax + hb + lane] = sS[wave][lane];
    }
}

// counts / sums at the listed slots from the chunk partials (integers: any order is exact)
__global__ __launch_bounds__(256) void k_e16_finish(const uint32_t *__restrict__ list,
                                                    const uint32_t *__restrict__ list_n, uint32_t kmax,
                                                    const uint32_t *__restrict__ cpart,
                                                    const unsigned long long *__restrict__ spart, uint32_t nch,
                                                    double inv_fxs, int32_t *__restrict__ counts,
                                                    float *__restrict__ sums) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t K = list ? *list_n : kmax;
    if (i >= K) return;
    uint32_t c = 0;
    unsigned long long s = 0;
    for (uint32_t y = 0; y < nch; y++) {
        c += cpart[(size_t)y * kmax + i];
        s += spart[(size_t)y * kmax + i];
    }
    const uint32_t slot = list ? list[i] : i;
    counts[slot] = (int32_t)c;
    sums[slot] = (float)((double)s * inv_fxs);
}

size_t e16_part_bytes(uint32_t kmax, int chunks) {
    return (size_t)chunks * kmax * (sizeof(uint32_t) + sizeof(uint64_t));
}

size_t e16_row_bytes(uint32_t kmax) { return (size_t)kmax * 64; }

hipError_t launch_score_e16(hipStream_t st, const void *feat, const float4 *pts, uint32_t n, const void *rows,
                            const float *cm, const float *models, size_t stride, const uint32_t *list,
                            const uint32_t *list_n, uint32_t kmax, float thr, int chunks, void *part,
                            int32_t *counts, float *sums) {
    if (chunks < 1 || n == 0 || n > 0x2000000u || kmax == 0) return hipErrorInvalidValue;
    const uint32_t nblk = (n + 31) / 32, per = (nblk + (uint32_t)chunks - 1) / (uint32_t)chunks;
    if ((uint64_t)per * 32 > (1u << 23)) return hipErrorInvalidValue;  // the fixed-point Σ bound (below)
    if (!(thr > 0x1p-100f && thr < 0x1p100f)) return hipErrorInvalidValue;
    // Σ in fixed point: an inlier's term is < thr (1 + 2^-15), 2^fx with thr 2^fx <= 2^40 leaves 2^23
    // terms per hypothesis and chunk below 2^63
    const int fx = 39 - ilogbf(thr);
    unsigned long long *sp = static_cast<unsigned long long *>(part);
    uint32_t *cp = reinterpret_cast<uint32_t *>(sp + (size_t)chunks * kmax);
    hipLaunchKernelGGL(k_score_e16, dim3((kmax + 4 * kE16HW - 1) / (4 * kE16HW), chunks), dim3(256), 0, st,
                       static_cast<const half8 *>(feat), pts, n, static_cast<const half8 *>(rows), cm, models, stride,
                       list, list_n, kmax, thr, ldexp(1.0, fx), cp, sp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_e16_finish, dim3((kmax + 255) / 256), dim3(256), 0, st, list, list_n, kmax, cp, sp,
                       (uint32_t)chunks, ldexp(1.0, -fx), counts, sums);
    return hipGetLastError();
}

}  // namespace usac
