// usac_hscore.hpp -- the homography score's per-pair stages (device), shared by the lanes-over-
// hypotheses scorer (kernels.hip k_score_hf) and the matrix-core prefilter scorer (kernels_h16.hip):
// the model registers, stage A's error bounds and the stage-B guard-band test (DESIGN.md "Guard band").
#pragma once
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_pk.hpp"

namespace usac {

// Model registers of a lane: h[9] = H, hi[9] = H^-1; plus the lane's stage-A error
// bounds dZ, E (below), and H / dZ / E duplicated into both halves of 2-wide vectors for the
// packed stage A (two points per v_pk_fma_f32).

struct HModel {
    float h[9], hi[9];
    float dZ, E;
    v2f h2[9];
    float trm, F;  // packed stage A: r = |Z| trm + F (see stage_a_bounds)
};

// Stage-A bounds of one hypothesis over the dataset box |x1| <= c.x, |y1| <= c.y,
// |x2| <= c.z, |y2| <= c.w:  K_X = |h0| c.x + |h1| c.y + |h2| bounds every magnitude in the
// reference's X = (h0 x1 + h1 y1) + h2 and in the FMA chain below, so the two differ by at
// most 2^-21 K_X; dX = 2^-20 K_X (2x slack), likewise dY, dZ;
// E = ((c.z dZ + dX) + (c.w dZ + dY)) (1 + 2^-18).
// For the packed stage A the per-point radius factor tr_i = (T + band_i)(1 + 2^-18) is
// replaced by its dataset maximum trm (band_max from the box: Mp <= c.x + c.y + c.z + c.w)
// and tr (|Z| + dZ) + E by |Z| trm + F with F = (trm dZ + E)(1 + 2^-20) -- never a smaller
// radius, so never a wrong rejection, and one v_fma_f32 (|Z| as an abs modifier) per point.
__device__ __forceinline__ void stage_a_bounds(HModel &M, float4 c, float T) {
    const float kx = fabsf(M.h[0]) * c.x + fabsf(M.h[1]) * c.y + fabsf(M.h[2]);
    const float ky = fabsf(M.h[3]) * c.x + fabsf(M.h[4]) * c.y + fabsf(M.h[5]);
    const float kz = fabsf(M.h[6]) * c.x + fabsf(M.h[7]) * c.y + fabsf(M.h[8]);
    const float s = 9.5367431640625e-07f;  // 2^-20
    const float dx = s * kx, dy = s * ky, dz = s * kz;
    M.dZ = dz;
    M.E = ((c.z * dz + dx) + (c.w * dz + dy)) * 1.000003814697265625f;
#pragma unroll
    for (int k = 0; k < 9; k++) M.h2[k] = v2f{M.h[k], M.h[k]};
    const float band_max = kBandMp * (((c.x + c.y) + (c.z + c.w)) * 1.00000095367431640625f) + kBandT * T;
    M.trm = (T + band_max) * 1.000003814697265625f;                  // (1 + 2^-18)
    M.F = (M.trm * M.dZ + M.E) * 1.00000095367431640625f;             // (1 + 2^-20)
}

// Stage A for two points at once: the FMA chains element-wise (v_pk_fma_f32), then the
// L-infinity test per point: keep iff !(max(|ex|, |ey|) > r) with r = |Z| trm + F.
// |e| >= max(|ex|, |ey|), so this rejects only where the Euclidean test |e| > r does
// (stage_a_reject derives that one) -- it lets through the few pairs between the circle and
// its circumscribed square -- for 11 VALU slots per point instead of 13 (no |e|^2, no r^2).
// One rounding (r, downwards by at most 2^-24 relative) against the (1 + 2^-18) slack
// already in trm and F.  Non-finite: if Z or its bound is infinite, r = inf and nothing is
// rejected; a NaN component can only come with an infinite X / Z, where the reference's
// error is not finite or not below thr.  Returns the KEEP flags.
__device__ __forceinline__ void stage_a_keep2(const HModel &M, v2f x1, v2f y1, v2f x2, v2f y2, bool &k0,
                                              bool &k1) {
    const v2f X = vfma(M.h2[1], y1, vfma(M.h2[0], x1, M.h2[2]));
    const v2f Y = vfma(M.h2[4], y1, vfma(M.h2[3], x1, M.h2[5]));
    const v2f Z = vfma(M.h2[7], y1, vfma(M.h2[6], x1, M.h2[8]));
    const v2f ex = vfma(x2, Z, -X);
    const v2f ey = vfma(y2, Z, -Y);
    const float m0 = __builtin_fmaxf(fabsf(ex.x), fabsf(ey.x)), m1 = __builtin_fmaxf(fabsf(ex.y), fabsf(ey.y));
    k0 = !(m0 > __builtin_fmaf(fabsf(Z.x), M.trm, M.F));
    k1 = !(m1 > __builtin_fmaf(fabsf(Z.y), M.trm, M.F));
}

// Stage A -- forward-only rejection, 14 VALU ops, no rcp / sqrt.  X, Y, Z by FMA chains,
// e = (x2 Z - X, y2 Z - Y); with r = tr (|Z| + dZ) + E:
//   |e|^2 > r^2   ==>   the reference's forward distance exceeds T + band >= 2 thr,
// so its error is not below the threshold: a sure outlier, whatever the backward term.
// (DESIGN.md "Guard band" derives it: |Z_ref u_ref - e| <= E, |Z_ref| <= |Z| + dZ; the
// (1 + 2^-18) factors dominate every rounding of the test itself; NaN -> not rejected.)
__device__ __forceinline__ bool stage_a_reject(const HModel &M, float x1, float y1, float x2, float y2, float tr) {
    const float X = __builtin_fmaf(M.h[1], y1, __builtin_fmaf(M.h[0], x1, M.h[2]));
    const float Y = __builtin_fmaf(M.h[4], y1, __builtin_fmaf(M.h[3], x1, M.h[5]));
    const float Z = __builtin_fmaf(M.h[7], y1, __builtin_fmaf(M.h[6], x1, M.h[8]));
    const float ex = __builtin_fmaf(x2, Z, -X);
    const float ey = __builtin_fmaf(y2, Z, -Y);
    const float lhs = __builtin_fmaf(ex, ex, ey * ey);
    const float r = __builtin_fmaf(tr, fabsf(Z) + M.dZ, M.E);
    return lhs > r * r;
}

// Stage B -- both directions with the reference's projection order, v_rcp, v_sqrt, and the
// guard-band test; lanes inside the band / non-finite / (EXACT_SUM) inliers re-evaluate the
// exact reference expression.  Adds to (cnt, sum): the exact err (EXACT_SUM, so Σ is the
// reference's sequential fp32 sum) or S ~= 2 err (throughput mode, halved at the end).
template <bool EXACT_SUM>
__device__ __forceinline__ void stage_b(const HModel &M, float x1, float y1, float x2, float y2, float band, float T,
                                        float thr, int &cnt, float &sum) {
    const float X = M.h[0] * x1 + M.h[1] * y1 + M.h[2];
    const float Y = M.h[3] * x1 + M.h[4] * y1 + M.h[5];
    const float Z = M.h[6] * x1 + M.h[7] * y1 + M.h[8];
    const float r2 = __builtin_amdgcn_rcpf(Z);
    const float dx2 = __builtin_fmaf(-X, r2, x2);
    const float dy2 = __builtin_fmaf(-Y, r2, y2);
    const float X1 = M.hi[0] * x2 + M.hi[1] * y2 + M.hi[2];
    const float Y1 = M.hi[3] * x2 + M.hi[4] * y2 + M.hi[5];
    const float Z1 = M.hi[6] * x2 + M.hi[7] * y2 + M.hi[8];
    const float r1 = __builtin_amdgcn_rcpf(Z1);
    const float dx1 = __builtin_fmaf(-X1, r1, x1);
    const float dy1 = __builtin_fmaf(-Y1, r1, y1);
    const float d2 = __builtin_fmaf(dx2, dx2, dy2 * dy2);
    const float d1 = __builtin_fmaf(dx1, dx1, dy1 * dy1);
    const float S = __builtin_amdgcn_sqrtf(d2) + __builtin_amdgcn_sqrtf(d1);
    const float diff = S - T;
    const bool sure = (fabsf(diff) > band) & (S < INFINITY);
    bool inl = sure & (diff < 0.f);
    float add = S;
    if (EXACT_SUM ? (!sure || inl) : !sure) {
        const float e = homography_error(M.h, M.hi, x1, y1, x2, y2);
        inl = e < thr;
        add = EXACT_SUM ? e : e + e;
    }
    if (inl) {
        cnt++;
        sum += add;
    }
}

}  // namespace usac
