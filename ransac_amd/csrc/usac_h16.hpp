#pragma once
// usac_h16.hpp -- the matrix-core scorer's per-hypothesis fp16 rows and prefilter slack (device),
// shared by k_h16_rows (kernels_h16.hip) and the homography solvers' epilogue (kernels.hip:
// usac_hypothesize* batches write the rows as they solve, one launch and one pass over the
// models fewer per batch).
#include <hip/hip_runtime.h>
#include <math.h>

#include "usac_hscore.hpp"
#include "usac_kernels.h"

namespace usac {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

// rows[(3 h + r) * 2 + half]: row r (0 ex, 1 ey, 2 zr) of hypothesis h, coefficients 8 half .. 8 half + 7.
// fp32 throughout (the dataset's centres are fp32 numbers, its scales powers of two): a coefficient's
// own rounding is <= 2^-21 of the sum a_k of its terms' magnitudes, the bound's sums are rounded up by
// (1 + 2^-18) -- both far inside the fp16 terms they sit beside.
__device__ __forceinline__ void h16_rows_of(const float (&Hm)[9], const H16Consts *__restrict__ kc, float thr, uint32_t h,
                                            half8 *__restrict__ rows, float *__restrict__ fm) {
    const float4 ext = kc->ext;
    HModel M;
#pragma unroll
    for (int c = 0; c < 9; c++) M.h[c] = Hm[c];
    const float T = 2.0f * thr;
    stage_a_bounds(M, ext, T);  // trm, F, dZ of the packed stage A (fp32, rounded up)
    const float s20 = 9.5367431640625e-07f;  // 2^-20, as stage_a_bounds
    const float dxf = s20 * (fabsf(M.h[0]) * ext.x + fabsf(M.h[1]) * ext.y + fabsf(M.h[2]));
    const float dyf = s20 * (fabsf(M.h[3]) * ext.x + fabsf(M.h[4]) * ext.y + fabsf(M.h[5]));
    const float cx1 = (float)kc->cx1, cy1 = (float)kc->cy1, cx2 = (float)kc->cx2, cy2 = (float)kc->cy2;
    const float s1 = (float)kc->s1, s2 = (float)kc->s2;
    // X, Y, Z over (u, v, 1) and the magnitudes of their terms
    float P[3][3], aP[3][3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const float a0 = M.h[3 * r] * cx1, a1 = M.h[3 * r + 1] * cy1;
        P[r][0] = M.h[3 * r] * s1;
        P[r][1] = M.h[3 * r + 1] * s1;
        P[r][2] = (a0 + a1) + M.h[3 * r + 2];
        aP[r][0] = fabsf(P[r][0]);
        aP[r][1] = fabsf(P[r][1]);
        aP[r][2] = (fabsf(a0) + fabsf(a1)) + fabsf(M.h[3 * r + 2]);
    }
    const float trmi = M.trm * 1.0009765625f;  // trm (1 + 2^-10)
    float g[3][9], a[3][9];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 9; c++) g[r][c] = a[r][c] = 0.f;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        g[0][c] = cx2 * P[2][c] - P[0][c];
        a[0][c] = fabsf(cx2) * aP[2][c] + aP[0][c];
        g[0][3 + c] = s2 * P[2][c];
        a[0][3 + c] = s2 * aP[2][c];
        g[1][c] = cy2 * P[2][c] - P[1][c];
        a[1][c] = fabsf(cy2) * aP[2][c] + aP[1][c];
        g[1][6 + c] = s2 * P[2][c];
        a[1][6 + c] = s2 * aP[2][c];
        g[2][c] = trmi * P[2][c];
        a[2][c] = trmi * aP[2][c];
    }
    float mx = 0.f;
    bool fin = isfinite(trmi) && isfinite(M.F) && isfinite(M.dZ) && isfinite(dxf) && isfinite(dyf);
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 9; c++) {
            fin = fin && isfinite(a[r][c]);  // a >= |g|: a finite a means a finite g
            mx = fmaxf(mx, fabsf(g[r][c]));
        }
    fin = fin && mx > 0x1p-100f && mx < 0x1p100f;
    half8 out[3][2];
    float fmv = INFINITY;
    if (!fin) {  // no prefilter for this hypothesis: zero rows, every pair to the exact stage
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
            for (int hf = 0; hf < 2; hf++)
#pragma unroll
                for (int j = 0; j < 8; j++) out[r][hf][j] = (_Float16)0.0f;
    } else {
        const int e = -(ilogbf(mx) + 1);  // max |g| 2^e in [0.5, 1)
        float D[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            float d = 0x1p-100f;
#pragma unroll
            for (int c = 0; c < 16; c++) {
                const float gh = c < 9 ? ldexpf(g[r][c], e) : 0.f;
                const _Float16 gt = (_Float16)gh;
                out[r][c >> 3][c & 7] = gt;
                if (c < 9) {
                    const float agt = fabsf((float)gt), fk = (float)kc->fmax[c];
                    d += agt * (0x1p-10f * fk + 0x1p-25f) +
                         fk * (0x1p-10f * fabsf(gh) + 0x1p-25f + 0x1p-21f * ldexpf(a[r][c], e)) +
                         0x1p-19f * agt * (fk + 0x1p-24f);
                }
            }
            D[r] = d * 1.00000381469726562f;  // (1 + 2^-18): the sum's own roundings
        }
        const float sc = ldexpf(1.0f, e);
        const float ex_fma = ext.z * M.dZ + dxf, ey_fma = ext.w * M.dZ + dyf;
        const float Fm = (M.F * sc + fmaxf(D[0] + ex_fma * sc, D[1] + ey_fma * sc) + trmi * M.dZ * sc + D[2]) *
                         1.00000381469726562f;
        fmv = isfinite(Fm) ? Fm : INFINITY;
    }
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int hf = 0; hf < 2; hf++) rows[((size_t)h * 3 + r) * 2 + hf] = out[r][hf];
    fm[h] = fmv;
}


}  // namespace usac
