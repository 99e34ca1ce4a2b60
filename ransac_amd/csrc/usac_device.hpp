// usac_device.hpp -- per-hypothesis device math of the hot path (gfx950, wave64).
//
// Every routine states the reference code it computes and the exact floating-point
// recipe (DESIGN.md "Numerics"); the CPU oracle (oracle/usac_oracle.c) restates the same
// reference independently, and the parity tests compare the two bit for bit.
// Compiled with -ffp-contract=off: no FMA contraction (a fused operation is an explicit fma()
// in both this file and the oracle), IEEE fp32/fp64 division and square root (hipcc's default
// correctly-rounded lowering), denormals kept.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "usac_kernels.h"

namespace usac {

// ---------------------------------------------------------------- counter-based sampler
// Throughput-mode sampler: one SplitMix64 stream per hypothesis keyed by
// (seed, global hypothesis index), xorshift-style mixing, Lemire multiply-shift into
// [0, N), duplicates rejected (a minimal sample has distinct points).
__device__ __forceinline__ uint64_t splitmix64(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// m distinct indices in [0, n) from the (seed, hyp) stream
template <int M>
__device__ __forceinline__ void draw_unique(uint64_t &st, uint32_t n, int32_t *s) {
#pragma unroll
    for (int i = 0; i < M; i++) {
        int32_t v;
        bool dup;
        do {
            uint64_t r = splitmix64(st);
            v = (int32_t)(((r >> 32) * (uint64_t)n) >> 32);
            dup = false;
#pragma unroll
            for (int j = 0; j < i; j++) dup |= (s[j] == v);
        } while (dup);
        s[i] = v;
    }
}

// UniformSampler (device stream) or PROSAC: the last point of the current subset plus
// m - 1 distinct points of the ones before it (prosac_sampler.hpp:160-168)
template <int M>
__device__ __forceinline__ void draw_sample(const DevSampler &ds, uint64_t hyp, uint32_t n, int32_t (&s)[M]) {
    uint64_t st = ds.seed ^ (hyp * 0xD1B54A32D192ED03ull);
    if (ds.nap_start && ds.nap_n_eligible) {  // NAPSAC (grid), see DevSampler
        const int32_t init = ds.nap_eligible[((splitmix64(st) >> 32) * ds.nap_n_eligible) >> 32];
        const uint32_t c = ds.nap_cell[init], rk = ds.nap_rank[init], b = ds.nap_start[c];
        const uint32_t cnt = ds.nap_start[c + 1] - b - 1;  // neighbours, >= M
        uint32_t j = (uint32_t)(((splitmix64(st) >> 32) * cnt) >> 32);
        s[0] = init;
#pragma unroll
        for (int k = 1; k < M; k++) {
            s[k] = ds.nap_members[b + (j < rk ? j : j + 1)];
            j = j + 1 == cnt ? 0 : j + 1;
        }
    } else if (ds.prosac && hyp < ds.prosac_len) {
        const uint32_t sub = ds.prosac[hyp];  // >= M
        draw_unique<M - 1>(st, sub - 1, s);
        s[M - 1] = (int32_t)sub - 1;
    } else {
        draw_unique<M>(st, n, s);
    }
}

// ---------------------------------------------------------------- 3x3 inverse
// cv::Mat::inv() of a CV_32F 3x3 (homography_estimator.hpp:35): fp64 determinant and
// cofactors from exact float*float products, times (1/det) in fp64, one cast to float;
// det == 0 -> zero matrix.
__device__ __forceinline__ void inv3x3(const float *m, float *dst) {
#define M_(r, c) ((double)m[3 * (r) + (c)])
    double d = M_(0, 0) * (M_(1, 1) * M_(2, 2) - M_(1, 2) * M_(2, 1)) -
               M_(0, 1) * (M_(1, 0) * M_(2, 2) - M_(1, 2) * M_(2, 0)) +
               M_(0, 2) * (M_(1, 0) * M_(2, 1) - M_(1, 1) * M_(2, 0));
    if (d == 0.0) {
#pragma unroll
        for (int i = 0; i < 9; i++) dst[i] = 0.f;
        return;
    }
    d = 1.0 / d;
    dst[0] = (float)((M_(1, 1) * M_(2, 2) - M_(1, 2) * M_(2, 1)) * d);
    dst[1] = (float)((M_(0, 2) * M_(2, 1) - M_(0, 1) * M_(2, 2)) * d);
    dst[2] = (float)((M_(0, 1) * M_(1, 2) - M_(0, 2) * M_(1, 1)) * d);
    dst[3] = (float)((M_(1, 2) * M_(2, 0) - M_(1, 0) * M_(2, 2)) * d);
    dst[4] = (float)((M_(0, 0) * M_(2, 2) - M_(0, 2) * M_(2, 0)) * d);
    dst[5] = (float)((M_(0, 2) * M_(1, 0) - M_(0, 0) * M_(1, 2)) * d);
    dst[6] = (float)((M_(1, 0) * M_(2, 1) - M_(1, 1) * M_(2, 0)) * d);
    dst[7] = (float)((M_(0, 1) * M_(2, 0) - M_(0, 0) * M_(2, 1)) * d);
    dst[8] = (float)((M_(0, 0) * M_(1, 1) - M_(0, 1) * M_(1, 0)) * d);
#undef M_
}

// ---------------------------------------------------------------- 4-pt DLT
// Rows of the DLT system exactly as dlt.cpp:24-41 (fp32 products), widened to fp64.
__device__ __forceinline__ void dlt_rows(float x1, float y1, float x2, float y2, double *r0, double *r1) {
    r0[0] = (double)(-x1); r0[1] = (double)(-y1); r0[2] = -1.0;
    r0[3] = 0.0; r0[4] = 0.0; r0[5] = 0.0;
    r0[6] = (double)(x2 * x1); r0[7] = (double)(x2 * y1); r0[8] = (double)x2;
    r1[0] = 0.0; r1[1] = 0.0; r1[2] = 0.0;
    r1[3] = (double)(-x1); r1[4] = (double)(-y1); r1[5] = -1.0;
    r1[6] = (double)(y2 * x1); r1[7] = (double)(y2 * y1); r1[8] = (double)y2;
}

// Round-robin (tournament) pair schedule, circle method, as (min, max) pairs; R-1 rounds
// of R/2 disjoint pairs (odd R: bye slot).  Consecutive pairs of a round touch disjoint
// rows, so their rotations are independent dependency chains (ILP for one lane).
template <int R>
struct Tournament {
    static constexpr int M = (R % 2) ? R + 1 : R;
    static constexpr int NP = R * (R - 1) / 2;
    int p[NP > 0 ? NP : 1], q[NP > 0 ? NP : 1];
    constexpr Tournament() : p(), q() {
        int arr[M] = {};
        for (int i = 0; i < M; i++) arr[i] = i;
        int np = 0;
        for (int round = 0; round < M - 1; round++) {
            for (int i = 0; i < M / 2; i++) {
                const int a = arr[i], b = arr[M - 1 - i];
                if (a >= R || b >= R) continue;
                p[np] = a < b ? a : b;
                q[np] = a < b ? b : a;
                np++;
            }
            const int last = arr[M - 1];
            for (int i = M - 1; i > 1; i--) arr[i] = arr[i - 1];
            arr[1] = last;
        }
    }
};

// One-sided (Hestenes) Jacobi on the R rows of W (fp64), the row-space part of the thin
// cv::SVD::compute of dlt.cpp:43.  Spec (identical in the oracle's row_jacobi; fused
// operations written out, fma = one rounding): sweeps < 30, pairs in tournament order
// (above); row norms n_i = fma chain over k = 0..8 recomputed at each sweep start; per pair
// a = n_p, b = n_q, g = fma chain of W[p][k] W[q][k]; skip when g*g <= 1e-28*(a*b);
// d = b - a, g2 = 2g, r = sqrt(fma(d, d, g2*g2)), u = |d| + r, inv = 1/sqrt((2r)*u),
// c = u*inv, s = g2*inv negated when d < 0, t = s*((2r)*inv)  (the classical
// t = sign(zeta)/(|zeta|+sqrt(1+zeta^2)), zeta = d/2g, c = 1/sqrt(1+t^2), s = c t with
// one division instead of two: (c, s) = (u, g2)/|(u, g2)| and |(u, g2)|^2 = 2 r u);
// row_p <- fma(c, row_p, -(s*row_q)), row_q <- fma(s, row_p, c*row_q);
// n_p <- a - t g, n_q <- b + t g; stop after a sweep without rotation.  Fully unrolled
// so W stays in VGPRs.
template <int R>
__device__ __forceinline__ void row_jacobi(double (&W)[R][9]) {
    constexpr Tournament<R> T{};
    for (int sweep = 0; sweep < 30; sweep++) {
        bool rotated = false;
        double nrm[R];
#pragma unroll
        for (int i = 0; i < R; i++) {
            double a = 0.0;
#pragma unroll
            for (int k = 0; k < 9; k++) a = fma(W[i][k], W[i][k], a);
            nrm[i] = a;
        }
#pragma unroll
        for (int pi = 0; pi < Tournament<R>::NP; pi++) {
            const int p = T.p[pi], q = T.q[pi];
            const double a = nrm[p], b = nrm[q];
            double g = 0.0;
#pragma unroll
            for (int k = 0; k < 9; k++) g = fma(W[p][k], W[q][k], g);
            if (!(g * g <= 1e-28 * (a * b))) {
                rotated = true;
                const double d = b - a, g2 = 2.0 * g;
                const double r = sqrt(fma(d, d, g2 * g2));
                const double u = fabs(d) + r, r2 = 2.0 * r;
                const double inv = 1.0 / sqrt(r2 * u);
                const double c = u * inv;
                double s = g2 * inv;
                if (d < 0.0) s = -s;
                const double t = s * (r2 * inv);
#pragma unroll
                for (int k = 0; k < 9; k++) {
                    const double wp = W[p][k], wq = W[q][k];
                    W[p][k] = fma(c, wp, -(s * wq));
                    W[q][k] = fma(s, wp, c * wq);
                }
                nrm[p] = a - t * g;
                nrm[q] = b + t * g;
            }
        }
        if (!rotated) break;
    }
}

// Thin row of the 4-pt DLT by Householder QR of A^T + two-vector subspace inverse iteration on
// R R^T with a Rayleigh-Ritz step (the oracle's dlt4_thin_qr, spec there; fma = one rounding on
// both sides).  Returns false when the spec falls back to row_jacobi + pick_vector (a zero /
// non-finite norm, or no convergence within 32 steps).  W is consumed (reflectors in place,
// R above them).
__device__ __forceinline__ void qr_back(const double (&W)[8][9], const double *rd, const double *q, double *y) {
#pragma unroll
    for (int k = 7; k >= 0; k--) {
        double t = q[k];
#pragma unroll
        for (int i = k + 1; i < 8; i++) t = fma(-W[i][k], y[i], t);
        y[k] = t * rd[k];
    }
}
__device__ __forceinline__ void qr_fwd(const double (&W)[8][9], const double *rd, const double *u, double *y) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
        double t = u[k];
#pragma unroll
        for (int i = 0; i < k; i++) t = fma(-W[k][i], y[i], t);
        y[k] = t * rd[k];
    }
}
__device__ __forceinline__ double dot8(const double *x, const double *y) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 8; k++) t = fma(x[k], y[k], t);
    return t;
}
__device__ __forceinline__ bool pos_finite(double x) { return x > 0.0 && x < INFINITY; }

__device__ __forceinline__ bool dlt4_thin_qr(double (&W)[8][9], double *v) {
    double be[8], rd[8];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        double s2 = 0.0;
#pragma unroll
        for (int k = j; k < 9; k++) s2 = fma(W[j][k], W[j][k], s2);
        const double sig = sqrt(s2);
        ok = ok && pos_finite(sig);
        const double x0 = W[j][j];
        const double alpha = x0 >= 0.0 ? -sig : sig;
        be[j] = 1.0 / (sig * (sig + fabs(x0)));
        W[j][j] = x0 - alpha;
#pragma unroll
        for (int i = j + 1; i < 8; i++) {
            double s = 0.0;
#pragma unroll
            for (int k = j; k < 9; k++) s = fma(W[j][k], W[i][k], s);
            const double f = be[j] * s;
#pragma unroll
            for (int k = j; k < 9; k++) W[i][k] = fma(-f, W[j][k], W[i][k]);
        }
        rd[j] = 1.0 / alpha;
    }
    if (!ok) return false;
    double q1[8], q2[8], w0[8], y1[8], y2[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        q1[k] = k == 7 ? 1.0 : 0.0;
        q2[k] = k == 6 ? 1.0 : 0.0;
        w0[k] = 0.0;
    }
    bool conv = false;
    for (int it = 0; it < 32; it++) {
        qr_back(W, rd, q1, y1);
        qr_back(W, rd, q2, y2);
        const double a = dot8(y1, y1), b = dot8(y1, y2), d = dot8(y2, y2);
        const double h = (a - d) * 0.5, r = sqrt(fma(h, h, b * b));
        double c1 = h >= 0.0 ? h + r : b, c2 = h >= 0.0 ? b : r - h;
        const double nn = sqrt(fma(c1, c1, c2 * c2));
        if (!pos_finite(nn)) return false;
        const double inn = 1.0 / nn;
        c1 = c1 * inn;
        c2 = c2 * inn;
        double w[8];
#pragma unroll
        for (int k = 0; k < 8; k++) w[k] = fma(c1, q1[k], c2 * q2[k]);
        const double dt = dot8(w, w0);
        double dmax = 0.0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const double ek = fabs(w[k] - (dt < 0.0 ? -w0[k] : w0[k]));
            dmax = ek > dmax ? ek : dmax;
            w0[k] = w[k];
        }
        if (dmax <= 1e-13) {
            conv = true;
            break;
        }
        double u1[8], u2[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            u1[k] = fma(c1, y1[k], c2 * y2[k]);
            u2[k] = fma(c1, y2[k], -(c2 * y1[k]));
        }
        qr_fwd(W, rd, u1, y1);
        qr_fwd(W, rd, u2, y2);
        const double n1 = dot8(y1, y1);
        if (!pos_finite(n1)) return false;
        const double i1 = 1.0 / sqrt(n1);
#pragma unroll
        for (int k = 0; k < 8; k++) q1[k] = y1[k] * i1;
        const double p = dot8(q1, y2);
#pragma unroll
        for (int k = 0; k < 8; k++) y2[k] = fma(-p, q1[k], y2[k]);
        const double n2 = dot8(y2, y2);
        if (!pos_finite(n2)) return false;
        const double i2 = 1.0 / sqrt(n2);
#pragma unroll
        for (int k = 0; k < 8; k++) q2[k] = y2[k] * i2;
    }
    if (!conv) return false;
    double x[9];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = w0[k];
    x[8] = 0.0;
#pragma unroll
    for (int j = 7; j >= 0; j--) {
        double s = 0.0;
#pragma unroll
        for (int k = j; k < 9; k++) s = fma(W[j][k], x[k], s);
        const double f = be[j] * s;
#pragma unroll
        for (int k = j; k < 9; k++) x[k] = fma(-f, W[j][k], x[k]);
    }
#pragma unroll
    for (int k = 0; k < 9; k++) v[k] = x[k];
    return true;
}

// Null-space basis of an R x 9 system (R < 9) in the FULL_UV completion order (the oracle's
// qr_null, spec there): Householder QR of W^T as in dlt4_thin_qr, the 9 - R null columns
// Q e_R.. Q e_8, then vector j from the axis least represented by the row space and the earlier
// vectors, projected onto the null space and twice Gram-Schmidt'ed against the earlier vectors.
// False (fall back to row_jacobi + the row-based completion) on a zero / non-finite column norm.
template <int R>
__device__ __forceinline__ bool qr_null(double (&W)[R][9], double (&N)[9 - R][9]) {
    constexpr int C = 9 - R;
    double be[R];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < R; j++) {
        double s2 = 0.0;
#pragma unroll
        for (int k = j; k < 9; k++) s2 = fma(W[j][k], W[j][k], s2);
        const double sig = sqrt(s2);
        ok = ok && pos_finite(sig);
        const double x0 = W[j][j];
        const double alpha = x0 >= 0.0 ? -sig : sig;
        be[j] = 1.0 / (sig * (sig + fabs(x0)));
        W[j][j] = x0 - alpha;
#pragma unroll
        for (int i = j + 1; i < R; i++) {
            double s = 0.0;
#pragma unroll
            for (int k = j; k < 9; k++) s = fma(W[j][k], W[i][k], s);
            const double f = be[j] * s;
#pragma unroll
            for (int k = j; k < 9; k++) W[i][k] = fma(-f, W[j][k], W[i][k]);
        }
    }
    if (!ok) return false;
    double Q[C][9];
#pragma unroll
    for (int m = 0; m < C; m++) {
#pragma unroll
        for (int k = 0; k < 9; k++) Q[m][k] = k == R + m ? 1.0 : 0.0;
#pragma unroll
        for (int j = R - 1; j >= 0; j--) {
            double s = 0.0;
#pragma unroll
            for (int k = j; k < 9; k++) s = fma(W[j][k], Q[m][k], s);
            const double f = be[j] * s;
#pragma unroll
            for (int k = j; k < 9; k++) Q[m][k] = fma(-f, W[j][k], Q[m][k]);
        }
    }
#pragma unroll
    for (int j = 0; j < C; j++) {
        int ks = 0;
        double best = 0.0;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            double t = 0.0, u = 0.0;
#pragma unroll
            for (int m = 0; m < C; m++) t = fma(Q[m][k], Q[m][k], t);
#pragma unroll
            for (int l = 0; l < j; l++) u = fma(N[l][k], N[l][k], u);
            const double c = u - t;
            if (k == 0 || c < best) {
                best = c;
                ks = k;
            }
        }
        double qk[C], x[9];
#pragma unroll
        for (int m = 0; m < C; m++) {
            qk[m] = Q[m][0];
#pragma unroll
            for (int k = 1; k < 9; k++) qk[m] = ks == k ? Q[m][k] : qk[m];
        }
#pragma unroll
        for (int k = 0; k < 9; k++) {
            double t = 0.0;
#pragma unroll
            for (int m = 0; m < C; m++) t = fma(qk[m], Q[m][k], t);
            x[k] = t;
        }
#pragma unroll
        for (int pass = 0; pass < 2; pass++) {
#pragma unroll
            for (int l = 0; l < j; l++) {
                double d = 0.0;
#pragma unroll
                for (int k = 0; k < 9; k++) d = fma(N[l][k], x[k], d);
#pragma unroll
                for (int k = 0; k < 9; k++) x[k] = fma(-d, N[l][k], x[k]);
            }
        }
        double nrm = 0.0;
#pragma unroll
        for (int k = 0; k < 9; k++) nrm = fma(x[k], x[k], nrm);
        nrm = sqrt(nrm);
#pragma unroll
        for (int k = 0; k < 9; k++) N[j][k] = x[k] / nrm;
    }
    return true;
}

// Model vector from the converged rows (oracle pick_vector):
//  thin      -> row of smallest squared norm, first on ties  (vt.row(vt.rows-1))
//  nullspace -> unit vector orthogonal to all non-zero rows: rows normalised in place,
//               start axis = least represented coordinate, two Gram-Schmidt passes.
template <int R>
__device__ __forceinline__ void pick_vector(double (&W)[R][9], int nullspace, double *h) {
    double n2[R];
#pragma unroll
    for (int i = 0; i < R; i++) {
        double a = 0.0;
#pragma unroll
        for (int k = 0; k < 9; k++) a += W[i][k] * W[i][k];
        n2[i] = a;
    }
    if (!nullspace) {
        double bestn = n2[0];
#pragma unroll
        for (int k = 0; k < 9; k++) h[k] = W[0][k];
#pragma unroll
        for (int i = 1; i < R; i++) {
            if (n2[i] < bestn) {
                bestn = n2[i];
#pragma unroll
                for (int k = 0; k < 9; k++) h[k] = W[i][k];
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < R; i++) {
        if (n2[i] > 0.0) {
            double inv = 1.0 / sqrt(n2[i]);
#pragma unroll
            for (int k = 0; k < 9; k++) W[i][k] = W[i][k] * inv;
        }
    }
    int ks = 0;
    double bestc = 0.0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        double c = 0.0;
#pragma unroll
        for (int i = 0; i < R; i++)
            if (n2[i] > 0.0) c += W[i][k] * W[i][k];
        if (k == 0 || c < bestc) {
            bestc = c;
            ks = k;
        }
    }
#pragma unroll
    for (int k = 0; k < 9; k++) h[k] = (k == ks) ? 1.0 : 0.0;
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
#pragma unroll
        for (int i = 0; i < R; i++) {
            if (n2[i] > 0.0) {
                double d = 0.0;
#pragma unroll
                for (int k = 0; k < 9; k++) d += W[i][k] * h[k];
#pragma unroll
                for (int k = 0; k < 9; k++) h[k] -= d * W[i][k];
            }
        }
    }
}

// ---------------------------------------------------------------- fundamental (7-pt / 8-pt)
// Row of the epipolar system x2^T F x1 = 0 (seven_points.cpp:62-73, eight_points.cpp:26-45):
// fp32 products, widened to fp64.
__device__ __forceinline__ void fund_row(float x1, float y1, float x2, float y2, double *r) {
    r[0] = (double)(x2 * x1); r[1] = (double)(x2 * y1); r[2] = (double)x2;
    r[3] = (double)(y2 * x1); r[4] = (double)(y2 * y1); r[5] = (double)y2;
    r[6] = (double)x1; r[7] = (double)y1; r[8] = 1.0;
}

// The two FULL_UV null-space rows of the 7x9 system (vt rows 7 and 8 of
// seven_points.cpp:88-90) from the converged Jacobi rows: rows normalised in place (zero
// rows skipped); vector j starts at the axis least represented by the rows and the
// earlier vectors (first minimum), two Gram-Schmidt passes (rows, then earlier vectors),
// normalised as x_k / |x|.  Identical to the oracle's null_complement.
__device__ __forceinline__ void null_complement7(double (&W)[7][9], double (&N)[2][9]) {
    double n2[7];
#pragma unroll
    for (int i = 0; i < 7; i++) {
        double a = 0.0;
#pragma unroll
        for (int k = 0; k < 9; k++) a += W[i][k] * W[i][k];
        n2[i] = a;
        if (a > 0.0) {
            const double inv = 1.0 / sqrt(a);
#pragma unroll
            for (int k = 0; k < 9; k++) W[i][k] = W[i][k] * inv;
        }
    }
#pragma unroll
    for (int j = 0; j < 2; j++) {
        int ks = 0;
        double bestc = 0.0;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            double c = 0.0;
#pragma unroll
            for (int i = 0; i < 7; i++)
                if (n2[i] > 0.0) c += W[i][k] * W[i][k];
            if (j == 1) c += N[0][k] * N[0][k];
            if (k == 0 || c < bestc) {
                bestc = c;
                ks = k;
            }
        }
        double x[9];
#pragma unroll
        for (int k = 0; k < 9; k++) x[k] = (k == ks) ? 1.0 : 0.0;
#pragma unroll
        for (int pass = 0; pass < 2; pass++) {
#pragma unroll
            for (int i = 0; i < 7; i++) {
                if (n2[i] > 0.0) {
                    double d = 0.0;
#pragma unroll
                    for (int k = 0; k < 9; k++) d += W[i][k] * x[k];
#pragma unroll
                    for (int k = 0; k < 9; k++) x[k] -= d * W[i][k];
                }
            }
            if (j == 1) {
                double d = 0.0;
#pragma unroll
                for (int k = 0; k < 9; k++) d += N[0][k] * x[k];
#pragma unroll
                for (int k = 0; k < 9; k++) x[k] -= d * N[0][k];
            }
        }
        double nrm = 0.0;
#pragma unroll
        for (int k = 0; k < 9; k++) nrm += x[k] * x[k];
        nrm = sqrt(nrm);
#pragma unroll
        for (int k = 0; k < 9; k++) N[j][k] = x[k] / nrm;
    }
}

// Real roots of c0 x^3 + c1 x^2 + c2 x + c3 (the contract of cv::solveCubic,
// seven_points.cpp:131) with IEEE basic operations only -- monic form, Cauchy bound,
// critical-point brackets, bisection.  Identical to the oracle's cubic_roots.
__device__ __forceinline__ double cubic_eval(double a, double b, double c, double x) {
    return ((x + a) * x + b) * x + c;
}

__device__ __noinline__ double cubic_bisect(double a, double b, double c, double lo, double hi) {
    double flo = cubic_eval(a, b, c, lo);
    for (int it = 0; it < 200; it++) {
        const double mid = 0.5 * (lo + hi);
        if (!(mid > lo && mid < hi)) break;
        const double fm = cubic_eval(a, b, c, mid);
        if (fm == 0.0) return mid;
        if ((fm < 0.0) == (flo < 0.0)) {
            lo = mid;
            flo = fm;
        } else {
            hi = mid;
        }
    }
    return 0.5 * (lo + hi);
}

__device__ __forceinline__ int cubic_roots(double c0, double c1, double c2, double c3, double *r) {
    if (c0 == 0.0) {
        if (c1 == 0.0) {
            if (c2 == 0.0) return 0;
            r[0] = -c3 / c2;
            return 1;
        }
        const double D = c2 * c2 - 4.0 * c1 * c3;
        if (D < 0.0) return 0;
        if (D == 0.0) {
            r[0] = -c2 / (2.0 * c1);
            return 1;
        }
        const double s = sqrt(D);
        const double q = -0.5 * (c2 + (c2 >= 0.0 ? s : -s));
        const double x1 = q / c1, x2 = c3 / q;
        r[0] = x1 < x2 ? x1 : x2;
        r[1] = x1 < x2 ? x2 : x1;
        return 2;
    }
    const double a = c1 / c0, b = c2 / c0, c = c3 / c0;
    double R = fabs(a);
    if (fabs(b) > R) R = fabs(b);
    if (fabs(c) > R) R = fabs(c);
    R = R + 1.0;
    const double D = a * a - 3.0 * b;
    int n = 0;
    if (!(D > 0.0)) {
        r[n++] = cubic_bisect(a, b, c, -R, R);
        return n;
    }
    const double s = sqrt(D);
    const double m1 = (-a - s) / 3.0, m2 = (-a + s) / 3.0;
    const double v1 = cubic_eval(a, b, c, m1), v2 = cubic_eval(a, b, c, m2);
    if (v1 >= 0.0) r[n++] = cubic_bisect(a, b, c, -R, m1);
    if (v1 > 0.0 && v2 < 0.0) r[n++] = cubic_bisect(a, b, c, m1, m2);
    if (v2 <= 0.0) r[n++] = cubic_bisect(a, b, c, m2, R);
    return n;
}

// det(f1 + lambda f2)-style cubic coefficients exactly as seven_points.cpp:98-128 (fp32,
// left to right), after f1 -= f2.
__device__ __forceinline__ void fund_cubic(float (&f1)[9], const float (&f2)[9], float (&c)[4]) {
#pragma unroll
    for (int i = 0; i < 9; i++) f1[i] -= f2[i];
    float t0 = f2[4] * f2[8] - f2[5] * f2[7];
    float t1 = f2[3] * f2[8] - f2[5] * f2[6];
    float t2 = f2[3] * f2[7] - f2[4] * f2[6];
    c[3] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2;
    c[2] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2 - f1[3] * (f2[1] * f2[8] - f2[2] * f2[7]) +
           f1[4] * (f2[0] * f2[8] - f2[2] * f2[6]) - f1[5] * (f2[0] * f2[7] - f2[1] * f2[6]) +
           f1[6] * (f2[1] * f2[5] - f2[2] * f2[4]) - f1[7] * (f2[0] * f2[5] - f2[2] * f2[3]) +
           f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]);
    t0 = f1[4] * f1[8] - f1[5] * f1[7];
    t1 = f1[3] * f1[8] - f1[5] * f1[6];
    t2 = f1[3] * f1[7] - f1[4] * f1[6];
    c[1] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2 - f2[3] * (f1[1] * f1[8] - f1[2] * f1[7]) +
           f2[4] * (f1[0] * f1[8] - f1[2] * f1[6]) - f2[5] * (f1[0] * f1[7] - f1[1] * f1[6]) +
           f2[6] * (f1[1] * f1[5] - f1[2] * f1[4]) - f2[7] * (f1[0] * f1[5] - f1[2] * f1[3]) +
           f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]);
    c[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2;
}

// F for one cubic root (seven_points.cpp:138-154, fp32)
__device__ __forceinline__ void fund_from_root(const float (&f1)[9], const float (&f2)[9], float r, float (&F)[9]) {
    float lambda = r, mu = 1.f;
    const float s = f1[8] * r + f2[8];
    if ((double)fabsf(s) > 2.220446049250313e-16) {
        mu = 1.f / s;
        lambda *= mu;
        F[8] = 1.f;
    } else {
        F[8] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) F[i] = f1[i] * lambda + f2[i] * mu;
}

// Oriented epipolar constraint (fundamental_estimator.hpp:189-231), fp32: epipole
// row0 x row2 (row1 x row2 when every |e_i| <= 1.9984e-15), sign of
// (F0 x2 + F3 y2 + F6)(e1 - e2 y1) consistent over the sample.
__device__ __forceinline__ bool fund_oriented(const float (&F)[9], const float4 *__restrict__ pts,
                                              const int32_t (&smp)[7]) {
    float e1 = F[2] * F[6] - F[0] * F[8];
    float e2 = F[0] * F[7] - F[1] * F[6];
    const float e0 = F[1] * F[8] - F[2] * F[7];
    const bool big = (e0 > 1.9984e-15 || e0 < -1.9984e-15) || (e1 > 1.9984e-15 || e1 < -1.9984e-15) ||
                     (e2 > 1.9984e-15 || e2 < -1.9984e-15);
    if (!big) {
        e1 = F[5] * F[6] - F[3] * F[8];
        e2 = F[3] * F[7] - F[4] * F[6];
    }
    float sig1 = 0.f;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        const float4 P = pts[smp[i]];
        const float s1 = F[0] * P.z + F[3] * P.w + F[6];
        const float s2 = e1 - e2 * P.y;
        const float sig = s1 * s2;
        if (i == 0) sig1 = sig;
        else ok = ok && !(sig1 * sig < 0);
    }
    return ok;
}

// FundamentalEstimator::GetError (fundamental_estimator.hpp:101-134): Sampson distance,
// fp32 left to right, one IEEE division.
__device__ __forceinline__ float fundamental_error(const float *f, float x1, float y1, float x2, float y2) {
    const float Fx = f[0] * x1 + f[1] * y1 + f[2];
    const float Fy = f[3] * x1 + f[4] * y1 + f[5];
    const float Gx = f[0] * x2 + f[3] * y2 + f[6];
    const float Gy = f[1] * x2 + f[4] * y2 + f[7];
    const float s = x2 * Fx + y2 * Fy + f[6] * x1 + f[7] * y1 + f[8];
    return (s * s) / (Fx * Fx + Fy * Fy + Gx * Gx + Gy * Gy);
}

// ---------------------------------------------------------------- residuals
// HomographyEstimator::GetError (homography_estimator.hpp:85-110): fp32 projections
// evaluated left to right, IEEE divisions, the two distances are double square roots
// summed in double and rounded to float, halved.  No z guard: inf/NaN -> outlier.
__device__ __forceinline__ float homography_error(const float *h, const float *hi, float x1, float y1, float x2,
                                                  float y2) {
    float ex2 = h[0] * x1 + h[1] * y1 + h[2];
    float ey2 = h[3] * x1 + h[4] * y1 + h[5];
    float ez2 = h[6] * x1 + h[7] * y1 + h[8];
    ex2 = ex2 / ez2;
    ey2 = ey2 / ez2;
    float ex1 = hi[0] * x2 + hi[1] * y2 + hi[2];
    float ey1 = hi[3] * x2 + hi[4] * y2 + hi[5];
    float ez1 = hi[6] * x2 + hi[7] * y2 + hi[8];
    ex1 = ex1 / ez1;
    ey1 = ey1 / ez1;
    float d2 = (x2 - ex2) * (x2 - ex2) + (y2 - ey2) * (y2 - ey2);
    float d1 = (x1 - ex1) * (x1 - ex1) + (y1 - ey1) * (y1 - ey1);
    float error = (float)(sqrt((double)d2) + sqrt((double)d1));
    return error / 2;
}

// ---------------------------------------------------------------- fast decision path
// The score kernel decides `err < thr` with approximate fp32 reciprocal / square root and
// falls back to homography_error() (the exact reference expression) whenever the fast
// value is within a guard band of the threshold or not finite.  Error analysis
// (DESIGN.md "Guard band"): the projections X, Y, Z are computed with the exact
// reference operation sequence; q0 = X*rcp(Z) is within 2^-21|q0| of fl(X/Z)
// (v_rcp_f32 1 ulp); the fast sum S = sqrt~(dx2^2+dy2^2) + sqrt~(dx1^2+dy1^2) then
// differs from the reference's fp32 `error` by at most 2^-21*Mp + 2^-18*S near S = 2 thr,
// Mp = |x1|+|y1|+|x2|+|y2|.  The band uses 8x that: 2^-18*Mp + 2^-15*(2 thr).
constexpr float kBandMp = 3.814697265625e-06f;  // 2^-18
constexpr float kBandT = 3.0517578125e-05f;     // 2^-15

// Line2DEstimator::GetError (line2d_estimator.hpp:154-156)
__device__ __forceinline__ float line2d_error(float a, float b, float c, float x, float y) {
    return fabsf(a * x + b * y + c);
}

// Line2DEstimator::EstimateModel (line2d_estimator.hpp:36-54)
__device__ __forceinline__ void line2d_estimate(float x1, float y1, float x2, float y2, float *m) {
    float a = y1 - y2;
    float b = x2 - x1;
    float mag = (float)sqrt((double)(a * a + b * b));
    a = a / mag;
    b = b / mag;
    float c = (x1 * y2 - x2 * y1) / mag;
    m[0] = a;
    m[1] = b;
    m[2] = c;
}

// Score::bigger (quality.hpp:22-26) extended to a strict total order with the earliest
// hypothesis index winning exact ties (the sequential loop keeps the first).
__device__ __forceinline__ bool record_better(int c1, float s1, uint32_t i1, int c2, float s2, uint32_t i2) {
    if (c1 != c2) return c1 > c2;
    if (s1 != s2) return s1 > s2;
    return i1 < i2;
}

}  // namespace usac
