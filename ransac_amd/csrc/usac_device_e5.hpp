// usac_device_e5.hpp -- per-sample device math of the essential 5-point solver
// (EssentialSolver::FivePoints / Solve5PointEssential, five_points.cpp:13-274) and the
// essential residual (essential_estimator.hpp:76-107).
//
// Written to the spec the oracle restates (oracle/usac_oracle.c "essential (5-pt)"): the
// same IEEE operation sequence -- fp64 throughout the solver, no FMA contraction, correctly
// rounded division and square root -- so device and oracle agree bit for bit.  The
// reference's OpenCV SVD / determinant / inv are replaced by: row Jacobi + null complement
// (basis), LU with partial pivoting (det M(z) at z = -5..5), Newton divided differences
// (degree-10 coefficients), elimination with partial pivoting (null vector of M(z)), and a
// cheirality test through Jacobi 3x3 SVD + 4x4 linear triangulation; its rpoly root step is
// restated operation for operation (usac_rpoly.hpp: the same zeros in the same order).
#pragma once
#include <float.h>

#include <type_traits>

#include "usac_device.hpp"

namespace usac {
namespace e5 {

// row Jacobi on R rows of C (<= 4) columns with the round-1 row_jacobi rules (unfused
// products, t and c by two divisions; the oracle's row_jacobi_small); ACC: also rotate the
// rows of J (R x R)
template <int R, int C, bool ACC>
__device__ __forceinline__ void jacobi_small(double (&W)[R][C], double (&J)[R][R]) {
    constexpr Tournament<R> T{};
    for (int sweep = 0; sweep < 30; sweep++) {
        bool rotated = false;
        double nrm[R];
#pragma unroll
        for (int i = 0; i < R; i++) {
            double a = 0.0;
#pragma unroll
            for (int k = 0; k < C; k++) a += W[i][k] * W[i][k];
            nrm[i] = a;
        }
#pragma unroll
        for (int pi = 0; pi < Tournament<R>::NP; pi++) {
            const int p = T.p[pi], q = T.q[pi];
            const double a = nrm[p], b = nrm[q];
            double g = 0.0;
#pragma unroll
            for (int k = 0; k < C; k++) g += W[p][k] * W[q][k];
            if (!(g * g <= 1e-28 * (a * b))) {
                rotated = true;
                const double d = b - a, g2 = 2.0 * g;
                double t = g2 / (fabs(d) + sqrt(d * d + g2 * g2));
                if (d < 0.0) t = -t;
                const double c = 1.0 / sqrt(1.0 + t * t);
                const double s = c * t;
#pragma unroll
                for (int k = 0; k < C; k++) {
                    const double wp = W[p][k], wq = W[q][k];
                    W[p][k] = c * wp - s * wq;
                    W[q][k] = s * wp + c * wq;
                }
                if (ACC) {
#pragma unroll
                    for (int k = 0; k < R; k++) {
                        const double jp = J[p][k], jq = J[q][k];
                        J[p][k] = c * jp - s * jq;
                        J[q][k] = s * jp + c * jq;
                    }
                }
                nrm[p] = a - t * g;
                nrm[q] = b + t * g;
            }
        }
        if (!rotated) break;
    }
}

// the four null-space rows of the 5 x 9 system (oracle null_complement(W, 5, 4, N))
__device__ __forceinline__ void null_basis4(double (&W)[5][9], double (&N)[4][9]) {
    double n2[5];
#pragma unroll
    for (int i = 0; i < 5; i++) {
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
    for (int j = 0; j < 4; j++) {
        int ks = 0;
        double bestc = 0.0;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            double c = 0.0;
#pragma unroll
            for (int i = 0; i < 5; i++)
                if (n2[i] > 0.0) c += W[i][k] * W[i][k];
#pragma unroll
            for (int l = 0; l < j; l++) c += N[l][k] * N[l][k];
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
            for (int i = 0; i < 5; i++) {
                if (n2[i] > 0.0) {
                    double d = 0.0;
#pragma unroll
                    for (int k = 0; k < 9; k++) d += W[i][k] * x[k];
#pragma unroll
                    for (int k = 0; k < 9; k++) x[k] -= d * W[i][k];
                }
            }
#pragma unroll
            for (int l = 0; l < j; l++) {
                double d = 0.0;
#pragma unroll
                for (int k = 0; k < 9; k++) d += N[l][k] * x[k];
#pragma unroll
                for (int k = 0; k < 9; k++) x[k] -= d * N[l][k];
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

// bivariate cubic algebra over [x^3, y^3, x^2y, xy^2, x^2, y^2, xy, x, y, 1]
struct Lin {
    double a, b, c;
};
struct Quad {
    double x2, y2, xy, x, y, k;
};
__device__ __forceinline__ Quad qmul(const Lin &u, const Lin &v) {
    Quad q;
    q.x2 = u.a * v.a;
    q.y2 = u.b * v.b;
    q.xy = u.a * v.b + u.b * v.a;
    q.x = u.a * v.c + u.c * v.a;
    q.y = u.b * v.c + u.c * v.b;
    q.k = u.c * v.c;
    return q;
}
__device__ __forceinline__ Quad qadd(const Quad &p, const Quad &q) {
    return Quad{p.x2 + q.x2, p.y2 + q.y2, p.xy + q.xy, p.x + q.x, p.y + q.y, p.k + q.k};
}
__device__ __forceinline__ Quad qsub(const Quad &p, const Quad &q) {
    return Quad{p.x2 - q.x2, p.y2 - q.y2, p.xy - q.xy, p.x - q.x, p.y - q.y, p.k - q.k};
}
__device__ __forceinline__ void cmul(const Quad &q, const Lin &l, double *c) {
    c[0] = q.x2 * l.a;
    c[1] = q.y2 * l.b;
    c[2] = q.x2 * l.b + q.xy * l.a;
    c[3] = q.y2 * l.a + q.xy * l.b;
    c[4] = q.x2 * l.c + q.x * l.a;
    c[5] = q.y2 * l.c + q.y * l.b;
    c[6] = q.xy * l.c + q.x * l.b + q.y * l.a;
    c[7] = q.x * l.c + q.k * l.a;
    c[8] = q.y * l.c + q.k * l.b;
    c[9] = q.k * l.c;
}

// M(z) (oracle e5_matrix)
__device__ __forceinline__ void matrix(const double (&N)[4][9], double z, double (&M)[10][10]) {
    Lin E[9];
#pragma unroll
    for (int k = 0; k < 9; k++) E[k] = Lin{N[0][k], N[1][k], z * N[2][k] + N[3][k]};
    Quad EEt[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            Quad acc = qmul(E[3 * i], E[3 * j]);
            acc = qadd(acc, qmul(E[3 * i + 1], E[3 * j + 1]));
            acc = qadd(acc, qmul(E[3 * i + 2], E[3 * j + 2]));
            EEt[i][j] = acc;
        }
    const Quad tr = qadd(qadd(EEt[0][0], EEt[1][1]), EEt[2][2]);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            double t0[10], t1[10], t2[10], tt[10];
            cmul(EEt[i][0], E[j], t0);
            cmul(EEt[i][1], E[3 + j], t1);
            cmul(EEt[i][2], E[6 + j], t2);
            cmul(tr, E[3 * i + j], tt);
#pragma unroll
            for (int m = 0; m < 10; m++) M[3 * i + j][m] = 2.0 * (t0[m] + t1[m] + t2[m]) - tt[m];
        }
    double d0[10], d1[10], d2[10];
    cmul(qsub(qmul(E[4], E[8]), qmul(E[5], E[7])), E[0], d0);
    cmul(qsub(qmul(E[3], E[8]), qmul(E[5], E[6])), E[1], d1);
    cmul(qsub(qmul(E[3], E[7]), qmul(E[4], E[6])), E[2], d2);
#pragma unroll
    for (int m = 0; m < 10; m++) M[9][m] = d0[m] - d1[m] + d2[m];
}

// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E-1.  Used where a
// "#pragma unroll" loop is not enough: the indices must be constants when the IR is first
// built, or instcombine folds select chains of array loads into one indexed load
// (A[p][j]) before unrolling, and the matrix can never leave scratch memory.
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// A value the optimiser must treat as freshly computed: select chains over opaque values
// cannot be folded into one dynamically indexed load, which would force the whole matrix
// into scratch memory.  Emits no instruction.
__device__ __forceinline__ double opaque(double x) {
    asm("" : "+v"(x));
    return x;
}

// in-place elimination with partial pivoting over the first NCOL columns (first maximal
// |pivot|, rows swapped); returns false on an exactly zero pivot column, sign = (-1)^swaps.
// Columns < k are dead after step k and never touched again.
template <int NCOL>
__device__ __forceinline__ bool eliminate(double (&A)[10][10], double &sign) {
    bool ok = true;
    static_for<0, NCOL>([&](auto K) {
        constexpr int k = decltype(K)::value;
        if (!ok) return;
        int p = k;
        double best = fabs(A[k][k]);
        static_for<k + 1, 10>([&](auto I) {
            constexpr int i = decltype(I)::value;
            if (fabs(A[i][k]) > best) {
                best = fabs(A[i][k]);
                p = i;
            }
        });
        double pr[10];
        static_for<k, 10>([&](auto J) {
            constexpr int j = decltype(J)::value;
            double v = A[k][j];
            static_for<k + 1, 10>([&](auto I) {
                constexpr int i = decltype(I)::value;
                v = (i == p) ? opaque(A[i][j]) : v;
            });
            pr[j] = v;
        });
        if (pr[k] == 0.0) {
            ok = false;
            return;
        }
        sign = (p != k) ? -sign : sign;
        static_for<k + 1, 10>([&](auto I) {
            constexpr int i = decltype(I)::value;
            static_for<k, 10>([&](auto J) {
                constexpr int j = decltype(J)::value;
                A[i][j] = (i == p) ? opaque(A[k][j]) : opaque(A[i][j]);
            });
        });
        static_for<k, 10>([&](auto J) { A[k][decltype(J)::value] = pr[decltype(J)::value]; });
        static_for<k + 1, 10>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const double f = A[i][k] / A[k][k];
            static_for<k + 1, 10>([&](auto J) {
                constexpr int j = decltype(J)::value;
                A[i][j] -= f * A[k][j];
            });
        });
    });
    return ok;
}

__device__ __forceinline__ double det10(double (&A)[10][10]) {
    double sign = 1.0;
    if (!eliminate<10>(A, sign)) return 0.0;
    double det = sign;
#pragma unroll
    for (int k = 0; k < 10; k++) det *= A[k][k];
    return det;
}

__device__ __forceinline__ bool null10(double (&A)[10][10], double (&v)[10]) {
    double sign = 1.0;
    if (!eliminate<9>(A, sign)) return false;
    v[9] = 1.0;
#pragma unroll
    for (int k = 8; k >= 0; k--) {
        double sum = A[k][9];
#pragma unroll
        for (int j = k + 1; j < 9; j++) sum += A[k][j] * v[j];
        v[k] = -sum / A[k][k];
    }
    return true;
}

// ---- the candidate values: real roots of det M(z), ascending (the oracle's asc_real_roots):
// derivative-recursion isolation + safeguarded Newton.  The reference's ORDER of the candidates
// (rpoly's, which decides the selected model when several pass cheirality) comes from the
// Jenkins-Traub restatement in usac_rpoly.hpp, run only for the samples that need it (k_e5_order).
// Horner with fused multiply-adds (oracle poly_eval / poly_eval2)
__device__ __forceinline__ double poly_eval(const double *c, int deg, double x) {
    double r = c[deg];
    for (int i = deg - 1; i >= 0; i--) r = fma(r, x, c[i]);
    return r;
}

__device__ __forceinline__ void poly_eval2(const double *c, int deg, double x, double &f, double &df) {
    double v = c[deg], d = 0.0;
    for (int j = deg - 1; j >= 0; j--) {
        d = fma(d, x, v);
        v = fma(v, x, c[j]);
    }
    f = v;
    df = d;
}

// safeguarded Newton from the secant point of a sign-changing bracket (oracle poly_refine,
// same op sequence)
__device__ __noinline__ double poly_refine(const double *c, int deg, double lo, double hi, double flo, double fhi) {
    double x = lo - flo * ((hi - lo) / (fhi - flo));
    if (!(x > lo && x < hi)) x = 0.5 * (lo + hi);
    double dxold = hi - lo, dx = dxold, f, df;
    poly_eval2(c, deg, x, f, df);
    for (int it = 0; it < 200; it++) {
        if (f == 0.0) return x;
        if ((f < 0.0) == (flo < 0.0)) {
            lo = x;
            flo = f;
        } else {
            hi = x;
        }
        const double step = f / df;
        const double xn = x - step;
        const bool inside = xn > lo && xn < hi;
        if (xn == x || fabs(step) <= 0x1p-50 * fabs(x)) return inside ? xn : x;
        const bool newton = inside && !(fabs(2.0 * f) > fabs(dxold * df));
        dxold = dx;
        if (newton) {
            dx = step;
            x = xn;
        } else {
            const double mid = 0.5 * (lo + hi);
            if (!(mid > lo && mid < hi)) return mid;
            dx = mid - x;
            x = mid;
        }
        poly_eval2(c, deg, x, f, df);
    }
    return x;
}

// IEEE-only root bound (oracle root_bound): smallest r = 2^k with |a_n| r > sum |a_i| r^(i-n+1)
__device__ __forceinline__ double root_bound(const double *a, int n) {
    double r = 1.0;
    const double an = fabs(a[n]);
    for (int it = 0; it < 2100; it++) {
        double t = fabs(a[0]);
        for (int i = 1; i < n; i++) t = t / r + fabs(a[i]);
        if (an * r > t) break;
        r = r * 2.0;
    }
    return r;
}

// real roots of a[0] + ... + a[n] z^n (oracle real_roots, any n <= 10), ascending; the
// general-degree path with indexed arrays, taken only when a[10] == 0
__device__ __noinline__ int real_roots_dyn(const double *a, double *roots) {
    int n = 10;
    while (n > 0 && a[n] == 0.0) n--;
    if (n == 0) return 0;
    const double R = root_bound(a, n);
    double crit[10], next[10];
    int found[10] = {0};
    for (int g = 1; g <= n; g++) {
        const int d = n - g;
        double c[11];
        for (int j = 0; j <= g; j++) {
            double f = 1.0;
            for (int m = j + d; m > j; m--) f *= (double)m;
            c[j] = a[j + d] * f;
        }
        double lo = -R, flo = poly_eval(c, g, lo);
        for (int k = 0; k < g; k++) {
            const double hi = k < g - 1 ? crit[k] : R;
            const double fhi = poly_eval(c, g, hi);
            if (hi > lo && ((flo < 0.0) != (fhi < 0.0))) {
                next[k] = poly_refine(c, g, lo, hi, flo, fhi);
                found[k] = 1;
            } else {
                next[k] = lo;
                found[k] = 0;
            }
            lo = hi;
            flo = fhi;
        }
        for (int k = 0; k < g; k++) crit[k] = next[k];
    }
    int nr = 0;
    for (int k = 0; k < n; k++)
        if (found[k]) roots[nr++] = crit[k];
    return nr;
}

// The same spec for a true degree-10 polynomial with every degree a compile-time constant:
// coefficients, partition points and Horner loops all stay in registers.  Within a level
// the sign-changing intervals are refined by ONE flat loop: each trip performs one step of
// the lane's current interval and, when that interval is done, moves the lane on to its
// next one -- a wave pays the max over lanes of the per-level sum of steps, not the sum
// over intervals of the per-interval max.  Every interval's result is poly_refine's (the
// oracle's), only the schedule differs.
template <int G>
__device__ __forceinline__ double poly_eval_t(const double (&c)[11], double x) {
    double r = c[G];
#pragma unroll
    for (int i = G - 1; i >= 0; i--) r = fma(r, x, c[i]);
    return r;
}

// Per-lane level arrays live in LDS (the caller's 64-lane block, stride 64 doubles):
// E[0..G] the interval ends, FE[0..G] p at the ends.  The level's output points overwrite
// E in place: output k starts as the filler E[k] (the interval's left end) and a refined
// interval k stores its root into E[k] when it completes -- intervals complete in
// ascending order and interval k+1 only reads E[k+1], E[k+2], so no later read sees it.
// The flat loop picks a new interval's ends with dynamically indexed LDS reads -- one
// ds_read each, where register arrays would cost G selects per value on every trip on
// which some lane starts an interval (nearly every trip).
struct RootsLds {
    double *E, *FE;  // already offset by the lane; element k at [64 k]
};

template <int G>
__device__ __forceinline__ void roots_level(const double (&a)[11], double R, const RootsLds &L, uint32_t &found) {
    constexpr int d = 10 - G;
    double c[11];
#pragma unroll
    for (int j = 0; j <= G; j++) {
        double f = 1.0;
#pragma unroll
        for (int m = j + d; m > j; m--) f *= (double)m;
        c[j] = a[j + d] * f;
    }
    // interval k = [E[k], E[k+1]]: the previous level's points between -R and R; left ends
    // are the fillers unless the interval is refined
    double e[G + 1];
    e[0] = -R;
#pragma unroll
    for (int k = 1; k < G; k++) e[k] = L.E[64 * (k - 1)];
    e[G] = R;
    uint32_t todo = 0;
    double fprev = poly_eval_t<G>(c, e[0]);
    L.E[0] = e[0];
    L.FE[0] = fprev;
#pragma unroll
    for (int k = 0; k < G; k++) {
        const double fk = poly_eval_t<G>(c, e[k + 1]);
        L.E[64 * (k + 1)] = e[k + 1];
        L.FE[64 * (k + 1)] = fk;
        if (e[k + 1] > e[k] && ((fprev < 0.0) != (fk < 0.0))) todo |= 1u << k;
        fprev = fk;
    }
    found = todo;
    // per-lane refinement state of the current interval k
    int k = 0, it = 0;
    double lo = 0.0, hi = 0.0, flo = 0.0, x = 0.0, dxold = 0.0, dx = 0.0;
    bool fresh = true;  // set up interval `k = lowest bit of todo` at the top of the trip
    while (todo) {
        if (fresh) {
            k = __builtin_ctz(todo);
            lo = L.E[64 * k];
            hi = L.E[64 * (k + 1)];
            flo = L.FE[64 * k];
            const double fhi = L.FE[64 * (k + 1)];
            x = lo - flo * ((hi - lo) / (fhi - flo));
            if (!(x > lo && x < hi)) x = 0.5 * (lo + hi);
            dxold = hi - lo;
            dx = dxold;
            it = 0;
            fresh = false;
        }
        double v = c[G], dd = 0.0;
#pragma unroll
        for (int j = G - 1; j >= 0; j--) {
            dd = fma(dd, x, v);
            v = fma(v, x, c[j]);
        }
        const double f = v, df = dd;
        bool done = false;
        double res = x;
        if (it == 200 || f == 0.0) {
            done = true;
        } else {
            it++;
            if ((f < 0.0) == (flo < 0.0)) {
                lo = x;
                flo = f;
            } else {
                hi = x;
            }
            const double step = f / df;
            const double xn = x - step;
            const bool inside = xn > lo && xn < hi;
            if (xn == x || fabs(step) <= 0x1p-50 * fabs(x)) {
                done = true;
                res = inside ? xn : x;
            } else {
                const bool newton = inside && !(fabs(2.0 * f) > fabs(dxold * df));
                dxold = dx;
                if (newton) {
                    dx = step;
                    x = xn;
                } else {
                    const double mid = 0.5 * (lo + hi);
                    if (!(mid > lo && mid < hi)) {
                        done = true;
                        res = mid;
                    } else {
                        dx = mid - x;
                        x = mid;
                    }
                }
            }
        }
        if (done) {
            L.E[64 * k] = res;
            todo &= todo - 1;
            fresh = true;
        }
    }
    if constexpr (G < 10) roots_level<G + 1>(a, R, L, found);
}

// a[10] != 0 required; root k (ascending) is L.E[64 k] where bit k of found
__device__ __forceinline__ void real_roots10(const double (&a)[11], const RootsLds &L, uint32_t &found) {
    double r = 1.0;
    const double an = fabs(a[10]);
    for (int it = 0; it < 2100; it++) {
        double t = fabs(a[0]);
#pragma unroll
        for (int i = 1; i < 10; i++) t = t / r + fabs(a[i]);
        if (an * r > t) break;
        r = r * 2.0;
    }
    roots_level<1>(a, r, L, found);
}

__device__ __forceinline__ double det3p(const double (&P)[3][4]) {
    return P[0][0] * (P[1][1] * P[2][2] - P[1][2] * P[2][1]) - P[0][1] * (P[1][0] * P[2][2] - P[1][2] * P[2][0]) +
           P[0][2] * (P[1][0] * P[2][1] - P[1][1] * P[2][0]);
}

// CalcDepth (five_points.cpp:278-302)
__device__ __forceinline__ double calc_depth(const double (&X)[4], const double (&P)[3][4]) {
    double w = 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++) w += P[2][k] * X[k];
    const double det = det3p(P);
    const double a = P[0][2], b = P[1][2], c = P[2][2];
    const double m3 = sqrt(a * a + b * b + c * c);
    const double sign = det > 0 ? 1.0 : -1.0;
    return (w / X[3]) * (sign / m3);
}

// both depths of a correspondence for P_ref = [I|0] and P (TriangulatePoint :304-334 as the
// rank-3 null vector on the first ray, oracle triangulate)
__device__ __forceinline__ bool in_front(double x1, double y1, double x2, double y2, const double (&P)[3][4]) {
    constexpr double Pr[3][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}};
    double b[2][2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const double u = r == 0 ? x2 : y2;
        double row[4];
#pragma unroll
        for (int c = 0; c < 4; c++) row[c] = u * P[2][c] - P[r][c];
        b[r][0] = row[0] * x1 + row[1] * y1 + row[2];
        b[r][1] = row[3];
    }
    const double n0 = b[0][0] * b[0][0] + b[0][1] * b[0][1];
    const double n1 = b[1][0] * b[1][0] + b[1][1] * b[1][1];
    const bool first = n0 >= n1;
    const double sc = first ? b[0][1] : b[1][1];
    const double w = first ? -b[0][0] : -b[1][0];
    const double X[4] = {x1 * sc, y1 * sc, sc, w};
    return calc_depth(X, Pr) > 0 && calc_depth(X, P) > 0;
}

// ProjectionsFromEssential (five_points.cpp:336-371), projection j in 0..3
__device__ __forceinline__ void projection(const double (&U)[3][3], const double (&V)[3][3], int j,
                                           double (&P)[3][4]) {
    constexpr double Wm[3][3] = {{0, -1, 0}, {1, 0, 0}, {0, 0, 1}};
    const int w = j >> 1, sgn = j & 1;
    double T[3][3];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) {
            double sum = 0.0;
#pragma unroll
            for (int k = 0; k < 3; k++) sum += U[r][k] * (w == 0 ? Wm[k][c] : Wm[c][k]);
            T[r][c] = sum;
        }
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            double sum = 0.0;
#pragma unroll
            for (int k = 0; k < 3; k++) sum += T[r][k] * V[c][k];
            P[r][c] = sum;
        }
        P[r][3] = sgn == 0 ? U[r][2] : -U[r][2];
    }
}

// 3x3 SVD columns U, V (oracle projections(): rows Jacobi with accumulated rotations,
// singular values descending, v3 = v1 x v2)
__device__ __forceinline__ void svd3(const double (&E)[9], double (&U)[3][3], double (&V)[3][3]) {
    double B[3][3], J[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            B[i][k] = E[3 * i + k];
            J[i][k] = i == k ? 1.0 : 0.0;
        }
    jacobi_small<3, 3, true>(B, J);
    double sg[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        double a = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) a += B[i][k] * B[i][k];
        sg[i] = sqrt(a);
    }
    int o[3] = {0, 1, 2};
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = i + 1; j < 3; j++)
            if (sg[o[j]] > sg[o[i]]) {
                const int t = o[i];
                o[i] = o[j];
                o[j] = t;
            }
    // o[] is a permutation: gather rows by value (no dynamic register indexing)
#pragma unroll
    for (int k = 0; k < 3; k++) {
        double jr[3], br[3], s = 0.0;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            jr[r] = o[k] == 0 ? J[0][r] : o[k] == 1 ? J[1][r] : J[2][r];
            br[r] = o[k] == 0 ? B[0][r] : o[k] == 1 ? B[1][r] : B[2][r];
        }
        s = o[k] == 0 ? sg[0] : o[k] == 1 ? sg[1] : sg[2];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            U[r][k] = jr[r];
            if (k < 2) V[r][k] = br[r] / s;
        }
    }
    V[0][2] = V[1][0] * V[2][1] - V[2][0] * V[1][1];
    V[1][2] = V[2][0] * V[0][1] - V[0][0] * V[2][1];
    V[2][2] = V[0][0] * V[1][1] - V[1][0] * V[0][1];
}

}  // namespace e5

// EssentialEstimator::GetError (essential_estimator.hpp:76-107).  The reference's
// `float a2 = sqrt(float)` is C's double sqrt rounded to float; for a float argument that
// equals the correctly rounded fp32 square root (53 >= 2*24 + 2 bits: no double rounding),
// so the correctly rounded fp32 sqrtf is used -- bit-identical, a fraction of the cost.
// (Not __fsqrt_rn: on gfx950 it lowers to the 1-ulp v_sqrt_f32.)
__device__ __forceinline__ float essential_error(const float *E, float x1, float y1, float x2, float y2) {
    const float l1 = E[0] * x2 + E[3] * y2 + E[6];
    const float l2 = E[1] * x2 + E[4] * y2 + E[7];
    const float l3 = E[2] * x2 + E[5] * y2 + E[8];
    const float t1 = E[0] * x1 + E[1] * y1 + E[2];
    const float t2 = E[3] * x1 + E[4] * y1 + E[5];
    const float t3 = E[6] * x1 + E[7] * y1 + E[8];
    const float a1 = l1 * x1 + l2 * y1 + l3;
    const float a2 = sqrtf(l1 * l1 + l2 * l2);
    const float b1 = t1 * x2 + t2 * y2 + t3;
    const float b2 = sqrtf(t1 * t1 + t2 * t2);
    return (fabsf(a1 / a2) + fabsf(b1 / b2)) / 2;
}

// The guarded essential residual of the throughput drains (C > 1: Σ is re-associated anyway and
// its terms may carry a stated error; the counts stay exact).  The reference's l, t, a1, b1 and
// squared norms (the same unfused operations), then e' = (|a1| rsq(a2²) + |b1| rsq(b2²)) / 2
// with v_rsq_f32 (1 ulp) instead of two correctly rounded square roots and two IEEE divisions.
// Per term the two differ by < 2^-21 relative (rsq 2^-23, the product and the reference's sqrt
// and division 2^-24 each), so |e' - e| <= e' 2^-19: e' <= thr (1 - 2^-16) proves e < thr and
// e' >= thr (1 + 2^-16) proves !(e < thr).  Pairs inside that band, squared norms outside
// [2^-96, inf) (denormal / zero / overflowing rsq) and non-finite values take the exact
// expression.  Returns the error added to Σ: e' for a proven inlier, else the exact e.
__device__ __forceinline__ float essential_error_guarded(const float *E, float x1, float y1, float x2, float y2,
                                                         float thr, float lo, float hi, bool &inl) {
    const float l1 = E[0] * x2 + E[3] * y2 + E[6];
    const float l2 = E[1] * x2 + E[4] * y2 + E[7];
    const float l3 = E[2] * x2 + E[5] * y2 + E[8];
    const float t1 = E[0] * x1 + E[1] * y1 + E[2];
    const float t2 = E[3] * x1 + E[4] * y1 + E[5];
    const float t3 = E[6] * x1 + E[7] * y1 + E[8];
    const float a1 = l1 * x1 + l2 * y1 + l3;
    const float qa = l1 * l1 + l2 * l2;
    const float b1 = t1 * x2 + t2 * y2 + t3;
    const float qb = t1 * t1 + t2 * t2;
    const float ef = (fabsf(a1) * __builtin_amdgcn_rsqf(qa) + fabsf(b1) * __builtin_amdgcn_rsqf(qb)) * 0.5f;
    const bool normal = qa >= 1.2621774483536189e-29f && qb >= 1.2621774483536189e-29f &&  // 2^-96
                        qa < INFINITY && qb < INFINITY;
    if (__builtin_expect(normal && (ef <= lo || ef >= hi), 1)) {
        inl = ef <= lo;
        return ef;
    }
    const float e = (fabsf(a1 / sqrtf(qa)) + fabsf(b1 / sqrtf(qb))) / 2;  // essential_error, bit for bit
    inl = e < thr;
    return e;
}

}  // namespace usac
