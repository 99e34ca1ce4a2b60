#pragma once
// usac_rpoly.hpp -- the 5-point solver's root step on the device: the reference's Jenkins-Traub
// rpoly_ak1 (usac/estimator/essential/rpoly.cpp:7-750), restated operation for operation as the
// oracle's jt_rpoly (oracle/usac_oracle.c) -- the same expressions, no FMA contraction, correctly
// rounded division / sqrt -- so the device reports the oracle's zeros bit for bit and in rpoly's
// order (five_points.cpp:143-157 keeps the real ones in that order; the first whose E passes
// cheirality is the model, :239-273).  rpoly's log / exp (rpoly.cpp:82,98) are the oracle's portable
// correctly rounded pair (jt_log / jt_exp).
//
// MI355X layout: rpoly indexes its polynomials by the running degree N, so every routine is a
// template on N (10 .. 3, the deflation visits each at most once) and the polynomials live in
// registers with constant indices; jt_rpoly10 walks the degrees in lockstep.  Two schedules:
//   * jt_rpoly10<false>: one polynomial per lane, at most `budget` fixed-shift steps (a wave waits
//     for its slowest lane; cfg4's step counts: median 16, p99 75, p99.9 136, a 20-shift failure
//     4 200) -- returns -1 past the budget, and the caller defers the polynomial;
//   * jt_rpoly10<true>: one polynomial per wave, its 20 shift attempts of a zero search (rpoly.cpp:
//     172-212: each starts from the same saved K with the shift rotated once more, and the first
//     that converges wins) run side by side on lanes 0..19; a lane stops when a lower lane has
//     converged; the lowest converged lane's zeros, quotient and rotation state are the sequential
//     result.  A zero search costs its longest needed attempt (<= 400 steps), not their sum.
#include <float.h>
#include <hip/hip_runtime.h>

#include "usac_rpoly_tables.hpp"

namespace usac {
namespace e5 {

// ---- double-double helpers and the correctly rounded log / exp (oracle jt_log / jt_exp)
struct JtDD {
    double hi, lo;
};
__device__ __forceinline__ JtDD jt_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return JtDD{s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ JtDD jt_qsum(double a, double b) {
    const double s = a + b;
    return JtDD{s, b - (s - a)};
}
__device__ __forceinline__ JtDD jt_dadd(JtDD x, JtDD y) {
    JtDD s = jt_sum(x.hi, y.hi);
    const JtDD t = jt_sum(x.lo, y.lo);
    s.lo += t.hi;
    s = jt_qsum(s.hi, s.lo);
    s.lo += t.lo;
    return jt_qsum(s.hi, s.lo);
}
__device__ __forceinline__ JtDD jt_dmul(JtDD x, JtDD y) {
    const double p = x.hi * y.hi;
    double e = fma(x.hi, y.hi, -p);
    e += x.hi * y.lo + x.lo * y.hi;
    return jt_qsum(p, e);
}
__device__ __forceinline__ JtDD jt_inv(double k) {
    const double h = 1.0 / k;
    return JtDD{h, fma(-h, k, 1.0) / k};
}
constexpr double kJtLn2Hi = 0x1.62e42fefa39efp-1, kJtLn2Lo = 0x1.abc9e3b39803fp-56;

__device__ __noinline__ double jt_log_slow(double x) {
    if (!(x > 0.0) || isinf(x)) return x == 0.0 ? -INFINITY : (x > 0.0 ? x : NAN);
    int e;
    double m = frexp(x, &e);
    if (m < 0x1.6a09e667f3bcdp-1) {
        m *= 2.0;
        e--;
    }
    const double f = m - 1.0;
    const JtDD den = jt_sum(2.0, f);
    const double sh = f / den.hi;
    const double r = fma(-sh, den.hi, f) - sh * den.lo;
    const JtDD s = jt_qsum(sh, r / den.hi);
    const JtDD t = jt_dmul(s, s);
    double tail = 0.0;
#pragma unroll
    for (int k = 24; k >= 11; k--) tail = tail * t.hi + 1.0 / (double)(2 * k + 1);
    JtDD P{tail, 0.0};
#pragma unroll
    for (int k = 10; k >= 1; k--) P = jt_dadd(jt_dmul(P, t), jt_inv((double)(2 * k + 1)));
    P = jt_dadd(jt_dmul(P, t), JtDD{1.0, 0.0});
    JtDD lm = jt_dmul(s, P);
    lm.hi *= 2.0;
    lm.lo *= 2.0;
    const JtDD res = jt_dadd(jt_dmul(JtDD{(double)e, 0.0}, JtDD{kJtLn2Hi, kJtLn2Lo}), lm);
    return res.hi + res.lo;
}

__device__ __noinline__ double jt_exp_slow(double y) {
    if (y != y) return y;
    if (y > 709.79) return INFINITY;
    if (y < -745.2) return 0.0;
    const double k = nearbyint(y / kJtLn2Hi);
    const JtDD r = jt_dadd(JtDD{y, 0.0}, jt_dmul(JtDD{-k, 0.0}, JtDD{kJtLn2Hi, kJtLn2Lo}));
    double fact = 1.0, tail = 0.0;
    double inv[28];
#pragma unroll
    for (int n = 1; n < 28; n++) {
        fact *= (double)n;
        inv[n] = 1.0 / fact;
    }
#pragma unroll
    for (int n = 27; n >= 14; n--) tail = tail * r.hi + inv[n];
    JtDD P{tail, 0.0};
    fact = 1.0;
#pragma unroll
    for (int n = 1; n < 14; n++) fact *= (double)n;
#pragma unroll
    for (int n = 13; n >= 1; n--) {
        P = jt_dadd(jt_dmul(P, r), jt_inv(fact));
        fact /= (double)n;
    }
    P = jt_dadd(jt_dmul(P, r), JtDD{1.0, 0.0});
    return ldexp(P.hi + P.lo, (int)k);
}

// The fast paths (Ziv's strategy): a table-driven evaluation in double-double whose absolute (log)
// or relative (exp) error is below 2^-67; when the result's rounding is decided within that bound it
// is the correctly rounded value, i.e. the slow path's and the oracle's, otherwise the slow path runs
// (measured on cfg4's polynomials: ~1e-4 of calls).  Tables: usac_rpoly_tables.hpp.
__device__ __forceinline__ double jt_round_checked(JtDD v, double delta, bool &ok) {
    const double a = v.hi + (v.lo - delta), b = v.hi + (v.lo + delta);
    ok = a == b;
    return a;
}

// log x = e ln2 - log c_k + log(1 + r), x = m 2^e, m in [sqrt(1/2), sqrt 2), r = m c_k - 1 exactly
// (|r| < 2^-7.5), log(1 + r) to degree 8
__device__ __forceinline__ double jt_log(double x) {
    if (!(x > 0x1p-1000 && x < 0x1p1000)) return jt_log_slow(x);
    int e;
    double m = frexp(x, &e);
    if (m < 0x1.6a09e667f3bcdp-1) {
        m *= 2.0;
        e--;
    }
    int k = (int)(m * 128.0);
    k = k < kJtLogK0 ? kJtLogK0 : (k > kJtLogK1 ? kJtLogK1 : k);
    const double c = kJtLogTab[k - kJtLogK0][0];
    const double P = m * c, Pe = fma(m, c, -P);
    const JtDD r = jt_sum(P - 1.0, Pe);
    const double sh = r.hi * r.hi, sl = fma(r.hi, r.hi, -sh);
    const double q = r.hi;
    const double poly = ((((( -0.125 * q + 0x1.2492492492492p-3) * q - 0x1.5555555555555p-3) * q + 0.2) * q - 0.25) * q +
                         0x1.5555555555555p-2);
    const double tail = (sh * q) * poly - r.hi * r.lo;
    JtDD l1 = jt_dadd(r, JtDD{-0.5 * sh, -0.5 * sl});
    l1 = jt_dadd(l1, JtDD{tail, 0.0});
    const JtDD lp = jt_dadd(JtDD{kJtLogTab[k - kJtLogK0][1], kJtLogTab[k - kJtLogK0][2]}, l1);
    const JtDD res = jt_dadd(jt_dmul(JtDD{(double)e, 0.0}, JtDD{kJtLn2Hi, kJtLn2Lo}), lp);
    bool ok;
    const double out = jt_round_checked(res, 0x1p-67, ok);
    return ok ? out : jt_log_slow(x);
}

// exp y = 2^kk 2^(j/128) exp(r), y = (128 kk + j) ln2 / 128 + r, |r| <= ln2 / 256 (+), exp(r) to degree 6
__device__ __forceinline__ double jt_exp(double y) {
    if (!(y > -700.0 && y < 700.0)) return jt_exp_slow(y);
    const double t = nearbyint(y * kJt128OverLn2);
    const int n = (int)t, j = n & 127, kk = (n - j) / 128;
    const JtDD r = jt_dadd(JtDD{y, 0.0}, jt_dmul(JtDD{-t, 0.0}, JtDD{kJtLn2_128Hi, kJtLn2_128Lo}));
    const double q = r.hi;
    const double sh = q * q, sl = fma(q, q, -sh);
    const double poly = ((0x1.6c16c16c16c17p-10 * q + 0x1.1111111111111p-7) * q + 0x1.5555555555555p-5) * q +
                        0x1.5555555555555p-3;
    const double tail = (sh * q) * poly + q * r.lo;
    JtDD E = jt_sum(1.0, q);
    E = jt_dadd(E, JtDD{r.lo, 0.0});
    E = jt_dadd(E, JtDD{0.5 * sh, 0.5 * sl});
    E = jt_dadd(E, JtDD{tail, 0.0});
    const JtDD res = jt_dmul(JtDD{kJtExpTab[j][0], kJtExpTab[j][1]}, E);
    bool ok;
    const double out = jt_round_checked(res, 0x1p-67 * fabs(res.hi), ok);
    return ok ? ldexp(out, kk) : jt_exp_slow(y);
}

// ---- the iteration at compile-time degree N (p: N + 1 coefficients, highest power first)
template <int N>
struct Jt {
    double K[N], qp[N + 1], qk[N + 1];
    double a, b, c, d, e, f, g, h, a1, a3, a7;
};

// QuadSD_ak1 (rpoly.cpp:378-394): q = src / (z^2 + u z + v), the last two running values -> ra, rb
template <int NN>
__device__ __forceinline__ void jt_divide(double u, double v, const double *src, double *q, double &ra, double &rb) {
    double bb = src[0], aa = src[1] - bb * u;
    q[0] = bb;
    q[1] = aa;
#pragma unroll
    for (int i = 2; i < NN; i++) {
        const double t = src[i] - (aa * u + bb * v);
        q[i] = t;
        bb = aa;
        aa = t;
    }
    ra = aa;
    rb = bb;
}

// calcSC_ak1 (rpoly.cpp:396-435)
template <int N>
__device__ __forceinline__ int jt_scalars(Jt<N> &s, double u, double v) {
    jt_divide<N>(u, v, s.K, s.qk, s.c, s.d);
    if (fabs(s.c) <= 100.0 * DBL_EPSILON * fabs(s.K[N - 1]) && fabs(s.d) <= 100.0 * DBL_EPSILON * fabs(s.K[N - 2]))
        return 3;
    s.h = v * s.b;
    if (fabs(s.d) >= fabs(s.c)) {
        s.e = s.a / s.d;
        s.f = s.c / s.d;
        s.g = u * s.b;
        s.a3 = s.e * (s.g + s.a) + s.h * (s.b / s.d);
        s.a1 = s.f * s.b - s.a;
        s.a7 = s.h + (s.f + u) * s.a;
        return 2;
    }
    s.e = s.a / s.c;
    s.f = s.d / s.c;
    s.g = s.e * u;
    s.a3 = s.e * s.a + (s.g + s.h / s.c) * s.b;
    s.a1 = s.b - s.a * (s.d / s.c);
    s.a7 = s.g * s.d + s.h * s.f + s.a;
    return 1;
}

// nextK_ak1 (rpoly.cpp:437-475)
template <int N>
__device__ __forceinline__ void jt_next_k(Jt<N> &s, int type) {
    if (type == 3) {
        s.K[0] = 0.0;
        s.K[1] = 0.0;
#pragma unroll
        for (int i = 2; i < N; i++) s.K[i] = s.qk[i - 2];
        return;
    }
    const double ref = type == 1 ? s.b : s.a;
    if (fabs(s.a1) > 10.0 * DBL_EPSILON * fabs(ref)) {
        s.a7 /= s.a1;
        s.a3 /= s.a1;
        s.K[0] = s.qp[0];
        s.K[1] = s.qp[1] - s.a7 * s.qp[0];
#pragma unroll
        for (int i = 2; i < N; i++) s.K[i] = (s.a3 * s.qk[i - 2] - s.a7 * s.qp[i - 1]) + s.qp[i];
    } else {
        s.K[0] = 0.0;
        s.K[1] = -s.a7 * s.qp[0];
#pragma unroll
        for (int i = 2; i < N; i++) s.K[i] = s.a3 * s.qk[i - 2] - s.a7 * s.qp[i - 1];
    }
}

// newest_ak1 (rpoly.cpp:477-513)
template <int N>
__device__ __forceinline__ void jt_newest(const Jt<N> &s, const double *p, int type, double u, double v, double &uu,
                                          double &vv) {
    uu = vv = 0.0;
    if (type == 3) return;
    double a4, a5;
    if (type != 2) {
        a4 = (s.a + u * s.b) + s.h * s.f;
        a5 = s.c + (u + v * s.f) * s.d;
    } else {
        a4 = (s.a + s.g) * s.f + s.h;
        a5 = (s.f + u) * s.c + v * s.d;
    }
    const double b1 = -s.K[N - 1] / p[N];
    const double b2 = -(s.K[N - 2] + b1 * p[N - 1]) / p[N];
    const double c1 = v * b2 * s.a1, c2 = b1 * s.a7, c3 = b1 * b1 * s.a3;
    const double c4 = c1 - (c2 + c3);
    const double t = (a5 - c4) + b1 * a4;
    if (t != 0.0) {
        uu = u - (u * (c3 + c2) + v * (b1 * s.a1 + b2 * s.a7)) / t;
        vv = v * (1.0 + c4 / t);
    }
}

// Quad_ak1 (rpoly.cpp:700-750)
__device__ __forceinline__ void jt_quadratic(double a, double b1, double c, double &sr, double &si, double &lr,
                                             double &li) {
    sr = si = lr = li = 0.0;
    if (a == 0.0) {
        if (b1 != 0.0) sr = -(c / b1);
        return;
    }
    if (c == 0.0) {
        lr = -(b1 / a);
        return;
    }
    const double b = b1 / 2.0;
    double d, e;
    if (fabs(b) < fabs(c)) {
        e = c >= 0.0 ? a : -a;
        e = b * (b / fabs(c)) - e;
        d = sqrt(fabs(e)) * sqrt(fabs(c));
    } else {
        e = 1.0 - (a / b) * (c / b);
        d = sqrt(fabs(e)) * fabs(b);
    }
    if (e >= 0.0) {
        if (b >= 0.0) d = -d;
        lr = (d - b) / a;
        if (lr != 0.0) sr = (c / lr) / a;
    } else {
        lr = sr = -(b / a);
        si = fabs(d / a);
        li = -si;
    }
}

// QuadIT_ak1 (rpoly.cpp:515-607)
template <int N>
__device__ __forceinline__ int jt_quad_iter(Jt<N> &s, const double *p, double uu, double vv, double &szr,
                                            double &szi, double &lzr, double &lzi, int &steps, int budget) {
    double u = uu, v = vv, relstp = 0.0, omp = 0.0, ui = 0.0, vi = 0.0;
    int j = 0;
    bool tried = false;
    do {
        if ((steps += 4) > budget) return -1;  // an iteration: one division of p, three of K
        jt_quadratic(1.0, u, v, szr, szi, lzr, lzi);
        if (fabs(fabs(szr) - fabs(lzr)) > 0.01 * fabs(lzr)) break;
        jt_divide<N + 1>(u, v, p, s.qp, s.a, s.b);
        const double mp = fabs(s.a - szr * s.b) + fabs(szi * s.b);
        const double zm = sqrt(fabs(v));
        double ee = 2.0 * fabs(s.qp[0]);
        const double t = -(szr * s.b);
#pragma unroll
        for (int i = 1; i < N; i++) ee = ee * zm + fabs(s.qp[i]);
        ee = ee * zm + fabs(s.a + t);
        ee = (9.0 * ee + 2.0 * fabs(t) - 7.0 * (fabs(s.a + t) + zm * fabs(s.b))) * DBL_EPSILON;
        if (mp <= 20.0 * ee) return 2;
        if (++j > 20) break;
        if (j >= 2 && relstp <= 0.01 && mp >= omp && !tried) {
            relstp = relstp < DBL_EPSILON ? sqrt(DBL_EPSILON) : sqrt(relstp);
            u -= u * relstp;
            v += v * relstp;
            jt_divide<N + 1>(u, v, p, s.qp, s.a, s.b);
            for (int i = 0; i < 5; i++) jt_next_k(s, jt_scalars(s, u, v));
            tried = true;
            j = 0;
        }
        omp = mp;
        jt_next_k(s, jt_scalars(s, u, v));
        jt_newest(s, p, jt_scalars(s, u, v), u, v, ui, vi);
        if (vi != 0.0) {
            relstp = fabs((vi - v) / vi);
            u = ui;
            v = vi;
        }
    } while (vi != 0.0);
    return 0;
}

// RealIT_ak1 (rpoly.cpp:609-698)
template <int N>
__device__ __forceinline__ int jt_real_iter(Jt<N> &s, const double *p, double &sx, int &flag, double &szr,
                                            double &szi, int &steps, int budget) {
    double x = sx, t = 0.0, omp = 0.0;
    int j = 0;
    flag = 0;
    for (;;) {
        if ((steps += 2) > budget) return -1;  // an iteration: two Horner passes
        double pv = p[0];
        s.qp[0] = pv;
#pragma unroll
        for (int i = 1; i <= N; i++) {
            pv = pv * x + p[i];
            s.qp[i] = pv;
        }
        const double mp = fabs(pv), ms = fabs(x);
        double ee = 0.5 * fabs(s.qp[0]);
#pragma unroll
        for (int i = 1; i <= N; i++) ee = ee * ms + fabs(s.qp[i]);
        if (mp <= 20.0 * DBL_EPSILON * (2.0 * ee - mp)) {
            szr = x;
            szi = 0.0;
            return 1;
        }
        if (++j > 10) return 0;
        if (j >= 2 && fabs(t) <= 0.001 * fabs(x - t) && mp > omp) {
            flag = 1;
            sx = x;
            return 0;
        }
        omp = mp;
        double kv = s.K[0];
        s.qk[0] = kv;
#pragma unroll
        for (int i = 1; i < N; i++) {
            kv = kv * x + s.K[i];
            s.qk[i] = kv;
        }
        if (fabs(kv) > fabs(s.K[N - 1]) * 10.0 * DBL_EPSILON) {
            const double tt = -(pv / kv);
            s.K[0] = s.qp[0];
#pragma unroll
            for (int i = 1; i < N; i++) s.K[i] = tt * s.qk[i - 1] + s.qp[i];
        } else {
            s.K[0] = 0.0;
#pragma unroll
            for (int i = 1; i < N; i++) s.K[i] = s.qk[i - 1];
        }
        kv = s.K[0];
#pragma unroll
        for (int i = 1; i < N; i++) kv = kv * x + s.K[i];
        t = fabs(kv) > fabs(s.K[N - 1]) * 10.0 * DBL_EPSILON ? -(pv / kv) : 0.0;
        x += t;
    }
}

// Fxshfr_ak1 (rpoly.cpp:232-376).  Returns the zeros found; -1 when `steps` passes `budget`; 0 as
// well when *stop (an LDS word of the wave, nullable) names a lower attempt that converged.
template <int N>
__device__ __forceinline__ int jt_fixed_shift(Jt<N> &s, const double *p, int l2, double sr, double v, double u,
                                              double &szr, double &szi, double &lzr, double &lzi, int &steps,
                                              int budget, const volatile int *stop, int me) {
    double svk[N];
    int iflag = 1;
    double betav = 0.25, betas = 0.25, oss = sr, ovv = v, ots = 0.0, otv = 0.0, ui = 0.0, vi = 0.0, xs = 0.0;
    jt_divide<N + 1>(u, v, p, s.qp, s.a, s.b);
    int type = jt_scalars(s, u, v);
    for (int j = 0; j < l2; j++) {
        if ((steps += 3) > budget) return -1;  // a step: the next K, two divisions of K
        if (stop && *stop < me) return 0;
        bool first = true;
        jt_next_k(s, type);
        type = jt_scalars(s, u, v);
        jt_newest(s, p, type, u, v, ui, vi);
        const double vv = vi;
        const double ss = s.K[N - 1] != 0.0 ? -(p[N] / s.K[N - 1]) : 0.0;
        double tv = 1.0, ts = 1.0;
        if (j != 0 && type != 3) {
            if (vv != 0.0) tv = fabs((vv - ovv) / vv);
            if (ss != 0.0) ts = fabs((ss - oss) / ss);
            const double tvv = tv < otv ? tv * otv : 1.0;
            const double tss = ts < ots ? ts * ots : 1.0;
            const bool vpass = tvv < betav, spass = tss < betas;
            if (spass || vpass) {
#pragma unroll
                for (int i = 0; i < N; i++) svk[i] = s.K[i];
                xs = ss;
                bool stry = false, vtry = false;
                for (;;) {
                    const bool linear_first = first && spass && (!vpass || tss < tvv);
                    first = false;
                    if (!linear_first) {
                        const int nz = jt_quad_iter(s, p, ui, vi, szr, szi, lzr, lzi, steps, budget);
                        if (nz != 0) return nz;
                        iflag = 1;
                        vtry = true;
                        betav *= 0.25;
                        if (stry || !spass) {
                            iflag = 0;
                        } else {
#pragma unroll
                            for (int i = 0; i < N; i++) s.K[i] = svk[i];
                        }
                    }
                    if (iflag != 0) {
                        const int nz = jt_real_iter(s, p, xs, iflag, szr, szi, steps, budget);
                        if (nz != 0) return nz;
                        stry = true;
                        betas *= 0.25;
                        if (iflag != 0) {
                            ui = -(xs + xs);
                            vi = xs * xs;
                            continue;
                        }
                    }
#pragma unroll
                    for (int i = 0; i < N; i++) s.K[i] = svk[i];
                    if (!vpass || vtry) break;
                }
                jt_divide<N + 1>(u, v, p, s.qp, s.a, s.b);
                type = jt_scalars(s, u, v);
            }
        }
        ovv = vv;
        oss = ss;
        otv = tv;
        ots = ts;
    }
    return 0;
}

// One zero search of rpoly's main loop (rpoly.cpp:58-221) at degree N >= 3: scaling, the zeros'
// modulus bound, the K polynomial, then the shift attempts.  On success the zero(s) go to emit(zr,
// zi), p becomes the quotient and the new degree is returned; -1: out of budget; -2: no convergence
// after 20 shifts (rpoly.cpp:214-220: the search ends with the zeros found so far).
template <int N, bool PAR, class Emit>
__device__ __forceinline__ int jt_search(double (&p)[11], double &xx, double &yy, int &steps, int budget,
                                         volatile int *stop, Emit &emit) {
    constexpr int NN = N + 1, NM1 = N - 1;
    const double cosr = -0x1.1db8f6d6a512ap-4, sinr = 0x1.fec0b7170fff6p-1;
    const double lo = DBL_MIN / DBL_EPSILON;
    double mmax = 0.0, mmin = DBL_MAX;
#pragma unroll
    for (int i = 0; i < NN; i++) {
        const double x = fabs(p[i]);
        if (x > mmax) mmax = x;
        if (x != 0.0 && x < mmin) mmin = x;
    }
    double sc = lo / mmin;
    if ((sc <= 1.0 && mmax >= 10.0) || (sc > 1.0 && DBL_MAX / sc >= mmax)) {
        if (sc == 0.0) sc = DBL_MIN;
        const int l = (int)(jt_log(sc) / kJtLn2Hi + 0.5);
        const double factor = ldexp(1.0, l);
        if (factor != 1.0) {
#pragma unroll
            for (int i = 0; i < NN; i++) p[i] = p[i] * factor;
        }
    }
    double pt[NN];
#pragma unroll
    for (int i = 0; i < NN; i++) pt[i] = fabs(p[i]);
    pt[N] = -pt[N];
    double x = jt_exp((jt_log(-pt[N]) - jt_log(pt[0])) / (double)N);
    if (pt[NM1] != 0.0) {
        const double xm = -pt[N] / pt[NM1];
        if (xm < x) x = xm;
    }
    double xm = x, ff = 0.0, df, dx;
    int trips = 0;
    do {
        x = xm;
        xm = 0.1 * x;
        ff = pt[0];
#pragma unroll
        for (int i = 1; i < NN; i++) ff = ff * xm + pt[i];
    } while (ff > 0.0 && ++trips < 2100);
    trips = 0;
    do {
        df = ff = pt[0];
#pragma unroll
        for (int i = 1; i < N; i++) {
            ff = x * ff + pt[i];
            df = x * df + ff;
        }
        ff = x * ff + pt[N];
        dx = ff / df;
        x -= dx;
    } while (fabs(dx / x) > 0.005 && ++trips < 500);
    const double bnd = x;
    Jt<N> s;
#pragma unroll
    for (int i = 1; i < N; i++) s.K[i] = (double)(N - i) * p[i] / (double)N;
    s.K[0] = p[0];
    const double aa = p[N], bb = p[NM1];
    bool zerok = s.K[NM1] == 0.0;
    for (int jj = 0; jj < 5; jj++) {
        const double cc = s.K[NM1];
        if (zerok) {
#pragma unroll
            for (int j = NM1; j >= 1; j--) s.K[j] = s.K[j - 1];
            s.K[0] = 0.0;
            zerok = s.K[NM1] == 0.0;
        } else {
            const double t = -aa / cc;
#pragma unroll
            for (int j = NM1; j >= 1; j--) s.K[j] = t * s.K[j - 1] + p[j];
            s.K[0] = p[0];
            zerok = fabs(s.K[NM1]) <= fabs(bb) * DBL_EPSILON * 10.0;
        }
    }
    double saved[N];
#pragma unroll
    for (int i = 0; i < N; i++) saved[i] = s.K[i];
    double szr = 0.0, szi = 0.0, lzr = 0.0, lzi = 0.0;
    int nz = 0;
    if constexpr (!PAR) {
        for (int jj = 1; jj <= 20; jj++) {
            const double xr = cosr * xx - sinr * yy;
            yy = sinr * xx + cosr * yy;
            xx = xr;
            const double sr = bnd * xx, u = -(2.0 * sr);
            nz = jt_fixed_shift(s, p, 20 * jj, sr, bnd, u, szr, szi, lzr, lzi, steps, budget, nullptr, 0);
            if (nz != 0) break;
#pragma unroll
            for (int i = 0; i < N; i++) s.K[i] = saved[i];
        }
        if (nz < 0) return -1;
        if (nz == 0) return -2;
    } else {
        // attempt jj = lane + 1 on lanes 0..19: the shift rotated jj times from (xx, yy), in order
        const int lane = (int)(threadIdx.x & 63);
        if (lane == 0) *stop = 64;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        if (lane < 20) {
            for (int r = 0; r <= lane; r++) {
                const double xr = cosr * xx - sinr * yy;
                yy = sinr * xx + cosr * yy;
                xx = xr;
            }
            const double sr = bnd * xx, u = -(2.0 * sr);
            nz = jt_fixed_shift(s, p, 20 * (lane + 1), sr, bnd, u, szr, szi, lzr, lzi, steps, budget, stop, lane);
            if (nz > 0) atomicMin((int *)stop, lane);
        }
        const uint64_t won = __builtin_amdgcn_ballot_w64(lane < 20 && nz > 0);
        if (won == 0) return -2;
        const int w = __builtin_ffsll((long long)won) - 1;
        nz = __shfl(nz, w, 64);
        szr = __shfl(szr, w, 64);
        szi = __shfl(szi, w, 64);
        lzr = __shfl(lzr, w, 64);
        lzi = __shfl(lzi, w, 64);
        xx = __shfl(xx, w, 64);
        yy = __shfl(yy, w, 64);
#pragma unroll
        for (int i = 0; i < NN; i++) s.qp[i] = __shfl(s.qp[i], w, 64);
    }
    emit(szr, szi);
    if (nz != 1) emit(lzr, lzi);
#pragma unroll
    for (int i = 0; i < NN; i++) p[i] = s.qp[i];  // the quotient: its first NN - nz entries
    return N - nz;
}

// rpoly's main loop (rpoly.cpp:52-222) in lockstep over the degree: the lanes whose polynomial is at
// degree n run its zero search there; degrees only decrease (by 1 or 2), so one pass n = 10 .. 3 takes
// every lane through its searches in order and a wave runs each degree's code once (a switch over the
// lanes' degrees inside a loop would serialise the cases every round).  status: 0 searching, -1 out of
// budget, 2 no convergence after 20 shifts (rpoly.cpp:214-220), 3 the caller has the zero it needs.
template <int n, bool PAR, class Emit>
__device__ __forceinline__ void jt_lockstep(int &N, int &status, double (&p)[11], double &xx, double &yy, int &steps,
                                            int budget, volatile int *stop, Emit &emit) {
    if (status == 0 && N == n) {
        const int r = jt_search<n, PAR>(p, xx, yy, steps, budget, stop, emit);
        if (r == -1) status = -1;
        else if (r == -2) status = 2;
        else N = r;
    }
    if constexpr (n > 3) jt_lockstep<n - 1, PAR>(N, status, p, xx, yy, steps, budget, stop, emit);
}

// rpoly_ak1 (rpoly.cpp:7-230) on a[0..10] (ascending powers; a[10] != 0 and every a finite, the caller
// checks): the real zeros in the order found, to roots[r * stride] (PAR: written by lane 0).  Returns
// their number, or -1 when more than `budget` fixed-shift steps would be needed (not PAR: the caller
// defers the polynomial and the roots written so far are rewritten).  stop: an LDS word (PAR only).
// take(zr) sees each real zero as it is found (PAR: on every lane, uniformly) and returns true when
// the caller needs no further zero: the search ends there (the caller's choice is made; the count
// returned is the zeros seen so far).
struct JtTakeAll {
    __device__ bool operator()(double) const { return false; }
};

template <bool PAR, class Take = JtTakeAll>
__device__ __forceinline__ int jt_rpoly10(const double (&a)[11], double *roots, size_t stride, int budget,
                                          volatile int *stop, Take take = Take()) {
    int nr = 0, status = 0;  // status 3: take() is satisfied
    const bool writer = !PAR || (threadIdx.x & 63) == 0;
    auto emit = [&](double zr, double zi) {
        if (zi == 0.0 && status != 3) {
            if (writer) roots[(size_t)nr * stride] = zr;
            nr++;
            if (take(zr)) status = 3;
        }
    };
    int z = 0;  // zeros at the origin (rpoly.cpp:36-42)
#pragma unroll
    for (int k = 0; k < 10; k++)
        if (z == k && a[k] == 0.0) z++;
    for (int k = 0; k < z; k++) emit(0.0, 0.0);
    double p[11];
#pragma unroll
    for (int i = 0; i < 11; i++) p[i] = a[10 - i];
    double xx = sqrt(0.5), yy = -xx;
    int N = 10 - z, steps = 0;
    jt_lockstep<10, PAR>(N, status, p, xx, yy, steps, budget, stop, emit);
    if (status == -1) return -1;
    if (status == 2 || status == 3) return nr;
    if (N == 2) {
        double sr, si, lr, li;
        jt_quadratic(p[0], p[1], p[2], sr, si, lr, li);
        emit(sr, si);
        emit(lr, li);
    } else if (N == 1) {
        emit(-(p[1] / p[0]), 0.0);
    }
    return nr;
}

}  // namespace e5
}  // namespace usac
