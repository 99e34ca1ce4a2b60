// kernels_ess.hip -- the essential 5-point solver (five_points.cpp:13-274) as a staged
// pipeline.  The per-sample arithmetic is exactly the one-lane spec of usac_device_e5.hpp /
// the oracle (same operations in the same order), only distributed over more lanes:
//
//   k_e5_basis   lane / sample          : 5 x 9 rows -> Jacobi -> 4-vector null basis N
//   k_e5_dets    lane / (node, sample)  : det M(z_k), z_k = -5..5 (11x the lanes)
//   k_e5_roots   lane / sample          : Newton divided differences -> degree-10 coefficients
//                                         -> the candidate values (real roots, ascending);
//                                         (sample, root) pairs appended to a list
//   k_e5_null    lane / listed pair     : null vector of M(z) (x, y)
//   k_e5_check   lane / listed pair     : E, cheirality over the sample
//   k_e5_select  lane / sample          : 0 passing candidates: count -1; 1: that model; >= 2: the
//                                         sample is listed for k_e5_order; counts 0 / -1 and the
//                                         occupied-slot list (as k_solve_f7)
//   k_e5_order   lane / listed sample   : the reference's candidate order -- rpoly's real zeros in the
//                                         order it finds them (usac_rpoly.hpp) -- under a work budget,
//                                         until a zero's nearest candidate passed -> the model
//   k_e5_order_tail  wave / deferred    : the same without a budget, rpoly's 20 shift attempts of a
//                                         search side by side (samples over k_e5_order's budget)
//
// The order matters only when several candidates pass cheirality (five_points.cpp:239-273 keeps the
// first in rpoly's order): ~10 % of cfg4's samples.  rpoly is iterative and branchy -- a wave waits
// for its slowest lane, and its work has a long tail (a 20-shift failure is ~20 000 K divisions) --
// so it runs for those samples only.
//
// Workspace (e5_workspace_bytes(B)): samples int32[5][B], N double[36][B], dets double[11][B],
// roots double[10][B], nroots int32[B], pair list uint32[10B] + counter, candidate E
// float[9][10B], flags int32[10B], order list uint32[B] + counter, deferred list uint32[B] +
// counter, rpoly zeros double[10][B], their numbers int32[B], the pairs' null vectors double[2][10B]
// and found flags int32[10B].
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_device_e5.hpp"
#include "usac_rpoly.hpp"
#include "usac_kernels.h"

#include <stdlib.h>

#include <algorithm>

namespace usac {

struct E5Work {
    int32_t *smp;
    double *N, *det, *roots;
    int32_t *nroots;
    uint32_t *pairs, *npairs;
    float *cand;
    int32_t *flags;
    uint32_t *multi, *nmulti;  // samples with several passing candidates (k_e5_order)
    uint32_t *defer, *ndefer;  // ... over k_e5_order's budget (k_e5_order_tail)
    double *jt;                // rpoly's real zeros of the listed samples, [r B + h]
    int32_t *njt;              // their numbers
    double *xy;                // per listed pair: the null vector's x, y ([i], [10 B + i]; k_e5_null)
    int32_t *xyok;             // ... found (null10)
};

__host__ __device__ inline size_t e5_align(size_t x) { return (x + 255) & ~(size_t)255; }

__host__ __device__ inline E5Work e5_carve(void *base, uint32_t B) {
    char *p = static_cast<char *>(base);
    E5Work w;
    size_t off = 0;
    w.smp = reinterpret_cast<int32_t *>(p + off); off += e5_align(sizeof(int32_t) * 5 * (size_t)B);
    w.N = reinterpret_cast<double *>(p + off); off += e5_align(sizeof(double) * 36 * (size_t)B);
    w.det = reinterpret_cast<double *>(p + off); off += e5_align(sizeof(double) * 11 * (size_t)B);
    w.roots = reinterpret_cast<double *>(p + off); off += e5_align(sizeof(double) * 10 * (size_t)B);
    w.nroots = reinterpret_cast<int32_t *>(p + off); off += e5_align(sizeof(int32_t) * (size_t)B);
    w.pairs = reinterpret_cast<uint32_t *>(p + off); off += e5_align(sizeof(uint32_t) * 10 * (size_t)B);
    w.npairs = reinterpret_cast<uint32_t *>(p + off); off += e5_align(sizeof(uint32_t));
    w.cand = reinterpret_cast<float *>(p + off); off += e5_align(sizeof(float) * 90 * (size_t)B);
    w.flags = reinterpret_cast<int32_t *>(p + off); off += e5_align(sizeof(int32_t) * 10 * (size_t)B);
    w.multi = reinterpret_cast<uint32_t *>(p + off); off += e5_align(sizeof(uint32_t) * (size_t)B);
    w.nmulti = reinterpret_cast<uint32_t *>(p + off); off += e5_align(sizeof(uint32_t));
    w.defer = reinterpret_cast<uint32_t *>(p + off); off += e5_align(sizeof(uint32_t) * (size_t)B);
    w.ndefer = reinterpret_cast<uint32_t *>(p + off); off += e5_align(sizeof(uint32_t));
    w.jt = reinterpret_cast<double *>(p + off); off += e5_align(sizeof(double) * 10 * (size_t)B);
    w.njt = reinterpret_cast<int32_t *>(p + off); off += e5_align(sizeof(int32_t) * (size_t)B);
    w.xy = reinterpret_cast<double *>(p + off); off += e5_align(sizeof(double) * 20 * (size_t)B);
    w.xyok = reinterpret_cast<int32_t *>(p + off);
    return w;
}

size_t e5_workspace_bytes(uint32_t B) {
    return e5_align(sizeof(int32_t) * 5 * (size_t)B) + e5_align(sizeof(double) * 36 * (size_t)B) +
           e5_align(sizeof(double) * 11 * (size_t)B) + e5_align(sizeof(double) * 10 * (size_t)B) +
           e5_align(sizeof(int32_t) * (size_t)B) + e5_align(sizeof(uint32_t) * 10 * (size_t)B) +
           e5_align(sizeof(uint32_t)) + e5_align(sizeof(float) * 90 * (size_t)B) +
           e5_align(sizeof(int32_t) * 10 * (size_t)B) + 2 * (e5_align(sizeof(uint32_t) * (size_t)B) +
           e5_align(sizeof(uint32_t))) + e5_align(sizeof(double) * 10 * (size_t)B) +
           e5_align(sizeof(int32_t) * (size_t)B) + e5_align(sizeof(double) * 20 * (size_t)B) +
           e5_align(sizeof(int32_t) * 10 * (size_t)B);
}

__global__ __launch_bounds__(64) void k_e5_basis(const float4 *__restrict__ pts, uint32_t n,
                                                 const int32_t *__restrict__ samples_in, int32_t *samples_out,
                                                 uint32_t B, DevSampler ds, uint64_t first_hyp, E5Work w) {
    const uint32_t h = blockIdx.x * 64 + threadIdx.x;
    if (h >= B) return;
    int32_t s[5];
    if (samples_in) {
#pragma unroll
        for (int i = 0; i < 5; i++) s[i] = samples_in[5 * (size_t)h + i];
    } else {
        draw_sample<5>(ds, first_hyp + h, n, s);
        if (samples_out) {
#pragma unroll
            for (int i = 0; i < 5; i++) samples_out[5 * (size_t)h + i] = s[i];
        }
    }
#pragma unroll
    for (int i = 0; i < 5; i++) w.smp[(size_t)i * B + h] = s[i];
    double W[5][9], N[4][9];
#pragma unroll
    for (int i = 0; i < 5; i++) {
        const float4 p = pts[s[i]];
        const double x1 = p.x, y1 = p.y, x2 = p.z, y2 = p.w;
        W[i][0] = x1 * x2; W[i][1] = x2 * y1; W[i][2] = x2;
        W[i][3] = x1 * y2; W[i][4] = y1 * y2; W[i][5] = y2;
        W[i][6] = x1; W[i][7] = y1; W[i][8] = 1.0;
    }
    if (!qr_null<5>(W, N)) {  // a zero / non-finite column: the row-Jacobi completion
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const float4 p = pts[s[i]];
            const double x1 = p.x, y1 = p.y, x2 = p.z, y2 = p.w;
            W[i][0] = x1 * x2; W[i][1] = x2 * y1; W[i][2] = x2;
            W[i][3] = x1 * y2; W[i][4] = y1 * y2; W[i][5] = y2;
            W[i][6] = x1; W[i][7] = y1; W[i][8] = 1.0;
        }
        row_jacobi<5>(W);
        e5::null_basis4(W, N);
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int k = 0; k < 9; k++) w.N[(size_t)(9 * j + k) * B + h] = N[j][k];
}

__device__ __forceinline__ void e5_load_basis(const E5Work &w, uint32_t B, uint32_t h, double (&N)[4][9]) {
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
        for (int k = 0; k < 9; k++) N[j][k] = w.N[(size_t)(9 * j + k) * B + h];
}

// Two waves per SIMD (the 10x10 fp64 matrix alone is 200 VGPRs): ~60 VGPRs spill to
// scratch, but the second wave hides the latency of the 45 dependent fp64 divisions --
// measured 1.9x faster than the spill-free single-wave build.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_e5_dets(uint32_t B, E5Work w) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= 11 * B) return;
    const uint32_t k = i / B, h = i - k * B;
    double N[4][9], M[10][10];
    e5_load_basis(w, B, h, N);
    e5::matrix(N, (double)((int)k - 5), M);
    w.det[(size_t)k * B + h] = e5::det10(M);
}

// degree-10 coefficients of det M(z) (ascending) from its values at z_k = k - 5: Newton divided
// differences, then the monomial form (five_points.cpp:113-136 interpolates at the same nodes)
__device__ __forceinline__ void e5_coeffs(const E5Work &w, uint32_t B, uint32_t h, double (&a)[11]) {
    double c[11];
#pragma unroll
    for (int k = 0; k < 11; k++) c[k] = w.det[(size_t)k * B + h];
#pragma unroll
    for (int j = 1; j < 11; j++)
#pragma unroll
        for (int i = 10; i >= j; i--) c[i] = (c[i] - c[i - 1]) / ((double)(i - 5) - (double)(i - j - 5));
#pragma unroll
    for (int i = 0; i < 11; i++) a[i] = 0.0;
    a[0] = c[10];
#pragma unroll
    for (int k = 9; k >= 0; k--) {
        const int deg = 9 - k;
        const double zk = (double)(k - 5);
        a[deg + 1] = 0.0;
#pragma unroll
        for (int i = deg + 1; i >= 1; i--) a[i] = a[i - 1] - zk * a[i];
        a[0] = c[k] - zk * a[0];
    }
}

// rpoly: a zero leading coefficient reports no zeros (rpoly.cpp:224-227); non-finite coefficients
// none either (its bounded loops all fail on NaN)
__device__ __forceinline__ bool e5_coeffs_ok(const double (&a)[11]) {
    bool fin = a[10] != 0.0;
#pragma unroll
    for (int i = 0; i < 11; i++) fin = fin && isfinite(a[i]);
    return fin;
}

// append (root, sample) pairs of the calling lanes, wave-aggregated (every lane of the wave calls)
__device__ __forceinline__ void e5_append_pairs(const E5Work &w, uint32_t B, uint32_t h, int nr) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t incl = (uint32_t)nr;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += v;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    uint32_t base = 0;
    if (lane == 63 && total) base = atomicAdd(w.npairs, total);
    base = __shfl(base, 63, 64);
    const uint32_t excl = base + incl - (uint32_t)nr;
    for (int r = 0; r < nr; r++) w.pairs[excl + r] = (uint32_t)r * B + h;
}

// coef (nullable): the polynomials given (11 ascending coefficients per sample; the self-test hook)
__device__ __forceinline__ void e5_coeffs_of(const E5Work &w, const double *coef, uint32_t B, uint32_t h,
                                             double (&a)[11]) {
    if (coef) {
#pragma unroll
        for (int k = 0; k < 11; k++) a[k] = coef[11 * (size_t)h + k];
    } else {
        e5_coeffs(w, B, h, a);
    }
}

// the candidate values: real roots ascending (oracle asc_real_roots); no candidates where rpoly
// reports none (e5_coeffs_ok)
__global__ __launch_bounds__(64) void k_e5_roots(uint32_t B, E5Work w) {
    __shared__ double s_lvl[22 * 64];  // root-isolation level arrays (e5::RootsLds), 11 KB
    const uint32_t lane = threadIdx.x;
    const uint32_t h = blockIdx.x * 64 + lane;
    int nr = 0;
    if (h < B) {
        double a[11];
        e5_coeffs(w, B, h, a);
#pragma unroll
        for (int r = 0; r < 10; r++) w.flags[(size_t)r * B + h] = 0;
        if (e5_coeffs_ok(a)) {
            const e5::RootsLds L{s_lvl + lane, s_lvl + 11 * 64 + lane};
            uint32_t found;
            e5::real_roots10(a, L, found);
#pragma unroll
            for (int k = 0; k < 10; k++)
                if (found & (1u << k)) {
                    w.roots[(size_t)nr * B + h] = L.E[64 * k];
                    nr++;
                }
        }
        w.nroots[h] = nr;
    }
    e5_append_pairs(w, B, h, nr);
}

// rpoly's work budget per listed sample in k_e5_order (usac_rpoly.hpp counts K-polynomial divisions:
// 3 per fixed-shift step, 4 per quadratic and 2 per real variable-shift iteration; cfg4: median ~90,
// p99 ~310, a 20-shift failure ~20 000); USAC_E5_BUDGET overrides (A/B)
constexpr int kE5RootBudget = 320;

int e5_budget() {
    static const int b = getenv("USAC_E5_BUDGET") ? atoi(getenv("USAC_E5_BUDGET")) : kE5RootBudget;
    return b;
}

// five_points.cpp:239-273 over rpoly's order (the oracle's essential_5pt_all): rpoly's real zeros in
// the order found, each standing for the candidate value nearest to it (first on ties); the first whose
// candidate passed cheirality is the model -- the search stops there.  Inactive (models == nullptr, the
// self-test hook): every zero.
struct E5Take {
    const E5Work &w;
    uint32_t B, h;
    int nr;
    bool on;
    int pick = -1;
    __device__ bool operator()(double z) {
        if (!on) return false;
        int near = -1;
        double dmin = INFINITY;
        for (int r = 0; r < nr; r++) {
            const double d = fabs(w.roots[(size_t)r * B + h] - z);
            if (d < dmin) {
                dmin = d;
                near = r;
            }
        }
        if (near >= 0 && w.flags[(size_t)near * B + h]) pick = near;
        return pick >= 0;
    }
};

// the model of a listed sample: the picked candidate, else (no zero stood for a passing one) the first
// passing candidate ascending.  models nullable (the self-test hook keeps the zeros' number only).
__device__ __forceinline__ void e5_select_pick(const E5Work &w, uint32_t B, uint32_t h, int nz, int pick,
                                               float *__restrict__ models) {
    w.njt[h] = nz;
    if (!models) return;
    int best = pick;
    for (int r = 0; r < w.nroots[h] && best < 0; r++)
        if (w.flags[(size_t)r * B + h]) best = r;
    const size_t rb = (size_t)best * B + h;
#pragma unroll
    for (int k = 0; k < 9; k++) models[(size_t)k * B + h] = w.cand[(size_t)k * 10 * B + rb];
}

// lane per listed sample (w.multi), rpoly under the budget; over it: deferred to k_e5_order_tail
__global__ __launch_bounds__(64) void k_e5_order(uint32_t B, E5Work w, const double *coef, int budget,
                                                 float *__restrict__ models) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= *w.nmulti) return;
    const uint32_t h = w.multi[i];
    double a[11];
    e5_coeffs_of(w, coef, B, h, a);
    E5Take take{w, B, h, models ? w.nroots[h] : 0, models != nullptr};
    const int nz = e5_coeffs_ok(a) ? e5::jt_rpoly10<false>(a, w.jt + h, B, budget, nullptr, [&](double z) {
        return take(z);
    }) : 0;
    if (nz < 0) {
        w.defer[atomicAdd(w.ndefer, 1u)] = h;
        return;
    }
    e5_select_pick(w, B, h, nz, take.pick, models);
}

// the deferred samples, one per wave: rpoly's 20 shift attempts of each search side by side on lanes
// 0..19 (e5::jt_rpoly10<true>), no budget
__global__ __launch_bounds__(64) void k_e5_order_tail(uint32_t B, E5Work w, const double *coef,
                                                      float *__restrict__ models) {
    __shared__ int s_stop;
    const uint32_t nd = *w.ndefer;
    for (uint32_t d = blockIdx.x; d < nd; d += gridDim.x) {
        const uint32_t h = w.defer[d];
        double a[11];
        e5_coeffs_of(w, coef, B, h, a);
        E5Take take{w, B, h, models ? w.nroots[h] : 0, models != nullptr};
        const int nz = e5::jt_rpoly10<true>(a, w.jt + h, B, 0x7fffffff, &s_stop, [&](double z) { return take(z); });
        if (threadIdx.x == 0) e5_select_pick(w, B, h, nz, take.pick, models);
    }
}

// the candidate's null vector (five_points.cpp:181-190): M(z) and its elimination, the register-
// heavy half of the candidate check, as its own kernel (two waves per SIMD, as k_e5_dets) so that
// k_e5_check -- E, its SVD and the cheirality test -- runs at several waves per SIMD
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_e5_null(uint32_t B,
                                                                                         uint32_t maxpairs,
                                                                                         E5Work w) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    const uint32_t np = *w.npairs;
    if (i >= np || i >= maxpairs) return;
    const uint32_t rb = w.pairs[i];
    const uint32_t r = rb / B, h = rb - r * B;
    double N[4][9];
    e5_load_basis(w, B, h, N);
    const double zz = w.roots[(size_t)r * B + h];
    double M[10][10], v[10];
    e5::matrix(N, zz, M);
    const bool ok = e5::null10(M, v);
    w.xyok[i] = ok ? 1 : 0;
    if (ok) {
        w.xy[i] = v[7];
        w.xy[(size_t)10 * B + i] = v[8];
    }
}

__global__ __launch_bounds__(64) void k_e5_check(const float4 *__restrict__ pts, uint32_t B, uint32_t maxpairs,
                                                 E5Work w) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    const uint32_t np = *w.npairs;
    if (i >= np || i >= maxpairs) return;
    if (!w.xyok[i]) return;
    const uint32_t rb = w.pairs[i];
    const uint32_t r = rb / B, h = rb - r * B;
    double N[4][9];
    e5_load_basis(w, B, h, N);
    const double zz = w.roots[(size_t)r * B + h];
    const double x = w.xy[i], y = w.xy[(size_t)10 * B + i];
    double E[9];
#pragma unroll
    for (int k = 0; k < 9; k++) E[k] = N[0][k] * x + N[1][k] * y + N[2][k] * zz + N[3][k];
    double U[3][3], V[3][3];
    e5::svd3(E, U, V);
    bool found = false;
    for (int j = 0; j < 4 && !found; j++) {
        double P[3][4];
        e5::projection(U, V, j, P);
        bool all = true;
        for (int k = 0; k < 5 && all; k++) {
            const float4 p = pts[w.smp[(size_t)k * B + h]];
            all = e5::in_front((double)p.x, (double)p.y, (double)p.z, (double)p.w, P);
        }
        found = all;
    }
    if (found) {
#pragma unroll
        for (int k = 0; k < 9; k++) w.cand[(size_t)k * 10 * B + rb] = (float)E[k];
        w.flags[rb] = 1;
    }
}

__global__ __launch_bounds__(64) void k_e5_select(uint32_t B, E5Work w, float *__restrict__ models,
                                                  int32_t *__restrict__ counts, uint32_t *__restrict__ list,
                                                  uint32_t *__restrict__ list_n) {
    const uint32_t lane = threadIdx.x;
    const uint32_t h = blockIdx.x * 64 + lane;
    int npass = 0, first = -1;
    if (h < B) {
        const int nr = w.nroots[h];
        for (int r = 0; r < nr; r++)
            if (w.flags[(size_t)r * B + h]) {
                if (first < 0) first = r;
                npass++;
            }
        if (npass == 1) {
            const size_t rb = (size_t)first * B + h;
#pragma unroll
            for (int k = 0; k < 9; k++) models[(size_t)k * B + h] = w.cand[(size_t)k * 10 * B + rb];
        } else if (npass > 1) {
            w.multi[atomicAdd(w.nmulti, 1u)] = h;  // k_e5_order writes its model
        }
        counts[h] = npass ? 0 : -1;
    }
    const uint32_t nvalid = npass ? 1u : 0u;
    uint32_t incl = nvalid;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += v;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    uint32_t base = 0;
    if (lane == 63 && total) base = atomicAdd(list_n, total);
    base = __shfl(base, 63, 64);
    if (nvalid) list[base + incl - 1] = h;
}

hipError_t launch_solve_e5(hipStream_t st, const float4 *pts, uint32_t n, const int32_t *samples_in,
                           int32_t *samples_out, uint32_t B, DevSampler ds, uint64_t first_hyp, float *models,
                           int32_t *counts, uint32_t *list, uint32_t *list_n, void *workspace, hipStream_t thin,
                           hipEvent_t ev_in, hipEvent_t ev_out) {
    const E5Work w = e5_carve(workspace, B);
    hipError_t e = hipMemsetAsync(list_n, 0, sizeof(uint32_t), st);
    if (e == hipSuccess) e = hipMemsetAsync(w.npairs, 0, sizeof(uint32_t), st);
    if (e == hipSuccess) e = hipMemsetAsync(w.nmulti, 0, sizeof(uint32_t), st);
    if (e == hipSuccess) e = hipMemsetAsync(w.ndefer, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    const dim3 g1((B + 63) / 64), g11((11 * B + 63) / 64), g10((10 * B + 63) / 64);
    hipLaunchKernelGGL(k_e5_basis, g1, dim3(64), 0, st, pts, n, samples_in, samples_out, B, ds, first_hyp, w);
    hipLaunchKernelGGL(k_e5_dets, g11, dim3(64), 0, st, B, w);
    hipLaunchKernelGGL(k_e5_roots, g1, dim3(64), 0, st, B, w);
    hipLaunchKernelGGL(k_e5_null, g10, dim3(64), 0, st, B, 10 * B, w);
    hipLaunchKernelGGL(k_e5_check, g10, dim3(64), 0, st, pts, B, 10 * B, w);
    hipLaunchKernelGGL(k_e5_select, g1, dim3(64), 0, st, B, w, models, counts, list, list_n);
    // the order kernels hold one ~260-register wave per SIMD for hundreds of microseconds: on a CU-masked
    // stream they keep off most of the chip, where the other batches' wide kernels run
    hipStream_t os = st;
    if (thin && ev_in && ev_out) {
        if ((e = hipEventRecord(ev_in, st)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(thin, ev_in, 0)) != hipSuccess) return e;
        os = thin;
    }
    hipLaunchKernelGGL(k_e5_order, g1, dim3(64), 0, os, B, w, nullptr, e5_budget(), models);
    hipLaunchKernelGGL(k_e5_order_tail, dim3(std::min(1024u, (B + 63) / 64)), dim3(64), 0, os, B, w, nullptr, models);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (os != st) {
        if ((e = hipEventRecord(ev_out, os)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(st, ev_out, 0)) != hipSuccess) return e;
    }
    return hipSuccess;
}

// self-test hooks: rpoly's zeros (k_e5_order's schedule: budget, deferral, tail) of given polynomials;
// the root step's log / exp
__global__ __launch_bounds__(64) void k_e5_list_all(uint32_t B, E5Work w) {
    const uint32_t h = blockIdx.x * 64 + threadIdx.x;
    if (h == 0) *w.nmulti = B;
    if (h < B) w.multi[h] = h;
}

__global__ __launch_bounds__(64) void k_e5_njt_copy(uint32_t B, E5Work w, int32_t *nroots) {
    const uint32_t h = blockIdx.x * 64 + threadIdx.x;
    if (h < B) nroots[h] = w.njt[h];
}

hipError_t launch_e5_roots_selftest(hipStream_t st, const double *coef, uint32_t B, double *roots, int32_t *nroots,
                                    void *workspace) {
    const E5Work w = e5_carve(workspace, B);
    hipError_t e = hipMemsetAsync(w.ndefer, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    const dim3 g1((B + 63) / 64);
    hipLaunchKernelGGL(k_e5_list_all, g1, dim3(64), 0, st, B, w);
    hipLaunchKernelGGL(k_e5_order, g1, dim3(64), 0, st, B, w, coef, e5_budget(), nullptr);
    hipLaunchKernelGGL(k_e5_order_tail, dim3(std::min(1024u, (B + 63) / 64)), dim3(64), 0, st, B, w, coef, nullptr);
    hipLaunchKernelGGL(k_e5_njt_copy, g1, dim3(64), 0, st, B, w, nroots);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipMemcpyAsync(roots, w.jt, sizeof(double) * 10 * (size_t)B, hipMemcpyDeviceToDevice, st);
}

__global__ __launch_bounds__(256) void k_jt_logexp(const double *x, uint32_t n, double *lg, double *ex) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    lg[i] = e5::jt_log(x[i]);
    ex[i] = e5::jt_exp(x[i]);
}

hipError_t launch_jt_logexp_selftest(hipStream_t st, const double *x, uint32_t n, double *lg, double *ex) {
    hipLaunchKernelGGL(k_jt_logexp, dim3((n + 255) / 256), dim3(256), 0, st, x, n, lg, ex);
    return hipGetLastError();
}

}  // namespace usac
