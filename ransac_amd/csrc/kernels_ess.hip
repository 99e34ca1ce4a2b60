// kernels_ess.hip -- the essential 5-point solver (five_points.cpp:13-274) as a staged
// pipeline.  The per-sample arithmetic is exactly the one-lane spec of usac_device_e5.hpp /
// the oracle (same operations in the same order), only distributed over more lanes:
//
//   k_e5_basis   lane / sample          : 5 x 9 rows -> Jacobi -> 4-vector null basis N
//   k_e5_dets    lane / (node, sample)  : det M(z_k), z_k = -5..5 (11x the lanes)
//   k_e5_roots   lane / sample          : Newton divided differences -> degree-10 coefficients
//                                         -> real roots; (sample, root) pairs appended to a list
//   k_e5_check   lane / listed pair     : null vector of M(z), E, cheirality over the sample
//   k_e5_select  lane / sample          : the first passing root (root order) -> the model;
//                                         counts 0 / -1, occupied-slot list (as k_solve_f7)
//
// Workspace (e5_workspace_bytes(B)): samples int32[5][B], N double[36][B], dets double[11][B],
// roots double[10][B], nroots int32[B], pair list uint32[10B] + counter, candidate E
// float[9][10B], flags int32[10B].
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_device_e5.hpp"
#include "usac_kernels.h"

namespace usac {

struct E5Work {
    int32_t *smp;
    double *N, *det, *roots;
    int32_t *nroots;
    uint32_t *pairs, *npairs;
    float *cand;
    int32_t *flags;
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
    w.flags = reinterpret_cast<int32_t *>(p + off);
    return w;
}

size_t e5_workspace_bytes(uint32_t B) {
    return e5_align(sizeof(int32_t) * 5 * (size_t)B) + e5_align(sizeof(double) * 36 * (size_t)B) +
           e5_align(sizeof(double) * 11 * (size_t)B) + e5_align(sizeof(double) * 10 * (size_t)B) +
           e5_align(sizeof(int32_t) * (size_t)B) + e5_align(sizeof(uint32_t) * 10 * (size_t)B) +
           e5_align(sizeof(uint32_t)) + e5_align(sizeof(float) * 90 * (size_t)B) +
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

__global__ __launch_bounds__(64) void k_e5_roots(uint32_t B, E5Work w) {
    __shared__ double s_lvl[22 * 64];  // root-isolation level arrays (e5::RootsLds), 11 KB
    const uint32_t lane = threadIdx.x;
    const uint32_t h = blockIdx.x * 64 + lane;
    int nr = 0;
    if (h < B) {
        double c[11];
#pragma unroll
        for (int k = 0; k < 11; k++) c[k] = w.det[(size_t)k * B + h];
        // Newton divided differences over the nodes z_k = k - 5, then the monomial form
#pragma unroll
        for (int j = 1; j < 11; j++)
#pragma unroll
            for (int i = 10; i >= j; i--) c[i] = (c[i] - c[i - 1]) / ((double)(i - 5) - (double)(i - j - 5));
        double a[11];
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
#pragma unroll
        for (int r = 0; r < 10; r++) w.flags[(size_t)r * B + h] = 0;
        if (a[10] != 0.0) {
            const e5::RootsLds L{s_lvl + lane, s_lvl + 11 * 64 + lane};
            uint32_t found;
            e5::real_roots10(a, L, found);
#pragma unroll
            for (int k = 0; k < 10; k++)
                if (found & (1u << k)) {
                    w.roots[(size_t)nr * B + h] = L.E[64 * k];
                    nr++;
                }
        } else {
            double roots[10];
            nr = e5::real_roots_dyn(a, roots);
            for (int r = 0; r < nr; r++) w.roots[(size_t)r * B + h] = roots[r];
        }
        w.nroots[h] = nr;
    }
    // append (root, sample) pairs, wave-aggregated
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

__global__ __launch_bounds__(64) void k_e5_check(const float4 *__restrict__ pts, uint32_t B, uint32_t maxpairs,
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
    if (!e5::null10(M, v)) return;
    const double x = v[7], y = v[8];
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
    int nvalid = 0;
    if (h < B) {
        const int nr = w.nroots[h];
        for (int r = 0; r < nr && !nvalid; r++) {
            const size_t rb = (size_t)r * B + h;
            if (w.flags[rb]) {
#pragma unroll
                for (int k = 0; k < 9; k++) models[(size_t)k * B + h] = w.cand[(size_t)k * 10 * B + rb];
                nvalid = 1;
            }
        }
        counts[h] = nvalid ? 0 : -1;
    }
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
    if (nvalid) list[base + incl - 1] = h;
}

hipError_t launch_solve_e5(hipStream_t st, const float4 *pts, uint32_t n, const int32_t *samples_in,
                           int32_t *samples_out, uint32_t B, DevSampler ds, uint64_t first_hyp, float *models,
                           int32_t *counts, uint32_t *list, uint32_t *list_n, void *workspace) {
    const E5Work w = e5_carve(workspace, B);
    hipError_t e = hipMemsetAsync(list_n, 0, sizeof(uint32_t), st);
    if (e == hipSuccess) e = hipMemsetAsync(w.npairs, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    const dim3 g1((B + 63) / 64), g11((11 * B + 63) / 64), g10((10 * B + 63) / 64);
    hipLaunchKernelGGL(k_e5_basis, g1, dim3(64), 0, st, pts, n, samples_in, samples_out, B, ds, first_hyp, w);
    hipLaunchKernelGGL(k_e5_dets, g11, dim3(64), 0, st, B, w);
    hipLaunchKernelGGL(k_e5_roots, g1, dim3(64), 0, st, B, w);
    hipLaunchKernelGGL(k_e5_check, g10, dim3(64), 0, st, pts, B, 10 * B, w);
    hipLaunchKernelGGL(k_e5_select, g1, dim3(64), 0, st, B, w, models, counts, list, list_n);
    return hipGetLastError();
}

}  // namespace usac
