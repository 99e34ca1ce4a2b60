// jt_bench.hip -- latency / divergence of the device root step (usac_rpoly.hpp) on the 5-point
// solver's polynomials (tools/ubench/polys.bin, gen_polys.py): per variant the kernel time over
// 65 536 polynomials (8192 distinct, repeated), one per lane, 64-lane workgroups.
//   uniform  : every lane of the launch on polynomial 0 (no divergence: the latency of one)
//   real     : the real polynomials, no budget
//   budget   : the real polynomials, budget 128 fixed-shift steps (the k_e5_roots schedule)
//   par      : one polynomial per wave, 20 attempts on lanes 0..19 (the tail schedule), 1024 of them
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../../ransac_amd/csrc/usac_rpoly.hpp"

__global__ __launch_bounds__(64) void k_jt(const double *polys, uint32_t npoly, uint32_t B, int mode, int budget,
                                           double *roots, int *nr_out) {
    __shared__ int s_stop;
    const uint32_t lane = threadIdx.x, h = blockIdx.x * 64 + lane;
    if (mode == 3) {  // par: polynomial blockIdx.x
        double a[11];
        const uint32_t pi = blockIdx.x % npoly;
        for (int k = 0; k < 11; k++) a[k] = polys[11 * pi + k];
        const int nr = usac::e5::jt_rpoly10<true>(a, roots + blockIdx.x, B, 0x7fffffff, &s_stop);
        if (lane == 0) nr_out[blockIdx.x] = nr;
        return;
    }
    if (h >= B) return;
    const uint32_t pi = mode == 0 ? 0 : h % npoly;
    double a[11];
    for (int k = 0; k < 11; k++) a[k] = polys[11 * pi + k];
    nr_out[h] = usac::e5::jt_rpoly10<false>(a, roots + h, B, mode == 2 ? budget : 0x7fffffff, nullptr);
}

int main() {
    FILE *f = fopen("tools/ubench/polys.bin", "rb");
    if (!f) return 2;
    std::vector<double> P(8192 * 11);
    if (fread(P.data(), 8, P.size(), f) != P.size()) return 2;
    fclose(f);
    const uint32_t B = 65536;
    double *d_p, *d_r;
    int *d_n;
    hipMalloc(&d_p, 8 * P.size());
    hipMemcpy(d_p, P.data(), 8 * P.size(), hipMemcpyHostToDevice);
    hipMalloc(&d_r, 8 * 10 * (size_t)B);
    hipMalloc(&d_n, 4 * (size_t)B);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[4] = {"uniform", "real", "budget", "par x1024"};
    const int budgets[] = {64, 128, 192, 320};
    for (int mi = 0; mi < 7; mi++) {
        const int mode = mi < 2 ? mi : (mi < 6 ? 2 : 3);
        const int budget = mi >= 2 && mi < 6 ? budgets[mi - 2] : 128;
        const dim3 grid = mode == 3 ? dim3(1024) : dim3(B / 64);
        hipLaunchKernelGGL(k_jt, grid, dim3(64), 0, nullptr, d_p, 8192u, B, mode, budget, d_r, d_n);
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_jt, grid, dim3(64), 0, nullptr, d_p, 8192u, B, mode, budget, d_r, d_n);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        std::vector<int> n(B);
        hipMemcpy(n.data(), d_n, 4 * (size_t)B, hipMemcpyDeviceToHost);
        long def = 0;
        for (uint32_t i = 0; i < (mode == 3 ? 1024u : B); i++) def += n[i] < 0;
        printf("%-10s %4d %8.3f ms  (deferred %ld)\n", names[mode], budget, best, def);
    }
    return 0;
}
