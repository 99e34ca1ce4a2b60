// jt_bench2.hip -- per-unit latency of one zero search at degree 10 (e5::jt_search<10>), all lanes on the
// same polynomial, repeated R times: the cost of the code path of one degree alone (I-cache footprint
// of one instantiation) against jt_bench's whole-polynomial dispatch.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../../ransac_amd/csrc/usac_rpoly.hpp"

__global__ __launch_bounds__(64) void k_one(const double *polys, int R, double *out) {
    double a[11];
    for (int k = 0; k < 11; k++) a[k] = polys[k];
    double acc = 0.0;
    int steps = 0;
    for (int r = 0; r < R; r++) {
        double p[11];
#pragma unroll
        for (int i = 0; i < 11; i++) p[i] = a[10 - i] * (1.0 + r * 1e-300);
        double xx = sqrt(0.5), yy = -xx;
        double z = 0.0;
        auto emit = [&](double zr, double zi) { z += zr + zi; };
        const int n = usac::e5::jt_search<10, false>(p, xx, yy, steps, 0x7fffffff, nullptr, emit);
        acc += z + n;
    }
    out[blockIdx.x * 64 + threadIdx.x] = acc + steps;
}

int main() {
    FILE *f = fopen("tools/ubench/polys.bin", "rb");
    if (!f) return 2;
    std::vector<double> P(8192 * 11);
    if (fread(P.data(), 8, P.size(), f) != P.size()) return 2;
    fclose(f);
    double *d_p, *d_o;
    (void)hipMalloc(&d_p, 8 * P.size());
    (void)hipMemcpy(d_p, P.data(), 8 * P.size(), hipMemcpyHostToDevice);
    (void)hipMalloc(&d_o, 8 * 65536);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int R : {1, 10}) {
        hipLaunchKernelGGL(k_one, dim3(1024), dim3(64), 0, nullptr, d_p, R, d_o);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_one, dim3(1024), dim3(64), 0, nullptr, d_p, R, d_o);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("one search at N = 10, polynomial 0, R = %d: %.3f ms\n", R, ms);
    }
    return 0;
}
