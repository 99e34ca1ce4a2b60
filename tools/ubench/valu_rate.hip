// Microbenchmark: wave64 issue rate of v_fma_f32 vs v_pk_fma_f32 on gfx950 (8 independent
// chains per lane, 8 waves per SIMD).  Prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_scalar(float *out, float a, float b) {
    float x[8];
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = __builtin_fmaf(x[i], a, b);
    }
    float s = 0; for (int i = 0; i < 8; i++) s += x[i];
    if (s == 12345.f) out[0] = s;
}
__global__ __launch_bounds__(256) void k_packed(float *out, float a, float b) {
    v2f x[8];
    for (int i = 0; i < 8; i++) x[i] = v2f{threadIdx.x * 0.001f + i, i * 0.5f};
    const v2f A = {a, a}, Bv = {b, b};
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = __builtin_elementwise_fma(x[i], A, Bv);
    }
    float s = 0; for (int i = 0; i < 8; i++) s += x[i].x + x[i].y;
    if (s == 12345.f) out[0] = s;
}
int main() {
    float *d; hipMalloc(&d, 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU -> 8 waves per SIMD
    for (int rep = 0; rep < 2; rep++) {
        for (int kind = 0; kind < 2; kind++) {
            hipEventRecord(e0);
            if (kind == 0) hipLaunchKernelGGL(k_scalar, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 0.001f);
            else hipLaunchKernelGGL(k_packed, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 0.001f);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_simd = (double)blocks * 4 / 1024 * ITERS * 8;  // wave-instr per SIMD
            printf("%s: %.3f ms, %.3f ns per wave-instr per SIMD (%.2f cycles at 2.4 GHz)\n",
                   kind == 0 ? "v_fma_f32   " : "v_pk_fma_f32", ms, ms * 1e6 / instr_per_simd,
                   ms * 1e6 / instr_per_simd * 2.4);
        }
    }
    return 0;
}
