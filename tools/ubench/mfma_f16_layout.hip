// mfma_f16_layout.hip -- checks, with exact small-integer data, the lane maps of
// v_mfma_f32_32x32x16_f16 that kernels_h16.hip relies on (cdna_hip_programming.md states them for
// bf16 and asks for a check per dtype):
//   A: lane l holds A[row l&31][k = 8 (l>>5) + j], j = 0..7
//   B: lane l holds B[k = 8 (l>>5) + j][col l&31]
//   D: lane l, register r holds D[row (r&3) + 8 (r>>2) + 4 (l>>5)][col l&31]
// and times a back-to-back chain of the instruction on one wave per SIMD (cycles per MFMA).
// Build: hipcc --offload-arch=gfx950 -O2 mfma_f16_layout.hip -o mfma_f16_layout
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_layout(const float *A, const float *B, float *D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    half8 a, b;
    for (int j = 0; j < 8; j++) {
        a[j] = (_Float16)A[r * 16 + 8 * h + j];
        b[j] = (_Float16)B[(8 * h + j) * 32 + r];
    }
    f32x16 acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    for (int q = 0; q < 16; q++) D[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = acc[q];
}

__global__ void k_rate(float *out, int iters, long long *cyc) {
    half8 a, b;
    for (int j = 0; j < 8; j++) {
        a[j] = (_Float16)(threadIdx.x * 0.001f + j);
        b[j] = (_Float16)(j * 0.5f);
    }
    f32x16 acc0 = {}, acc1 = {};
    const long long t0 = clock64();
    for (int i = 0; i < iters; i++) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc1, 0, 0, 0);
    }
    const long long t1 = clock64();
    float s = 0.f;
    for (int q = 0; q < 16; q++) s += acc0[q] + acc1[q];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    float hA[32 * 16], hB[16 * 32], hD[32 * 32], ref[32 * 32];
    for (int i = 0; i < 32; i++)
        for (int k = 0; k < 16; k++) hA[i * 16 + k] = (float)((i * 7 + k * 3) % 23 - 11);
    for (int k = 0; k < 16; k++)
        for (int j = 0; j < 32; j++) hB[k * 32 + j] = (float)((k * 5 + j * 11) % 19 - 9);
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++) {
            float s = 0.f;
            for (int k = 0; k < 16; k++) s += hA[i * 16 + k] * hB[k * 32 + j];
            ref[i * 32 + j] = s;
        }
    float *dA, *dB, *dD, *dO;
    long long *dc, cyc = 0;
    hipMalloc(&dA, sizeof(hA));
    hipMalloc(&dB, sizeof(hB));
    hipMalloc(&dD, sizeof(hD));
    hipMalloc(&dO, sizeof(float) * 64 * 1024);
    hipMalloc(&dc, sizeof(long long));
    hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32 * 32; i++) bad += hD[i] != ref[i];
    printf("{\"layout_mismatches\": %d", bad);
    const int iters = 4096;
    hipLaunchKernelGGL(k_rate, dim3(1024), dim3(64), 0, 0, dO, iters, dc);
    hipDeviceSynchronize();
    hipMemcpy(&cyc, dc, sizeof(cyc), hipMemcpyDeviceToHost);
    printf(", \"cycles_per_mfma_one_wave\": %.2f}\n", (double)cyc / (2.0 * iters));
    return bad != 0;
}
