// Issue-cost calibration for the roofline bookkeeping: throughput of independent plain fp32
// FMAs, packed fp32 FMAs (v_pk_fma_f32), fp64 FMAs, fp64 divisions' building blocks and a
// v_cndmask stream, at 1, 2, 4 and 8 waves per SIMD on every CU.  Reports SIMD-cycles per
// wave-instruction at the nominal 2.4 GHz (wall time; DVFS lowers the clock under load, so the
// ratios between rows are the result, not the absolute values).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/valu_issue_bench.hip -o /tmp/vib && /tmp/vib > profiles/r4/valu_issue_costs.json
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float v2f __attribute__((ext_vector_type(2)));

constexpr int kIters = 32768;

__global__ void k_plain(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(x), "v"(y));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_packed(float *out, float x, float y) {
    v2f a[4];
#pragma unroll
    for (int i = 0; i < 4; i++) a[i] = v2f{(float)threadIdx.x + i, (float)threadIdx.x - i};
    const v2f X{x, x}, Y{y, y};
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 4; i++) __asm__ volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(X), "v"(Y));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; i++) s += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_f64(float *out, float x, float y) {
    double a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const double X = x, Y = y;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(X), "v"(Y));
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
}

// 4 packed + 4 plain per trip, interleaved (do the two kinds' costs add?)
__global__ void k_mix(float *out, float x, float y) {
    v2f a[4];
    float b[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        a[i] = v2f{(float)threadIdx.x + i, (float)threadIdx.x - i};
        b[i] = threadIdx.x * 0.5f + i;
    }
    const v2f X{x, x}, Y{y, y};
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            __asm__ volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(X), "v"(Y));
            __asm__ volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(b[i]) : "v"(x), "v"(y));
        }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; i++) s += a[i].x + a[i].y + b[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_cndmask_b32 stream (the select of register-array pivoting)
__global__ void k_select(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + x + y;
}

__global__ void k_select64(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x;
    unsigned long long m;
    __asm__ volatile("v_cmp_gt_f32 %0, %1, %2" : "=s"(m) : "v"(a[0]), "v"(b));
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(m));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + x + y;
}

__global__ void k_rcp(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i + 1.0f;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_rcp_f32 %0, %0" : "+v"(a[i]));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + x + y;
}

__global__ void k_rcp64(float *out, float x, float y) {
    double a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i + 1.0;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_rcp_f64 %0, %0" : "+v"(a[i]));
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s + x + y;
}

// v_pk_fma_f32 with a wave-uniform SGPR-pair operand (the cfg2 stage-A form)
__global__ void k_packed_s(float *out, float x, float y) {
    v2f a[4];
#pragma unroll
    for (int i = 0; i < 4; i++) a[i] = v2f{(float)threadIdx.x + i, (float)threadIdx.x - i};
    const v2f Y{y, y};
    const uint64_t xs = *reinterpret_cast<const uint64_t *>(out);  // uniform address: a scalar load
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 4; i++) __asm__ volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "s"(xs), "v"(Y));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; i++) s += a[i].x + a[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_plain_s(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float yv = y * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "s"(x), "v"(yv));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_cmp_*_e64 writing an SGPR pair (the stage-A keep test)
__global__ void k_cmp(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x;
    for (int it = 0; it < kIters; it++) {
        unsigned long long m[8];
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_cmp_ngt_f32_e64 %0, %1, %2" : "=s"(m[i]) : "v"(a[i]), "v"(b));
        __asm__ volatile("" ::"s"(m[0]), "s"(m[1]), "s"(m[2]), "s"(m[3]), "s"(m[4]), "s"(m[5]), "s"(m[6]), "s"(m[7]));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a[0] + y;
}

// v_max_f32_e64 with |.| modifiers
__global__ void k_maxabs(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_max_f32_e64 %0, |%0|, |%1|" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op0(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op1(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op2(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_max_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op3(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_and_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op4(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_fma_f32 %0, |%0|, %1, %1" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op5(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_fmac_f32 %0, %1, %1" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op6(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_mov_b32 %0, %1" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op7(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op8(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_max3_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

__global__ void k_op9(float *out, float x, float y) {
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x + i;
    const float b = x * threadIdx.x;
    for (int it = 0; it < kIters; it++)
#pragma unroll
        for (int i = 0; i < 8; i++) __asm__ volatile("v_sub_f32 %0, %1, %0" : "+v"(a[i]) : "v"(b));
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + y;
}

#define CK(e)                                                                      \
    do {                                                                           \
        hipError_t r_ = (e);                                                       \
        if (r_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(r_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

template <typename K>
double run(K kern, int waves_per_simd, int cus, float *out) {
    // one workgroup of 4 x waves_per_simd waves per CU (the 4 SIMDs of the CU)
    const dim3 grid(cus), block(256 * waves_per_simd > 1024 ? 1024 : 256 * waves_per_simd);
    const int reps = 256 * waves_per_simd > 1024 ? (256 * waves_per_simd) / 1024 : 1;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(kern, dim3(grid.x * reps), block, 0, 0, out, 1.0000001f, 1e-7f);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(grid.x * reps), block, 0, 0, out, 1.0000001f, 1e-7f);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / 5;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    float *out;
    CK(hipMalloc(&out, sizeof(float) * (size_t)cus * 8 * 1024));
    struct Row {
        const char *name;
        void (*k)(float *, float, float);
        int instr_per_iter;  // wave-instructions per loop trip
    } rows[] = {{"v_fma_f32", k_plain, 8}, {"v_pk_fma_f32", k_packed, 4}, {"v_fma_f64", k_f64, 8}, {"pk+plain 1:1", k_mix, 8},
                {"v_cndmask_b32 (vcc)", k_select, 8},
                {"v_cndmask_b32_e64 (sgpr pair)", k_select64, 8}, {"v_rcp_f32", k_rcp, 8}, {"v_rcp_f64", k_rcp64, 8},
                {"v_pk_fma_f32 (sgpr pair src)", k_packed_s, 4}, {"v_fma_f32 (sgpr src)", k_plain_s, 8},
                {"v_cmp_ngt_f32_e64 (sgpr dst)", k_cmp, 8}, {"v_max_f32_e64 |a|,|b|", k_maxabs, 8},
                {"v_add_f32", k_op0, 8}, {"v_mul_f32", k_op1, 8}, {"v_max_f32 (vop2)", k_op2, 8}, {"v_and_b32", k_op3, 8}, {"v_fma_f32 |a|", k_op4, 8}, {"v_fmac_f32", k_op5, 8}, {"v_mov_b32", k_op6, 8}, {"v_add_u32", k_op7, 8}, {"v_max3_f32", k_op8, 8}, {"v_sub_f32", k_op9, 8}};
    printf("{\"cus\": %d, \"clock_nominal_ghz\": 2.4, \"rows\": [\n", cus);
    bool first = true;
    for (const Row &r : rows)
        for (int w : {1, 2, 4, 8}) {
            const double ms = run(r.k, w, cus, out);
            const double wave_instr_per_simd = (double)w * kIters * r.instr_per_iter;
            const double cyc = ms * 1e-3 * 2.4e9 / wave_instr_per_simd;
            printf("%s {\"instr\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"simd_cycles_per_wave_instr\": %.3f}",
                   first ? "" : ",\n", r.name, w, ms, cyc);
            first = false;
        }
    printf("\n]}\n");
    CK(hipFree(out));
    return 0;
}
