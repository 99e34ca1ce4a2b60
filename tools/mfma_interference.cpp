// mfma_interference.cpp -- which VALU instruction classes return wrong results while another
// kernel's waves run MFMAs on the same device (the round-5/6 recount miscount).
//
// Stream S runs a busy kernel (B0 nothing, B1 v_mfma_f32_32x32x16_f16 on registers, B2 fp64 VALU
// chains, B3 fp32 VALU chains); stream R runs a probe kernel R times, each launch writing its own
// output.  Every probe launch is compared bit for bit with the probe run alone.  Probes (each lane a
// dependent chain of 64 operations on its own inputs):
//   P0 fp32 fma/mul/add    P1 fp32 IEEE division     P2 v_rcp_f32        P3 fp32 correctly
//   rounded sqrtf          P4 v_sqrt_f32 / v_rsq_f32 P5 fp64 fma/mul/add P6 fp64 division
//   P7 fp64 sqrt           P8 f32 <-> f64 conversion P9 integer mul/add/xor
// Output: per (busy, probe) the number of differing launches and lanes, and the lane pattern.
// Build: hipcc -O2 --offload-arch=gfx950 -ffp-contract=off tools/mfma_interference.cpp -o tools/mfma_interference
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                          \
        }                                                                                     \
    } while (0)

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float v2f __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_busy(int kind, int iters, float *out) {
    if (kind == 1) {
        h8 a, b;
        for (int j = 0; j < 8; j++) {
            a[j] = (_Float16)(0.001f * (threadIdx.x + j));
            b[j] = (_Float16)(0.002f * (blockIdx.x + j));
        }
        f16v acc = {};
        for (int i = 0; i < iters; i++) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
        float s = 0.f;
        for (int j = 0; j < 16; j++) s += acc[j];
        if (s == 12345.f) out[blockIdx.x * 256 + threadIdx.x] = s;
    } else if (kind == 2) {
        double x = threadIdx.x * 1e-3, y = blockIdx.x * 1e-3;
        for (int i = 0; i < iters * 8; i++) {
            x = x * 0.999 + y;
            y = y * 1.001 - x * 1e-3;
        }
        if (x == 12345.0) out[blockIdx.x * 256 + threadIdx.x] = (float)(x + y);
    } else if (kind == 3) {
        float x = threadIdx.x * 1e-3f, y = blockIdx.x * 1e-3f;
        for (int i = 0; i < iters * 8; i++) {
            x = x * 0.999f + y;
            y = y * 1.001f - x * 1e-3f;
        }
        if (x == 12345.f) out[blockIdx.x * 256 + threadIdx.x] = x + y;
    }
}

__global__ __launch_bounds__(256) void k_probe(int kind, const float *in, uint32_t *out) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    const float a = in[2 * t], b = in[2 * t + 1];
    uint32_t r = 0;
    switch (kind) {
        case 0: {
            float x = a;
            for (int i = 0; i < 64; i++) x = x * b + a * 0.5f;
            r = __float_as_uint(x);
        } break;
        case 1: {
            float x = a;
            for (int i = 0; i < 64; i++) x = (x + b) / (b + 1.0f);
            r = __float_as_uint(x);
        } break;
        case 2: {
            float x = a;
            for (int i = 0; i < 64; i++) x = __builtin_amdgcn_rcpf(x + b) + 0.5f;
            r = __float_as_uint(x);
        } break;
        case 3: {
            float x = a;
            for (int i = 0; i < 64; i++) x = sqrtf(x * b + 1.0f) + 0.25f;
            r = __float_as_uint(x);
        } break;
        case 4: {
            float x = a;
            for (int i = 0; i < 64; i++) x = __builtin_amdgcn_sqrtf(x + b) + __builtin_amdgcn_rsqf(x + 1.0f);
            r = __float_as_uint(x);
        } break;
        case 5: {
            double x = a, y = b;
            for (int i = 0; i < 64; i++) x = x * y + 0.5 * (double)a;
            const double z = x;
            r = (uint32_t)(__double_as_longlong(z) ^ (__double_as_longlong(z) >> 32));
        } break;
        case 6: {
            double x = a, y = b;
            for (int i = 0; i < 64; i++) x = (x + y) / (y + 1.0);
            r = (uint32_t)(__double_as_longlong(x) ^ (__double_as_longlong(x) >> 32));
        } break;
        case 7: {
            double x = a, y = b;
            for (int i = 0; i < 64; i++) x = sqrt(x * y + 1.0) + 0.25;
            r = (uint32_t)(__double_as_longlong(x) ^ (__double_as_longlong(x) >> 32));
        } break;
        case 8: {
            float x = a;
            for (int i = 0; i < 64; i++) x = (float)((double)x * 1.0000001 + (double)b);
            r = __float_as_uint(x);
        } break;
        case 9: {
            uint32_t x = __float_as_uint(a), y = __float_as_uint(b);
            for (int i = 0; i < 64; i++) x = (x * 2654435761u + y) ^ (x >> 13);
            r = x;
        } break;
        case 10: {  // v_pk_fma_f32
            v2f x = {a, b}, y = {b, a}, z = {0.5f * a, 0.25f * b};
            for (int i = 0; i < 64; i++) x = __builtin_elementwise_fma(x, y, z);
            r = __float_as_uint(x.x) ^ (__float_as_uint(x.y) * 3u);
        } break;
        case 11: {  // v_pk_mul_f32 / v_pk_add_f32 with swizzled halves
            v2f x = {a, b}, y = {b, a};
            for (int i = 0; i < 64; i++) {
                const v2f w = x * y;
                x = v2f{w.y, w.x} + v2f{a, b} - x * 0.5f;
            }
            r = __float_as_uint(x.x) ^ (__float_as_uint(x.y) * 3u);
        } break;
    }
    out[t] = r;
}

int main(int argc, char **argv) {
    const uint32_t lanes = 256 * 1024, R = argc > 1 ? atoi(argv[1]) : 100;
    std::vector<float> in(2 * lanes);
    srand(3);
    for (auto &v : in) v = 0.25f + (float)(rand() % 1000000) * 1e-6f;
    float *d_in, *d_sink;
    uint32_t *d_out, *d_q;
    CK(hipMalloc(&d_in, 8 * (size_t)lanes));
    CK(hipMemcpy(d_in, in.data(), 8 * (size_t)lanes, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_out, 4 * (size_t)lanes * R));
    CK(hipMalloc(&d_q, 4 * (size_t)lanes));
    CK(hipMalloc(&d_sink, 4 * 256 * 4096));
    hipStream_t sR, sS;
    CK(hipStreamCreateWithFlags(&sR, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sS, hipStreamNonBlocking));
    const char *bn[4] = {"none", "mfma", "fp64-valu", "fp32-valu"};
    const char *pn[12] = {"fp32 fma", "fp32 div", "v_rcp_f32", "fp32 sqrtf", "v_sqrt/v_rsq f32", "fp64 fma",
                          "fp64 div", "fp64 sqrt", "cvt f32<->f64", "int", "v_pk_fma_f32", "v_pk_mul/add_f32"};
    int bad_any = 0;
    for (int probe = 0; probe < 12; probe++) {
        hipLaunchKernelGGL(k_probe, dim3(lanes / 256), dim3(256), 0, nullptr, probe, d_in, d_q);
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> q(lanes);
        CK(hipMemcpy(q.data(), d_q, 4 * (size_t)lanes, hipMemcpyDeviceToHost));
        for (int busy = 0; busy < 4; busy++) {
            for (int l = 0; l < 4; l++) hipLaunchKernelGGL(k_busy, dim3(1024), dim3(256), 0, sS, busy, 20000, d_sink);
            for (uint32_t r = 0; r < R; r++)
                hipLaunchKernelGGL(k_probe, dim3(lanes / 256), dim3(256), 0, sR, probe, d_in, d_out + (size_t)lanes * r);
            CK(hipStreamSynchronize(sR));
            CK(hipStreamSynchronize(sS));
            CK(hipGetLastError());
            std::vector<uint32_t> o((size_t)lanes * R);
            CK(hipMemcpy(o.data(), d_out, 4 * (size_t)lanes * R, hipMemcpyDeviceToHost));
            long bad_l = 0, bad_r = 0, first = -1;
            uint32_t lane_hist[4] = {0, 0, 0, 0};
            for (uint32_t r = 0; r < R; r++) {
                long b = 0;
                for (uint32_t i = 0; i < lanes; i++)
                    if (o[(size_t)lanes * r + i] != q[i]) {
                        b++;
                        lane_hist[(i % 64) / 16]++;
                        if (first < 0) first = (long)i;
                    }
                bad_l += b;
                bad_r += b > 0;
            }
            printf("probe %-18s busy %-9s: %ld of %u launches differ, %ld lanes (quarter-wave hist %u %u %u %u)%s\n",
                   pn[probe], bn[busy], bad_r, R, bad_l, lane_hist[0], lane_hist[1], lane_hist[2], lane_hist[3],
                   first >= 0 ? "" : "");
            fflush(stdout);
            bad_any |= bad_l > 0;
        }
    }
    return bad_any ? 1 : 0;
}
