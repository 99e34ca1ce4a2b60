// h16_race.cpp -- diagnostic for the round-5 miscount: the
// exact recount (launch_inliers_batch: k_inl_flags + k_inl_compact + seqsum, the loop's
// exact_sums) on stream R while stream S runs one of
//   0 nothing, 1 k_score_h16 (the matrix-core scorer), 2 a pure MFMA kernel (no LDS, no memory in
//   its loop), 3 a pure fp32 VALU kernel, 4 k_score_h16 with the recount's point set copied (no
//   shared input buffer).
// Every recount keeps its own scratch (per-point residuals) and counts, so a recount that differs
// from the quiet one is dumped point by point afterwards: which points, which lanes of which
// wave, and the residuals both times.  Every h16 launch keeps its own counts too and is compared
// with the quiet h16 launch (does the scorer itself miscount?).
//
// Build: make -C tools h16_race   (links ../ransac_amd/libransac_amd.so)
// Run:   ./tools/h16_race [mode ...]   (default: 0 1 2 3 4); exit 1 if any mode saw a difference.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../ransac_amd/csrc/usac_kernels.h"

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

// mode 2: MFMA back to back on register operands, the result folded into one store at the end
__global__ __launch_bounds__(256) void k_busy_mfma(int iters, float *out) {
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
}

// mode 3: dependent fp32 VALU chains
__global__ __launch_bounds__(256) void k_busy_valu(int iters, float *out) {
    float x = threadIdx.x * 1e-3f, y = blockIdx.x * 1e-3f;
    for (int i = 0; i < iters; i++) {
        x = x * 0.999f + y;
        y = y * 1.001f - x * 1e-3f;
    }
    if (x == 12345.f) out[blockIdx.x * 256 + threadIdx.x] = x + y;
}

int main(int argc, char **argv) {
    std::vector<int> modes;
    for (int i = 1; i < argc; i++) modes.push_back(atoi(argv[i]));
    if (modes.empty()) modes = {0, 1, 2, 3, 4};
    const uint32_t n = 20000, K = 64, R = 300, B = 65536, L = 60;
    const float thr = 2.0f;
    // points: 30 % on a homography (+-0.7 px noise), the rest uniform
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(0.f, 1000.f), E(-0.7f, 0.7f);
    const double Ht[9] = {0.9, 0.05, 30, -0.04, 1.1, -20, 1e-5, 2e-5, 1};
    std::vector<float> pts(4 * n);
    for (uint32_t i = 0; i < n; i++) {
        const float x = U(rng), y = U(rng);
        pts[4 * i] = x;
        pts[4 * i + 1] = y;
        if (i % 10 < 3) {
            const double z = Ht[6] * x + Ht[7] * y + Ht[8];
            pts[4 * i + 2] = (float)((Ht[0] * x + Ht[1] * y + Ht[2]) / z) + E(rng);
            pts[4 * i + 3] = (float)((Ht[3] * x + Ht[4] * y + Ht[5]) / z) + E(rng);
        } else {
            pts[4 * i + 2] = U(rng);
            pts[4 * i + 3] = U(rng);
        }
    }
    float4 ext = {0, 0, 0, 0};
    for (uint32_t i = 0; i < n; i++) {
        ext.x = fmaxf(ext.x, fabsf(pts[4 * i]));
        ext.y = fmaxf(ext.y, fabsf(pts[4 * i + 1]));
        ext.z = fmaxf(ext.z, fabsf(pts[4 * i + 2]));
        ext.w = fmaxf(ext.w, fabsf(pts[4 * i + 3]));
    }
    // models: the truth perturbed (recount: small, many borderline points; h16 batch: larger)
    auto perturb = [&](float s, std::vector<float> &m, uint32_t cnt) {
        std::normal_distribution<double> Nd(0.0, 1.0);
        m.resize(9 * (size_t)cnt);
        for (uint32_t h = 0; h < cnt; h++)
            for (int k = 0; k < 9; k++) {
                const double sc = k == 2 || k == 5 ? 1.0 : (k >= 6 ? 1e-6 : 1e-3);
                m[9 * (size_t)h + k] = (float)(Ht[k] + (k == 8 ? 0.0 : s * sc * Nd(rng)));
            }
    };
    std::vector<float> mk, mb;
    perturb(1.0f, mk, K);
    perturb(4.0f, mb, B);

    float4 *d_pts, *d_pts2;
    CK(hipMalloc(&d_pts, 16 * (size_t)n));
    CK(hipMalloc(&d_pts2, 16 * (size_t)n));
    CK(hipMemcpy(d_pts, pts.data(), 16 * (size_t)n, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_pts2, pts.data(), 16 * (size_t)n, hipMemcpyHostToDevice));
    float *d_mk, *d_mb9, *d_mb;
    CK(hipMalloc(&d_mk, 4 * 9 * (size_t)K));
    CK(hipMemcpy(d_mk, mk.data(), 4 * 9 * (size_t)K, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_mb9, 4 * 9 * (size_t)B));
    CK(hipMalloc(&d_mb, 4 * 18 * (size_t)B));
    CK(hipMemcpy(d_mb9, mb.data(), 4 * 9 * (size_t)B, hipMemcpyHostToDevice));
    CK(usac::launch_prepare_h(nullptr, d_mb9, B, d_mb));
    // h16 state (one set per point buffer)
    usac::H16Consts *d_k[2];
    void *d_feat[2], *d_rows[2];
    float *d_fm[2];
    const int ch = 8;
    void *d_part;
    CK(hipMalloc(&d_part, usac::h16_part_bytes(B, ch)));
    for (int s = 0; s < 2; s++) {
        float4 *p = s ? d_pts2 : d_pts;
        CK(hipMalloc(&d_k[s], sizeof(usac::H16Consts)));
        CK(hipMalloc(&d_feat[s], usac::h16_feature_bytes(n)));
        CK(hipMalloc(&d_rows[s], 96 * (size_t)B));
        CK(hipMalloc(&d_fm[s], 4 * (size_t)B));
        CK(usac::launch_h16_consts(nullptr, p, n, ext, d_k[s]));
        CK(usac::launch_h16_points(nullptr, p, n, d_k[s], d_feat[s]));
        CK(usac::launch_h16_rows(nullptr, d_mb, B, d_k[s], thr, d_rows[s], d_fm[s]));
    }
    int32_t *d_hc;
    float *d_hs;
    CK(hipMalloc(&d_hc, 4 * (size_t)B * (L + 1)));
    CK(hipMalloc(&d_hs, 4 * (size_t)B * (L + 1)));
    // recount scratch / results, one per recount (+ the quiet one at index R)
    const size_t sbytes = usac::inliers_scratch_bytes(n, K);
    const size_t sw = usac::inliers_scratch_bytes(n, 1) / 4;  // words per model
    const uint32_t nb = (n + 1023) / 1024;
    const size_t all_off = (size_t)((nb + 63) & ~63u) + ((n + 1) & ~1u);
    char *d_scr;
    int32_t *d_rc;
    float *d_rs;
    int32_t *d_idx;
    CK(hipMalloc(&d_scr, sbytes * (R + 1)));
    CK(hipMalloc(&d_rc, 4 * (size_t)K * (R + 1)));
    CK(hipMalloc(&d_rs, 4 * (size_t)K * (R + 1)));
    CK(hipMalloc(&d_idx, 4 * (size_t)K * n));
    float *d_sink;
    CK(hipMalloc(&d_sink, 4 * 256 * 4096));
    CK(hipDeviceSynchronize());

    // quiet references
    CK(usac::launch_inliers_batch(nullptr, USAC_HOMOGRAPHY, d_pts, n, d_mk, K, thr, nullptr, nullptr, d_idx, n,
                                  d_rc + (size_t)K * R, d_rs + (size_t)K * R, d_scr + sbytes * R, nullptr));
    CK(usac::launch_score_h16(nullptr, d_feat[0], d_pts, n, d_rows[0], d_fm[0], d_mb, B, thr, ch, d_part,
                              d_hc + (size_t)B * L, d_hs + (size_t)B * L, true));
    CK(hipDeviceSynchronize());
    std::vector<int32_t> rq(K), hq(B);
    std::vector<float> eq((size_t)K * n);
    CK(hipMemcpy(rq.data(), d_rc + (size_t)K * R, 4 * K, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hq.data(), d_hc + (size_t)B * L, 4 * (size_t)B, hipMemcpyDeviceToHost));
    for (uint32_t k = 0; k < K; k++)
        CK(hipMemcpy(eq.data() + (size_t)k * n, d_scr + sbytes * R + 4 * (sw * k + all_off), 4 * (size_t)n,
                     hipMemcpyDeviceToHost));
    long tot = 0;
    for (uint32_t k = 0; k < K; k++) tot += rq[k];
    printf("quiet recount: %u models, mean count %.1f; h16 quiet batch of %u\n", K, (double)tot / K, B);

    hipStream_t sR, sS;
    CK(hipStreamCreateWithFlags(&sR, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sS, hipStreamNonBlocking));
    int any_bad = 0;
    for (int mode : modes) {
        CK(hipMemset(d_rc, 0xff, 4 * (size_t)K * R));
        CK(hipMemset(d_hc, 0xff, 4 * (size_t)B * L));
        CK(hipDeviceSynchronize());
        // stream S first (it keeps the device busy), then the recounts
        for (uint32_t l = 0; l < L; l++) {
            if (mode == 1 || mode == 4) {
                const int s = mode == 4 ? 1 : 0;
                CK(usac::launch_score_h16(sS, d_feat[s], s ? d_pts2 : d_pts, n, d_rows[s], d_fm[s], d_mb, B, thr, ch,
                                          d_part, d_hc + (size_t)B * l, d_hs + (size_t)B * l, true));
            } else if (mode == 2) {
                hipLaunchKernelGGL(k_busy_mfma, dim3(2048), dim3(256), 0, sS, 2000, d_sink);
            } else if (mode == 3) {
                hipLaunchKernelGGL(k_busy_valu, dim3(2048), dim3(256), 0, sS, 4000, d_sink);
            }
        }
        for (uint32_t r = 0; r < R; r++)
            CK(usac::launch_inliers_batch(sR, USAC_HOMOGRAPHY, d_pts, n, d_mk, K, thr, nullptr, nullptr, d_idx, n,
                                          d_rc + (size_t)K * r, d_rs + (size_t)K * r, d_scr + sbytes * r, nullptr));
        CK(hipStreamSynchronize(sR));
        CK(hipStreamSynchronize(sS));
        CK(hipGetLastError());
        std::vector<int32_t> rc((size_t)K * R);
        CK(hipMemcpy(rc.data(), d_rc, 4 * (size_t)K * R, hipMemcpyDeviceToHost));
        int bad_r = 0, shown = 0;
        for (uint32_t r = 0; r < R; r++)
            for (uint32_t k = 0; k < K; k++) {
                if (rc[(size_t)K * r + k] == rq[k]) continue;
                bad_r++;
                if (shown >= 6) continue;
                shown++;
                std::vector<float> e(n);
                CK(hipMemcpy(e.data(), d_scr + sbytes * r + 4 * (sw * k + all_off), 4 * (size_t)n,
                             hipMemcpyDeviceToHost));
                printf("  mode %d recount %u model %u: count %d, quiet %d\n", mode, r, k, rc[(size_t)K * r + k], rq[k]);
                int nd = 0;
                for (uint32_t i = 0; i < n; i++) {
                    const float a = e[i], b = eq[(size_t)k * n + i];
                    if (memcmp(&a, &b, 4) == 0) continue;
                    if (nd++ < 40)
                        printf("    point %u (block %u, u %u, wave %u, lane %u): residual %.9g quiet %.9g%s\n", i,
                               i / 1024, (i % 1024) / 256, (i % 256) / 64, i % 64, a, b,
                               (a < thr) != (b < thr) ? "  <- crosses thr" : "");
                }
                printf("    %d residuals differ\n", nd);
            }
        int bad_h = 0;
        if (mode == 1 || mode == 4) {
            std::vector<int32_t> hc((size_t)B * L);
            CK(hipMemcpy(hc.data(), d_hc, 4 * (size_t)B * L, hipMemcpyDeviceToHost));
            for (uint32_t l = 0; l < L; l++)
                for (uint32_t h = 0; h < B; h++)
                    if (hc[(size_t)B * l + h] != hq[h]) {
                        if (bad_h < 6)
                            printf("  mode %d h16 launch %u hyp %u: count %d, quiet %d\n", mode, l, h,
                                   hc[(size_t)B * l + h], hq[h]);
                        bad_h++;
                    }
        }
        printf("mode %d: %d of %u recounts differ, %d h16 counts differ (of %u launches)\n", mode, bad_r, R * K, bad_h,
               mode == 1 || mode == 4 ? L : 0);
        fflush(stdout);
        any_bad |= bad_r || bad_h;
    }
    return any_bad ? 1 : 0;
}
