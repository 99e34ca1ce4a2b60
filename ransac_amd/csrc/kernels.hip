// kernels.hip -- HIP kernels of the hypothesize-and-verify hot path (gfx950 / CDNA4).
//
// Data layout in HBM (DESIGN.md "Layout"):
//   points   : N x float4 {x1,y1,x2,y2} (two-view) or N x float2 {x,y} (line), read-only,
//              L2/LDS resident (160 KB at N = 10k);
//   samples  : B x m int32;
//   models   : SoA [18][B] fp32 -- H (9) then H^-1 (9) per hypothesis, so lane h reads
//              component c at models[c*B + h] (coalesced);
//   scores   : counts int32[B], sums fp32[B].
//
// Scoring maps LANES TO HYPOTHESES: each wave owns 64 hypotheses and walks the points in
// order; a point is wave-uniform, so it arrives by scalar loads into SGPRs and feeds the
// VALU as a scalar operand (no LDS, no VGPR staging, one 16 B load shared by 64
// hypotheses).  Each lane's inlier count and Σerr are accumulated in point order, so with
// one chunk per hypothesis the sum is bit-identical to the reference's sequential fp32 sum
// (quality.hpp:89-96).  `CHUNKS` waves of a workgroup split the point range of the same 64
// hypotheses for occupancy; their partial sums are then combined in chunk order.
#include <hip/hip_runtime.h>

#include "usac_device.hpp"
#include "usac_h16.hpp"
#include "usac_hscore.hpp"
#include "usac_kernels.h"

namespace usac {

// ------------------------------------------------------------------------ solve (H, 4-pt)
__device__ __forceinline__ void store_h(float *__restrict__ models, uint32_t B, uint32_t h, const double *v,
                                        const H16Emit &emit) {
    float H[9], Hi[9];
#pragma unroll
    for (int k = 0; k < 9; k++) H[k] = (float)(v[k] / v[8]);
    inv3x3(H, Hi);
#pragma unroll
    for (int k = 0; k < 9; k++) {
        models[(size_t)k * B + h] = H[k];
        models[(size_t)(9 + k) * B + h] = Hi[k];
    }
    if (emit.rows) h16_rows_of(H, emit.k, emit.thr, h, static_cast<half8 *>(emit.rows), emit.fm);
}

// Thin 4-pt DLT by QR + inverse iteration (dlt4_thin_qr).  A lane whose system falls back is
// appended to fb_list (wave-aggregated atomic on fb_n[0]); k_solve_h4_jac then solves it by the
// row Jacobi.  The sample is written to samples_out here for every lane.
__global__ __launch_bounds__(64) void k_solve_h4(const float4 *__restrict__ pts, uint32_t n,
                                                 const int32_t *__restrict__ samples_in, int32_t *samples_out,
                                                 uint32_t B, DevSampler ds, uint64_t first_hyp,
                                                 float *__restrict__ models, uint32_t *__restrict__ fb_list,
                                                 uint32_t *__restrict__ fb_n, H16Emit emit) {
    const uint32_t h = blockIdx.x * 64 + threadIdx.x;
    bool fb = false;
    if (h < B) {
        int32_t s[4];
        if (samples_in) {
#pragma unroll
            for (int i = 0; i < 4; i++) s[i] = samples_in[4 * (size_t)h + i];
        } else {
            draw_sample<4>(ds, first_hyp + h, n, s);
            if (samples_out) {
#pragma unroll
                for (int i = 0; i < 4; i++) samples_out[4 * (size_t)h + i] = s[i];
            }
        }
        double W[8][9];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            float4 p = pts[s[i]];
            dlt_rows(p.x, p.y, p.z, p.w, W[2 * i], W[2 * i + 1]);
        }
        double v[9];
        if (dlt4_thin_qr(W, v)) store_h(models, B, h, v, emit);
        else fb = true;
    }
    const uint64_t m = __ballot(fb);
    if (m) {
        const uint32_t lane = threadIdx.x;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(fb_n, (uint32_t)__popcll(m));
        base = __shfl(base, 0, 64);
        if (fb) fb_list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = h;
    }
}

// Row-Jacobi 4-pt DLT (row_jacobi + pick_vector): every hypothesis (fb_list == nullptr: the
// nullspace mode; it also writes samples_out) or the fb_n[0] listed fall-backs of k_solve_h4
// (a grid-stride loop over the list: the grid is sized before the count is known).  With a list, the last
// workgroup to finish (fb_n[1] counts them) resets both counters, so the next solve on this
// buffer starts from zero without a memset.
__global__ __launch_bounds__(64) void k_solve_h4_jac(const float4 *__restrict__ pts, uint32_t n,
                                                     const int32_t *__restrict__ samples_in, int32_t *samples_out,
                                                     uint32_t B, DevSampler ds, uint64_t first_hyp, int nullspace,
                                                     float *__restrict__ models, const uint32_t *__restrict__ fb_list,
                                                     uint32_t *__restrict__ fb_n, H16Emit emit) {
    const uint32_t K = fb_list ? __builtin_amdgcn_readfirstlane(__atomic_load_n(fb_n, __ATOMIC_RELAXED)) : B;
    for (uint32_t base = blockIdx.x * 64; base < K; base += gridDim.x * 64) {
        const uint32_t i = base + threadIdx.x;
        if (i >= K) continue;
        const uint32_t h = fb_list ? fb_list[i] : i;
        int32_t s[4];
        if (samples_in) {
#pragma unroll
            for (int k = 0; k < 4; k++) s[k] = samples_in[4 * (size_t)h + k];
        } else {
            draw_sample<4>(ds, first_hyp + h, n, s);
            if (samples_out && !fb_list) {
#pragma unroll
                for (int k = 0; k < 4; k++) samples_out[4 * (size_t)h + k] = s[k];
            }
        }
        double W[8][9];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            float4 p = pts[s[k]];
            dlt_rows(p.x, p.y, p.z, p.w, W[2 * k], W[2 * k + 1]);
        }
        row_jacobi<8>(W);
        double v[9];
        pick_vector<8>(W, nullspace, v);
        store_h(models, B, h, v, emit);
    }
    if (fb_list) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            if (atomicAdd(fb_n + 1, 1u) == gridDim.x - 1) {
                __atomic_store_n(fb_n, 0u, __ATOMIC_RELAXED);
                __atomic_store_n(fb_n + 1, 0u, __ATOMIC_RELAXED);
            }
        }
    }
}

// Host-provided models (B x 9, row-major) -> SoA H / H^-1.
__global__ __launch_bounds__(256) void k_prepare_h(const float *__restrict__ in, uint32_t B,
                                                   float *__restrict__ models) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
    float H[9], Hi[9];
#pragma unroll
    for (int k = 0; k < 9; k++) H[k] = in[9 * (size_t)h + k];
    inv3x3(H, Hi);
#pragma unroll
    for (int k = 0; k < 9; k++) {
        models[(size_t)k * B + h] = H[k];
        models[(size_t)(9 + k) * B + h] = Hi[k];
    }
}

// ------------------------------------------------------------------------ score (H)
template <int CHUNKS>
__global__ __launch_bounds__(64 * CHUNKS) void k_score_h(const float4 *__restrict__ pts, uint32_t n,
                                                         const float *__restrict__ models, uint32_t B, float thr,
                                                         int32_t *__restrict__ counts, float *__restrict__ sums) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t h = blockIdx.x * 64 + lane;
    const uint32_t hc = h < B ? h : B - 1;
    float H[9], Hi[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
        H[k] = models[(size_t)k * B + hc];
        Hi[k] = models[(size_t)(9 + k) * B + hc];
    }
    const uint32_t per = (n + CHUNKS - 1) / CHUNKS;
    const uint32_t begin = wave * per;
    const uint32_t end = begin + per < n ? begin + per : n;
    int cnt = 0;
    float sum = 0.f;
    for (uint32_t i = begin; i < end; ++i) {
        const float4 p = pts[i];
        const float err = homography_error(H, Hi, p.x, p.y, p.z, p.w);
        if (err < thr) {
            cnt++;
            sum += err;
        }
    }
    if constexpr (CHUNKS == 1) {
        if (h < B) {
            counts[h] = cnt;
            sums[h] = sum;
        }
    } else {
        __shared__ int s_cnt[CHUNKS][64];
        __shared__ float s_sum[CHUNKS][64];
        s_cnt[wave][lane] = cnt;
        s_sum[wave][lane] = sum;
        __syncthreads();
        if (wave == 0 && h < B) {
            int c = s_cnt[0][lane];
            float s = s_sum[0][lane];
#pragma unroll
            for (int w = 1; w < CHUNKS; w++) {
                c += s_cnt[w][lane];
                s += s_sum[w][lane];
            }
            counts[h] = c;
            sums[h] = s;
        }
    }
}

// ------------------------------------------------------------------------ score (H), fast path
// Point records for the fast kernel, in groups of 4 points (128 B per group), one
// coordinate of the four points per float4 so that consecutive points' values are adjacent
// SGPRs (the packed stage-A FMAs take them as 64-bit scalar operands without s_mov):
//   float4 [0..3] = x1[4], y1[4], x2[4], y2[4] of points 4g..4g+3,
//   float4 [4]    = guard bands for the current threshold          band_i
//   float4 [5]    = forward-rejection radii (T + band_i)(1 + 2^-18), T = 2 thr
//   float4 [6..7] = padding.
// One s_load_dwordx16 + one s_load_dwordx8 bring four points into SGPRs.  The tail group
// is padded with NaN points, which are never inliers (NaN < thr is false in every path).
// Built once per context and threshold.
__global__ __launch_bounds__(256) void k_prepare_rec(const float4 *__restrict__ pts, uint32_t n, float T,
                                                     float4 *__restrict__ rec) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t ngroups = (n + 3) / 4;
    if (i >= 4 * ngroups) return;
    const uint32_t g = i >> 2, j = i & 3;
    float4 p;
    float band, tr;
    if (i < n) {
        p = pts[i];
        const float mp = fabsf(p.x) + fabsf(p.y) + fabsf(p.z) + fabsf(p.w);
        band = kBandMp * mp + kBandT * T;
        tr = (T + band) * 1.000003814697265625f;  // (1 + 2^-18)
    } else {
        p = make_float4(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
        band = 0.f;
        tr = __builtin_nanf("");
    }
    float *r = reinterpret_cast<float *>(rec + 8 * g);
    r[0 + j] = p.x;
    r[4 + j] = p.y;
    r[8 + j] = p.z;
    r[12 + j] = p.w;
    reinterpret_cast<float *>(rec + 8 * g + 4)[j] = band;
    reinterpret_cast<float *>(rec + 8 * g + 5)[j] = tr;
    if (j < 2) rec[8 * g + 6 + j] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Four points of a group: stage A for all four first (independent chains); the wave takes
// the stage-B path at all only if one of its 64 hypotheses kept one of the four points
// (one scalar branch per group in the common case), then per point behind its own branch.
template <bool EXACT_SUM>
__device__ __forceinline__ void score_group(const HModel &M, float4 X1, float4 Y1, float4 X2, float4 Y2, float4 bd,
                                            float4 tr, float T, float thr, int &cnt, float &sum) {
    bool k0, k1, k2, k3;
    stage_a_keep2(M, v2f{X1.x, X1.y}, v2f{Y1.x, Y1.y}, v2f{X2.x, X2.y}, v2f{Y2.x, Y2.y}, k0, k1);
    stage_a_keep2(M, v2f{X1.z, X1.w}, v2f{Y1.z, Y1.w}, v2f{X2.z, X2.w}, v2f{Y2.z, Y2.w}, k2, k3);
    // marked unlikely: the stage-B blocks are placed out of line, so the common path falls
    // through from one group's stage A to the next instead of jumping over them
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(k0 | k1 | k2 | k3) == 0, 1)) return;
    if (k0) stage_b<EXACT_SUM>(M, X1.x, Y1.x, X2.x, Y2.x, bd.x, T, thr, cnt, sum);
    if (k1) stage_b<EXACT_SUM>(M, X1.y, Y1.y, X2.y, Y2.y, bd.y, T, thr, cnt, sum);
    if (k2) stage_b<EXACT_SUM>(M, X1.z, Y1.z, X2.z, Y2.z, bd.z, T, thr, cnt, sum);
    if (k3) stage_b<EXACT_SUM>(M, X1.w, Y1.w, X2.w, Y2.w, bd.w, T, thr, cnt, sum);
}

// Lanes = hypotheses (64 per wave), point groups wave-uniform (scalar loads, two groups per
// iteration).  CHUNKS waves of a workgroup split the groups of the same 64
// hypotheses and combine (count, Σ) in chunk order.  ext = dataset box (see above).
//
// perm (nullable): lane i of the grid scores hypothesis perm[i] (k_presort_h groups the
// hypotheses that survive stage A often into the same waves, so the other waves rarely
// take the stage-B branch); results land at the hypothesis' own index.
template <int CHUNKS, bool EXACT_SUM>
__global__ __launch_bounds__(64 * CHUNKS) void k_score_hf(const float4 *__restrict__ rec, uint32_t n, float4 ext,
                                                          const float *__restrict__ models, uint32_t B, float thr,
                                                          const uint32_t *__restrict__ perm,
                                                          int32_t *__restrict__ counts, float *__restrict__ sums,
                                                          int32_t *__restrict__ pc, float *__restrict__ ps) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t i = blockIdx.x * 64 + lane;
    const uint32_t ic = i < B ? i : B - 1;
    const uint32_t h = perm ? perm[ic] : i;
    const uint32_t hc = perm ? h : ic;
    HModel M;
#pragma unroll
    for (int k = 0; k < 9; k++) {
        M.h[k] = models[(size_t)k * B + hc];
        M.hi[k] = models[(size_t)(9 + k) * B + hc];
    }
    const float T = 2.0f * thr;
    stage_a_bounds(M, ext, T);
    // point chunks: CHUNKS waves per workgroup x gridDim.y workgroups per hypothesis tile
    const uint32_t ngroups = (n + 3) / 4;
    const uint32_t nchunks = CHUNKS * gridDim.y, chunk = blockIdx.y * CHUNKS + wave;
    const uint32_t per = (ngroups + nchunks - 1) / nchunks;
    const uint32_t gbeg = chunk * per < ngroups ? chunk * per : ngroups;
    const uint32_t gend = gbeg + per < ngroups ? gbeg + per : ngroups;
    int cnt = 0;
    float sum = 0.f;
    // the two groups of an iteration load into fixed SGPR tuples, so the packed stage A reads
    // its point pairs straight from the loaded registers (no copies); 8 waves per SIMD hide
    // the scalar-load latency
    uint32_t g = gbeg;
    for (; g + 2 <= gend; g += 2) {
        const float4 *p = rec + 8 * (size_t)g;
        const float4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3], ab = p[4], at = p[5];
        const float4 b0 = p[8], b1 = p[9], b2 = p[10], b3 = p[11], bb = p[12], bt = p[13];
        score_group<EXACT_SUM>(M, a0, a1, a2, a3, ab, at, T, thr, cnt, sum);
        score_group<EXACT_SUM>(M, b0, b1, b2, b3, bb, bt, T, thr, cnt, sum);
    }
    if (g < gend) {
        const float4 *p = rec + 8 * (size_t)g;
        score_group<EXACT_SUM>(M, p[0], p[1], p[2], p[3], p[4], p[5], T, thr, cnt, sum);
    }
    if (!EXACT_SUM) sum *= 0.5f;
    if (pc) {  // gridDim.y > 1: this workgroup's partial at [blockIdx.y][h] (k_score_ycombine adds them)
        counts = pc + (size_t)blockIdx.y * B;
        sums = ps + (size_t)blockIdx.y * B;
    }
    if constexpr (CHUNKS == 1) {
        if (i < B) {
            counts[hc] = cnt;
            sums[hc] = sum;
        }
    } else {
        __shared__ int s_cnt[CHUNKS][64];
        __shared__ float s_sum[CHUNKS][64];
        s_cnt[wave][lane] = cnt;
        s_sum[wave][lane] = sum;
        __syncthreads();
        if (wave == 0 && i < B) {
            int c = s_cnt[0][lane];
            float s = s_sum[0][lane];
#pragma unroll
            for (int w = 1; w < CHUNKS; w++) {
                c += s_cnt[w][lane];
                s += s_sum[w][lane];
            }
            counts[hc] = c;
            sums[hc] = s;
        }
    }
}

// the gridDim.y partials of k_score_hf, added in workgroup order (deterministic)
__global__ __launch_bounds__(256) void k_score_ycombine(const int32_t *__restrict__ pc, const float *__restrict__ ps,
                                                        uint32_t B, uint32_t ny, int32_t *__restrict__ counts,
                                                        float *__restrict__ sums) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
    int c = pc[h];
    float s = ps[h];
    for (uint32_t y = 1; y < ny; y++) {
        c += pc[(size_t)y * B + h];
        s += ps[(size_t)y * B + h];
    }
    counts[h] = c;
    sums[h] = s;
}

// Hypothesis pre-sort for the fast score kernel: forward-distance hits of every hypothesis
// on the first kPresortGroups point groups (fp32 with v_rcp -- a heuristic, it only
// decides WHERE a hypothesis is scored, never its result).  Within each region of R
// hypotheses (R a multiple of 64; the launch uses one region) those with >= kPresortHits hits
// go to the front, the rest to the back: one packed 64-bit atomic per workgroup on the
// region's counter ((good << 32) | bad); the workgroup that completes a region puts its
// counter back to 0, so the next launch needs no memset (the counters are zeroed once, when
// the buffer is allocated).
constexpr uint32_t kPresortGroups = 32;  // 128 points
constexpr int kPresortHits = 3;

constexpr int kPresortWaves = 4;       // waves per workgroup, 64 hypotheses each
constexpr uint32_t kPresortCtr = 256;  // region counters at the head of the pre-sort buffer

// One workgroup = 4 x 64 hypotheses, each lane over all kPresortGroups groups; the four waves'
// good / bad counts are combined in LDS so the workgroup takes its places with ONE atomic
// (the atomics on the region counter, not the arithmetic, set this kernel's time).
__global__ __launch_bounds__(64 * kPresortWaves) void k_presort_h(const float4 *__restrict__ rec, uint32_t n,
                                                                  const float *__restrict__ models, uint32_t B,
                                                                  float thr, uint32_t *__restrict__ perm,
                                                                  unsigned long long *__restrict__ ctr, uint32_t R) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t h = blockIdx.x * (64 * kPresortWaves) + threadIdx.x;
    const uint32_t hc = h < B ? h : B - 1;
    float m[9];
#pragma unroll
    for (int k = 0; k < 9; k++) m[k] = models[(size_t)k * B + hc];
    const float T2 = 4.0f * thr * thr;  // forward distance < 2 thr
    const uint32_t ngroups = (n + 3) / 4;
    const uint32_t g1 = ngroups < kPresortGroups ? ngroups : kPresortGroups;
    int hits = 0;
    for (uint32_t g = 0; g < g1; g++) {
        const float *p = reinterpret_cast<const float *>(rec + 8 * (size_t)g);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float x1 = p[u], y1 = p[4 + u], x2 = p[8 + u], y2 = p[12 + u];
            const float X = __builtin_fmaf(m[1], y1, __builtin_fmaf(m[0], x1, m[2]));
            const float Y = __builtin_fmaf(m[4], y1, __builtin_fmaf(m[3], x1, m[5]));
            const float Z = __builtin_fmaf(m[7], y1, __builtin_fmaf(m[6], x1, m[8]));
            const float r = __builtin_amdgcn_rcpf(Z);
            const float dx = __builtin_fmaf(-X, r, x2), dy = __builtin_fmaf(-Y, r, y2);
            hits += __builtin_fmaf(dx, dx, dy * dy) < T2 ? 1 : 0;
        }
    }
    const bool valid = h < B;
    const bool good = valid && hits >= kPresortHits;
    const uint64_t bg = __ballot(good), bb = __ballot(valid && !good);
    const uint32_t below = (uint32_t)__popcll(good ? bg & ((1ull << lane) - 1) : bb & ((1ull << lane) - 1));
    __shared__ uint32_t s_g[kPresortWaves], s_b[kPresortWaves];
    __shared__ unsigned long long s_old;
    if (lane == 0) {
        s_g[wave] = (uint32_t)__popcll(bg);
        s_b[wave] = (uint32_t)__popcll(bb);
    }
    __syncthreads();
    const uint32_t h0 = blockIdx.x * (64 * kPresortWaves);
    const uint32_t r = h0 / R, rs = r * R, re = rs + R < B ? rs + R : B;
    uint32_t ng = 0, nbad = 0, gw = 0, bw = 0;
#pragma unroll
    for (int w = 0; w < kPresortWaves; w++) {
        if ((uint32_t)w < wave) {
            gw += s_g[w];
            bw += s_b[w];
        }
        ng += s_g[w];
        nbad += s_b[w];
    }
    if (threadIdx.x == 0) {
        const unsigned long long old = atomicAdd(&ctr[r], ((unsigned long long)ng << 32) | nbad);
        const uint32_t done = (uint32_t)(old >> 32) + (uint32_t)old + ng + nbad;
        if (done == re - rs) __hip_atomic_store(&ctr[r], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_old = old;
    }
    __syncthreads();
    const unsigned long long old = s_old;
    const uint32_t fbase = rs + (uint32_t)(old >> 32) + gw, bbase = (uint32_t)old + bw;
    const uint32_t at = good ? fbase + below : re - 1 - (bbase + below);
    if (valid && at < re) perm[at] = h;  // (each region's counts reach its size exactly)
}

size_t presort_bytes(uint32_t B) { return sizeof(unsigned long long) * kPresortCtr + sizeof(uint32_t) * (size_t)B; }
size_t presort_counter_bytes() { return sizeof(unsigned long long) * kPresortCtr; }

// ------------------------------------------------------------------------ line2d
__global__ __launch_bounds__(256) void k_solve_line(const float2 *__restrict__ pts, uint32_t n,
                                                    const int32_t *__restrict__ samples_in, int32_t *samples_out,
                                                    uint32_t B, DevSampler ds, uint64_t first_hyp,
                                                    float *__restrict__ models) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
    int32_t s[2];
    if (samples_in) {
        s[0] = samples_in[2 * (size_t)h];
        s[1] = samples_in[2 * (size_t)h + 1];
    } else {
        draw_sample<2>(ds, first_hyp + h, n, s);
        if (samples_out) {
            samples_out[2 * (size_t)h] = s[0];
            samples_out[2 * (size_t)h + 1] = s[1];
        }
    }
    const float2 p1 = pts[s[0]], p2 = pts[s[1]];
    float m[3];
    line2d_estimate(p1.x, p1.y, p2.x, p2.y, m);
#pragma unroll
    for (int k = 0; k < 3; k++) models[(size_t)k * B + h] = m[k];
}

__global__ __launch_bounds__(256) void k_prepare_line(const float *__restrict__ in, uint32_t B,
                                                      float *__restrict__ models) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
#pragma unroll
    for (int k = 0; k < 3; k++) models[(size_t)k * B + h] = in[9 * (size_t)h + k];
}

template <int CHUNKS>
__global__ __launch_bounds__(64 * CHUNKS) void k_score_line(const float2 *__restrict__ pts, uint32_t n,
                                                            const float *__restrict__ models, uint32_t B, float thr,
                                                            int32_t *__restrict__ counts, float *__restrict__ sums) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t h = blockIdx.x * 64 + lane;
    const uint32_t hc = h < B ? h : B - 1;
    const float a = models[hc], b = models[(size_t)B + hc], c = models[2 * (size_t)B + hc];
    const uint32_t per = (n + CHUNKS - 1) / CHUNKS;
    const uint32_t begin = wave * per;
    const uint32_t end = begin + per < n ? begin + per : n;
    int cnt = 0;
    float sum = 0.f;
    for (uint32_t i = begin; i < end; ++i) {
        const float2 p = pts[i];
        const float err = line2d_error(a, b, c, p.x, p.y);
        if (err < thr) {
            cnt++;
            sum += err;
        }
    }
    if constexpr (CHUNKS == 1) {
        if (h < B) {
            counts[h] = cnt;
            sums[h] = sum;
        }
    } else {
        __shared__ int s_cnt[CHUNKS][64];
        __shared__ float s_sum[CHUNKS][64];
        s_cnt[wave][lane] = cnt;
        s_sum[wave][lane] = sum;
        __syncthreads();
        if (wave == 0 && h < B) {
            int cc = s_cnt[0][lane];
            float ss = s_sum[0][lane];
#pragma unroll
            for (int w = 1; w < CHUNKS; w++) {
                cc += s_cnt[w][lane];
                ss += s_sum[w][lane];
            }
            counts[h] = cc;
            sums[h] = ss;
        }
    }
}

// ------------------------------------------------------------------------ batch argmax
// Two launches: k_argmax_part reduces 2048 hypotheses per workgroup (8 independent loads
// per lane in flight, LDS tree), k_argmax_final reduces the partials and gathers the
// model.  record_better is a strict total order, so the tree shape does not change the
// result (= the sequential first-best under Score::bigger).
struct BestEntry {
    int c;
    float s;
    uint32_t i;
};

__device__ __forceinline__ void tree_best(BestEntry *sh, uint32_t t, uint32_t width) {
    for (uint32_t w = width / 2; w > 0; w >>= 1) {
        if (t < w) {
            const BestEntry o = sh[t + w];
            if (o.c >= 0 && (sh[t].c < 0 || record_better(o.c, o.s, o.i, sh[t].c, sh[t].s, sh[t].i))) sh[t] = o;
        }
        __syncthreads();
    }
}

// H16: counts / sums first from the matrix-core scorer's chunk partials (cpart u32, spart u64 fixed
// point, chunk-major), added in chunk order and written out exactly as k_h16_finish does
template <bool H16>
__global__ __launch_bounds__(256) void k_argmax_part(const int32_t *__restrict__ counts_in,
                                                     const float *__restrict__ sums_in, uint32_t B,
                                                     BestEntry *__restrict__ part, const uint32_t *__restrict__ cpart,
                                                     const unsigned long long *__restrict__ spart, uint32_t nch,
                                                     double inv_fxs, int32_t *__restrict__ counts_out,
                                                     float *__restrict__ sums_out) {
    __shared__ BestEntry sh[256];
    const uint32_t t = threadIdx.x;
    const uint32_t base = blockIdx.x * 2048 + t;
    int c[8];
    float s[8];
    if constexpr (H16) {
        uint32_t cc[8];
        unsigned long long ss[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            cc[j] = 0;
            ss[j] = 0;
        }
        for (uint32_t y = 0; y < nch; y++)
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t i = base + 256 * j;
                if (i < B) {
                    cc[j] += cpart[(size_t)y * B + i];
                    ss[j] += spart[(size_t)y * B + i];
                }
            }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t i = base + 256 * j;
            c[j] = i < B ? (int32_t)cc[j] : -1;
            s[j] = (float)((double)ss[j] * inv_fxs * 0.5);  // as k_h16_finish
            if (i < B) {
                counts_out[i] = c[j];
                sums_out[i] = s[j];
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t i = base + 256 * j;
            c[j] = i < B ? counts_in[i] : -1;
            s[j] = i < B ? sums_in[i] : 0.f;
        }
    }
    BestEntry b{-1, 0.f, 0xFFFFFFFFu};
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t i = base + 256 * j;
        if (c[j] >= 0 && (b.c < 0 || record_better(c[j], s[j], i, b.c, b.s, b.i))) b = BestEntry{c[j], s[j], i};
    }
    sh[t] = b;
    __syncthreads();
    tree_best(sh, t, 256);
    if (t == 0) part[blockIdx.x] = sh[0];
}

__global__ __launch_bounds__(256) void k_argmax_final(const BestEntry *__restrict__ part, uint32_t nparts, uint32_t B,
                                                      const float *__restrict__ models, int ncomp, uint64_t first_hyp,
                                                      uint32_t spk, usac_record *out) {
    __shared__ BestEntry sh[256];
    const uint32_t t = threadIdx.x;
    BestEntry b{-1, 0.f, 0xFFFFFFFFu};
    for (uint32_t k = t; k < nparts; k += 256) {
        const BestEntry o = part[k];
        if (o.c >= 0 && (b.c < 0 || record_better(o.c, o.s, o.i, b.c, b.s, b.i))) b = o;
    }
    sh[t] = b;
    __syncthreads();
    tree_best(sh, t, 256);
    if (t == 0) {
        usac_record r;
        const BestEntry best = sh[0];
        const int sc0 = best.c;
        const float ss0 = best.s;
        const uint32_t i = best.i;
        r.valid = sc0 >= 0 ? 1 : 0;
        r.inliers = sc0 < 0 ? 0 : sc0;
        r.score = ss0;
        r.hyp_index = first_hyp + (i == 0xFFFFFFFFu ? 0 : i / spk);  // spk model slots per hypothesis
        for (int k = 0; k < 9; k++) r.model[k] = (k < ncomp && r.valid) ? models[(size_t)k * B + i] : 0.f;
        *out = r;
    }
}

// ------------------------------------------------------------------------ launchers
#define LAUNCH_CHECK() hipGetLastError()

hipError_t launch_solve_h4(hipStream_t st, const float4 *pts, uint32_t n, const int32_t *samples_in,
                           int32_t *samples_out, uint32_t B, DevSampler ds, uint64_t first_hyp, int nullspace,
                           float *models, uint32_t *fb_list, uint32_t *fb_n, const H16Emit *emit) {
    const uint32_t blocks = (B + 63) / 64;
    const H16Emit em = emit ? *emit : H16Emit{nullptr, 0.f, nullptr, nullptr};
    if (nullspace) {
        hipLaunchKernelGGL(k_solve_h4_jac, dim3(blocks), dim3(64), 0, st, pts, n, samples_in, samples_out, B, ds,
                           first_hyp, 1, models, (const uint32_t *)nullptr, (uint32_t *)nullptr, em);
        return LAUNCH_CHECK();
    }
    if (!fb_list || !fb_n) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_solve_h4, dim3(blocks), dim3(64), 0, st, pts, n, samples_in, samples_out, B, ds, first_hyp,
                       models, fb_list, fb_n, em);
    hipError_t e = LAUNCH_CHECK();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_solve_h4_jac, dim3(blocks < 256 ? blocks : 256), dim3(64), 0, st, pts, n, samples_in,
                       samples_out, B, ds, first_hyp, 0, models, (const uint32_t *)fb_list, fb_n, em);
    return LAUNCH_CHECK();
}

hipError_t launch_prepare_h(hipStream_t st, const float *in, uint32_t B, float *models) {
    hipLaunchKernelGGL(k_prepare_h, dim3((B + 255) / 256), dim3(256), 0, st, in, B, models);
    return LAUNCH_CHECK();
}

hipError_t launch_score_h(hipStream_t st, int chunks, const float4 *pts, uint32_t n, const float *models, uint32_t B,
                          float thr, int32_t *counts, float *sums) {
    dim3 grid((B + 63) / 64);
    switch (chunks) {
        case 1: hipLaunchKernelGGL(k_score_h<1>, grid, dim3(64), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 2: hipLaunchKernelGGL(k_score_h<2>, grid, dim3(128), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 4: hipLaunchKernelGGL(k_score_h<4>, grid, dim3(256), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 8: hipLaunchKernelGGL(k_score_h<8>, grid, dim3(512), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 16: hipLaunchKernelGGL(k_score_h<16>, grid, dim3(1024), 0, st, pts, n, models, B, thr, counts, sums); break;
        default: return hipErrorInvalidValue;
    }
    return LAUNCH_CHECK();
}

hipError_t launch_prepare_rec(hipStream_t st, const float4 *pts, uint32_t n, float thr, float4 *rec) {
    const uint32_t total = 4 * ((n + 3) / 4);
    hipLaunchKernelGGL(k_prepare_rec, dim3((total + 255) / 256), dim3(256), 0, st, pts, n, 2.0f * thr, rec);
    return LAUNCH_CHECK();
}

hipError_t launch_score_hf(hipStream_t st, int chunks, bool exact_sum, const float4 *rec, uint32_t n, float4 ext,
                           const float *models, uint32_t B, float thr, uint32_t *perm, int32_t *counts, float *sums,
                           uint32_t ysplit, void *yscratch) {
    if (exact_sum || !yscratch) ysplit = 1;
    dim3 grid((B + 63) / 64, ysplit);
    int32_t *pc = ysplit > 1 ? static_cast<int32_t *>(yscratch) : nullptr;
    float *ps = ysplit > 1 ? reinterpret_cast<float *>(pc + (size_t)ysplit * B) : nullptr;
    if (perm) {  // the pre-sort buffer (presort_bytes): region counters, then the B entries
        unsigned long long *ctr = reinterpret_cast<unsigned long long *>(perm);
        perm += 2 * kPresortCtr;
        // one region: the front-loaded order (stage-B-heavy hypotheses first) is what pays; a
        // region per 4096 hypotheses measured 0.33 ms against 0.22 for the score kernel
        const uint32_t R = (B + 255) & ~255u;  // a multiple of the workgroup's 256 hypotheses
        hipLaunchKernelGGL(k_presort_h, dim3((B + 64 * kPresortWaves - 1) / (64 * kPresortWaves)),
                           dim3(64 * kPresortWaves), 0, st, rec, n, models, B, thr, perm, ctr, R);
    }
#define SHF(C, E) \
    hipLaunchKernelGGL((k_score_hf<C, E>), grid, dim3(64 * C), 0, st, rec, n, ext, models, B, thr, perm, counts, sums, \
                       pc, ps)
    if (exact_sum) {
        switch (chunks) {
            case 1: SHF(1, true); break;
            case 2: SHF(2, true); break;
            case 4: SHF(4, true); break;
            case 8: SHF(8, true); break;
            case 16: SHF(16, true); break;
            default: return hipErrorInvalidValue;
        }
    } else {
        switch (chunks) {
            case 1: SHF(1, false); break;
            case 2: SHF(2, false); break;
            case 4: SHF(4, false); break;
            case 8: SHF(8, false); break;
            case 16: SHF(16, false); break;
            default: return hipErrorInvalidValue;
        }
    }
#undef SHF
    if (ysplit > 1)
        hipLaunchKernelGGL(k_score_ycombine, dim3((B + 255) / 256), dim3(256), 0, st, pc, ps, B, ysplit, counts, sums);
    return LAUNCH_CHECK();
}

template <int M>
__global__ __launch_bounds__(256) void k_draw_samples(uint32_t n, uint32_t B, DevSampler ds, uint64_t first_hyp,
                                                      int32_t *__restrict__ out) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= B) return;
    int32_t s[M];
    draw_sample<M>(ds, first_hyp + h, n, s);
#pragma unroll
    for (int i = 0; i < M; i++) out[(size_t)M * h + i] = s[i];
}

hipError_t launch_draw_samples(hipStream_t st, int m, uint32_t n, uint32_t B, DevSampler ds, uint64_t first_hyp,
                               int32_t *out) {
    const dim3 g((B + 255) / 256), b(256);
    switch (m) {
        case 2: hipLaunchKernelGGL(k_draw_samples<2>, g, b, 0, st, n, B, ds, first_hyp, out); break;
        case 4: hipLaunchKernelGGL(k_draw_samples<4>, g, b, 0, st, n, B, ds, first_hyp, out); break;
        case 5: hipLaunchKernelGGL(k_draw_samples<5>, g, b, 0, st, n, B, ds, first_hyp, out); break;
        case 7: hipLaunchKernelGGL(k_draw_samples<7>, g, b, 0, st, n, B, ds, first_hyp, out); break;
        default: return hipErrorInvalidValue;
    }
    return LAUNCH_CHECK();
}

hipError_t launch_solve_line(hipStream_t st, const float2 *pts, uint32_t n, const int32_t *samples_in,
                             int32_t *samples_out, uint32_t B, DevSampler ds, uint64_t first_hyp, float *models) {
    hipLaunchKernelGGL(k_solve_line, dim3((B + 255) / 256), dim3(256), 0, st, pts, n, samples_in, samples_out, B, ds,
                       first_hyp, models);
    return LAUNCH_CHECK();
}

hipError_t launch_prepare_line(hipStream_t st, const float *in, uint32_t B, float *models) {
    hipLaunchKernelGGL(k_prepare_line, dim3((B + 255) / 256), dim3(256), 0, st, in, B, models);
    return LAUNCH_CHECK();
}

hipError_t launch_score_line(hipStream_t st, int chunks, const float2 *pts, uint32_t n, const float *models,
                             uint32_t B, float thr, int32_t *counts, float *sums) {
    dim3 grid((B + 63) / 64);
    switch (chunks) {
        case 1: hipLaunchKernelGGL(k_score_line<1>, grid, dim3(64), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 2: hipLaunchKernelGGL(k_score_line<2>, grid, dim3(128), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 4: hipLaunchKernelGGL(k_score_line<4>, grid, dim3(256), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 8: hipLaunchKernelGGL(k_score_line<8>, grid, dim3(512), 0, st, pts, n, models, B, thr, counts, sums); break;
        case 16: hipLaunchKernelGGL(k_score_line<16>, grid, dim3(1024), 0, st, pts, n, models, B, thr, counts, sums); break;
        default: return hipErrorInvalidValue;
    }
    return LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void k_pack_slice(const int32_t *__restrict__ counts, const float *__restrict__ models,
                                                    uint32_t S, uint32_t P, int ncomp, int32_t status,
                                                    int32_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) out[0] = status;
    if (i >= P) return;
    out[1 + i] = i < S ? counts[i] : -1;
    for (int k = 0; k < ncomp; k++)
        out[1 + (size_t)(1 + k) * P + i] = i < S ? __float_as_int(models[(size_t)k * S + i]) : 0;
}

hipError_t launch_pack_slice(hipStream_t st, const int32_t *counts, const float *models, uint32_t S, uint32_t P,
                             int ncomp, int32_t status, int32_t *out) {
    hipLaunchKernelGGL(k_pack_slice, dim3(P / 256 + 1), dim3(256), 0, st, counts, models, S, P, ncomp, status, out);
    return LAUNCH_CHECK();
}

hipError_t launch_argmax(hipStream_t st, const int32_t *counts, const float *sums, uint32_t B, const float *models,
                         int ncomp, uint64_t first_hyp, uint32_t spk, void *scratch, usac_record *out) {
    const uint32_t nparts = (B + 2047) / 2048;
    BestEntry *part = static_cast<BestEntry *>(scratch);
    hipLaunchKernelGGL(k_argmax_part<false>, dim3(nparts), dim3(256), 0, st, counts, sums, B, part,
                       (const uint32_t *)nullptr, (const unsigned long long *)nullptr, 0u, 0.0, (int32_t *)nullptr,
                       (float *)nullptr);
    hipLaunchKernelGGL(k_argmax_final, dim3(1), dim3(256), 0, st, part, nparts, B, models, ncomp, first_hyp, spk,
                       out);
    return LAUNCH_CHECK();
}

hipError_t launch_argmax_h16(hipStream_t st, const void *part16, uint32_t B, int chunks, float thr, int32_t *counts,
                             float *sums, const float *models, int ncomp, uint64_t first_hyp, uint32_t spk,
                             void *scratch, usac_record *out) {
    const uint32_t nparts = (B + 2047) / 2048;
    BestEntry *part = static_cast<BestEntry *>(scratch);
    // the h16 partials' layout (launch_score_h16): u64 sums [chunks][B] first, then u32 counts
    const unsigned long long *sp = static_cast<const unsigned long long *>(part16);
    const uint32_t *cp = reinterpret_cast<const uint32_t *>(sp + (size_t)chunks * B);
    hipLaunchKernelGGL(k_argmax_part<true>, dim3(nparts), dim3(256), 0, st, (const int32_t *)nullptr,
                       (const float *)nullptr, B, part, cp, sp, (uint32_t)chunks, ldexp(1.0, -h16_fixed_point(thr)),
                       counts, sums);
    hipLaunchKernelGGL(k_argmax_final, dim3(1), dim3(256), 0, st, part, nparts, B, models, ncomp, first_hyp, spk,
                       out);
    return LAUNCH_CHECK();
}

}  // namespace usac
