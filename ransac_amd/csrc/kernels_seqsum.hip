// kernels_seqsum.hip -- the reference's SEQUENTIAL fp32 sums (a running float updated once
// per element, in element order) evaluated in parallel, bit for bit.
//
// The sums are the LO / polish latency floor: NormalizedDLT's coordinate means and average
// distances (normalizing_transformation.cpp:7-113: `float` accumulators, one `+=` per point)
// and Quality's Σerr over the inliers (quality.hpp:85).  Evaluated one dependent add per
// element they cost ~10 cycles per element on one lane (k_normalize 0.3 ms at 17 k points).
//
// Speculation with exact verification.  A chain s_{k+1} = op(s_k, v_k) -- op(s, x) = s + x
// (fp32), or (float)((double)s + y) (the reference's `float += double`) -- is cut into S <= 32
// segments of L elements.  Segment j's true start s_{jL} is not known, but it lies a few
// dozen ulps from c_j = (float)(Σ_{k<jL} v_k) (fp64 prefix): the fp32 chain drifts from the
// exact prefix by its accumulated roundings (measured max ~35 ulp at 20 k elements).  So
// every segment is run from 256 candidate starts -- the floats whose order keys are key(c_j)
// - 128 .. key(c_j) + 127, one per lane -- and a link pass walks the segments in order: the
// running value s picks the candidate whose start has s's exact bits, and that candidate's
// end IS op_{jL+L-1}(...op_{jL}(s)) -- same bits in, same IEEE operations, same bits out.  A
// start outside the window (or a non-finite one) falls back to the plain sequential walk of
// that one segment.  The result is therefore the sequential sum, whatever the data; the
// centres only decide how often the fallback runs.
//
// Layout of one fit's scratch (seqsum_scratch_bytes(nch)): psum[kSegMax][nch] doubles (the
// fp64 segment sums), then R[kSegMax][nch][kCand] floats (every candidate's segment end).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "usac_kernels.h"
#include "usac_seqsum.hpp"

namespace usac {

using namespace seq;

// fp64 segment sums: workgroup (segment j, fit b), any order (they only place the centres)
template <int NCH, bool F64>
__global__ __launch_bounds__(256) void k_seq_psum(const typename Op<F64>::V *__restrict__ vals, size_t vstride,
                                                  const uint32_t *__restrict__ ns, uint32_t n1,
                                                  const uint32_t *__restrict__ slots, char *scratch, size_t sstride) {
    __shared__ double red[NCH][256];
    const uint32_t j = blockIdx.x, w = fit_slot(slots, blockIdx.y);
    const uint32_t n = fit_n(ns, n1, w), L = seg_len(n);
    if (j * L >= n) return;
    const uint32_t e = (j + 1) * L < n ? (j + 1) * L : n;
    const typename Op<F64>::V *v = vals + w * vstride;
    double acc[NCH];
#pragma unroll
    for (int q = 0; q < NCH; q++) acc[q] = 0.0;
    for (uint32_t k0 = j * L + threadIdx.x; k0 < e; k0 += 4 * 256) {  // four elements' loads in flight
        typename Op<F64>::V x[4][NCH];
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int q = 0; q < NCH; q++) {
                const uint32_t k = k0 + 256 * u;
                x[u][q] = k < e ? v[(size_t)k * NCH + q] : typename Op<F64>::V(0);
            }
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int q = 0; q < NCH; q++) acc[q] += Op<F64>::wide(x[u][q]);
    }
#pragma unroll
    for (int q = 0; q < NCH; q++) red[q][threadIdx.x] = acc[q];
    __syncthreads();
    for (uint32_t h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h)
#pragma unroll
            for (int q = 0; q < NCH; q++) red[q][threadIdx.x] += red[q][threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x < NCH) reinterpret_cast<double *>(scratch + w * sstride)[j * NCH + threadIdx.x] = red[threadIdx.x][0];
}

// every candidate's segment end: workgroup (segment j, fit b), lane = candidate, NCH
// independent chains per lane.  The segment streams through LDS in chunks (every thread
// loads a strided share of the next chunk into registers while the chains run over the
// current one; one barrier per chunk), so each step reads its element by a broadcast
// ds_read instead of waiting on a load.
template <int NCH, bool F64>
__global__ __launch_bounds__(kCand) void k_seq_seg(const typename Op<F64>::V *__restrict__ vals, size_t vstride,
                                                   const uint32_t *__restrict__ ns, uint32_t n1,
                                                   const uint32_t *__restrict__ slots, char *scratch, size_t sstride) {
    typedef typename Op<F64>::V V;
    constexpr uint32_t kChunk = (NCH == 1 ? 8 : 4) * kCand;  // elements per LDS chunk (2048 / 1024 at 256 candidates)
    constexpr uint32_t kPer = kChunk * NCH / kCand;      // values per thread per chunk
    __shared__ V sv[2][kChunk * NCH];
    __shared__ double sp[kSegMax * NCH];
    const uint32_t j = blockIdx.x, w = fit_slot(slots, blockIdx.y);
    const uint32_t n = fit_n(ns, n1, w), L = seg_len(n);
    if (j * L >= n) return;
    const uint32_t b = j * L, e = b + L < n ? b + L : n;
    const double *psum = reinterpret_cast<const double *>(scratch + w * sstride);
    float *R = reinterpret_cast<float *>(scratch + w * sstride + sizeof(double) * kSegMax * NCH);
    const V *__restrict__ v = vals + w * vstride + (size_t)b * NCH;
    const uint32_t tot = (e - b) * NCH;  // values of the segment
    const uint32_t t = threadIdx.x;
    V pre[kPer];
    auto fetch = [&](uint32_t c) {
#pragma unroll
        for (uint32_t u = 0; u < kPer; u++) {
            const uint32_t i = c * kChunk * NCH + t + kCand * u;
            pre[u] = i < tot ? v[i] : V(0);
        }
    };
    fetch(0);
    // the earlier segments' sums through LDS (one parallel load, not a dependent load per add)
    for (uint32_t i = t; i < j * NCH; i += kCand) sp[i] = psum[i];
    __syncthreads();
    float s[NCH];
#pragma unroll
    for (int q = 0; q < NCH; q++) s[q] = cand_start(centre(sp, j, NCH, q), t);
    const uint32_t nch = (e - b + kChunk - 1) / kChunk;
    for (uint32_t c = 0; c < nch; c++) {
        V *buf = sv[c & 1];
#pragma unroll
        for (uint32_t u = 0; u < kPer; u++) buf[t + kCand * u] = pre[u];
        __syncthreads();
        if (c + 1 < nch) fetch(c + 1);
        const uint32_t m = e - b - c * kChunk < kChunk ? e - b - c * kChunk : kChunk;
        uint32_t k = 0;
        for (; k + 8 <= m; k += 8) {
            V x[8][NCH];
#pragma unroll
            for (int u = 0; u < 8; u++)
#pragma unroll
                for (int q = 0; q < NCH; q++) x[u][q] = buf[(k + u) * NCH + q];
#pragma unroll
            for (int u = 0; u < 8; u++)
#pragma unroll
                for (int q = 0; q < NCH; q++) s[q] = Op<F64>::step(s[q], x[u][q]);
        }
        for (; k < m; k++)
#pragma unroll
            for (int q = 0; q < NCH; q++) s[q] = Op<F64>::step(s[q], buf[k * NCH + q]);
    }
#pragma unroll
    for (int q = 0; q < NCH; q++) R[((size_t)j * NCH + q) * kCand + t] = s[q];
}

// The same segment ends with the chains split over the waves: workgroup (segment j, fit b) of
// kCand * NCH / CPL threads, thread t runs chain q = t / (kCand / CPL) (wave-uniform) from the
// CPL candidates c + u kCand / CPL, c = t % (kCand / CPL) -- CPL independent dependent chains
// per lane, every element read once from LDS for all of them.  The chunk is staged transposed
// ([chain][element]) so a wave reads its chain's next elements with 16-byte broadcast reads.
// Same starts, same ops, same ends.
template <int NCH, bool F64, int CPL>
__global__ __launch_bounds__(kCand *NCH / CPL) void k_seq_seg_split(const typename Op<F64>::V *__restrict__ vals,
                                                                    size_t vstride, const uint32_t *__restrict__ ns,
                                                                    uint32_t n1, const uint32_t *__restrict__ slots,
                                                                    char *scratch, size_t sstride) {
    typedef typename Op<F64>::V V;
    constexpr uint32_t kLanes = kCand / CPL;             // threads per chain
    static_assert(kLanes % 64 == 0, "a chain's threads are whole waves");
    constexpr uint32_t kT = kLanes * NCH;                // threads
    constexpr uint32_t kChunk = 1024;                    // elements per LDS chunk
    constexpr uint32_t kPer = kChunk * NCH / kT;         // values per thread per chunk (4 CPL)
    constexpr uint32_t kVec = 16 / sizeof(V);            // elements per 16-byte read
    typedef V Vv __attribute__((ext_vector_type(kVec)));
    __shared__ __attribute__((aligned(16))) V sv[2][NCH][kChunk + kVec];  // rows padded 16 B: no bank conflicts
    __shared__ double sp[kSegMax * NCH];
    const uint32_t j = blockIdx.x, w = fit_slot(slots, blockIdx.y);
    const uint32_t n = fit_n(ns, n1, w), L = seg_len(n);
    if (j * L >= n) return;
    const uint32_t b = j * L, e = b + L < n ? b + L : n;
    const double *psum = reinterpret_cast<const double *>(scratch + w * sstride);
    float *R = reinterpret_cast<float *>(scratch + w * sstride + sizeof(double) * kSegMax * NCH);
    const V *__restrict__ v = vals + w * vstride + (size_t)b * NCH;
    const uint32_t tot = (e - b) * NCH;
    const uint32_t t = threadIdx.x;
    const uint32_t q = __builtin_amdgcn_readfirstlane(t / kLanes), c = t % kLanes;
    V pre[kPer];
    auto fetch = [&](uint32_t ch) {
#pragma unroll
        for (uint32_t u = 0; u < kPer; u++) {
            const uint32_t i = ch * kChunk * NCH + t + kT * u;
            pre[u] = i < tot ? v[i] : V(0);
        }
    };
    fetch(0);
    for (uint32_t i = t; i < j * NCH; i += kT) sp[i] = psum[i];
    __syncthreads();
    float s[CPL];
    {
        const float ctr = centre(sp, j, NCH, q);
#pragma unroll
        for (int u = 0; u < CPL; u++) s[u] = cand_start(ctr, c + kLanes * u);
    }
    const uint32_t nch = (e - b + kChunk - 1) / kChunk;
    for (uint32_t ch = 0; ch < nch; ch++) {
#pragma unroll
        for (uint32_t u = 0; u < kPer; u++) {
            const uint32_t i = t + kT * u;  // value i of the chunk: element i / NCH, chain i % NCH
            sv[ch & 1][i % NCH][i / NCH] = pre[u];
        }
        __syncthreads();
        if (ch + 1 < nch) fetch(ch + 1);
        const V *buf = sv[ch & 1][q];
        const uint32_t m = e - b - ch * kChunk < kChunk ? e - b - ch * kChunk : kChunk;
        uint32_t k = 0;
        for (; k + 8 <= m; k += 8) {
            Vv x[8 / kVec];
#pragma unroll
            for (uint32_t u = 0; u < 8 / kVec; u++) x[u] = *reinterpret_cast<const Vv *>(buf + k + kVec * u);
#pragma unroll
            for (uint32_t u = 0; u < 8 / kVec; u++)
#pragma unroll
                for (uint32_t z = 0; z < kVec; z++)
#pragma unroll
                    for (int a = 0; a < CPL; a++) s[a] = Op<F64>::step(s[a], x[u][z]);
        }
        for (; k < m; k++) {
            const V x = buf[k];
#pragma unroll
            for (int a = 0; a < CPL; a++) s[a] = Op<F64>::step(s[a], x);
        }
    }
#pragma unroll
    for (int a = 0; a < CPL; a++) R[((size_t)j * NCH + q) * kCand + c + kLanes * a] = s[a];
}

// link: workgroup (chain q, fit b); the four waves stage the chain's candidate ends into
// LDS, then wave 0 walks the segments (every lane the same value)
template <int NCH, bool F64>
__global__ __launch_bounds__(256) void k_seq_link(const typename Op<F64>::V *__restrict__ vals, size_t vstride,
                                                  const uint32_t *__restrict__ ns, uint32_t n1,
                                                  const uint32_t *__restrict__ slots, const char *scratch,
                                                  size_t sstride, float *__restrict__ out) {
    __shared__ float sR[kSegMax][kCand];
    __shared__ double sp[kSegMax];
    const uint32_t q = blockIdx.x, w = fit_slot(slots, blockIdx.y);
    const uint32_t n = fit_n(ns, n1, w), L = seg_len(n);
    const uint32_t S = (n + L - 1) / L;
    const double *psum = reinterpret_cast<const double *>(scratch + w * sstride);
    const float *R = reinterpret_cast<const float *>(scratch + w * sstride + sizeof(double) * kSegMax * NCH);
    static_assert(kCand == 256, "thread = candidate");
    // every row's load in flight at once (the scratch holds kSegMax rows; rows >= S are read and
    // dropped): a strided loop here was one dependent round trip per row, ~14 us per link
    float r[kSegMax];
#pragma unroll
    for (uint32_t j = 0; j < kSegMax; j++) r[j] = R[((size_t)j * NCH + q) * kCand + threadIdx.x];
    if (threadIdx.x < S) sp[threadIdx.x] = psum[threadIdx.x * NCH + q];
#pragma unroll
    for (uint32_t j = 0; j < kSegMax; j++)
        if (j < S) sR[j][threadIdx.x] = r[j];
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const typename Op<F64>::V *__restrict__ v = vals + w * vstride;
    float s = 0.f;
    double pre = 0.0;  // centre(psum, j, NCH, q) incrementally: the same fp64 adds in the same order
    for (uint32_t j = 0; j < S; j++) {
        if (j) pre += sp[j - 1];
        const float ctr = (float)pre;
        const int64_t idx = (int64_t)key(s) - (int64_t)key(ctr) + (int64_t)(kCand / 2);
        bool hit = false;
        if (idx >= 0 && idx < (int64_t)kCand) {
            const uint32_t c = (uint32_t)idx;
            if (__float_as_uint(cand_start(ctr, c)) == __float_as_uint(s)) {
                s = sR[j][c];
                hit = true;
            }
        }
        if (!hit) {  // the plain sequential walk of segment j
            const uint32_t b = j * L, e = b + L < n ? b + L : n;
            uint32_t k = b;
            for (; k + 8 <= e; k += 8) {  // eight loads in flight per eight dependent steps
                typename Op<F64>::V x[8];
#pragma unroll
                for (int u = 0; u < 8; u++) x[u] = v[(size_t)(k + u) * NCH + q];
#pragma unroll
                for (int u = 0; u < 8; u++) s = Op<F64>::step(s, x[u]);
            }
            for (; k < e; k++) s = Op<F64>::step(s, v[(size_t)k * NCH + q]);
        }
    }
    if (threadIdx.x == 0) out[(size_t)w * NCH + q] = s;
}

size_t seqsum_scratch_bytes(int nch) { return scratch_bytes(nch); }

// multi-chain segment kernel: chains split over waves (default) or interleaved per lane
// (USAC_SEQ_SPLIT=0, the round-3 kernel; kept for A/B)
static bool seg_split() {
    static const bool on = [] {
        const char *e = getenv("USAC_SEQ_SPLIT");
        return !e || atoi(e) != 0;
    }();
    return on;
}
// candidates per lane of the split kernel: 2 for the fp32 chains (the four coordinate means:
// 15.9 -> 12.8 us per fit batch), 1 for the fp64-addend ones (21.3 / 21.2 us with 1 / 2, 27.8
// with 4); USAC_SEQ_CPL = 1, 2 or 4 sets both, for A/B
static int seg_cpl(bool f64) {
    static const int cpl = [] {
        const char *e = getenv("USAC_SEQ_CPL");
        const int v = e ? atoi(e) : 0;
        return v == 1 || v == 2 || v == 4 ? v : 0;
    }();
    return cpl ? cpl : f64 ? 1 : 2;
}
// one-chain sums (Σerr) through the split kernel with this many candidates per lane
// (USAC_SEQ1_CPL = 1, 2 or 4; unset or 0: k_seq_seg).  One per lane runs as fast as k_seq_seg
// (6.7 / 6.8 us) with half its LDS; the cfg5 / cfg3-exact lines split both ways over two boxes
// (DESIGN §7 round 6), so k_seq_seg stays the default
static int seg1_cpl() {
    static const int cpl = [] {
        const char *e = getenv("USAC_SEQ1_CPL");
        const int v = e ? atoi(e) : 0;
        return v == 1 || v == 2 || v == 4 ? v : 0;
    }();
    return cpl;
}

hipError_t launch_seqsum(hipStream_t st, int nch, bool f64, const void *vals, size_t vstride, const uint32_t *ns,
                         uint32_t n1, uint32_t W, const uint32_t *slots, void *scratch, size_t sstride,
                         bool have_psum, float *out) {
    if (W == 0) return hipSuccess;
    const dim3 gs(kSegMax, W), gl(nch, W);
    char *scr = static_cast<char *>(scratch);
#define SEQ(N, D)                                                                                                   \
    do {                                                                                                            \
        typedef typename Op<D>::V V_;                                                                               \
        const V_ *v_ = static_cast<const V_ *>(vals);                                                               \
        if (!have_psum)                                                                                             \
            hipLaunchKernelGGL((k_seq_psum<N, D>), gs, dim3(256), 0, st, v_, vstride, ns, n1, slots, scr, sstride); \
        if (N == 1 && seg1_cpl() == 2)                                                                              \
            hipLaunchKernelGGL((k_seq_seg_split<N, D, 2>), gs, dim3(kCand * N / 2), 0, st, v_, vstride, ns, n1, slots, \
                               scr, sstride);                                                                       \
        else if (N == 1 && seg1_cpl() == 4)                                                                         \
            hipLaunchKernelGGL((k_seq_seg_split<N, D, 4>), gs, dim3(kCand * N / 4), 0, st, v_, vstride, ns, n1, slots, \
                               scr, sstride);                                                                       \
        else if (N == 1 && seg1_cpl() == 1)                                                                         \
            hipLaunchKernelGGL((k_seq_seg_split<N, D, 1>), gs, dim3(kCand * N), 0, st, v_, vstride, ns, n1, slots,     \
                               scr, sstride);                                                                       \
        else if (N > 1 && seg_split() && seg_cpl(D) == 4)                                                                 \
            hipLaunchKernelGGL((k_seq_seg_split<N, D, 4>), gs, dim3(kCand * N / 4), 0, st, v_, vstride, ns, n1, slots, \
                               scr, sstride);                                                                       \
        else if (N > 1 && seg_split() && seg_cpl(D) == 2)                                                            \
            hipLaunchKernelGGL((k_seq_seg_split<N, D, 2>), gs, dim3(kCand * N / 2), 0, st, v_, vstride, ns, n1, slots, \
                               scr, sstride);                                                                       \
        else if (N > 1 && seg_split())                                                                              \
            hipLaunchKernelGGL((k_seq_seg_split<N, D, 1>), gs, dim3(kCand * N), 0, st, v_, vstride, ns, n1, slots,     \
                               scr, sstride);                                                                       \
        else                                                                                                        \
            hipLaunchKernelGGL((k_seq_seg<N, D>), gs, dim3(kCand), 0, st, v_, vstride, ns, n1, slots, scr, sstride);  \
        hipLaunchKernelGGL((k_seq_link<N, D>), gl, dim3(256), 0, st, v_, vstride, ns, n1, slots, scr, sstride, out); \
    } while (0)
    if (nch == 1 && !f64) SEQ(1, false);
    else if (nch == 4 && !f64) SEQ(4, false);
    else if (nch == 2 && f64) SEQ(2, true);
    else return hipErrorInvalidValue;
#undef SEQ
    return hipGetLastError();
}

}  // namespace usac
