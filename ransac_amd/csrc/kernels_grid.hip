// kernels_grid.hip -- grid neighbours on the device (NearestNeighbors::getGridNearestNeighbors,
// usac/utils/nearest_neighbors.cpp:160-202) and the eligible-point list of the NAPSAC
// throughput sampler (napsac_sampler.hpp:100-138).
//
// The reference's neighbours of point i are the other points of its 4-D cell
// ((int)(x1/cs), (int)(y1/cs), (int)(x2/cs), (int)(y2/cs)) -- fp32 division, truncation --
// in ascending index order.  Built here as a CSR that is bit-identical to the host
// GridNeighbors (usac_host.hpp): cell[i] (cells numbered in order of first appearance in
// point order), rank[i] (i's position in its cell), start[c] (n_cells + 1), members (cells in
// order, ascending index within a cell).  Point i's k-th neighbour is
// members[start[cell[i]] + (k < rank[i] ? k : k + 1)].
//
// No sort: the cells are grouped through an open-addressing hash table of the packed cell
// keys, and first-appearance order is a scan in point order.  Seven launches, one host wait:
//   K0 k_grid_clear    the table (its memory is recycled between builds);
//   K1 k_grid_insert   per point: the packed key (per dimension the bits of the box's cell
//                      range plus an out-of-box sentinel), its slot (linear probing, 64-bit
//                      CAS), the cell's smallest index (atomicMin) and size (atomicAdd, whose
//                      return value is the point's unordered place in the cell);
//   K2 k_grid_part     per 1024-point block: heads (points that are their cell's smallest
//                      index), the heads' cell sizes, NAPSAC-eligible points (>= m neighbours,
//                      Q18);
//   K3 k_grid_emit     each block sums its predecessors' partials, then scans its points in
//                      index order: a head's cell number (= order of first appearance) and
//                      start, the eligible list (ascending), the totals from the last block;
//   K4 k_grid_scatter  cell[i], and i written to its unordered place in its cell's segment;
//   K5 k_grid_small    one lane per cell of <= 16 members: rank by counting smaller members,
//                      members written in order; larger cells queued;
//   K6 k_grid_big      one workgroup per queued cell: the members as a bitmap over the index
//                      range in LDS, rank = popcount prefix.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <thread>

#include "usac_kernels.h"

namespace usac {

namespace {

constexpr uint64_t kEmpty = ~0ull;       // no key reaches it: keys are at most 63 bits
constexpr uint32_t kPartPts = 1024;      // points per K2/K3 block (4 per thread)
constexpr uint32_t kSmallCell = 16;      // cells up to this size are ranked by one lane
constexpr uint32_t kBmWords = 8192;      // LDS bitmap chunk of K6: 262 144 indices
constexpr uint32_t kBigBlocks = 256;
// k_grid_big holds the bitmap and its per-word prefix (2 x 32 KiB) plus 16 B in LDS: 65 552 B per
// workgroup, above the 64 KiB of gfx90a / gfx942 and within gfx950's 160 KiB (MI355X_MICROARCH.md).
// This build targets gfx950 only (ransac_amd/Makefile ARCH); the bound is checked here.
static_assert(2 * kBmWords * sizeof(uint32_t) + 4 * sizeof(uint32_t) <= 160 * 1024,
              "k_grid_big's LDS exceeds gfx950's 160 KiB per workgroup");

__device__ __forceinline__ uint32_t hash_slot(uint64_t k, uint32_t mask) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return (uint32_t)k & mask;
}

// wave-inclusive scan of three counters (64 lanes)
__device__ __forceinline__ void wave_scan3(uint32_t &a, uint32_t &b, uint32_t &c) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t ta = __shfl_up(a, d), tb = __shfl_up(b, d), tc = __shfl_up(c, d);
        if (lane >= d) {
            a += ta;
            b += tb;
            c += tc;
        }
    }
}

}  // namespace

__global__ __launch_bounds__(256) void k_grid_clear(uint64_t *__restrict__ tkey, uint32_t *__restrict__ tmin,
                                                    uint32_t *__restrict__ tcnt, uint32_t T,
                                                    uint32_t *__restrict__ counts) {
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s < T) {
        tkey[s] = kEmpty;
        tmin[s] = 0xffffffffu;
        tcnt[s] = 0;
    }
    if (s < 4) counts[s] = 0;
}

__global__ __launch_bounds__(256) void k_grid_insert(const float4 *__restrict__ pts, uint32_t n, float cs, int4 cmin,
                                                     int4 bits, uint64_t *__restrict__ tkey,
                                                     uint32_t *__restrict__ tmin, uint32_t *__restrict__ tcnt,
                                                     uint32_t mask, uint32_t *__restrict__ slot,
                                                     uint32_t *__restrict__ pos) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 p = pts[i];
    const float v[4] = {p.x, p.y, p.z, p.w};
    const int lo[4] = {cmin.x, cmin.y, cmin.z, cmin.w};
    const int bw[4] = {bits.x, bits.y, bits.z, bits.w};
    uint64_t k = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int top = (1 << bw[j]) - 1;  // above every cell of the box: the out-of-box sentinel
        int c = (int)(v[j] / cs) - lo[j];  // IEEE fp32 division, truncation (as the reference)
        c = c < 0 ? 0 : c > top ? top : c;  // only non-finite coordinates leave the box
        k = (k << bw[j]) | (uint64_t)c;
    }
    // A slot's key changes once, from kEmpty to its final value, so a plain read returns either
    // the final key or a (possibly stale) kEmpty, which the CAS then settles.
    uint32_t s = hash_slot(k, mask);
    for (;;) {  // the table has >= 2n slots: a free one is always reached
        uint64_t cur = tkey[s];
        if (cur == kEmpty)
            cur = atomicCAS(reinterpret_cast<unsigned long long *>(tkey + s), (unsigned long long)kEmpty,
                            (unsigned long long)k);
        if (cur == kEmpty || cur == k) break;
        s = (s + 1) & mask;
    }
    // The lanes sharing the first active lane's slot (one cell holding most points is the
    // degenerate case that would serialise on one address) take one atomic for the group: its
    // smallest index is the first lane's, places are handed out in lane order.
    const uint32_t s0 = __builtin_amdgcn_readfirstlane(s);
    const uint64_t peers = __ballot(s == s0);
    const bool lead = (__lanemask_lt() & peers) == 0;
    uint32_t at;
    if (s == s0) {
        uint32_t base = 0;
        if (lead) {
            if (i < tmin[s]) atomicMin(tmin + s, i);
            base = atomicAdd(tcnt + s, (uint32_t)__popcll(peers));
        }
        at = __shfl(base, (int)__ffsll((long long)peers) - 1) + (uint32_t)__popcll(peers & __lanemask_lt());
    } else {
        // a stale tmin only over-states the minimum: skipping the atomic when i is above it is safe
        if (i < tmin[s]) atomicMin(tmin + s, i);
        at = atomicAdd(tcnt + s, 1u);
    }
    pos[i] = at;  // i's (unordered) place in its cell's segment
    slot[i] = s;
}

// per block of kPartPts points: (heads, sizes of the heads' cells, eligible points)
__global__ __launch_bounds__(256) void k_grid_part(const uint32_t *__restrict__ slot, const uint32_t *__restrict__ tmin,
                                                   const uint32_t *__restrict__ tcnt, uint32_t n, uint32_t m,
                                                   uint32_t *__restrict__ part) {
    __shared__ uint32_t red[3][4];
    uint32_t h = 0, sz = 0, el = 0;
    const uint32_t base = blockIdx.x * kPartPts;
#pragma unroll
    for (uint32_t j = 0; j < kPartPts / 256; j++) {
        const uint32_t i = base + j * 256 + threadIdx.x;
        if (i < n) {
            const uint32_t s = slot[i], cnt = tcnt[s];
            const bool head = tmin[s] == i;
            h += head;
            sz += head ? cnt : 0u;
            el += (cnt - 1 >= m);
        }
    }
    wave_scan3(h, sz, el);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) {
        red[0][w] = h;
        red[1][w] = sz;
        red[2][w] = el;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const uint32_t *r = red[threadIdx.x];
        part[3 * blockIdx.x + threadIdx.x] = r[0] + r[1] + r[2] + r[3];
    }
}

__global__ __launch_bounds__(256) void k_grid_emit(const uint32_t *__restrict__ slot, const uint32_t *__restrict__ tmin,
                                                   const uint32_t *__restrict__ tcnt, const uint32_t *__restrict__ part,
                                                   uint32_t n, uint32_t m, uint32_t *__restrict__ tcell,
                                                   uint32_t *__restrict__ cslot, uint32_t *__restrict__ start,
                                                   int32_t *__restrict__ eligible, uint32_t *__restrict__ counts) {
    __shared__ uint32_t red[3][4];
    __shared__ uint32_t pre[3];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // predecessors' totals
    uint32_t ph = 0, ps = 0, pe = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += 256) {
        ph += part[3 * b];
        ps += part[3 * b + 1];
        pe += part[3 * b + 2];
    }
    wave_scan3(ph, ps, pe);
    if (lane == 63) {
        red[0][w] = ph;
        red[1][w] = ps;
        red[2][w] = pe;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const uint32_t *r = red[threadIdx.x];
        pre[threadIdx.x] = r[0] + r[1] + r[2] + r[3];
    }
    __syncthreads();
    // this thread's four consecutive points, scanned in index order
    const uint32_t i0 = blockIdx.x * kPartPts + 4 * threadIdx.x;
    uint32_t s4[4], c4[4];
    bool hd[4];
    uint32_t h = 0, sz = 0, el = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t i = i0 + j;
        s4[j] = 0;
        c4[j] = 0;
        hd[j] = false;
        if (i < n) {
            s4[j] = slot[i];
            c4[j] = tcnt[s4[j]];
            hd[j] = tmin[s4[j]] == i;
            h += hd[j];
            sz += hd[j] ? c4[j] : 0u;
            el += (c4[j] - 1 >= m);
        }
    }
    uint32_t ih = h, is = sz, ie = el;
    wave_scan3(ih, is, ie);
    __syncthreads();  // red[] reused
    if (lane == 63) {
        red[0][w] = ih;
        red[1][w] = is;
        red[2][w] = ie;
    }
    __syncthreads();
    uint32_t q = pre[0] + ih - h, st = pre[1] + is - sz, e = pre[2] + ie - el;
    for (int v = 0; v < w; v++) {
        q += red[0][v];
        st += red[1][v];
        e += red[2][v];
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t i = i0 + j;
        if (i >= n) break;
        if (hd[j]) {
            tcell[s4[j]] = q;
            cslot[q] = s4[j];
            start[q] = st;
            q++;
            st += c4[j];
        }
        if (c4[j] - 1 >= m) eligible[e++] = (int32_t)i;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 255) {  // the last point's totals
        start[q] = n;
        counts[0] = q;  // cells
        counts[1] = e;  // eligible points
    }
}

__global__ __launch_bounds__(256) void k_grid_scatter(const uint32_t *__restrict__ slot,
                                                      const uint32_t *__restrict__ pos,
                                                      const uint32_t *__restrict__ tcell,
                                                      const uint32_t *__restrict__ start, uint32_t n,
                                                      uint32_t *__restrict__ cell, int32_t *__restrict__ unordered) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t q = tcell[slot[i]];
    cell[i] = q;
    unordered[start[q] + pos[i]] = (int32_t)i;
}

// one lane per cell of <= kSmallCell members; larger cells queued for k_grid_big
__global__ __launch_bounds__(256) void k_grid_small(const uint32_t *__restrict__ start,
                                                    const int32_t *__restrict__ unordered,
                                                    uint32_t *__restrict__ counts, uint32_t *__restrict__ rank,
                                                    int32_t *__restrict__ members, uint32_t *__restrict__ big) {
    const uint32_t nc = counts[0];
    for (uint32_t q = blockIdx.x * 256 + threadIdx.x; q < nc; q += gridDim.x * 256) {
        const uint32_t b = start[q], s = start[q + 1] - b;
        if (s > kSmallCell) {
            big[atomicAdd(counts + 2, 1u)] = q;
            continue;
        }
        if (s == 1) {
            const int32_t a = unordered[b];
            members[b] = a;
            rank[a] = 0;
            continue;
        }
        int32_t v[kSmallCell];
#pragma unroll
        for (uint32_t k = 0; k < kSmallCell; k++) v[k] = k < s ? unordered[b + k] : 0x7fffffff;
#pragma unroll
        for (uint32_t j = 0; j < kSmallCell; j++) {
            if (j < s) {
                uint32_t r = 0;
#pragma unroll
                for (uint32_t k = 0; k < kSmallCell; k++) r += v[k] < v[j];
                members[b + r] = v[j];
                rank[v[j]] = r;
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_grid_big(const uint32_t *__restrict__ start,
                                                  const int32_t *__restrict__ unordered,
                                                  const uint32_t *__restrict__ counts,
                                                  const uint32_t *__restrict__ big,
                                                  const uint32_t *__restrict__ cslot,
                                                  const uint32_t *__restrict__ tmin, uint32_t n,
                                                  uint32_t *__restrict__ rank, int32_t *__restrict__ members) {
    __shared__ uint32_t bm[kBmWords];
    __shared__ uint32_t wpre[kBmWords];
    __shared__ uint32_t red[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t nbig = counts[2];
    for (uint32_t t = blockIdx.x; t < nbig; t += gridDim.x) {
        const uint32_t q = big[t], b = start[q], s = start[q + 1] - b;
        uint32_t carry = 0;
        for (uint32_t cb = tmin[cslot[q]]; cb < n; cb += kBmWords * 32) {  // the smallest member starts
            for (uint32_t k = threadIdx.x; k < kBmWords; k += 256) bm[k] = 0;
            __syncthreads();
            for (uint32_t j = threadIdx.x; j < s; j += 256) {
                const uint32_t a = (uint32_t)unordered[b + j] - cb;
                if (a < kBmWords * 32) atomicOr(bm + (a >> 5), 1u << (a & 31));
            }
            __syncthreads();
            // popcount prefix over the chunk's words: 32 consecutive words per thread
            const uint32_t w0 = threadIdx.x * (kBmWords / 256);
            uint32_t tot = 0;
            for (uint32_t k = 0; k < kBmWords / 256; k++) tot += __popc(bm[w0 + k]);
            uint32_t inc = tot;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t x = __shfl_up(inc, d);
                if (lane >= d) inc += x;
            }
            if (lane == 63) red[w] = inc;
            __syncthreads();
            uint32_t run = carry + inc - tot;
            for (int v = 0; v < w; v++) run += red[v];
            const uint32_t chunk_total = red[0] + red[1] + red[2] + red[3];
            for (uint32_t k = 0; k < kBmWords / 256; k++) {
                wpre[w0 + k] = run;
                run += __popc(bm[w0 + k]);
            }
            __syncthreads();
            for (uint32_t j = threadIdx.x; j < s; j += 256) {
                const int32_t ai = unordered[b + j];
                const uint32_t a = (uint32_t)ai - cb;
                if (a < kBmWords * 32) {
                    const uint32_t r = wpre[a >> 5] + __popc(bm[a >> 5] & ((1u << (a & 31)) - 1u));
                    members[b + r] = ai;
                    rank[ai] = r;
                }
            }
            carry += chunk_total;
            __syncthreads();  // bm / wpre / red reused by the next chunk or cell
            if (carry == s) break;
        }
    }
}

namespace {

// scratch carve-out of the build
struct GridScratch {
    uint64_t *tkey;
    uint32_t *tmin, *tcnt, *pos, *tcell, *slot, *cslot, *part, *big, *counts;
    int32_t *unordered;
    uint32_t T;
};

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

uint32_t table_slots(uint32_t n) {
    uint32_t T = 1024;
    while (T < 2 * (size_t)n) T <<= 1;
    return T;
}

template <class F>
size_t lay_out(uint32_t n, F &&take) {
    const uint32_t T = table_slots(n);
    const size_t u = sizeof(uint32_t) * ((size_t)n + 1), t = sizeof(uint32_t) * (size_t)T;
    const size_t nb = (n + kPartPts - 1) / kPartPts;
    size_t total = 0;
    total += take(0, sizeof(uint64_t) * (size_t)T);
    for (int k = 1; k <= 3; k++) total += take(k, t);  // tmin, tcnt, tcell
    for (int k = 4; k <= 8; k++) total += take(k, u);  // pos, slot, cslot, big, unordered
    total += take(9, sizeof(uint32_t) * 3 * nb);       // part
    total += take(10, sizeof(uint32_t) * 4);           // counts
    return total;
}

GridScratch carve(void *ws, uint32_t n) {
    GridScratch s;
    s.T = table_slots(n);
    char *p = static_cast<char *>(ws);
    void *ptr[11];
    lay_out(n, [&](int k, size_t bytes) {
        ptr[k] = p;
        p += align256(bytes);
        return align256(bytes);
    });
    s.tkey = (uint64_t *)ptr[0];
    s.tmin = (uint32_t *)ptr[1];
    s.tcnt = (uint32_t *)ptr[2];
    s.tcell = (uint32_t *)ptr[3];
    s.pos = (uint32_t *)ptr[4];
    s.slot = (uint32_t *)ptr[5];
    s.cslot = (uint32_t *)ptr[6];
    s.big = (uint32_t *)ptr[7];
    s.unordered = (int32_t *)ptr[8];
    s.part = (uint32_t *)ptr[9];
    s.counts = (uint32_t *)ptr[10];
    return s;
}

}  // namespace

size_t grid_workspace_bytes(uint32_t n) {
    return lay_out(n, [](int, size_t bytes) { return align256(bytes); }) + 256;
}

#define GRID_TRY(expr)                      \
    do {                                    \
        hipError_t e_ = (expr);             \
        if (e_ != hipSuccess) return e_;    \
    } while (0)

// wait for the stream by polling (a blocking synchronise adds a ~20 us wake-up; usac_api.cpp
// stream_wait does the same for the loop's waits)
static hipError_t poll_stream(hipStream_t st) {
    for (uint32_t spins = 0;; spins++) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) return e;
        if ((spins & 1023u) == 1023u) std::this_thread::yield();
    }
}

hipError_t build_grid(hipStream_t st, const float4 *pts, uint32_t n, int cell_size, int4 cmin, int4 bits, uint32_t m,
                      void *ws, uint32_t *cell, uint32_t *rank, uint32_t *start, int32_t *members, int32_t *eligible,
                      uint32_t *pinned2, uint32_t *n_cells_out, uint32_t *n_elig_out) {
    if (n == 0 || n > 0x7fffffffu) return hipErrorInvalidValue;
    if (bits.x + bits.y + bits.z + bits.w > 63) return hipErrorInvalidValue;  // kEmpty stays unreachable
    GridScratch s = carve(ws, n);
    const dim3 b(256), g((n + 255) / 256);
    const uint32_t nb = (n + kPartPts - 1) / kPartPts;
    hipLaunchKernelGGL(k_grid_clear, dim3((s.T + 255) / 256), b, 0, st, s.tkey, s.tmin, s.tcnt, s.T, s.counts);
    GRID_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_grid_insert, g, b, 0, st, pts, n, (float)cell_size, cmin, bits, s.tkey, s.tmin, s.tcnt,
                       s.T - 1, s.slot, s.pos);
    GRID_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_grid_part, dim3(nb), b, 0, st, s.slot, s.tmin, s.tcnt, n, m, s.part);
    GRID_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_grid_emit, dim3(nb), b, 0, st, s.slot, s.tmin, s.tcnt, s.part, n, m, s.tcell, s.cslot, start,
                       eligible, s.counts);
    GRID_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_grid_scatter, g, b, 0, st, s.slot, s.pos, s.tcell, start, n, cell, s.unordered);
    GRID_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_grid_small, dim3(std::min<uint32_t>(g.x, 1024)), b, 0, st, start, s.unordered, s.counts, rank,
                       members, s.big);
    GRID_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_grid_big, dim3(kBigBlocks), b, 0, st, start, s.unordered, s.counts, s.big, s.cslot, s.tmin, n,
                       rank, members);
    GRID_TRY(hipGetLastError());
    GRID_TRY(hipMemcpyAsync(pinned2, s.counts, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    GRID_TRY(poll_stream(st));
    *n_cells_out = pinned2[0];
    *n_elig_out = pinned2[1];
    return hipSuccess;
}

}  // namespace usac
