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
// Pipeline (rocPRIM device primitives for the sort and scans):
//   1. k_grid_keys     per point: the packed cell key (per dimension just the bits of the
//                      box's cell range plus a sentinel, offset by its lowest cell) and index;
//   2. radix sort      (key, index) pairs -- stable, so a cell's members stay ascending;
//   3. k_grid_heads    1 where the sorted key changes; inclusive scan -> cell id (key order);
//   4. k_grid_cells    per key-order cell: first position and first (= smallest) member;
//   5. radix sort      key-order cells by their smallest member = order of first appearance;
//   6. k_grid_renumber size of each cell in first-appearance order; exclusive scan -> start;
//   7. k_grid_scatter  cell / rank / members per point, eligibility (>= m neighbours, Q18);
//   8. exclusive scan + k_grid_compact: the eligible points, ascending.
#include <hip/hip_runtime.h>

#include <thread>

#include <string.h>

#include <algorithm>
#include <rocprim/rocprim.hpp>

#include "usac_kernels.h"

namespace usac {

__global__ __launch_bounds__(256) void k_grid_keys(const float4 *__restrict__ pts, uint32_t n, float cs, int4 cmin,
                                                   int4 bits, uint64_t *__restrict__ keys, uint32_t *__restrict__ idx) {
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
    keys[i] = k;
    idx[i] = i;
}

__global__ __launch_bounds__(256) void k_grid_heads(const uint64_t *__restrict__ keys, uint32_t n,
                                                    uint32_t *__restrict__ head) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    head[p] = (p == 0 || keys[p] != keys[p - 1]) ? 1u : 0u;
}

// cellid[p] = 1-based key-order cell of sorted position p (inclusive scan of the heads)
__global__ __launch_bounds__(256) void k_grid_cells(const uint32_t *__restrict__ head,
                                                    const uint32_t *__restrict__ cellid,
                                                    const uint32_t *__restrict__ idx_sorted, uint32_t n,
                                                    uint32_t *__restrict__ old_start, uint32_t *__restrict__ old_min,
                                                    uint32_t *__restrict__ ord, uint32_t *__restrict__ n_cells) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const uint32_t c = cellid[p] - 1;
    if (head[p]) {
        old_start[c] = p;
        old_min[c] = idx_sorted[p];  // stable sort: the first member is the smallest index
        ord[c] = c;
    }
    if (p == n - 1) {
        old_start[c + 1] = n;
        *n_cells = c + 1;
    }
}

// q-th cell in order of first appearance = key-order cell ord[q]
__global__ __launch_bounds__(256) void k_grid_renumber(const uint32_t *__restrict__ ord,
                                                       const uint32_t *__restrict__ old_start, uint32_t n_cells,
                                                       uint32_t *__restrict__ new_of_old,
                                                       uint32_t *__restrict__ size_new) {
    const uint32_t q = blockIdx.x * 256 + threadIdx.x;
    if (q > n_cells) return;
    if (q == n_cells) {
        size_new[q] = 0;  // the exclusive scan's last entry becomes start[n_cells] = n
        return;
    }
    const uint32_t o = ord[q];
    new_of_old[o] = q;
    size_new[q] = old_start[o + 1] - old_start[o];
}

__global__ __launch_bounds__(256) void k_grid_scatter(const uint32_t *__restrict__ cellid,
                                                      const uint32_t *__restrict__ idx_sorted,
                                                      const uint32_t *__restrict__ old_start,
                                                      const uint32_t *__restrict__ new_of_old,
                                                      const uint32_t *__restrict__ start, uint32_t n, uint32_t m,
                                                      uint32_t *__restrict__ cell, uint32_t *__restrict__ rank,
                                                      int32_t *__restrict__ members, uint32_t *__restrict__ elig) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const uint32_t o = cellid[p] - 1;
    const uint32_t q = new_of_old[o];
    const uint32_t i = idx_sorted[p];
    const uint32_t r = p - old_start[o];
    cell[i] = q;
    rank[i] = r;
    members[start[q] + r] = (int32_t)i;
    elig[i] = (old_start[o + 1] - old_start[o] - 1 >= m) ? 1u : 0u;  // >= m neighbours (Q18)
}

__global__ __launch_bounds__(256) void k_grid_compact(const uint32_t *__restrict__ elig,
                                                      const uint32_t *__restrict__ pos, uint32_t n,
                                                      int32_t *__restrict__ eligible, uint32_t *__restrict__ n_elig) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (elig[i]) eligible[pos[i]] = (int32_t)i;
    if (i == n - 1) *n_elig = pos[i] + elig[i];
}

namespace {

// scratch carve-out of the build (all sizes in elements of n or n + 1)
struct GridScratch {
    uint64_t *keys_a, *keys_b;
    uint32_t *idx_a, *idx_b, *head, *cellid, *old_start, *old_min, *ord_a, *ord_b, *min_b, *new_of_old, *size_new,
        *elig, *pos, *counts;
    void *tmp;
    size_t tmp_bytes;
};

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t rocprim_tmp_bytes(uint32_t n) {
    size_t a = 0, b = 0, c = 0, d = 0;
    (void)rocprim::radix_sort_pairs((void *)nullptr, a, (uint64_t *)nullptr, (uint64_t *)nullptr, (uint32_t *)nullptr,
                              (uint32_t *)nullptr, n, 0, 64);
    (void)rocprim::radix_sort_pairs((void *)nullptr, b, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                              (uint32_t *)nullptr, n, 0, 32);
    (void)rocprim::inclusive_scan((void *)nullptr, c, (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n,
                            rocprim::plus<uint32_t>());
    (void)rocprim::exclusive_scan((void *)nullptr, d, (uint32_t *)nullptr, (uint32_t *)nullptr, 0u, (size_t)n + 1,
                            rocprim::plus<uint32_t>());
    return std::max(std::max(a, b), std::max(c, d));
}

GridScratch carve(void *ws, uint32_t n) {
    GridScratch s;
    char *p = static_cast<char *>(ws);
    auto take = [&](size_t bytes) {
        void *r = p;
        p += align256(bytes);
        return r;
    };
    const size_t u = sizeof(uint32_t) * ((size_t)n + 1);
    s.keys_a = (uint64_t *)take(sizeof(uint64_t) * n);
    s.keys_b = (uint64_t *)take(sizeof(uint64_t) * n);
    s.idx_a = (uint32_t *)take(u);
    s.idx_b = (uint32_t *)take(u);
    s.head = (uint32_t *)take(u);
    s.cellid = (uint32_t *)take(u);
    s.old_start = (uint32_t *)take(u);
    s.old_min = (uint32_t *)take(u);
    s.ord_a = (uint32_t *)take(u);
    s.ord_b = (uint32_t *)take(u);
    s.min_b = (uint32_t *)take(u);
    s.new_of_old = (uint32_t *)take(u);
    s.size_new = (uint32_t *)take(u);
    s.elig = (uint32_t *)take(u);
    s.pos = (uint32_t *)take(u);
    s.counts = (uint32_t *)take(sizeof(uint32_t) * 2);
    s.tmp_bytes = rocprim_tmp_bytes(n);
    s.tmp = take(s.tmp_bytes);
    return s;
}

}  // namespace

size_t grid_workspace_bytes(uint32_t n) {
    return align256(sizeof(uint64_t) * n) * 2 + align256(sizeof(uint32_t) * ((size_t)n + 1)) * 13 + 256 +
           align256(rocprim_tmp_bytes(n)) + 256;
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
    if (n == 0) return hipErrorInvalidValue;
    GridScratch s = carve(ws, n);
    const dim3 b(256), g((n + 255) / 256);
    hipLaunchKernelGGL(k_grid_keys, g, b, 0, st, pts, n, (float)cell_size, cmin, bits, s.keys_a, s.idx_a);
    GRID_TRY(hipGetLastError());
    size_t tb = s.tmp_bytes;
    // only the key's used bits (per dimension: the box's cell range and a sentinel) are sorted
    const int key_bits = bits.x + bits.y + bits.z + bits.w;
    GRID_TRY(rocprim::radix_sort_pairs(s.tmp, tb, s.keys_a, s.keys_b, s.idx_a, s.idx_b, n, 0, key_bits, st));
    hipLaunchKernelGGL(k_grid_heads, g, b, 0, st, s.keys_b, n, s.head);
    GRID_TRY(hipGetLastError());
    tb = s.tmp_bytes;
    GRID_TRY(rocprim::inclusive_scan(s.tmp, tb, s.head, s.cellid, (size_t)n, rocprim::plus<uint32_t>(), st));
    hipLaunchKernelGGL(k_grid_cells, g, b, 0, st, s.head, s.cellid, s.idx_b, n, s.old_start, s.old_min, s.ord_a,
                       s.counts);
    GRID_TRY(hipGetLastError());
    GRID_TRY(hipMemcpyAsync(pinned2, s.counts, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    GRID_TRY(poll_stream(st));
    const uint32_t nc = pinned2[0];
    tb = s.tmp_bytes;
    int min_bits = 1;  // the smallest members are point indices < n
    while (min_bits < 32 && (n - 1) >> min_bits) min_bits++;
    GRID_TRY(rocprim::radix_sort_pairs(s.tmp, tb, s.old_min, s.min_b, s.ord_a, s.ord_b, nc, 0, min_bits, st));
    hipLaunchKernelGGL(k_grid_renumber, dim3((nc + 1 + 255) / 256), b, 0, st, s.ord_b, s.old_start, nc, s.new_of_old,
                       s.size_new);
    GRID_TRY(hipGetLastError());
    tb = s.tmp_bytes;
    GRID_TRY(rocprim::exclusive_scan(s.tmp, tb, s.size_new, start, 0u, (size_t)nc + 1, rocprim::plus<uint32_t>(), st));
    hipLaunchKernelGGL(k_grid_scatter, g, b, 0, st, s.cellid, s.idx_b, s.old_start, s.new_of_old, start, n, m, cell,
                       rank, members, s.elig);
    GRID_TRY(hipGetLastError());
    tb = s.tmp_bytes;
    GRID_TRY(rocprim::exclusive_scan(s.tmp, tb, s.elig, s.pos, 0u, (size_t)n, rocprim::plus<uint32_t>(), st));
    hipLaunchKernelGGL(k_grid_compact, g, b, 0, st, s.elig, s.pos, n, eligible, s.counts + 1);
    GRID_TRY(hipGetLastError());
    GRID_TRY(hipMemcpyAsync(pinned2 + 1, s.counts + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    GRID_TRY(poll_stream(st));
    const uint32_t ne = pinned2[1];
    *n_cells_out = nc;
    *n_elig_out = ne;
    return hipSuccess;
}

}  // namespace usac
