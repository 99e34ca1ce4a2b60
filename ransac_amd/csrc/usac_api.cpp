// usac_api.cpp -- C-ABI (include/usac_gpu.h) over the HIP kernels, plus the batched
// Ransac::run replay.  Host code only; every model estimation and every residual runs on
// the device -- there is no CPU compute path (a context without a usable GPU fails at
// usac_create with USAC_ERR_HIP).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/usac_gpu.h"
#include "usac_host.hpp"
#include "usac_maxflow.hpp"
#include "usac_kernels.h"

namespace {

constexpr uint32_t kDefaultBatch = 8192;
constexpr uint32_t kRampFirst = 1024;  // first batch of a run with the default batch
// the SPRT batch's whole [nw][S] word block copied with its list in one host wait up to this size
constexpr size_t kMaskWholeCopy = 512 * 1024;
constexpr uint32_t kRampFirstProsac = 32;

// Device memory of the contexts comes from a process-wide cache per device: a context is
// typically created per Ransac::run (as the reference constructs its Ransac per run), and
// hipMalloc / hipFree -- the latter synchronising the whole device -- cost milliseconds per
// context.  Blocks are kept in power-of-two size classes (>= 4 KB); a released block goes back
// to its class after its context's stream has drained (usac_destroy synchronises first), a
// block replaced by a larger one only after the device has (reserve() below), so no block is
// handed out while a kernel may still use it.  At most kPoolCap bytes per device are cached.
constexpr size_t kPoolCap = size_t(16) << 30;

struct DevPool {
    std::mutex mu;
    std::multimap<std::pair<int, size_t>, void *> free;  // (device, class bytes) -> block
    std::map<int, size_t> cached;                         // bytes held per device
    static DevPool &get() {
        static DevPool *pool = new DevPool();  // never destroyed: no hipFree after runtime teardown
        return *pool;
    }
    static size_t size_class(size_t b) {
        size_t c = 4096;
        while (c < b) c <<= 1;
        return c;
    }
    hipError_t alloc(size_t b, void **p, size_t *got) {
        const size_t c = size_class(b);
        int dev = 0;
        (void)hipGetDevice(&dev);
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = free.find({dev, c});
            if (it != free.end()) {
                *p = it->second;
                free.erase(it);
                cached[dev] -= c;
                *got = c;
                return hipSuccess;
            }
        }
        hipError_t e = hipMalloc(p, c);
        if (e == hipSuccess) *got = c;
        return e;
    }
    void give_back(void *p, size_t c) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        {
            std::lock_guard<std::mutex> g(mu);
            if (cached[dev] + c <= kPoolCap) {
                free.emplace(std::make_pair(dev, c), p);
                cached[dev] += c;
                return;
            }
        }
        (void)hipFree(p);
    }
};

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    hipError_t reserve(size_t b) {
        if (b <= bytes) return hipSuccess;
        if (p) {  // kernels of this context may still read the old block
            (void)hipDeviceSynchronize();
            DevPool::get().give_back(p, bytes);
        }
        p = nullptr;
        bytes = 0;
        return DevPool::get().alloc(b, &p, &bytes);
    }
    void release() {  // the owner's stream has drained (usac_destroy)
        if (p) DevPool::get().give_back(p, bytes);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};

// streams and events likewise: creating / destroying them per context costs more than a run
struct StreamPool {
    std::mutex mu;
    std::multimap<int, hipStream_t> streams;
    std::multimap<int, hipEvent_t> events;
    static StreamPool &get() {
        static StreamPool *pool = new StreamPool();
        return *pool;
    }
    hipError_t stream(hipStream_t *s) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = streams.find(dev);
            if (it != streams.end()) {
                *s = it->second;
                streams.erase(it);
                return hipSuccess;
            }
        }
        return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    }
    hipError_t event(hipEvent_t *ev) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = events.find(dev);
            if (it != events.end()) {
                *ev = it->second;
                events.erase(it);
                return hipSuccess;
            }
        }
        return hipEventCreate(ev);
    }
    void give_back(hipStream_t s) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        std::lock_guard<std::mutex> g(mu);
        streams.emplace(dev, s);
    }
    // streams restricted to a few CUs spread over the device (hipExtStreamCreateWithCUMask), pooled
    // apart; cus <= 0 or >= the device's CU count: none (nullptr)
    std::multimap<int, hipStream_t> masked;
    hipError_t masked_stream(int cus, hipStream_t *s) {
        *s = nullptr;
        int dev = 0;
        (void)hipGetDevice(&dev);
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = masked.find(dev);
            if (it != masked.end()) {
                *s = it->second;
                masked.erase(it);
                return hipSuccess;
            }
        }
        int ncu = 0;
        hipError_t e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        if (cus <= 0 || cus >= ncu) return hipSuccess;
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int k = 0; k < cus; k++) {
            const int cu = (int)((long long)k * ncu / cus);
            mask[cu / 32] |= 1u << (cu % 32);
        }
        return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
    }
    void give_back_masked(hipStream_t s) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        std::lock_guard<std::mutex> g(mu);
        masked.emplace(dev, s);
    }
    void give_back(hipEvent_t ev) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        std::lock_guard<std::mutex> g(mu);
        events.emplace(dev, ev);
    }
};

// pinned host staging blocks (hipHostMalloc costs far more than a run's copies), by size class
struct PinnedPool {
    std::mutex mu;
    std::multimap<size_t, void *> free;
    static PinnedPool &get() {
        static PinnedPool *pool = new PinnedPool();
        return *pool;
    }
    void *take(size_t b, size_t *got) {
        const size_t c = DevPool::size_class(b);
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = free.find(c);
            if (it != free.end()) {
                void *p = it->second;
                free.erase(it);
                *got = c;
                return p;
            }
        }
        void *p = nullptr;
        if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) return nullptr;
        *got = c;
        return p;
    }
    void give_back(void *p, size_t c) {
        std::lock_guard<std::mutex> g(mu);
        free.emplace(c, p);
    }
};

// Captured LO stage graphs, process-wide: a context lives for one Ransac::run (as the reference
// builds its Ransac per run), but its device blocks come from DevPool and recur from run to run,
// so a graph keyed by the stage shape and every buffer address it touches is reused across runs
// (a graph's kernels only reach what its key's shape implies; the key also holds every buffer's
// reserved byte count, so a block handed out again at the same address with a smaller backing
// never matches an old graph).  The cache only grows, up to kMax entries; past that, stages of new
// shapes are launched kernel by kernel.  The execs are destroyed at process exit by an atexit
// handler registered after the HIP runtime's own (so it runs before the runtime's teardown).
struct GraphCache {
    static constexpr size_t kMax = 256;
    std::mutex mu;
    std::map<std::vector<uintptr_t>, hipGraphExec_t> g;
    static GraphCache &get() {
        static GraphCache *c = [] {
            GraphCache *gc = new GraphCache();
            std::atexit([] {
                GraphCache &cc = GraphCache::get();
                std::lock_guard<std::mutex> lk(cc.mu);
                for (auto &kv : cc.g) (void)hipGraphExecDestroy(kv.second);
                cc.g.clear();
            });
            return gc;
        }();
        return *c;
    }
};

// std::vector storage in pinned host memory (PinnedPool), for the loop's DMA sources and
// targets: a copy from / to pageable memory goes through a staging buffer and holds the host
// for the copy; these copies sit between every device step and the host replay.
template <class T>
struct PinnedAlloc {
    typedef T value_type;
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U> &) {}
    T *allocate(size_t k) {
        size_t got = 0;
        void *p = PinnedPool::get().take(sizeof(T) * (k ? k : 1), &got);
        if (!p) throw std::bad_alloc();
        return static_cast<T *>(p);
    }
    void deallocate(T *p, size_t k) { PinnedPool::get().give_back(p, DevPool::size_class(sizeof(T) * (k ? k : 1))); }
    // default-initialise (no zero fill of staging that a copy overwrites anyway); explicit
    // values as usual
    template <class U>
    void construct(U *p) noexcept {
        ::new (static_cast<void *>(p)) U;
    }
    template <class U, class... A>
    void construct(U *p, A &&...a) {
        ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
    }
    template <class U>
    bool operator==(const PinnedAlloc<U> &) const { return true; }
    template <class U>
    bool operator!=(const PinnedAlloc<U> &) const { return false; }
};
template <class T>
using pinned_vector = std::vector<T, PinnedAlloc<T>>;

// Wait for a stream by polling it: the loop's host replay waits on the device dozens of
// times per run (LO stages, batches, polish), and a blocking hipStreamSynchronize adds a wake-up
// latency of ~20 us each time; polling returns within about a microsecond of completion.
hipError_t stream_wait(hipStream_t st) {
    for (uint32_t spins = 0;; spins++) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) return e;
        if ((spins & 1023u) == 1023u) std::this_thread::yield();
    }
}

}  // namespace

struct usac_ctx {
    int device = 0;
    int estimator = 0;
    uint32_t n = 0, cols = 0, m = 0;
    int dlt_mode = USAC_DLT_THIN;
    int chunks = 4;
    int score_variant = 0;  // 0 = guard-band fast path (+ pre-sort; multi-chunk H: the matrix-core prefilter),
                            // 1 = exact expression only, 2 = fast, no pre-sort, 3 = (tests) usac_score_models
                            // of H through the multi-chunk scorer
    hipStream_t stream = nullptr;
    DevBuf pts;
    DevBuf rec;             // fast-kernel point records (32 B / point)
    DevBuf prosac_tab;      // device PROSAC schedule: subset size per hypothesis (< T_N)
    uint32_t prosac_len = 0;  // its entries
    int dev_sampler = USAC_SAMPLER_UNIFORM;
    DevBuf tv_part;         // two-view scorer scratch: pre-sort permutation, chunk partials
    DevBuf perm;            // hypothesis pre-sort of the fast kernel (usac::presort_bytes)
    void *perm_zeroed = nullptr;  // the perm block whose region counters were zeroed
    DevBuf hf_part;         // fast-kernel partials of a point range split over workgroups
    float rec_thr = -1.f;   // threshold the record bands were built for
    float4 ext = {0, 0, 0, 0};  // dataset box: max |x1|, |y1|, |x2|, |y2| (fast-kernel bounds)
    // the matrix-core prefilter scorer of homographies (kernels_h16.hip): dataset constants, fp16
    // point features (built on first use), per-batch rows / slacks and chunk partials; h16 = 1 when
    // usable (USAC_H16=0 turns it off: the lanes-over-hypotheses k_score_hf then scores every batch)

    int h16 = 0;
    bool h16_feat_ok = false;
    bool h16_off = false;  // k_score_hf for every batch (usac_ransac_run sets it for its loop)
    uint32_t h16_rows_for = 0;  // > 0: the solver wrote the rows of a batch of this size for h16_rows_thr
    float h16_rows_thr = 0.f;
    uint32_t h16_deferred_ch = 0;  // > 0: the last h16 batch's chunk partials await batch_argmax
    float h16_deferred_thr = 0.f;
    DevBuf h16_k, h16_feat, h16_rows, h16_fm, h16_part;  // h16_k: the dataset constants (usac::H16Consts)
    // the matrix-core prefilter scorer of essential matrices (kernels_e16.hip): the h16 dataset
    // constants, its own rho-scaled fp16 features, per-batch rows / bounds and chunk partials; e16 = 1
    // when usable (USAC_E16=0: the lanes-over-models k_score_f2 scores every throughput batch)
    int e16 = 0;
    bool h16_k_ok = false, e16_feat_ok = false;
    DevBuf e16_feat, e16_rows, e16_cm, e16_part;
    // batch buffers
    DevBuf samples, models, counts, sums, best, hostmodels, argmax_part;
    DevBuf list, list_n;    // fundamental: occupied model slots (compacted) and their number
    DevBuf h4_fb, h4_fb_n;  // homography thin DLT: QR fall-back hypotheses and two counters (zeroed once)
    DevBuf pool_idx, pool_pts, masks;  // SPRT parity path: pool order, permuted points, flag words
    // LO-RANSAC (LoRansac): W speculative inner iterations in flight -- their inlier lists
    // (W x N), LSQ sample positions (W x lo_sample_size), point counts, thresholds, models,
    // fit flags, scores, fit and scoring scratch; lo_max = the current best's inlier list
    DevBuf lo_max, lo_lists, lo_pos, lo_ns, lo_thrs, lo_slots, lo_models, lo_ok, lo_cnts, lo_sums, lo_q, lo_part,
        lo_ws, lo_scr;
    DevBuf knn_idx, knn_d2;  // KNN neighbour table (usac_knn, NAPSAC KNN)
    // grid neighbours (build_grid): CSR of the cells of size grid_cs, NAPSAC-eligible points
    // grid CSR in one block, downloaded by one copy: cell[n], rank[n], members[n], start[n + 1]
    DevBuf grid_csr, grid_elig, grid_ws;
    uint32_t *grid_cell() const { return grid_csr.as<uint32_t>(); }
    uint32_t *grid_rank() const { return grid_csr.as<uint32_t>() + n; }
    int32_t *grid_members() const { return reinterpret_cast<int32_t *>(grid_csr.as<uint32_t>() + 2 * (size_t)n); }
    uint32_t *grid_start() const { return grid_csr.as<uint32_t>() + 3 * (size_t)n; }
    int grid_cs = 0;        // cell size the grid was built for (0 = none)
    uint64_t grid_gen = 0;  // bumped at every (re)build of the device grid
    // the host copy of the grid (download_grid), reused while grid_gen is unchanged
    std::shared_ptr<const usac::GridNeighbors> grid_host;
    uint64_t grid_host_gen = ~0ull;
    int cell_size = 50;     // model.hpp:43, the device NAPSAC sampler's grid
    uint32_t grid_n_cells = 0, grid_n_elig = 0;
    DevBuf gc_err;           // graph-cut LO: residuals of the model being labelled
    DevBuf e5_ws;                      // staged 5-point solver workspace
    // throughput SPRT (usac_set_sprt): batch-fixed test on the pool-ordered points
    bool sprt_on = false;
    usac::SprtConsts sprt_k{};      // up, down, A and their logs (the reference's doubles)
    double sprt_eps = 0.0, sprt_delta = 0.0;
    DevBuf sprt_pts, sprt_tested, sprt_surv, sprt_surv_n, sprt_starts;
    uint32_t spk = 1;       // model slots per hypothesis (3 for the 7-point solver)
    // single-model / polish buffers
    DevBuf one_model, inl_idx, inl_cnt, inl_sum, inl_scratch, q, partial, ws, nm_model, nm_ok;
    uint32_t *grid_pin = nullptr;    // pinned words the grid build reads its two counts into
    size_t grid_pin_bytes = 0;
    DevBuf pol_res;                  // polish pass results (usac_kernels.h kPol*: per pass model, ok, count, sum)
    DevBuf pol_lists;                // the polish passes' inlier lists (4 x n)
    void *pol_pin = nullptr;         // their pinned host copy (PinnedPool)
    size_t pol_pin_bytes = 0;
    DevBuf nm_seq;          // normalisation scratch of the non-minimal fits (polish and LO)
    DevBuf nm_w, nm_qw;     // usac_lsq_fit with weights: the weights, the weighted points
    DevBuf lo_io;           // one LO stage's inputs (two blocks, alternating) and outputs
    // the LO stages' Σerr passes run on their own stream beside the next stage's fit
    hipStream_t lo_stream = nullptr;
    // LO iterative stages replayed as HIP graphs (USAC_LO_GRAPH=1; one capture per stage shape and
    // buffer set, process-wide).  Off by default: measured slower than the direct launches (same-
    // process A/B over 60 cfg5 runs, tools/ab_lo_graph.py: 134 vs 127 us per LO stage)
    bool lo_graph_on = false;
    DevBuf lo_best;                  // the round's best count on the device (the graphs read it)
    int32_t *lo_best_pin = nullptr;  // its pinned host word
    size_t lo_best_pin_bytes = 0;
    void *rec_pin = nullptr;  // usac_fetch_best's pinned staging (a pageable D2H copy is staged by the runtime)
    size_t rec_pin_bytes = 0;
    // the loop's next batch drawn and run ahead of the current batch's replay (usac_ransac_run)
    hipStream_t spec_stream = nullptr;
    hipStream_t thin_stream = nullptr;  // CU-masked: the essential solver's root-order kernels
    hipEvent_t thin_ev[2] = {nullptr, nullptr};
    hipEvent_t spec_ev = nullptr;
    // per block parity: the stage's outputs in the host block (main), its Σ (side); round end
    hipEvent_t lo_ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    // comm
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    DevBuf rec_send, rec_all;
    DevBuf x_send, x_recv;  // sharded-run all-gather buffers (RCCL path, device-packed)
    void *x_pin = nullptr;  // their pinned host copy (the replay's counts / model words)
    size_t x_pin_bytes = 0;
    // batch-best exchange (usac_exchange_best_async / _wait): a dedicated stream ordered after
    // each batch by an event, a ring of in-flight all-gathers (device + pinned host records)
    hipStream_t xstream = nullptr;
    hipEvent_t xev_batch[USAC_XRING] = {}, xev_done[USAC_XRING] = {};
    DevBuf xring;
    usac_record *xring_host = nullptr;
    size_t xring_host_bytes = 0;
    // collectives on one communicator must run in one order on every rank: the two streams
    // that issue them are ordered by events -- a collective on `stream` waits for the last
    // exchange (x_last), an exchange waits for the last collective on `stream` (coll_ev)
    int x_last = -1;
    hipEvent_t coll_ev = nullptr;
    bool coll_pending = false;
    // timing
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    float last_ms[3] = {0, 0, 0};
    bool batch_valid = false;  // counts / sums hold a batch's scores (usac_last_counts)
    uint32_t sprt_S = 0;       // model slots of the last batch-SPRT launch (usac_batch_sprt_info)
    bool timed_pending = false;
    bool timing_on = true;  // usac_set_timing
    std::string err;
};

namespace {

int fail(usac_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                      \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail((ctx), USAC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define NCCL_TRY(ctx, expr)                                                                        \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess)                                                                     \
            return fail((ctx), USAC_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// before a collective on c->stream: after every exchange issued on the exchange stream
hipError_t order_after_exchanges(usac_ctx *c) {
    if (c->xstream && c->x_last >= 0) return hipStreamWaitEvent(c->stream, c->xev_done[c->x_last], 0);
    return hipSuccess;
}
// after a collective on c->stream: later exchanges wait for it
hipError_t mark_collective(usac_ctx *c) {
    if (!c->coll_ev) return hipSuccess;
    hipError_t e = hipEventRecord(c->coll_ev, c->stream);
    if (e == hipSuccess) c->coll_pending = true;
    return e;
}

bool is_h(const usac_ctx *c) { return c->estimator == USAC_HOMOGRAPHY; }
bool is_f(const usac_ctx *c) { return c->estimator == USAC_FUNDAMENTAL; }
bool is_e(const usac_ctx *c) { return c->estimator == USAC_ESSENTIAL; }
// solvers that may return no model for a sample: occupied slots are listed (list / list_n)
bool listed(const usac_ctx *c) { return is_f(c) || is_e(c); }
bool two_view(const usac_ctx *c) { return c->cols == 4; }
int ncomp(const usac_ctx *c) { return two_view(c) ? 9 : 3; }
int ncomp_dev(const usac_ctx *c) { return is_h(c) ? 18 : ncomp(c); }

// B = hypotheses (minimal samples); every per-model buffer holds B * spk slots
int ensure_batch(usac_ctx *c, uint32_t B) {
    const size_t S = (size_t)B * c->spk;
    HIP_TRY(c, c->samples.reserve(sizeof(int32_t) * (size_t)B * c->m));
    HIP_TRY(c, c->models.reserve(sizeof(float) * S * ncomp_dev(c)));
    HIP_TRY(c, c->counts.reserve(sizeof(int32_t) * S));
    HIP_TRY(c, c->sums.reserve(sizeof(float) * S));
    HIP_TRY(c, c->best.reserve(sizeof(usac_record)));
    HIP_TRY(c, c->argmax_part.reserve(16 * (S / 2048 + 1)));
    HIP_TRY(c, c->hostmodels.reserve(sizeof(float) * 9 * S));
    if (listed(c)) {
        HIP_TRY(c, c->list.reserve(sizeof(uint32_t) * S));
        HIP_TRY(c, c->list_n.reserve(sizeof(uint32_t)));
    }
    if (is_h(c)) {
        HIP_TRY(c, c->h4_fb.reserve(sizeof(uint32_t) * (size_t)B));
        if (!c->h4_fb_n.p) {  // the kernels reset the counters after each use; a pooled block is not zero
            HIP_TRY(c, c->h4_fb_n.reserve(2 * sizeof(uint32_t)));
            HIP_TRY(c, hipMemsetAsync(c->h4_fb_n.p, 0, 2 * sizeof(uint32_t), c->stream));
        }
    }
    return USAC_OK;
}

int ensure_single(usac_ctx *c) {
    HIP_TRY(c, c->one_model.reserve(sizeof(float) * 9));
    HIP_TRY(c, c->inl_idx.reserve(sizeof(int32_t) * (size_t)std::max<uint32_t>(c->n, 1)));
    HIP_TRY(c, c->pol_lists.reserve(sizeof(int32_t) * 4 * (size_t)std::max<uint32_t>(c->n, 1)));
    // the polish's later passes fit with c->n as the bound on their device-side counts: their
    // scratch reserved here, so no growth (a device synchronise) inside a run
    HIP_TRY(c, c->nm_seq.reserve(usac::nonminimal_seq_bytes(std::max<uint32_t>(c->n, 1), 1)));
    HIP_TRY(c, c->pol_res.reserve(sizeof(float) * usac::kPolWords));
    HIP_TRY(c, c->inl_cnt.reserve(sizeof(int32_t)));
    HIP_TRY(c, c->inl_sum.reserve(sizeof(float)));
    HIP_TRY(c, c->q.reserve(sizeof(float) * 4 * (size_t)std::max<uint32_t>(c->n, 1)));
    HIP_TRY(c, c->partial.reserve(sizeof(double) * 45 * ((size_t)c->n / 64 + 2)));
    HIP_TRY(c, c->ws.reserve(sizeof(float) * 32));
    HIP_TRY(c, c->nm_model.reserve(sizeof(float) * 9));
    HIP_TRY(c, c->nm_ok.reserve(sizeof(int32_t)));
    return USAC_OK;
}

usac::DevSampler dev_sampler(const usac_ctx *c, uint64_t seed) {
    const bool prosac = c->dev_sampler == USAC_SAMPLER_PROSAC;
    usac::DevSampler ds{};
    ds.seed = seed;
    ds.prosac = prosac ? c->prosac_tab.as<uint32_t>() : nullptr;
    ds.prosac_len = prosac ? c->prosac_len : 0u;
    if (c->dev_sampler == USAC_SAMPLER_NAPSAC) {
        ds.nap_n_eligible = c->grid_n_elig;
        ds.nap_cell = c->grid_cell();
        ds.nap_rank = c->grid_rank();
        ds.nap_start = c->grid_start();
        ds.nap_members = c->grid_members();
        ds.nap_eligible = c->grid_elig.as<int32_t>();
    }
    return ds;
}

// The grid of a dataset whose cell key does not fit the device build's 63-bit packed key (more
// than 65536 cells along a dimension, or four ranges wider than 63 bits in all): built on the host
// (usac::GridNeighbors' hash map takes any key) from the device's points, then uploaded in the
// device CSR layout -- the same cells, numbering and member order as the device build.
int host_grid(usac_ctx *c, int cs) {
    const size_t n = c->n;
    std::vector<float> pts(4 * n);
    HIP_TRY(c, hipMemcpyAsync(pts.data(), c->pts.p, sizeof(float) * 4 * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    const usac::GridNeighbors g(pts.data(), c->n, cs);
    std::vector<uint32_t> csr(4 * n + 1);
    const uint32_t nc = (uint32_t)g.starts().size() - 1;
    memcpy(csr.data(), g.cells().data(), 4 * n);
    memcpy(csr.data() + n, g.ranks().data(), 4 * n);
    memcpy(csr.data() + 2 * n, g.members().data(), 4 * n);
    memcpy(csr.data() + 3 * n, g.starts().data(), 4 * ((size_t)nc + 1));
    std::vector<int32_t> elig;
    for (uint32_t i = 0; i < c->n; i++)
        if (g.count(i) >= c->m) elig.push_back((int32_t)i);
    HIP_TRY(c, hipMemcpyAsync(c->grid_csr.p, csr.data(), sizeof(uint32_t) * (3 * n + nc + 1), hipMemcpyHostToDevice,
                              c->stream));
    if (!elig.empty())
        HIP_TRY(c, hipMemcpyAsync(c->grid_elig.p, elig.data(), sizeof(int32_t) * elig.size(), hipMemcpyHostToDevice,
                                  c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    c->grid_n_cells = nc;
    c->grid_n_elig = (uint32_t)elig.size();
    c->grid_cs = cs;
    c->grid_gen++;
    return USAC_OK;
}

// NearestNeighbors::getGridNearestNeighbors (nearest_neighbors.cpp:160-202) on the device for
// cell size cs (kept until another size is asked for).  Cells are packed per dimension relative
// to the dataset box's lowest cell; a box too wide for the packed key takes host_grid instead.
int ensure_grid(usac_ctx *c, int cs) {
    if (c->grid_cs == cs) return USAC_OK;
    if (c->cols != 4) return fail(c, USAC_ERR_ARG, "grid neighbours need 4-column points (SURVEY Q17)");
    if (cs <= 0) return fail(c, USAC_ERR_ARG, "grid cell_size must be > 0");
    const float e[4] = {c->ext.x, c->ext.y, c->ext.z, c->ext.w};
    int lo[4], bits[4];
    bool packable = true;
    for (int j = 0; j < 4; j++) {
        lo[j] = bits[j] = 0;
        if (!(e[j] / (float)cs < 1.0e9f)) {  // the int cell index itself is out of range
            packable = false;
            continue;
        }
        lo[j] = (int)(-e[j] / (float)cs);
        const long long range = (long long)(int)(e[j] / (float)cs) - lo[j];
        packable &= range <= 65535;
        bits[j] = 1;  // 2^bits - 1 > range: room for the out-of-box sentinel
        while (bits[j] < 40 && (1ll << bits[j]) - 1 <= range) bits[j]++;
    }
    // each dimension keeps its range plus the out-of-box sentinel; the build's hash table keeps
    // the all-ones word as its empty slot, so the key must fit 63 bits (clamping a dimension
    // would give the sentinel a real cell's value)
    packable &= bits[0] + bits[1] + bits[2] + bits[3] <= 63;
    const size_t n = c->n;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, c->grid_csr.reserve(sizeof(uint32_t) * (4 * n + 1)));
    HIP_TRY(c, c->grid_elig.reserve(sizeof(int32_t) * n));
    c->grid_cs = 0;
    c->grid_gen++;
    if (!packable) return host_grid(c, cs);
    if (!c->grid_pin && !(c->grid_pin = static_cast<uint32_t *>(PinnedPool::get().take(64, &c->grid_pin_bytes))))
        return fail(c, USAC_ERR_HIP, "pinned host allocation failed");
    HIP_TRY(c, c->grid_ws.reserve(usac::grid_workspace_bytes(c->n)));
    c->grid_cs = 0;
    c->grid_gen++;
    HIP_TRY(c, usac::build_grid(c->stream, c->pts.as<float4>(), c->n, cs, make_int4(lo[0], lo[1], lo[2], lo[3]),
                                make_int4(bits[0], bits[1], bits[2], bits[3]), c->m, c->grid_ws.p,
                                c->grid_cell(), c->grid_rank(), c->grid_start(), c->grid_members(),
                                c->grid_elig.as<int32_t>(), c->grid_pin,
                                &c->grid_n_cells, &c->grid_n_elig));
    c->grid_cs = cs;
    c->grid_gen++;
    return USAC_OK;
}

// the device grid as the host loop's GridNeighbors (bit-identical to building it on the host)
int download_grid(usac_ctx *c, int cs, std::shared_ptr<const usac::GridNeighbors> &out) {
    int rc = ensure_grid(c, cs);
    if (rc) return rc;
    if (c->grid_host && c->grid_host_gen == c->grid_gen) {  // the same device grid: its host copy
        out = c->grid_host;
        return USAC_OK;
    }
    // DMA into one pinned block, then into the host vectors (the sampler reads them at random:
    // they should be cache-warm, which DMA-written pinned memory is not)
    const size_t n = c->n, nc1 = (size_t)c->grid_n_cells + 1;
    // (a raw pooled block: a pinned_vector would zero-fill the 1.2 MB first)
    size_t got = 0;
    uint32_t *w = static_cast<uint32_t *>(PinnedPool::get().take(sizeof(uint32_t) * (3 * n + nc1), &got));
    if (!w) return fail(c, USAC_ERR_HIP, "pinned host allocation failed");
    struct Back {
        void *p;
        size_t b;
        ~Back() { PinnedPool::get().give_back(p, b); }
    } back{w, got};
    HIP_TRY(c, hipMemcpyAsync(w, c->grid_csr.p, sizeof(uint32_t) * (3 * n + nc1), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    std::vector<uint32_t> cell(w, w + n), rank(w + n, w + 2 * n), start(w + 3 * n, w + 3 * n + nc1);
    std::vector<int32_t> members(reinterpret_cast<const int32_t *>(w + 2 * n), reinterpret_cast<const int32_t *>(w + 3 * n));
    out = std::make_shared<const usac::GridNeighbors>(std::move(cell), std::move(rank), std::move(start),
                                                      std::move(members));
    c->grid_host = out;
    c->grid_host_gen = c->grid_gen;
    return USAC_OK;
}

// solve (samples on device, or device RNG when samples_dev == nullptr) into c->models
hipError_t h16_init(usac_ctx *c);

// h16_thr >= 0: the batch will be scored by the matrix-core scorer (h16_scores) -- the homography
// solvers then also write its rows and slacks (usac_h16.hpp), so enqueue_score_h16 skips k_h16_rows
hipError_t enqueue_solve(usac_ctx *c, const int32_t *samples_dev, uint32_t B, uint64_t seed, uint64_t first_hyp,
                         int32_t *samples_out, float h16_thr = -1.f) {
    const usac::DevSampler ds = dev_sampler(c, seed);
    c->h16_rows_for = 0;
    if (is_e(c)) {
        hipError_t e = c->e5_ws.reserve(usac::e5_workspace_bytes(B));
        if (e != hipSuccess) return e;
        // USAC_E5_THIN_CUS = k > 0: the root-order kernels on a stream masked to k CUs (default 0: the
        // context stream -- measured faster once every context has its own hardware queue)
        static const int thin_cus = getenv("USAC_E5_THIN_CUS") ? atoi(getenv("USAC_E5_THIN_CUS")) : 0;
        if (thin_cus > 0 && !c->thin_stream) {
            if ((e = StreamPool::get().masked_stream(thin_cus, &c->thin_stream)) != hipSuccess) return e;
            for (auto &ev : c->thin_ev)
                if (!ev && (e = StreamPool::get().event(&ev)) != hipSuccess) return e;
        }
        return usac::launch_solve_e5(c->stream, c->pts.as<float4>(), c->n, samples_dev, samples_out, B, ds,
                                     first_hyp, c->models.as<float>(), c->counts.as<int32_t>(),
                                     c->list.as<uint32_t>(), c->list_n.as<uint32_t>(), c->e5_ws.p, c->thin_stream,
                                     c->thin_ev[0], c->thin_ev[1]);
    }
    if (is_f(c))
        return usac::launch_solve_f7(c->stream, c->pts.as<float4>(), c->n, samples_dev, samples_out, B, ds,
                                     first_hyp, c->models.as<float>(), c->counts.as<int32_t>(),
                                     c->list.as<uint32_t>(), c->list_n.as<uint32_t>());
    if (is_h(c)) {
        usac::H16Emit em{nullptr, 0.f, nullptr, nullptr};
        if (h16_thr >= 0.f) {
            hipError_t e = h16_init(c);
            if (e == hipSuccess) e = c->h16_rows.reserve((size_t)B * 96);
            if (e == hipSuccess) e = c->h16_fm.reserve(sizeof(float) * (size_t)B);
            if (e != hipSuccess) return e;
            em = usac::H16Emit{c->h16_k.as<usac::H16Consts>(), h16_thr, c->h16_rows.p, c->h16_fm.as<float>()};
        }
        const hipError_t e = usac::launch_solve_h4(c->stream, c->pts.as<float4>(), c->n, samples_dev, samples_out, B,
                                                   ds, first_hyp, c->dlt_mode == USAC_DLT_NULLSPACE,
                                                   c->models.as<float>(), c->h4_fb.as<uint32_t>(),
                                                   c->h4_fb_n.as<uint32_t>(), em.rows ? &em : nullptr);
        if (e == hipSuccess && em.rows) {
            c->h16_rows_for = B;
            c->h16_rows_thr = h16_thr;
        }
        return e;
    }
    return usac::launch_solve_line(c->stream, c->pts.as<float2>(), c->n, samples_dev, samples_out, B, ds, first_hyp,
                                   c->models.as<float>());
}

// point chunks of the matrix-core scorer for a batch of B: ~16 waves per SIMD over the launch
// (20 hypotheses per wave; USAC_H16_CHUNKS overrides), at most one 32-point block per chunk and 256
uint32_t h16_chunks(const usac_ctx *c, uint32_t B) {
    static const int na = getenv("USAC_H16_NA") && atoi(getenv("USAC_H16_NA")) == 4 ? 4 : 2;
    const uint32_t waves = (B + 10 * na - 1) / (10 * na), nblk = (c->n + 31) / 32;
    static const int env_ch = getenv("USAC_H16_CHUNKS") ? atoi(getenv("USAC_H16_CHUNKS")) : 0;
    const uint32_t ch = env_ch > 0 ? (uint32_t)env_ch : (16384u + waves - 1) / waves;
    // at most 2^23 points per chunk: a hypothesis' fixed-point Σ partial of one chunk stays below 2^63
    // (launch_score_h16 refuses more); n <= 2^25 makes this at most 4
    const uint32_t min_ch = (nblk + (1u << 18) - 1) >> 18;
    return std::max(std::max(1u, min_ch), std::min(ch, std::min(nblk, 256u)));
}

// The matrix-core prefilter scorer (kernels_h16.hip): the point features once per context, each
// hypothesis' fp16 rows and slack per batch, then the scorer over point chunks -- enough chunks for
// ~16 waves per SIMD over the launch (20 hypotheses per wave; USAC_H16_CHUNKS overrides).
// the dataset constants and the point features, once per context (on its stream)
// the dataset constants (centres, power-of-two scales, feature maxima), shared by h16 and e16
hipError_t h16_consts_init(usac_ctx *c) {
    if (c->h16_k_ok) return hipSuccess;
    hipError_t e;
    if ((e = c->h16_k.reserve(sizeof(usac::H16Consts))) != hipSuccess) return e;
    if ((e = usac::launch_h16_consts(c->stream, c->pts.as<float4>(), c->n, c->ext, c->h16_k.as<usac::H16Consts>())) !=
        hipSuccess)
        return e;
    c->h16_k_ok = true;
    return hipSuccess;
}

hipError_t h16_init(usac_ctx *c) {
    if (c->h16_feat_ok) return hipSuccess;
    hipError_t e;
    if ((e = h16_consts_init(c)) != hipSuccess) return e;
    if ((e = c->h16_feat.reserve(usac::h16_feature_bytes(c->n))) != hipSuccess) return e;
    if ((e = usac::launch_h16_points(c->stream, c->pts.as<float4>(), c->n, c->h16_k.as<usac::H16Consts>(),
                                     c->h16_feat.p)) != hipSuccess)
        return e;
    c->h16_feat_ok = true;
    return hipSuccess;
}

// will enqueue_score(c, B, thr, chunks) take the matrix-core scorer?
bool h16_scores(const usac_ctx *c, int chunks);
// ... and should the solver write its rows (USAC_H16_FUSE=0: k_h16_rows after the solve, A/B)
float h16_solver_thr(const usac_ctx *c, int chunks, float thr) {
    static const bool fuse = !getenv("USAC_H16_FUSE") || atoi(getenv("USAC_H16_FUSE")) != 0;
    return fuse && h16_scores(c, chunks) ? thr : -1.f;
}
bool h16_scores(const usac_ctx *c, int chunks) {
    return is_h(c) && !c->sprt_on && c->h16 == 1 && !c->h16_off && (c->score_variant == 0 || c->score_variant == 3) &&
           chunks > 1;
}

// defer_finish: the chunk partials stay for the batch argmax (launch_argmax_h16, via batch_argmax)
hipError_t enqueue_score_h16(usac_ctx *c, uint32_t B, float thr, bool defer_finish) {
    hipError_t e;
    c->h16_deferred_ch = 0;
    if ((e = h16_init(c)) != hipSuccess) return e;
    const uint32_t ch = h16_chunks(c, B);
    if ((e = c->h16_part.reserve(usac::h16_part_bytes(B, (int)ch))) != hipSuccess) return e;
    const bool ready = c->h16_rows_for == B && c->h16_rows_thr == thr;  // written by the solver
    c->h16_rows_for = 0;
    if (!ready) {
        if ((e = c->h16_rows.reserve((size_t)B * 96)) != hipSuccess) return e;
        if ((e = c->h16_fm.reserve(sizeof(float) * (size_t)B)) != hipSuccess) return e;
        if ((e = usac::launch_h16_rows(c->stream, c->models.as<float>(), B, c->h16_k.as<usac::H16Consts>(), thr,
                                       c->h16_rows.p, c->h16_fm.as<float>())) != hipSuccess)
            return e;
    }
    e = usac::launch_score_h16(c->stream, c->h16_feat.p, c->pts.as<float4>(), c->n, c->h16_rows.p,
                               c->h16_fm.as<float>(), c->models.as<float>(), B, thr, (int)ch, c->h16_part.p,
                               c->counts.as<int32_t>(), c->sums.as<float>(), !defer_finish);
    if (e == hipSuccess && defer_finish) {
        c->h16_deferred_ch = ch;
        c->h16_deferred_thr = thr;
    }
    return e;
}

// The essential matrix-core prefilter scorer (kernels_e16.hip): throughput batches of listed models
// (chunks > 1: Σ re-associated, counts exact), the default score variant, USAC_E16 unset or 1
bool e16_scores(const usac_ctx *c, int chunks, float thr) {
    return is_e(c) && !c->sprt_on && c->e16 == 1 && c->score_variant == 0 && chunks > 1 && thr > 0x1p-100f &&
           thr < 0x1p100f;
}

// point chunks of the e16 scorer for kmax listed slots: ~12 waves per SIMD if every slot is
// occupied (64 models per wave), at most one 32-point block per chunk, 256 chunks, and >= 1 per
// 2^23 points (its fixed-point Σ bound)
uint32_t e16_chunks(const usac_ctx *c, uint32_t kmax) {
    const uint32_t waves = (kmax + 63) / 64, nblk = (c->n + 31) / 32;
    static const int env_ch = getenv("USAC_E16_CHUNKS") ? atoi(getenv("USAC_E16_CHUNKS")) : 0;
    const uint32_t ch = env_ch > 0 ? (uint32_t)env_ch : (12288u + waves - 1) / waves;
    const uint32_t min_ch = (nblk + (1u << 18) - 1) >> 18;
    return std::max(std::max(1u, min_ch), std::min(ch, std::min(nblk, 256u)));
}

// list / list_n: the batch's occupied slots (nullptr: models 0 .. kmax - 1)
hipError_t enqueue_score_e16(usac_ctx *c, uint32_t kmax, float thr, const uint32_t *list, const uint32_t *list_n) {
    hipError_t e;
    if ((e = h16_consts_init(c)) != hipSuccess) return e;
    if (!c->e16_feat_ok) {
        if ((e = c->e16_feat.reserve(usac::e16_feature_bytes(c->n))) != hipSuccess) return e;
        if ((e = usac::launch_e16_points(c->stream, c->pts.as<float4>(), c->n, c->h16_k.as<usac::H16Consts>(),
                                         c->e16_feat.p)) != hipSuccess)
            return e;
        c->e16_feat_ok = true;
    }
    const uint32_t ch = e16_chunks(c, kmax);
    if ((e = c->e16_rows.reserve(usac::e16_row_bytes(kmax))) != hipSuccess) return e;
    if ((e = c->e16_cm.reserve(sizeof(float) * (size_t)kmax)) != hipSuccess) return e;
    if ((e = c->e16_part.reserve(usac::e16_part_bytes(kmax, (int)ch))) != hipSuccess) return e;
    const size_t stride = kmax;
    if ((e = usac::launch_e16_rows(c->stream, c->models.as<float>(), stride, list, list_n, kmax,
                                   c->h16_k.as<usac::H16Consts>(), thr, c->e16_rows.p, c->e16_cm.as<float>())) !=
        hipSuccess)
        return e;
    return usac::launch_score_e16(c->stream, c->e16_feat.p, c->pts.as<float4>(), c->n, c->e16_rows.p,
                                  c->e16_cm.as<float>(), c->models.as<float>(), stride, list, list_n, kmax, thr,
                                  (int)ch, c->e16_part.p, c->counts.as<int32_t>(), c->sums.as<float>());
}

// chunks == 1 is the parity configuration: per-hypothesis sums are the exact sequential
// fp32 sums of the reference.  chunks > 1 re-associates Σerr across chunks (counts exact).
hipError_t enqueue_score(usac_ctx *c, uint32_t B, float thr, int chunks, bool defer_finish = false) {
    if (c->sprt_on) {
        hipError_t e = hipMemsetAsync(c->sprt_tested.p, 0, sizeof(uint32_t), c->stream);
        if (e != hipSuccess) return e;
        const uint32_t S = B * c->spk;
        c->sprt_S = S;
        e = c->sprt_surv.reserve(usac::sprt_survivor_bytes() * (size_t)S);
        if (e != hipSuccess) return e;
        e = c->sprt_starts.reserve(sizeof(uint32_t) * (size_t)S);
        if (e != hipSuccess) return e;
        return usac::launch_score_sprt(c->stream, c->estimator, c->sprt_pts.p, c->n, c->models.as<float>(),
                                       (size_t)S, listed(c) ? c->list.as<uint32_t>() : nullptr,
                                       listed(c) ? c->list_n.as<uint32_t>() : nullptr, S, thr, c->sprt_k,
                                       c->counts.as<int32_t>(), c->sums.as<float>(), c->sprt_tested.as<uint32_t>(),
                                       c->sprt_surv.p, c->sprt_surv_n.as<uint32_t>(), c->sprt_starts.as<uint32_t>());
    }
    if ((listed(c) || is_h(c)) && c->score_variant != 1 && c->rec_thr != thr) {  // fast-kernel point records
        hipError_t e = c->rec.reserve(sizeof(float) * 32 * (((size_t)c->n + 3) / 4));
        if (e != hipSuccess) return e;
        e = usac::launch_prepare_rec(c->stream, c->pts.as<float4>(), c->n, thr, c->rec.as<float4>());
        if (e != hipSuccess) return e;
        c->rec_thr = thr;
    }
    if (listed(c)) {  // the occupied slots of the last solve
        if (c->score_variant == 1)
            return usac::launch_score_f(c->stream, c->estimator, chunks, c->pts.as<float4>(), c->n,
                                        c->models.as<float>(), (size_t)B * c->spk, c->list.as<uint32_t>(),
                                        c->list_n.as<uint32_t>(), B * c->spk, thr, c->counts.as<int32_t>(),
                                        c->sums.as<float>());
        if (e16_scores(c, chunks, thr))  // counts exact
            return enqueue_score_e16(c, B * c->spk, thr, c->list.as<uint32_t>(), c->list_n.as<uint32_t>());
        hipError_t e = c->tv_part.reserve(usac::tv_scratch_bytes(B * c->spk, chunks));
        if (e != hipSuccess) return e;
        return usac::launch_score_f2(c->stream, c->estimator, chunks, c->rec.as<float4>(), c->pts.as<float4>(), c->n,
                                     c->ext, c->models.as<float>(),
                                     (size_t)B * c->spk, c->list.as<uint32_t>(), c->list_n.as<uint32_t>(), B * c->spk,
                                     thr, c->counts.as<int32_t>(), c->sums.as<float>(), c->tv_part.p);
    }
    if (is_h(c)) {
        if (c->score_variant == 1)
            return usac::launch_score_h(c->stream, chunks, c->pts.as<float4>(), c->n, c->models.as<float>(), B, thr,
                                        c->counts.as<int32_t>(), c->sums.as<float>());
        if (h16_scores(c, chunks)) return enqueue_score_h16(c, B, thr, defer_finish);  // counts exact
        uint32_t *perm = nullptr;
        if (c->score_variant == 0) {  // 2: fast kernel without the hypothesis pre-sort (A/B)
            hipError_t e = c->perm.reserve(usac::presort_bytes(B));
            if (e != hipSuccess) return e;
            if (c->perm_zeroed != c->perm.p) {  // a new block: its region counters start at 0
                e = hipMemsetAsync(c->perm.p, 0, usac::presort_counter_bytes(), c->stream);
                if (e != hipSuccess) return e;
                c->perm_zeroed = c->perm.p;
            }
            perm = c->perm.as<uint32_t>();
        }
        // small batches over many points (the loop's batches): split each tile's points over
        // several workgroups too, so the chip holds ~8 waves per SIMD
        uint32_t ys = 1;
        if (chunks > 1) {
            const uint32_t waves = (B + 63) / 64 * (uint32_t)chunks, groups = (c->n + 3) / 4;
            while (ys < 16 && waves * ys * 2 <= 8192u && groups / ((uint32_t)chunks * ys * 2) >= 64u) ys *= 2;
        }
        if (ys > 1) {
            hipError_t e = c->hf_part.reserve(sizeof(int32_t) * 2 * (size_t)ys * B);
            if (e != hipSuccess) return e;
        }
        return usac::launch_score_hf(c->stream, chunks, chunks == 1, c->rec.as<float4>(), c->n, c->ext,
                                     c->models.as<float>(), B, thr, perm, c->counts.as<int32_t>(), c->sums.as<float>(),
                                     ys, ys > 1 ? c->hf_part.p : nullptr);
    }
    return usac::launch_score_line(c->stream, chunks, c->pts.as<float2>(), c->n, c->models.as<float>(), B, thr,
                                   c->counts.as<int32_t>(), c->sums.as<float>());
}

// point chunks for the loop's batches (counts only -- the sums the replay reads are exact,
// exact_sums): lanes-over-hypotheses kernels need ~4 waves per SIMD, and the loop's batches
// are small (<= 8192 samples, often max_iterations), so H / line split the points finer
int loop_chunks(const usac_ctx *c, uint32_t B) {
    if (listed(c)) return c->chunks;
    const uint32_t tiles = (B + 63) / 64;
    int ch = c->chunks;
    while (ch < 16 && tiles * (uint32_t)ch < 4096u) ch *= 2;
    return ch;
}

// exact single-model inliers into c->inl_idx / inl_cnt / inl_sum (device)
hipError_t enqueue_inliers(usac_ctx *c, const float *model_dev, float thr) {
    hipError_t e = c->inl_scratch.reserve(usac::inliers_scratch_bytes(c->n, 1));
    if (e != hipSuccess) return e;
    return usac::launch_inliers(c->stream, c->estimator, c->pts.p, c->n, model_dev, thr, c->inl_idx.as<int32_t>(),
                                c->inl_cnt.as<int32_t>(), c->inl_sum.as<float>(), c->inl_scratch.p);
}

// ns_dev (nullable): the fit's point count on the device, n then only a bound on it
hipError_t enqueue_nonminimal(usac_ctx *c, const int32_t *idx_dev, uint32_t n, float *model_out = nullptr,
                              int32_t *ok_out = nullptr, const float *weights_dev = nullptr,
                              const uint32_t *ns_dev = nullptr, usac::NmBatch *batch_out = nullptr) {
    hipError_t e = c->nm_seq.reserve(usac::nonminimal_seq_bytes(n, 1));
    if (e != hipSuccess) return e;
    usac::NmBatch b{};
    // batch_out: the fit stops before its finish (NmBatch::skip_finish) and the batch is handed
    // back for launch_finish_score
    b.seq = c->nm_seq.p;
    b.base = idx_dev;
    b.n1 = n;
    b.W = 1;
    b.nmax = n;
    b.ns = ns_dev;
    b.fused_any = ns_dev != nullptr;
    b.q = c->q.p;
    b.partial = c->partial.as<double>();
    b.ws = c->ws.as<float>();
    b.model_out = model_out ? model_out : c->nm_model.as<float>();
    b.ok = ok_out ? ok_out : c->nm_ok.as<int32_t>();
    if (weights_dev) {
        if ((e = c->nm_qw.reserve(sizeof(float) * 4 * (size_t)n)) != hipSuccess) return e;
        b.weights = weights_dev;
        b.qw = c->nm_qw.p;
    }
    b.skip_finish = batch_out != nullptr;
    if (batch_out) *batch_out = b;
    return usac::launch_nonminimal_batch(c->stream, c->estimator, c->pts.p, b);
}

// The ranks of a sharded run and their all-gather of host bytes: the gather callback when one
// is given, else RCCL on the context's communicator (staged through device buffers).  Every
// payload is prefixed by the sender's status word, so a rank whose local part failed still
// joins the collective and every rank then fails with the first failing rank's status.
struct Shard {
    int nranks = 1, rank = 0;
    usac_allgather_fn gather = nullptr;
    void *user = nullptr;
};

int shard_allgather(usac_ctx *c, const Shard &sh, int status, const void *send, size_t bytes,
                    std::vector<uint8_t> &recv) {
    const size_t rb = 8 + ((bytes + 7) & ~(size_t)7);  // status word padded to 8, payload
    std::vector<uint8_t> mine(rb, 0);
    memcpy(mine.data(), &status, sizeof(status));
    if (bytes) memcpy(mine.data() + 8, send, bytes);
    recv.resize(rb * (size_t)sh.nranks);
    if (sh.gather) {
        if (sh.gather(sh.user, mine.data(), rb, recv.data()) != 0)
            return fail(c, USAC_ERR_ARG, "all-gather callback failed (gather callbacks must fail on every rank)");
    } else {
        if (!c->comm) return fail(c, USAC_ERR_ARG, "sharded run without a communicator");
        HIP_TRY(c, c->x_send.reserve(rb));
        HIP_TRY(c, c->x_recv.reserve(rb * (size_t)sh.nranks));
        pinned_vector<uint8_t> st(rb * (size_t)(sh.nranks + 1));
        memcpy(st.data(), mine.data(), rb);
        HIP_TRY(c, hipMemcpyAsync(c->x_send.p, st.data(), rb, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, order_after_exchanges(c));
        NCCL_TRY(c, ncclAllGather(c->x_send.p, c->x_recv.p, rb, ncclUint8, c->comm, c->stream));
        HIP_TRY(c, mark_collective(c));
        HIP_TRY(c, hipMemcpyAsync(st.data() + rb, c->x_recv.p, rb * (size_t)sh.nranks, hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, stream_wait(c->stream));
        memcpy(recv.data(), st.data() + rb, rb * (size_t)sh.nranks);
    }
    for (int r = 0; r < sh.nranks; r++) {
        int32_t st;
        memcpy(&st, recv.data() + (size_t)r * rb, sizeof(st));
        if (st != USAC_OK)
            return r == sh.rank ? st : fail(c, st, "sharded run: rank " + std::to_string(r) + " failed (status " +
                                                        std::to_string(st) + ")");
    }
    // payloads only, rank after rank (bytes each)
    for (int r = 0; r < sh.nranks; r++) memmove(recv.data() + (size_t)r * bytes, recv.data() + (size_t)r * rb + 8, bytes);
    recv.resize(bytes * (size_t)sh.nranks);
    return USAC_OK;
}

// LO-RANSAC: InnerLocalOptimization::GetModelScore (inner_local_optimization.hpp:74-133) with
// IterativeLocalOptimization (iterative_local_optimization.hpp:61-136).  lo_model's threshold
// persists across calls and compounds like the reference's; the LO mt19937 is
// seeded with seed + 1 (the reference: std::random_device).
//
// The reference runs its <= 20 inner iterations one after the other, each a chain of up to
// five dependent (least-squares fit -> scored inlier list) steps whose sequential fp32 sums
// make every step latency-bound.  Inner iteration j depends on the earlier ones only through
// (a) the best model / inlier list, which changes only when an iteration improves it,
// (b) the generator, which (unlimited variant) only the inner sample draws advance, and
// (c) the LO threshold each iteration starts from.  So all remaining iterations run at once
// as speculative chains: their samples are drawn up front under "no improvement", each starts
// from the threshold the previous one would leave after a completed iterative stage, and the
// chains advance in lockstep -- one batched fit launch, then one batched scoring launch, per
// stage (kernels_nonmin.hip / kernels_inliers.hip, W fits at once).  The host then replays
// the iterations in order with the reference's exact control flow: a chain whose start
// threshold was mis-predicted, or every chain after one that improved the best, is discarded
// and the speculation restarts there with the generator rewound to just after the last kept
// draw.  Every kept result is bit-identical to the sequential order.  The limited variant
// (InItFLORsc) draws inside the iterative stage, so it runs one chain at a time.
struct LoRansac {
    enum Phase { INNER_FIT, INNER_SCORE, ITER_FIT, ITER_SCORE, DONE };
    enum Outcome { RETURN, SKIP, FEW, ITERATED };
    struct Chain {
        float thr_start = 0.f, thr = 0.f;
        Phase phase = DONE;
        Outcome outcome = SKIP;
        int lo_cnt = 0;
        float lo_sum = 0.f;
        uint32_t it = 0, iter_count = 0;
        int32_t failed = 0, fit_pos = 0;
        float model[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        // the model and threshold that produced the chain's inlier list (its last successful
        // fit's scoring): a rank that does not own the chain rebuilds the list from them
        float list_model[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        float list_thr = 0.f;
    };

    usac_ctx *c;
    Shard sh;  // sharded run: chain w runs on rank w % nranks (unlimited variant only)
    usac::Mt19937 g;
    bool limited;
    uint32_t inner, iters, limit, mult, m, n, wmax;
    float theta, lo_thr, step;
    uint32_t inner_count = 0, iterative_count = 0;
    uint32_t rounds = 0, stages = 0, fits = 0;  // speculation rounds, device stages, fits (statistics)
    double t_enqueue = 0.0, t_poll = 0.0;          // host ms spent enqueuing stages / waiting for them (USAC_PROFILE)
    uint32_t graphs_built = 0;                      // iterative-stage graphs captured (USAC_PROFILE)
    int rc = USAC_OK;
    // entry best of the current call
    int best_cnt = 0;
    float best_sum = 0.f;
    std::vector<Chain> ch;
    std::vector<usac::Mt19937> g_after;  // generator after chain w's inner draw
    // A stage's inputs (ns, thresholds, slots, LSQ positions) and outputs (models, fit flags,
    // counts, Σ) as one pinned host block mirrored by one device block, one copy each way; two
    // such pairs (and two scoring scratch areas), by stage parity, so that a pipelined round
    // can have stage k + 1 on the device while the host reads stage k.
    void *pin = nullptr;
    size_t pin_bytes = 0, in_bytes = 0, out_bytes = 0, scr_bytes = 0;
    uint32_t *hns = nullptr, *hslots = nullptr;
    int32_t *hpos = nullptr, *hcnt = nullptr, *hok = nullptr;
    float *hthr = nullptr, *hsum = nullptr, *hmod = nullptr;
    float *hmodel = nullptr;  // pinned slot of the model a round starts from (its H2D copy)
    uint32_t *dns = nullptr, *dslots = nullptr;
    int32_t *dpos = nullptr, *dcnt = nullptr, *dok = nullptr;
    float *dthr = nullptr, *dsum = nullptr, *dmod = nullptr;
    int next_par = 0;  // block parity of the next pipelined stage (alternates across rounds too)

    LoRansac(usac_ctx *ctx, const usac_params *p, const Shard &shard)
        : c(ctx),
          sh(shard),
          g(p->seed + 1u),
          limited(p->lo == USAC_LO_INITFLORSC),
          inner(p->lo_inner_iterations),
          iters(p->lo_iterative_iterations),
          limit(p->lo_sample_size),
          mult(p->lo_threshold_multiplier),
          m(ctx->m),
          n(ctx->n),
          wmax(std::max<uint32_t>(1u, p->lo == USAC_LO_INITFLORSC ? 1u : p->lo_inner_iterations)),
          theta(p->threshold),
          lo_thr(p->threshold),
          step((p->threshold * p->lo_threshold_multiplier - p->threshold) / p->lo_iterative_iterations),
          ch(wmax),
          g_after(wmax, usac::Mt19937(0)) {}
    ~LoRansac() {
        if (pin) {  // a pipelined round's unread last stage may still copy into the blocks
            (void)hipStreamSynchronize(c->stream);
            if (c->lo_stream) (void)hipStreamSynchronize(c->lo_stream);
            PinnedPool::get().give_back(pin, pin_bytes);
        }
    }

    int reserve() {
        const size_t W = wmax, N = n, L = std::max<uint32_t>(1u, limit);
        HIP_TRY(c, c->lo_max.reserve(sizeof(int32_t) * N));
        HIP_TRY(c, c->lo_lists.reserve(sizeof(int32_t) * N * W));
        in_bytes = sizeof(uint32_t) * (3 * W + W * L);
        out_bytes = sizeof(float) * 12 * W;
        HIP_TRY(c, c->lo_io.reserve(2 * (in_bytes + out_bytes)));
        pin = PinnedPool::get().take(2 * (in_bytes + out_bytes) + sizeof(float) * 16, &pin_bytes);
        if (!pin) return fail(c, USAC_ERR_HIP, "hipHostMalloc (LO staging) failed");
        hmodel = reinterpret_cast<float *>(static_cast<char *>(pin) + 2 * (in_bytes + out_bytes));
        if (!limited && !c->lo_stream) {
            HIP_TRY(c, StreamPool::get().stream(&c->lo_stream));
            for (auto &ev : c->lo_ev) HIP_TRY(c, StreamPool::get().event(&ev));
        }
        set_block(0);
        HIP_TRY(c, c->lo_q.reserve(sizeof(float) * c->cols * N * W));
        HIP_TRY(c, c->lo_part.reserve(sizeof(double) * usac::nonminimal_partial_stride(n) * W));
        HIP_TRY(c, c->nm_seq.reserve(usac::nonminimal_seq_bytes(n, (uint32_t)W)));
        HIP_TRY(c, c->lo_ws.reserve(sizeof(float) * 18 * W));
        scr_bytes = usac::inliers_scratch_bytes(n, wmax);
        HIP_TRY(c, c->lo_scr.reserve(2 * scr_bytes));
        if (graphs()) {
            HIP_TRY(c, c->lo_best.reserve(sizeof(int32_t)));
            if (!c->lo_best_pin &&
                !(c->lo_best_pin = static_cast<int32_t *>(PinnedPool::get().take(sizeof(int32_t), &c->lo_best_pin_bytes))))
                return fail(c, USAC_ERR_HIP, "hipHostMalloc (LO best word) failed");
        }
        return USAC_OK;
    }
    // iterative stages as HIP graphs: the unlimited variant's pipelined stages, non-line fits
    bool graphs() const { return c->lo_graph_on && !limited && c->estimator != USAC_LINE2D; }

    // the host and device blocks of parity b: inputs then outputs (layout of both)
    void set_block(int b) {
        const size_t W = wmax, L = std::max<uint32_t>(1u, limit);
        auto lay = [&](uint32_t *w, uint32_t *&ns, float *&thr, uint32_t *&slots, int32_t *&pos, float *&mod,
                       int32_t *&ok, int32_t *&cnt, float *&sum) {
            ns = w;
            thr = reinterpret_cast<float *>(w + W);
            slots = w + 2 * W;
            pos = reinterpret_cast<int32_t *>(w + 3 * W);
            mod = reinterpret_cast<float *>(w + 3 * W + W * L);
            ok = reinterpret_cast<int32_t *>(mod + 9 * W);
            cnt = ok + W;
            sum = reinterpret_cast<float *>(cnt + W);
        };
        const size_t off = (size_t)b * (in_bytes + out_bytes) / sizeof(uint32_t);
        lay(static_cast<uint32_t *>(pin) + off, hns, hthr, hslots, hpos, hmod, hok, hcnt, hsum);
        lay(c->lo_io.as<uint32_t>() + off, dns, dthr, dslots, dpos, dmod, dok, dcnt, dsum);
    }
    void *scr(int b) const { return static_cast<char *>(c->lo_scr.p) + (size_t)b * scr_bytes; }
    int poll(hipEvent_t ev) {
        for (uint32_t spins = 0;; spins++) {
            const hipError_t e = hipEventQuery(ev);
            if (e == hipSuccess) return USAC_OK;
            if (e != hipErrorNotReady) return fail(c, USAC_ERR_HIP, std::string("LO stage: ") + hipGetErrorString(e));
            if ((spins & 1023u) == 1023u) std::this_thread::yield();
        }
    }
    static bool bigger(int c1, float s1, int c2, float s2) { return c1 > c2 || (c1 == c2 && s1 > s2); }
    // chains of this rank: all of them unless the run is sharded.  The limited variant draws
    // inside its iterative stage (one chain, the generator moves), so it is never split.
    bool own(uint32_t w) const { return sh.nranks == 1 || limited || (int)(w % (uint32_t)sh.nranks) == sh.rank; }

    // the threshold an inner iteration leaves when its iterative stage runs all its steps
    float predict(float t) const {
        t = (float)mult * t;
        for (uint32_t k = 0; k < iters; k++) t -= step;
        return fabsf(t - theta) > 0.00001 ? theta : t;
    }

    // IterativeLocalOptimization loop head: decrement, the break tests, then the next fit
    void iter_head(Chain &h, uint32_t w) {
        for (;;) {
            if (h.it >= iters) return finish(h);
            h.thr -= step;
            if (h.lo_cnt <= (int)m) return finish(h);
            h.fit_pos = false;
            if (limited && h.lo_cnt > (int)limit) {  // GetScoreLimited: a random subset of lo_inliers
                usac::unique_set(g, hpos + (size_t)w * limit, limit, (uint32_t)(h.lo_cnt - 1));
                h.fit_pos = true;
            }
            h.phase = ITER_FIT;
            return;
        }
    }
    void finish(Chain &h) {
        h.failed = fabsf(h.thr - theta) > 0.00001;  // double literal, as the reference
        if (h.failed) h.thr = theta;
        h.outcome = ITERATED;
        h.phase = DONE;
    }

    // one lockstep stage: the batched fit of every chain in INNER_FIT / ITER_FIT and, in the
    // same submission, the batched scoring of the fitted models at the threshold each chain
    // scores with after its fit (inner: K * thr, iterative: the already decremented thr); the
    // scoring leaves the index list of a failed fit alone (the limited variant refits from it).
    // One host synchronisation per stage; then every chain's state machine takes the fit
    // outcome and, if the fit succeeded, the score.  (A chain in a SCORE phase only arises
    // without a fused fit -- never here -- so it is scored on its own.)
    int stage(uint32_t W, int inner_cnt) {
        bool fit = false, score = false, inner_fit = false, iter_fit = false, pos = false;
        uint32_t nmax = 0, ns = 0;
        for (uint32_t w = 0; w < W; w++) {
            const Chain &h = ch[w];
            hns[w] = 0;
            if (!own(w)) continue;
            if (h.phase == INNER_FIT || h.phase == ITER_FIT) {
                fit = true;
                bool p;
                if (h.phase == INNER_FIT) {
                    inner_fit = true;
                    p = inner_cnt > (int)limit;
                    hns[w] = p ? limit : (uint32_t)inner_cnt;
                    hthr[w] = (float)mult * h.thr;
                } else {
                    iter_fit = true;
                    p = h.fit_pos;
                    hns[w] = p ? limit : (uint32_t)h.lo_cnt;
                    hthr[w] = h.thr;
                }
                pos = pos || p;
                fits++;
                hslots[ns++] = w;
                nmax = std::max(nmax, hns[w]);
            } else if (h.phase == INNER_SCORE || h.phase == ITER_SCORE) {
                score = true;
                hslots[ns++] = w;
                hthr[w] = h.thr;
            }
        }
        // never: fit and score stages alternate, and inner fits only open a round
        if ((fit && score) || (inner_fit && iter_fit)) return fail(c, USAC_ERR_HIP, "LO chains out of lockstep");
        if (pos) {
            // the position list is per launch: a fitting chain without its own positions
            // (GetScoreLimited with lo_cnt <= limit, or an inner fit of <= limit points) fits
            // its first hns[w] list entries -- identity positions (hns[w] <= limit)
            for (uint32_t w = 0; w < W; w++) {
                const Chain &h = ch[w];
                const bool fitting = own(w) && (h.phase == INNER_FIT || h.phase == ITER_FIT);
                const bool own = h.phase == INNER_FIT ? inner_cnt > (int)limit : h.fit_pos;
                if (fitting && !own)
                    for (uint32_t i = 0; i < hns[w]; i++) hpos[(size_t)w * limit + i] = (int32_t)i;
            }
        }
        hipStream_t st = c->stream;
        HIP_TRY(c, hipMemcpyAsync(dns, hns, in_bytes, hipMemcpyHostToDevice, st));
        if (fit) {
            usac::NmBatch b{};
            b.base = inner_fit ? c->lo_max.as<int32_t>() : c->lo_lists.as<int32_t>();
            b.base_stride = inner_fit ? 0 : n;
            b.pos = pos ? dpos : nullptr;
            b.pos_stride = limit;
            b.ns = dns;
            b.W = W;
            b.nmax = nmax;
            b.q = c->lo_q.p;
            b.q_stride = n;
            b.partial = c->lo_part.as<double>();
            b.p_stride = usac::nonminimal_partial_stride(n);
            b.ws = c->lo_ws.as<float>();
            b.model_out = dmod;
            b.ok = dok;
            b.seq = c->nm_seq.p;
            HIP_TRY(c, usac::launch_nonminimal_batch(st, c->estimator, c->pts.p, b));
        }
        HIP_TRY(c, usac::launch_inliers_batch(st, c->estimator, c->pts.p, n, dmod, ns, 0.f, dthr, dslots,
                                              c->lo_lists.as<int32_t>(), n, dcnt, dsum, scr(0), fit ? dok : nullptr));
        HIP_TRY(c, hipMemcpyAsync(hmod, dmod, out_bytes, hipMemcpyDeviceToHost, st));
        HIP_TRY(c, stream_wait(st));
        stages++;
        take(W, inner_cnt);
        return USAC_OK;
    }

    // the chains' state machines take a stage's outputs (host block in use: hmod, hok, hcnt,
    // hsum, hthr)
    void take(uint32_t W, int inner_cnt) {
        for (uint32_t w = 0; w < W; w++) {
            Chain &h = ch[w];
            if (!own(w)) continue;
            switch (h.phase) {
                case INNER_FIT:  // LeastSquaresFitting(lo_sample | max_inliers) -> lo_model
                    memcpy(h.model, hmod + 9 * (size_t)w, sizeof(h.model));
                    if (!hok[w]) {
                        h.outcome = inner_cnt > (int)limit ? SKIP : RETURN;
                        h.phase = DONE;
                    } else {
                        h.thr = (float)mult * h.thr;  // K * theta
                        scored_list(h, w);
                        inner_scored(h, w);
                    }
                    break;
                case INNER_SCORE:
                    inner_scored(h, w);
                    break;
                case ITER_FIT:
                    memcpy(h.model, hmod + 9 * (size_t)w, sizeof(h.model));
                    if (hok[w]) {
                        scored_list(h, w);
                        iter_scored(h, w);
                    } else if (h.fit_pos) {  // GetScoreLimited: continue
                        h.it++;
                        iter_head(h, w);
                    } else {
                        finish(h);  // break
                    }
                    break;
                case ITER_SCORE:
                    iter_scored(h, w);
                    break;
                default:
                    break;
            }
        }
    }
    // a fitted model was scored: lo_lists[w] now holds its inliers at the chain's threshold
    // (inner: K * theta, iterative: the already decremented one -- the stage's scoring threshold)
    void scored_list(Chain &h, uint32_t) {
        memcpy(h.list_model, h.model, sizeof(h.model));
        h.list_thr = h.thr;
    }
    // the inner iteration's scoring of lo_model at K * theta
    void inner_scored(Chain &h, uint32_t w) {
        h.lo_cnt = hcnt[w];
        h.lo_sum = hsum[w];
        if (h.lo_cnt <= (int)m) {
            h.outcome = FEW;
            h.phase = DONE;
        } else {
            h.it = 0;
            h.iter_count = 0;
            iter_head(h, w);
        }
    }
    // an iterative step's scoring of its fit
    void iter_scored(Chain &h, uint32_t w) {
        h.lo_cnt = hcnt[w];
        h.lo_sum = hsum[w];
        if (!limited && bigger(best_cnt, best_sum, h.lo_cnt, h.lo_sum)) {
            finish(h);  // GetScoreUnlimited: the best is bigger -> break
        } else {
            h.iter_count++;
            h.it++;
            iter_head(h, w);
        }
    }

    // ---- pipelined rounds (the unlimited variant): stage k + 1 is on the device while the
    // host reads stage k.  Everything a stage needs is known before stage k's outputs are read
    // except the point counts of its fits: each chain's threshold follows a fixed schedule
    // (K * theta_start, then one step less per iterative fit), its list is on the device, and
    // the fit's gather derives its n from stage k's outputs on the device -- zero, a no-op fit
    // and scoring that leave the chain's list alone, once the chain has certainly stopped
    // (failed fit, <= m inliers, fewer inliers than the best).  A count tie with the best
    // needs Σ to decide; the device continues such a chain, and if the host's state machine
    // (which reads every stage in order, exactly as the sequential stages did) stops it, its
    // later speculative fits are never read -- a chain stopped by the comparison never
    // improves the best, so its list is never used either.  The scoring's Σ runs on the side
    // stream beside the next stage's fit.  The stage after a round's last is usually already
    // queued: it runs for nothing, ordered before every later use of the LO buffers.
    int enqueue_pipe(uint32_t k, uint32_t W, int inner_cnt) {
        const int b = next_par;
        next_par ^= 1;
        set_block(b ^ 1);  // the previous stage's device block (the count derivation's inputs)
        const uint32_t *pns = dns;
        const int32_t *pok = dok, *pcnt = dcnt;
        const float *pthr = dthr;
        set_block(b);
        hipStream_t st = c->stream;
        const bool pos = k == 0 && inner_cnt > (int)limit;
        uint32_t nmax = 0;
        if (k == 0) {  // the round's inner fits: inputs from the host
            for (uint32_t w = 0; w < W; w++) {
                hslots[w] = w;
                hthr[w] = (float)mult * ch[w].thr_start;
                hns[w] = own(w) ? (pos ? limit : (uint32_t)inner_cnt) : 0u;
                nmax = std::max(nmax, hns[w]);
            }
            HIP_TRY(c, hipMemcpyAsync(dns, hns, in_bytes, hipMemcpyHostToDevice, st));
            if (graphs()) {  // the round's best count, read by the captured iterative stages
                *c->lo_best_pin = best_cnt;
                HIP_TRY(c, hipMemcpyAsync(c->lo_best.p, c->lo_best_pin, sizeof(int32_t), hipMemcpyHostToDevice, st));
            }
        }
        // iterative fits: counts and thresholds derived on the device from the previous stage
        // (by the fit's first kernel)
        const bool graph = k > 0 && graphs();
        const usac::LoPrep prep{pns,      pok, pcnt, pthr, dns, dthr, (int32_t)m, best_cnt, k > 1 ? 1 : 0, step,
                                graph ? c->lo_best.as<int32_t>() : nullptr};
        usac::NmBatch nb{};
        nb.base = k == 0 ? c->lo_max.as<int32_t>() : c->lo_lists.as<int32_t>();
        nb.base_stride = k == 0 ? 0 : n;
        nb.pos = pos ? dpos : nullptr;
        nb.pos_stride = limit;
        nb.ns = dns;
        nb.W = W;
        nb.nmax = k == 0 ? nmax : n;  // iterative fits: n bounds the counts on the device
        nb.fused_any = k > 0;
        nb.prep = k > 0 ? &prep : nullptr;
        nb.q = c->lo_q.p;
        nb.q_stride = n;
        nb.partial = c->lo_part.as<double>();
        nb.p_stride = usac::nonminimal_partial_stride(n);
        nb.ws = c->lo_ws.as<float>();
        nb.model_out = dmod;
        nb.ok = dok;
        nb.seq = c->nm_seq.p;
        auto launch = [&]() -> hipError_t {
            hipError_t e = usac::launch_nonminimal_batch(st, c->estimator, c->pts.p, nb);
            if (e == hipSuccess)
                e = usac::launch_inliers_batch(st, c->estimator, c->pts.p, n, dmod, W, 0.f, dthr, nullptr,
                                               c->lo_lists.as<int32_t>(), n, dcnt, nullptr, scr(b), dok);
            return e;
        };
        if (graph) {  // the stage's ten kernels as one graph launch (captured once per shape)
            float stepv = step;
            uint32_t stepbits;
            memcpy(&stepbits, &stepv, 4);
            int dev = 0;
            (void)hipGetDevice(&dev);
            const std::vector<uintptr_t> key = {
                (uintptr_t)dev, (uintptr_t)b, (uintptr_t)(k > 1), W, n, (uintptr_t)c->estimator, stepbits, m,
                (uintptr_t)c->pts.p,
                (uintptr_t)c->lo_io.p, (uintptr_t)c->lo_q.p, (uintptr_t)c->lo_part.p, (uintptr_t)c->lo_ws.p,
                (uintptr_t)c->nm_seq.p, (uintptr_t)c->lo_lists.p, (uintptr_t)c->lo_max.p, (uintptr_t)c->lo_scr.p,
                (uintptr_t)c->lo_best.p, scr_bytes, in_bytes, out_bytes,
                // the blocks' reserved sizes (DevPool may hand an address out again with less behind it)
                c->pts.bytes, c->lo_io.bytes, c->lo_q.bytes, c->lo_part.bytes, c->lo_ws.bytes, c->nm_seq.bytes,
                c->lo_lists.bytes, c->lo_max.bytes, c->lo_scr.bytes, c->lo_best.bytes};
            GraphCache &gc = GraphCache::get();
            hipGraphExec_t ex = nullptr;
            {
                std::lock_guard<std::mutex> lk(gc.mu);
                auto it = gc.g.find(key);
                if (it != gc.g.end()) ex = it->second;
            }
            bool full = false;
            if (!ex) {
                std::lock_guard<std::mutex> lk(gc.mu);
                full = gc.g.size() >= GraphCache::kMax;
            }
            if (!ex && full) {
                HIP_TRY(c, launch());
            } else if (!ex) {
                HIP_TRY(c, hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
                const hipError_t le = launch();
                hipGraph_t g = nullptr;
                const hipError_t ce = hipStreamEndCapture(st, &g);
                if (le != hipSuccess || ce != hipSuccess) {
                    if (g) (void)hipGraphDestroy(g);
                    return fail(c, USAC_ERR_HIP, std::string("LO stage capture: ") +
                                                     hipGetErrorString(le != hipSuccess ? le : ce));
                }
                const hipError_t ie = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
                (void)hipGraphDestroy(g);
                if (ie != hipSuccess) return fail(c, USAC_ERR_HIP, std::string("LO stage graph: ") + hipGetErrorString(ie));
                {
                    std::lock_guard<std::mutex> lk(gc.mu);
                    auto ins = gc.g.emplace(key, ex);
                    if (!ins.second) {  // another thread captured the same stage meanwhile
                        (void)hipGraphExecDestroy(ex);
                        ex = ins.first->second;
                    }
                }
                graphs_built++;
                HIP_TRY(c, hipGraphLaunch(ex, st));
            } else {
                HIP_TRY(c, hipGraphLaunch(ex, st));
            }
        } else {
            HIP_TRY(c, launch());
        }
        // the side stream: Σ, then every output of the stage into the host block
        HIP_TRY(c, hipEventRecord(c->lo_ev[b], st));
        HIP_TRY(c, hipStreamWaitEvent(c->lo_stream, c->lo_ev[b], 0));
        HIP_TRY(c, usac::launch_inliers_sums(c->lo_stream, n, W, nullptr, dcnt, dsum, scr(b)));
        HIP_TRY(c, hipMemcpyAsync(hmod, dmod, out_bytes, hipMemcpyDeviceToHost, c->lo_stream));
        HIP_TRY(c, hipEventRecord(c->lo_ev[2 + b], c->lo_stream));
        return USAC_OK;
    }

    int round_pipe(uint32_t W, int inner_cnt) {
        const int b0 = next_par;
        uint32_t queued = 0;  // stages 0 .. queued - 1 are on the device
        auto now = [] { return std::chrono::steady_clock::now(); };
        auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        auto t0 = now();
        int r = enqueue_pipe(queued++, W, inner_cnt);
        if (!r && iters > 0) r = enqueue_pipe(queued++, W, inner_cnt);
        t_enqueue += ms(t0, now());
        for (uint32_t k = 0; !r; k++) {
            const int b = (b0 + (int)k) & 1;
            t0 = now();
            r = poll(c->lo_ev[2 + b]);
            t_poll += ms(t0, now());
            if (r) break;
            set_block(b);
            for (uint32_t w = 0; w < W; w++)
                if (own(w) && (ch[w].phase == INNER_FIT || ch[w].phase == ITER_FIT)) fits++;
            stages++;
            take(W, inner_cnt);
            bool active = false;
            for (uint32_t w = 0; w < W; w++) active |= own(w) && ch[w].phase != DONE;
            if (!active) break;
            // an active chain fits again at stage k + 1 <= iters, which is queued
            if (queued < k + 2) {
                r = fail(c, USAC_ERR_HIP, "LO pipeline out of step");
                break;
            }
            if (k + 2 <= iters && queued == k + 2) {
                t0 = now();
                r = enqueue_pipe(queued++, W, inner_cnt);
                t_enqueue += ms(t0, now());
            }
        }
        // later main-stream users of the LO scratch wait for the side stream's last Σ pass
        if (!r) {
            hipError_t e = hipEventRecord(c->lo_ev[4], c->lo_stream);
            if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->lo_ev[4], 0);
            if (e != hipSuccess) r = fail(c, USAC_ERR_HIP, std::string("LO stage: ") + hipGetErrorString(e));
        } else {
            (void)hipStreamSynchronize(c->stream);
            (void)hipStreamSynchronize(c->lo_stream);
        }
        return r;
    }

    // GetModelScore(best_model, best_score): model / (cnt, sum) improved in place
    void run(float *model, int &cnt, float &sum) {
        if (cnt < 12 || rc) return;
        // quality->getInliers(best_model) -> max_inliers (device)
        memcpy(hmodel, model, sizeof(float) * 9);  // (the previous round's copy has completed)
        hipError_t e = hipMemcpyAsync(c->one_model.p, hmodel, sizeof(float) * 9, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = c->inl_scratch.reserve(usac::inliers_scratch_bytes(n, 1));
        if (e == hipSuccess)
            e = usac::launch_inliers(c->stream, c->estimator, c->pts.p, n, c->one_model.as<float>(), theta,
                                     c->lo_max.as<int32_t>(), c->inl_cnt.as<int32_t>(), c->inl_sum.as<float>(),
                                     c->inl_scratch.p);
        if (e != hipSuccess) {
            rc = fail(c, USAC_ERR_HIP, std::string("LO inliers: ") + hipGetErrorString(e));
            return;
        }
        uint32_t j0 = 0;
        while (j0 < inner && !rc) {
            // speculate iterations j0 .. j0 + W - 1 under "no improvement"
            const uint32_t W = std::min(wmax, inner - j0);
            const usac::Mt19937 g_before = g;
            best_cnt = cnt;
            best_sum = sum;
            float t = lo_thr;
            set_block(limited ? 0 : next_par);  // the round's first stage block (its LSQ positions)
            for (uint32_t w = 0; w < W; w++) {
                Chain &h = ch[w];
                h = Chain();
                h.thr_start = h.thr = t;
                h.phase = INNER_FIT;
                if (cnt > (int)limit) {
                    usac::unique_set(g, hpos + (size_t)w * limit, limit, (uint32_t)(cnt - 1));
                }
                g_after[w] = g;
                t = predict(t);
            }
            rounds++;
            int st = USAC_OK;
            if (!limited) {
                st = round_pipe(W, cnt);
            } else {
                for (;;) {
                    bool active = false;
                    for (uint32_t w = 0; w < W; w++) active |= own(w) && ch[w].phase != DONE;
                    if (!active) break;
                    if ((st = stage(W, cnt))) break;
                }
            }
            if (sh.nranks > 1 && !limited) {  // every rank's chains, one all-gather per round
                std::vector<uint8_t> all;
                if ((rc = shard_allgather(c, sh, st, ch.data(), sizeof(Chain) * W, all))) return;
                for (uint32_t w = 0; w < W; w++)
                    if (!own(w))
                        memcpy(&ch[w], all.data() + sizeof(Chain) * ((size_t)(w % (uint32_t)sh.nranks) * W + w),
                               sizeof(Chain));
            } else if ((rc = st)) {
                return;
            }
            if (limited) g_after[0] = g;  // the iterative stage's draws
            // replay in order
            bool restart = false;
            uint32_t w = 0;
            for (; w < W; w++) {
                const Chain &h = ch[w];
                if (memcmp(&h.thr_start, &lo_thr, sizeof(float)) != 0) {  // mis-predicted start
                    g = w ? g_after[w - 1] : g_before;
                    j0 += w;
                    restart = true;
                    break;
                }
                if (h.outcome == RETURN) {
                    g = g_after[w];
                    return;
                }
                if (h.outcome == SKIP) continue;
                lo_thr = h.thr;
                if (h.outcome == FEW) continue;
                iterative_count += h.iter_count;
                inner_count++;
                if (!h.failed && bigger(h.lo_cnt, h.lo_sum, cnt, sum)) {
                    memcpy(model, h.model, sizeof(h.model));
                    cnt = h.lo_cnt;
                    sum = h.lo_sum;
                    if (own(w)) {
                        e = hipMemcpyAsync(c->lo_max.p, c->lo_lists.as<int32_t>() + (size_t)w * n,
                                           sizeof(int32_t) * (size_t)cnt, hipMemcpyDeviceToDevice, c->stream);
                    } else {  // another rank's chain: its list is the inliers of (list_model, list_thr)
                        memcpy(hmodel, h.list_model, sizeof(float) * 9);
                        e = hipMemcpyAsync(c->one_model.p, hmodel, sizeof(float) * 9, hipMemcpyHostToDevice, c->stream);
                        if (e == hipSuccess)
                            e = usac::launch_inliers(c->stream, c->estimator, c->pts.p, n, c->one_model.as<float>(),
                                                     h.list_thr, c->lo_max.as<int32_t>(), c->inl_cnt.as<int32_t>(),
                                                     c->inl_sum.as<float>(), c->inl_scratch.p);
                        // hmodel is reused by the next H2D copy: that copy is queued behind this one
                        if (e == hipSuccess) e = stream_wait(c->stream);
                    }
                    if (e != hipSuccess) {
                        rc = fail(c, USAC_ERR_HIP, std::string("LO inliers copy: ") + hipGetErrorString(e));
                        return;
                    }
                    g = g_after[w];
                    j0 += w + 1;
                    restart = true;
                    break;
                }
            }
            if (!restart) {
                g = g_after[W - 1];
                j0 += W;
            }
        }
    }
};

constexpr uint32_t kExactSumsMax = 64;  // models per exact_sums launch

// exact_sums' buffers at their full size, before the loop: growing a DevBuf synchronises the
// device, and under the speculation that waited for the speculative batch (plus a hipMalloc) --
// 0.47 ms a cfg5 run (USAC_PROFILE, round 4)
int reserve_exact_sums(usac_ctx *c) {
    HIP_TRY(c, c->lo_models.reserve(sizeof(float) * 9 * kExactSumsMax));
    HIP_TRY(c, c->lo_cnts.reserve(sizeof(int32_t) * kExactSumsMax));
    HIP_TRY(c, c->lo_sums.reserve(sizeof(float) * kExactSumsMax));
    HIP_TRY(c, c->lo_scr.reserve(usac::inliers_scratch_bytes(c->n, kExactSumsMax)));
    return USAC_OK;
}

// Σerr where the replay can read it.  The loop compares a model's Σ only against the running
// best with an equal count, and stores it only when the model becomes the best (Score::bigger,
// quality.hpp:22-31); both need count >= the running best count, which is at least
// max(best count at batch start, every earlier count of the batch).  So only the slots whose
// count reaches that running maximum get the reference's sequential fp32 sum -- computed
// exactly on the device, 64 models per launch (launch_inliers_batch) -- and the batch itself
// is scored by the fast multi-chunk kernel, whose counts are exact.  Other slots' sums are
// never read.  The recount doubles as a check of the fast kernel's counts.
int exact_sums(usac_ctx *c, float thr, int best_count, const int32_t *hc, const float *hmod, size_t SB, size_t S,
               float *hsum, uint32_t *n_models) {
    constexpr uint32_t kMax = kExactSumsMax;
    std::vector<uint32_t> cand;
    int run_max = best_count;
    for (size_t sl = 0; sl < S; sl++) {
        if (hc[sl] < 0) continue;
        if (hc[sl] >= run_max) {
            cand.push_back((uint32_t)sl);
            run_max = hc[sl];
        }
    }
    if (cand.empty()) return USAC_OK;
    const int nc = ncomp(c);
    pinned_vector<float> am(9 * (size_t)kMax);
    pinned_vector<int32_t> cc(kMax);
    pinned_vector<float> cs(kMax);
    HIP_TRY(c, c->lo_models.reserve(sizeof(float) * 9 * kMax));
    HIP_TRY(c, c->lo_cnts.reserve(sizeof(int32_t) * kMax));
    HIP_TRY(c, c->lo_sums.reserve(sizeof(float) * kMax));
    HIP_TRY(c, c->lo_scr.reserve(usac::inliers_scratch_bytes(c->n, kMax)));
    for (size_t k0 = 0; k0 < cand.size(); k0 += kMax) {
        const uint32_t K = (uint32_t)std::min<size_t>(kMax, cand.size() - k0);
        for (uint32_t k = 0; k < K; k++)
            for (int e = 0; e < 9; e++) am[9 * k + e] = e < nc ? hmod[(size_t)e * SB + cand[k0 + k]] : 0.f;
        HIP_TRY(c, hipMemcpyAsync(c->lo_models.p, am.data(), sizeof(float) * 9 * K, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, usac::launch_inliers_batch(c->stream, c->estimator, c->pts.p, c->n, c->lo_models.as<float>(), K, thr,
                                              nullptr, nullptr, nullptr, 0, c->lo_cnts.as<int32_t>(),
                                              c->lo_sums.as<float>(), c->lo_scr.p));
        HIP_TRY(c, hipMemcpyAsync(cc.data(), c->lo_cnts.p, sizeof(int32_t) * K, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipMemcpyAsync(cs.data(), c->lo_sums.p, sizeof(float) * K, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, stream_wait(c->stream));
        for (uint32_t k = 0; k < K; k++) {
            if (cc[k] != hc[cand[k0 + k]])
                return fail(c, USAC_ERR_HIP, "score kernel count differs from the exact recount (slot " +
                                                 std::to_string(cand[k0 + k]) + ": " + std::to_string(hc[cand[k0 + k]]) +
                                                 " vs " + std::to_string(cc[k]) + ")");
            hsum[cand[k0 + k]] = cs[k];
        }
    }
    *n_models += (uint32_t)cand.size();
    return USAC_OK;
}

// Graph-cut LO: GraphCut::GetModelScore (graphcut.hpp:99-153) with GraphCut::labeling
// (graphcut.cpp:7-101).  Per labelling: the device computes every point's exact residual
// under the best model; the host turns them into the reference's energies -- unary
// exp(-(e*e) / (2 thr^2)) (float argument, double exp as the reference's unqualified exp of
// a float), pairwise terms over the KNN (device usac_knn) or grid neighbour lists, skipping
// non-submodular / NaN terms, lambda = spatial_coherence_gc as given (model.hpp:33 default 0.1;
// graphcut.hpp:43 uses it unchanged, 0 = no pairwise term) -- and runs
// the reference's BK min cut (usac_maxflow.hpp); inliers = SINK nodes.  The <=
// lo_inner_iterations least-squares fits on 7m-point subsets of the labelling's inliers do
// not depend on each other (only the comparisons with the best do), so all of them run as
// one batched fit and one batched scoring on the device, then the host replays them in
// order (a failed fit ends the round; the generator is rewound to just after its draw).
// Its mt19937 is seeded with seed + 1 (reference: std::random_device).
struct GcLo {
    usac_ctx *c;
    usac::Mt19937 g;
    uint32_t inner, m, n, limit;
    float thr, lambda, sqr_thr;
    const int32_t *knn_tab;
    uint32_t knn;
    const usac::GridNeighbors *grid;
    uint32_t gc_iters = 0, labelings = 0, stages = 0;
    int rc = USAC_OK;
    std::vector<float> err, en, hsum, hmod;
    std::vector<int32_t> inl, hpos, hcnt, hok;
    std::vector<usac::Mt19937> g_after;

    GcLo(usac_ctx *ctx, const usac_params *p, const int32_t *knn_table, uint32_t k, const usac::GridNeighbors *gr)
        : c(ctx),
          g(p->seed + 1u),
          inner(p->lo_inner_iterations),
          m(ctx->m),
          n(ctx->n),
          limit(7 * ctx->m),
          thr(p->threshold),
          lambda(p->spatial_coherence_gc),
          sqr_thr(2 * p->threshold * p->threshold),
          knn_tab(knn_table),
          knn(k),
          grid(gr),
          err(ctx->n),
          en(ctx->n),
          hsum(std::max<uint32_t>(1u, p->lo_inner_iterations)),
          hmod(9 * (size_t)std::max<uint32_t>(1u, p->lo_inner_iterations)),
          inl(ctx->n),
          hpos((size_t)7 * ctx->m * std::max<uint32_t>(1u, p->lo_inner_iterations)),
          hcnt(std::max<uint32_t>(1u, p->lo_inner_iterations)),
          hok(std::max<uint32_t>(1u, p->lo_inner_iterations)),
          g_after(std::max<uint32_t>(1u, p->lo_inner_iterations), usac::Mt19937(0)) {}

    int reserve() {
        const size_t W = std::max<uint32_t>(1u, inner);
        HIP_TRY(c, c->lo_max.reserve(sizeof(int32_t) * n));
        HIP_TRY(c, c->lo_pos.reserve(sizeof(int32_t) * hpos.size()));
        HIP_TRY(c, c->lo_models.reserve(sizeof(float) * 9 * W));
        HIP_TRY(c, c->lo_ok.reserve(sizeof(int32_t) * W));
        HIP_TRY(c, c->lo_cnts.reserve(sizeof(int32_t) * W));
        HIP_TRY(c, c->lo_sums.reserve(sizeof(float) * W));
        HIP_TRY(c, c->lo_q.reserve(sizeof(float) * c->cols * limit * W));
        HIP_TRY(c, c->lo_part.reserve(sizeof(double) * usac::nonminimal_partial_stride(limit) * W));
        HIP_TRY(c, c->nm_seq.reserve(usac::nonminimal_seq_bytes(limit, (uint32_t)W)));
        HIP_TRY(c, c->lo_ws.reserve(sizeof(float) * 18 * W));
        HIP_TRY(c, c->lo_scr.reserve(usac::inliers_scratch_bytes(n, (uint32_t)W)));
        HIP_TRY(c, c->gc_err.reserve(sizeof(float) * n));
        return USAC_OK;
    }

    static bool bigger(int c1, float s1, int c2, float s2) { return c1 > c2 || (c1 == c2 && s1 > s2); }

    // GraphCut::labeling -> number of SINK nodes, their ascending list in inl (host) and lo_max
    int labeling(const float *model) {
        HIP_TRY(c, hipMemcpyAsync(c->one_model.p, model, sizeof(float) * 9, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, usac::launch_point_errors(c->stream, c->estimator, c->pts.p, n, c->one_model.as<float>(),
                                             c->gc_err.as<float>()));
        HIP_TRY(c, hipMemcpyAsync(err.data(), c->gc_err.p, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, stream_wait(c->stream));
        for (uint32_t i = 0; i < n; i++) {
            const float d = err[i];
            en[i] = (float)std::exp((double)(-(d * d) / sqr_thr));
        }
        usac::BkGraph G((int)n, knn_tab ? (size_t)knn * n : (size_t)n);
        for (uint32_t i = 0; i < n; i++) G.add_node();
        for (uint32_t i = 0; i < n; i++) G.add_term1((int)i, en[i], 0.f);
        const float e01 = 1.f, e10 = 1.f;
        for (uint32_t i = 0; i < n; i++) {
            const float energy1 = en[i];
            const uint32_t cnt = knn_tab ? knn : grid->count(i);
            for (uint32_t k = 0; k < cnt; k++) {
                const int32_t j = knn_tab ? knn_tab[(size_t)knn * i + k] : grid->at(i, k);
                if (j == (int32_t)i || j < 0) continue;
                const float energy2 = en[j];
                const float e00 = (energy1 + energy2) / 2;
                const float e11 = 1 - e00;
                if (e00 + e11 > e01 + e10 || std::isnan(e00)) continue;
                G.add_term2((int)i, j, e00 * lambda, e01 * lambda, e10 * lambda, e11 * lambda);
            }
        }
        G.maxflow();
        int L = 0;
        for (uint32_t i = 0; i < n; i++)
            if (G.is_sink((int)i)) inl[L++] = (int32_t)i;
        if (L > 0)
            HIP_TRY(c, hipMemcpyAsync(c->lo_max.p, inl.data(), sizeof(int32_t) * L, hipMemcpyHostToDevice, c->stream));
        labelings++;
        return L;
    }

    void run(float *model, int &cnt, float &sum) {
        bool updated = true;
        while (updated && !rc) {
            updated = false;
            const int L = labeling(model);
            if (L < 0) {
                rc = L;
                return;
            }
            if (L <= (int)m) break;
            const bool sampled = (uint32_t)L > limit;
            const uint32_t W = std::min<uint32_t>(inner, sampled ? inner : 1u);
            if (W == 0) break;
            for (uint32_t w = 0; w < W; w++) {
                if (sampled) usac::unique_set(g, hpos.data() + (size_t)w * limit, limit, (uint32_t)(L - 1));
                g_after[w] = g;
            }
            if ((rc = fit_and_score(W, sampled ? limit : (uint32_t)L, sampled))) return;
            uint32_t w = 0;
            for (; w < W; w++) {
                if (!hok[w]) break;  // EstimateModelNonMinimalSample failed: end of this round
                if (bigger(hcnt[w], hsum[w], cnt, sum)) {
                    updated = true;
                    cnt = hcnt[w];
                    sum = hsum[w];
                    memcpy(model, hmod.data() + 9 * (size_t)w, sizeof(float) * 9);
                }
                gc_iters++;
            }
            g = g_after[w < W ? w : W - 1];
        }
    }

    // W least-squares fits (sampled positions into lo_max, or all npts of it) and their
    // (count, sequential sum) at the model threshold
    int fit_and_score(uint32_t W, uint32_t npts, bool sampled) {
        hipStream_t st = c->stream;
        if (sampled)
            HIP_TRY(c, hipMemcpyAsync(c->lo_pos.p, hpos.data(), sizeof(int32_t) * (size_t)W * limit,
                                      hipMemcpyHostToDevice, st));
        usac::NmBatch b{};
        b.base = c->lo_max.as<int32_t>();
        b.base_stride = 0;
        b.pos = sampled ? c->lo_pos.as<int32_t>() : nullptr;
        b.pos_stride = limit;
        b.n1 = npts;
        b.W = W;
        b.nmax = npts;
        b.q = c->lo_q.p;
        b.q_stride = limit;
        b.partial = c->lo_part.as<double>();
        b.p_stride = usac::nonminimal_partial_stride(limit);
        b.ws = c->lo_ws.as<float>();
        b.model_out = c->lo_models.as<float>();
        b.ok = c->lo_ok.as<int32_t>();
        b.seq = c->nm_seq.p;
        HIP_TRY(c, usac::launch_nonminimal_batch(st, c->estimator, c->pts.p, b));
        HIP_TRY(c, usac::launch_inliers_batch(st, c->estimator, c->pts.p, n, c->lo_models.as<float>(), W, thr, nullptr,
                                              nullptr, nullptr, 0, c->lo_cnts.as<int32_t>(), c->lo_sums.as<float>(),
                                              c->lo_scr.p));
        HIP_TRY(c, hipMemcpyAsync(hmod.data(), c->lo_models.p, sizeof(float) * 9 * W, hipMemcpyDeviceToHost, st));
        HIP_TRY(c, hipMemcpyAsync(hok.data(), c->lo_ok.p, sizeof(int32_t) * W, hipMemcpyDeviceToHost, st));
        HIP_TRY(c, hipMemcpyAsync(hcnt.data(), c->lo_cnts.p, sizeof(int32_t) * W, hipMemcpyDeviceToHost, st));
        HIP_TRY(c, hipMemcpyAsync(hsum.data(), c->lo_sums.p, sizeof(float) * W, hipMemcpyDeviceToHost, st));
        HIP_TRY(c, stream_wait(st));
        stages++;
        return USAC_OK;
    }
};

// model.hpp:40 max_hypothesis_test_before_sprt (usac_params, ABI 12; 0 = the default 20)
static int max_before_sprt(const usac_params *p) {
    return p->max_hypothesis_test_before_sprt ? (int)p->max_hypothesis_test_before_sprt : 20;
}

bool rec_better(const usac_record &a, const usac_record &b) {
    if (!a.valid) return false;
    if (!b.valid) return true;
    if (a.inliers != b.inliers) return a.inliers > b.inliers;
    if (a.score != b.score) return a.score > b.score;
    return a.hyp_index < b.hyp_index;
}

}  // namespace

extern "C" {

int usac_abi_version(void) { return USAC_ABI_VERSION; }

int usac_create(usac_ctx **out, int device, int estimator, const float *pts, uint32_t n, uint32_t cols) {
    if (!out) return USAC_ERR_ARG;
    *out = nullptr;
    if (estimator != USAC_LINE2D && estimator != USAC_HOMOGRAPHY && estimator != USAC_FUNDAMENTAL &&
        estimator != USAC_ESSENTIAL)
        return USAC_ERR_UNSUPPORTED;
    if ((estimator == USAC_LINE2D) != (cols == 2) || (cols != 2 && cols != 4)) return USAC_ERR_ARG;
    if (n == 0 || !pts) return USAC_ERR_ARG;
    usac_ctx *c = new usac_ctx();
    c->device = device;
    c->estimator = estimator;
    c->n = n;
    c->cols = cols;
    c->m = estimator == USAC_LINE2D ? 2 : estimator == USAC_FUNDAMENTAL ? 7 : estimator == USAC_ESSENTIAL ? 5 : 4;
    c->spk = estimator == USAC_FUNDAMENTAL ? 3 : 1;
    // two-view scoring: a batch yields few models (about 0.4-1.3 per sample) and the few with
    // many inliers are much slower to score, so their point ranges are cut finer
    if (estimator == USAC_FUNDAMENTAL || estimator == USAC_ESSENTIAL) c->chunks = 96;
    if (const char *g = getenv("USAC_LO_GRAPH")) c->lo_graph_on = atoi(g) != 0;
    int rc = USAC_OK;
    do {
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) { rc = fail(c, USAC_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e)); break; }
        e = StreamPool::get().stream(&c->stream);
        if (e != hipSuccess) { rc = fail(c, USAC_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e)); break; }
        for (auto &ev : c->ev) {
            e = StreamPool::get().event(&ev);
            if (e != hipSuccess) break;
        }
        if (e != hipSuccess) { rc = fail(c, USAC_ERR_HIP, "hipEventCreate failed"); break; }
        e = c->pts.reserve(sizeof(float) * (size_t)n * cols);
        if (e != hipSuccess) { rc = fail(c, USAC_ERR_HIP, "hipMalloc points failed"); break; }
        e = hipMemcpy(c->pts.p, pts, sizeof(float) * (size_t)n * cols, hipMemcpyHostToDevice);
        if (cols == 4) {  // dataset box for the score kernel's error bounds (NaN rows skipped)
            float mx[4] = {0, 0, 0, 0};
            for (uint32_t i = 0; i < n; i++)
                for (int k = 0; k < 4; k++) {
                    const float v = fabsf(pts[4 * (size_t)i + k]);
                    if (v > mx[k]) mx[k] = v;
                }
            c->ext = make_float4(mx[0], mx[1], mx[2], mx[3]);
            const char *h16env = getenv("USAC_H16");
            c->h16 = !h16env || atoi(h16env) != 0 ? 1 : 0;
            const char *e16env = getenv("USAC_E16");  // USAC_E16=0: k_score_f2 for every essential batch
            c->e16 = !e16env || atoi(e16env) != 0 ? 1 : 0;
        }
        if (e != hipSuccess) { rc = fail(c, USAC_ERR_HIP, std::string("hipMemcpy: ") + hipGetErrorString(e)); break; }
    } while (0);
    if (rc != USAC_OK) {
        // keep the message reachable for the caller through a static copy
        static thread_local std::string last;
        last = c->err;
        usac_destroy(c);
        fprintf(stderr, "usac_create: %s\n", last.c_str());
        return rc;
    }
    *out = c;
    return USAC_OK;
}

void usac_destroy(usac_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);  // the pools are per device
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->xstream) (void)hipStreamSynchronize(c->xstream);
    if (c->lo_stream) (void)hipStreamSynchronize(c->lo_stream);
    if (c->spec_stream) (void)hipStreamSynchronize(c->spec_stream);
    if (c->thin_stream) (void)hipStreamSynchronize(c->thin_stream);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->pol_pin) PinnedPool::get().give_back(c->pol_pin, c->pol_pin_bytes);
    if (c->x_pin) PinnedPool::get().give_back(c->x_pin, c->x_pin_bytes);
    if (c->xring_host) PinnedPool::get().give_back(c->xring_host, c->xring_host_bytes);
    for (int k = 0; k < USAC_XRING; k++) {
        if (c->xev_batch[k]) StreamPool::get().give_back(c->xev_batch[k]);
        if (c->xev_done[k]) StreamPool::get().give_back(c->xev_done[k]);
    }
    if (c->xstream) StreamPool::get().give_back(c->xstream);
    if (c->coll_ev) StreamPool::get().give_back(c->coll_ev);
    for (auto &ev : c->lo_ev)
        if (ev) StreamPool::get().give_back(ev);
    if (c->lo_stream) StreamPool::get().give_back(c->lo_stream);
    if (c->lo_best_pin) PinnedPool::get().give_back(c->lo_best_pin, c->lo_best_pin_bytes);
    if (c->rec_pin) PinnedPool::get().give_back(c->rec_pin, c->rec_pin_bytes);
    if (c->spec_ev) StreamPool::get().give_back(c->spec_ev);
    if (c->spec_stream) StreamPool::get().give_back(c->spec_stream);
    if (c->thin_stream) StreamPool::get().give_back_masked(c->thin_stream);
    for (auto &ev : c->thin_ev)
        if (ev) StreamPool::get().give_back(ev);
    if (c->grid_pin) PinnedPool::get().give_back(c->grid_pin, c->grid_pin_bytes);
    for (DevBuf *b : {&c->pts, &c->rec, &c->perm, &c->samples, &c->models, &c->counts, &c->sums, &c->best, &c->hostmodels,
                      &c->argmax_part, &c->list, &c->list_n, &c->h4_fb, &c->h4_fb_n, &c->pool_idx, &c->pool_pts, &c->masks, &c->sprt_pts,
                      &c->sprt_tested, &c->sprt_surv, &c->sprt_surv_n, &c->sprt_starts, &c->inl_scratch, &c->e5_ws, &c->one_model,
                      &c->h16_k, &c->h16_feat, &c->h16_rows, &c->h16_fm, &c->h16_part, &c->e16_feat, &c->e16_rows, &c->e16_cm, &c->e16_part,
                      &c->inl_idx, &c->pol_lists, &c->pol_res, &c->inl_cnt, &c->inl_sum, &c->q, &c->partial, &c->ws, &c->nm_model, &c->nm_ok, &c->nm_seq, &c->nm_w, &c->nm_qw, &c->lo_io,
                      &c->rec_send, &c->rec_all, &c->tv_part, &c->hf_part, &c->prosac_tab, &c->lo_max, &c->lo_lists, &c->lo_pos,
                      &c->lo_ns, &c->lo_thrs, &c->lo_slots, &c->lo_models, &c->lo_ok, &c->lo_cnts, &c->lo_sums,
                      &c->lo_q, &c->lo_part, &c->lo_ws, &c->lo_scr, &c->knn_idx, &c->knn_d2, &c->gc_err, &c->grid_csr,
                      &c->grid_elig, &c->grid_ws, &c->x_send, &c->lo_best,
                      &c->x_recv, &c->xring})
        b->release();
    for (auto &ev : c->ev)
        if (ev) StreamPool::get().give_back(ev);
    if (c->stream) StreamPool::get().give_back(c->stream);
    delete c;
}

const char *usac_last_error(const usac_ctx *c) { return c ? c->err.c_str() : "null context"; }

int usac_set_dlt_mode(usac_ctx *c, int mode) {
    if (!c || (mode != USAC_DLT_THIN && mode != USAC_DLT_NULLSPACE)) return USAC_ERR_ARG;
    c->dlt_mode = mode;
    return USAC_OK;
}

int usac_set_score_chunks(usac_ctx *c, int chunks) {
    if (!c) return USAC_ERR_ARG;
    const bool ok = listed(c) ? (chunks >= 1 && chunks <= 128)
                              : (chunks == 1 || chunks == 2 || chunks == 4 || chunks == 8 || chunks == 16);
    if (!ok) return USAC_ERR_ARG;
    c->chunks = chunks;
    return USAC_OK;
}

int usac_set_score_variant(usac_ctx *c, int variant) {
    if (!c || variant < 0 || variant > 3) return USAC_ERR_ARG;
    c->score_variant = variant;
    return USAC_OK;
}

uint32_t usac_sample_size(const usac_ctx *c) { return c ? c->m : 0; }
uint32_t usac_num_points(const usac_ctx *c) { return c ? c->n : 0; }

int usac_estimate_models(usac_ctx *c, const int32_t *samples, uint32_t B, float *models, int32_t *n_models) {
    if (!c || !samples || !models || B == 0) return USAC_ERR_ARG;
    for (uint64_t i = 0; i < (uint64_t)B * c->m; i++)
        if (samples[i] < 0 || (uint32_t)samples[i] >= c->n) return fail(c, USAC_ERR_ARG, "sample index out of range");
    int rc = ensure_batch(c, B);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMemcpyAsync(c->samples.p, samples, sizeof(int32_t) * (size_t)B * c->m, hipMemcpyHostToDevice,
                              c->stream));
    HIP_TRY(c, enqueue_solve(c, c->samples.as<int32_t>(), B, 0, 0, nullptr));
    const size_t S = (size_t)B * c->spk;
    std::vector<float> soa((size_t)ncomp(c) * S);
    std::vector<int32_t> slot_cnt(S, 0);
    HIP_TRY(c, hipMemcpyAsync(soa.data(), c->models.p, sizeof(float) * soa.size(), hipMemcpyDeviceToHost, c->stream));
    if (listed(c))
        HIP_TRY(c, hipMemcpyAsync(slot_cnt.data(), c->counts.p, sizeof(int32_t) * S, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    const int nc = ncomp(c);
    for (size_t sl = 0; sl < S; sl++) {
        const bool ok = slot_cnt[sl] >= 0;
        for (int k = 0; k < 9; k++) models[9 * sl + k] = (k < nc && ok) ? soa[(size_t)k * S + sl] : 0.f;
    }
    if (n_models)
        for (uint32_t h = 0; h < B; h++) {
            int32_t k = 0;
            for (uint32_t j = 0; j < c->spk; j++) k += slot_cnt[(size_t)h * c->spk + j] >= 0;
            n_models[h] = k;
        }
    return USAC_OK;
}

int usac_score_models(usac_ctx *c, const float *models, uint32_t nm, float thr, int32_t *counts, float *sums) {
    if (!c || !models || !counts || nm == 0) return USAC_ERR_ARG;
    int rc = ensure_batch(c, nm);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    // Quality::getNumberInliers never runs the SPRT (quality.hpp:60-101): the throughput SPRT of
    // usac_set_sprt applies to the hypothesize_* batches only, so it is off for this call.
    struct SprtOff {
        usac_ctx *c;
        bool saved;
        ~SprtOff() { c->sprt_on = saved; }
    } sprt_off{c, c->sprt_on};
    c->sprt_on = false;
    HIP_TRY(c, hipMemcpyAsync(c->hostmodels.p, models, sizeof(float) * 9 * (size_t)nm, hipMemcpyHostToDevice, c->stream));
    if (listed(c)) {
        HIP_TRY(c, usac::launch_prepare_f(c->stream, c->hostmodels.as<float>(), nm, c->models.as<float>()));
        if (c->score_variant == 1) {
            HIP_TRY(c, usac::launch_score_f(c->stream, c->estimator, 1, c->pts.as<float4>(), c->n,
                                            c->models.as<float>(), nm, nullptr, nullptr, nm, thr,
                                            c->counts.as<int32_t>(), c->sums.as<float>()));
        } else if (c->score_variant == 3 && is_e(c) && c->e16 == 1 && thr > 0x1p-100f && thr < 0x1p100f) {
            // variant 3 (tests): the matrix-core throughput scorer -- counts exact, Σ within its bound
            HIP_TRY(c, enqueue_score_e16(c, nm, thr, nullptr, nullptr));
        } else {  // the fast two-view kernel, one chunk: exact sequential sums
            if (c->rec_thr != thr) {
                HIP_TRY(c, c->rec.reserve(sizeof(float) * 32 * (((size_t)c->n + 3) / 4)));
                HIP_TRY(c, usac::launch_prepare_rec(c->stream, c->pts.as<float4>(), c->n, thr, c->rec.as<float4>()));
                c->rec_thr = thr;
            }
            HIP_TRY(c, c->tv_part.reserve(usac::tv_scratch_bytes(nm, 1)));
            HIP_TRY(c, usac::launch_score_f2(c->stream, c->estimator, 1, c->rec.as<float4>(), c->pts.as<float4>(),
                                             c->n, c->ext, c->models.as<float>(), nm, nullptr, nullptr, nm, thr,
                                             c->counts.as<int32_t>(), c->sums.as<float>(), c->tv_part.p));
        }
    } else {
        if (is_h(c))
            HIP_TRY(c, usac::launch_prepare_h(c->stream, c->hostmodels.as<float>(), nm, c->models.as<float>()));
        else
            HIP_TRY(c, usac::launch_prepare_line(c->stream, c->hostmodels.as<float>(), nm, c->models.as<float>()));
        // variant 3 (tests): the throughput scorer on the given models -- counts exact, Σ within its bound
        HIP_TRY(c, enqueue_score(c, nm, thr, c->score_variant == 3 ? std::max(c->chunks, 2) : 1));
    }
    HIP_TRY(c, hipMemcpyAsync(counts, c->counts.p, sizeof(int32_t) * nm, hipMemcpyDeviceToHost, c->stream));
    if (sums) HIP_TRY(c, hipMemcpyAsync(sums, c->sums.p, sizeof(float) * nm, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    return USAC_OK;
}

int usac_get_inliers(usac_ctx *c, const float *model, float thr, int32_t *idx, uint32_t *n, float *sum) {
    if (!c || !model) return USAC_ERR_ARG;
    int rc = ensure_single(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMemcpyAsync(c->one_model.p, model, sizeof(float) * 9, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, enqueue_inliers(c, c->one_model.as<float>(), thr));
    int32_t cnt = 0;
    float s = 0.f;
    HIP_TRY(c, hipMemcpyAsync(&cnt, c->inl_cnt.p, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(&s, c->inl_sum.p, sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    if (idx && cnt > 0)
        HIP_TRY(c, hipMemcpy(idx, c->inl_idx.p, sizeof(int32_t) * (size_t)cnt, hipMemcpyDeviceToHost));
    if (n) *n = (uint32_t)cnt;
    if (sum) *sum = s;
    return USAC_OK;
}

float usac_bk_label(int n, const float *unary, int m, const int32_t *ei, const int32_t *ej, const float *e00,
                    const float *e01, const float *e10, const float *e11, int32_t *sink_out) {
    usac::BkGraph G(n, (size_t)m);
    for (int i = 0; i < n; i++) G.add_node();
    for (int i = 0; i < n; i++) G.add_term1(i, unary[i], 0.f);
    for (int k = 0; k < m; k++) G.add_term2(ei[k], ej[k], e00[k], e01[k], e10[k], e11[k]);
    const float f = G.maxflow();
    for (int i = 0; i < n; i++) sink_out[i] = G.is_sink(i) ? 1 : 0;
    return f;
}

int usac_knn(usac_ctx *c, uint32_t k, int32_t *idx, float *d2) {
    if (!c || !idx || k == 0 || k > usac::kKnnMax) return USAC_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t nk = (size_t)c->n * k;
    HIP_TRY(c, c->knn_idx.reserve(sizeof(int32_t) * nk));
    if (d2) HIP_TRY(c, c->knn_d2.reserve(sizeof(float) * nk));
    HIP_TRY(c, usac::launch_knn(c->stream, c->pts.as<float>(), c->n, c->cols, k, c->knn_idx.as<int32_t>(),
                                d2 ? c->knn_d2.as<float>() : nullptr));
    HIP_TRY(c, hipMemcpyAsync(idx, c->knn_idx.p, sizeof(int32_t) * nk, hipMemcpyDeviceToHost, c->stream));
    if (d2) HIP_TRY(c, hipMemcpyAsync(d2, c->knn_d2.p, sizeof(float) * nk, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    return USAC_OK;
}

int usac_nonminimal(usac_ctx *c, const int32_t *idx, uint32_t n, float *model) {
    return usac_lsq_fit(c, idx, n, nullptr, model);
}

int usac_lsq_fit(usac_ctx *c, const int32_t *idx, uint32_t n, const float *weights, float *model) {
    if (!c || !idx || !model) return USAC_ERR_ARG;
    if (n == 0) return fail(c, USAC_ERR_ARG, "empty sample");
    if (weights && c->estimator != USAC_HOMOGRAPHY && c->estimator != USAC_FUNDAMENTAL)
        return fail(c, USAC_ERR_UNSUPPORTED, "weighted non-minimal fit: homography / fundamental only "
                                             "(the other estimators inherit estimator.hpp:26's NOT IMPLEMENTED)");
    for (uint32_t i = 0; i < n; i++)
        if (idx[i] < 0 || (uint32_t)idx[i] >= c->n) return fail(c, USAC_ERR_ARG, "index out of range");
    int rc = ensure_single(c);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, c->inl_idx.reserve(sizeof(int32_t) * std::max<size_t>(n, c->n)));
    HIP_TRY(c, c->q.reserve(sizeof(float) * 4 * (size_t)n));
    HIP_TRY(c, c->partial.reserve(sizeof(double) * 45 * ((size_t)n / 64 + 2)));
    HIP_TRY(c, hipMemcpyAsync(c->inl_idx.p, idx, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
    if (weights) {
        HIP_TRY(c, c->nm_w.reserve(sizeof(float) * (size_t)c->n));
        HIP_TRY(c, hipMemcpyAsync(c->nm_w.p, weights, sizeof(float) * c->n, hipMemcpyHostToDevice, c->stream));
    }
    HIP_TRY(c, enqueue_nonminimal(c, c->inl_idx.as<int32_t>(), n, nullptr, nullptr,
                                  weights ? c->nm_w.as<float>() : nullptr));
    int32_t ok = 0;
    HIP_TRY(c, hipMemcpyAsync(model, c->nm_model.p, sizeof(float) * 9, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(&ok, c->nm_ok.p, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    return ok ? USAC_OK : fail(c, USAC_ERR_NO_MODEL, "non-minimal estimation failed");
}

// USAC_H16_DEFER=0: the h16 scorer's own finish kernel, then the plain argmax (A/B)
bool h16_defer() {
    static const bool on = !getenv("USAC_H16_DEFER") || atoi(getenv("USAC_H16_DEFER")) != 0;
    return on;
}

// the batch argmax (record of the batch) -- over the h16 scorer's chunk partials when it deferred
// its finish (one launch fewer), else over counts / sums
hipError_t batch_argmax(usac_ctx *c, uint32_t S, uint64_t first_hyp) {
    if (c->h16_deferred_ch) {
        const uint32_t ch = c->h16_deferred_ch;
        c->h16_deferred_ch = 0;
        return usac::launch_argmax_h16(c->stream, c->h16_part.p, S, (int)ch, c->h16_deferred_thr,
                                       c->counts.as<int32_t>(), c->sums.as<float>(), c->models.as<float>(), ncomp(c),
                                       first_hyp, c->spk, c->argmax_part.p, c->best.as<usac_record>());
    }
    return usac::launch_argmax(c->stream, c->counts.as<int32_t>(), c->sums.as<float>(), S, c->models.as<float>(),
                               ncomp(c), first_hyp, c->spk, c->argmax_part.p, c->best.as<usac_record>());
}

int usac_hypothesize_score(usac_ctx *c, const int32_t *samples, uint32_t B, uint64_t seed, uint64_t first_hyp,
                           float thr, int32_t *counts, float *sums, usac_record *best) {
    if (!c || B == 0) return USAC_ERR_ARG;
    if (samples)
        for (uint64_t i = 0; i < (uint64_t)B * c->m; i++)
            if (samples[i] < 0 || (uint32_t)samples[i] >= c->n) return fail(c, USAC_ERR_ARG, "sample index out of range");
    int rc = ensure_batch(c, B);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    if (samples)
        HIP_TRY(c, hipMemcpyAsync(c->samples.p, samples, sizeof(int32_t) * (size_t)B * c->m, hipMemcpyHostToDevice,
                                  c->stream));
    // per-hypothesis outputs requested -> exact sequential sums (one chunk)
    const int chunks = (counts || sums) ? 1 : c->chunks;
    HIP_TRY(c, enqueue_solve(c, samples ? c->samples.as<int32_t>() : nullptr, B, seed, first_hyp,
                             samples ? nullptr : c->samples.as<int32_t>(), h16_solver_thr(c, chunks, thr)));
    HIP_TRY(c, enqueue_score(c, B, thr, chunks, h16_defer()));
    c->batch_valid = true;
    const uint32_t S = B * c->spk;
    HIP_TRY(c, batch_argmax(c, S, first_hyp));
    if (counts) HIP_TRY(c, hipMemcpyAsync(counts, c->counts.p, sizeof(int32_t) * S, hipMemcpyDeviceToHost, c->stream));
    if (sums) HIP_TRY(c, hipMemcpyAsync(sums, c->sums.p, sizeof(float) * S, hipMemcpyDeviceToHost, c->stream));
    if (best) HIP_TRY(c, hipMemcpyAsync(best, c->best.p, sizeof(usac_record), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    return USAC_OK;
}

int usac_hypothesize_async(usac_ctx *c, uint32_t B, uint64_t seed, uint64_t first_hyp, float thr) {
    if (!c || B == 0) return USAC_ERR_ARG;
    int rc = ensure_batch(c, B);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    const bool tm = c->timing_on;
    if (tm) HIP_TRY(c, hipEventRecord(c->ev[0], c->stream));
    HIP_TRY(c, enqueue_solve(c, nullptr, B, seed, first_hyp, nullptr, h16_solver_thr(c, c->chunks, thr)));
    if (tm) HIP_TRY(c, hipEventRecord(c->ev[1], c->stream));
    HIP_TRY(c, enqueue_score(c, B, thr, c->chunks, h16_defer()));
    c->batch_valid = true;
    if (tm) HIP_TRY(c, hipEventRecord(c->ev[2], c->stream));
    HIP_TRY(c, batch_argmax(c, B * c->spk, first_hyp));
    if (tm) HIP_TRY(c, hipEventRecord(c->ev[3], c->stream));
    c->timed_pending = tm;
    return USAC_OK;
}

int usac_selftest_rpoly(usac_ctx *c, const double *coeffs, uint32_t B, double *roots, int32_t *nroots) {
    if (!c || !coeffs || !roots || !nroots || B == 0) return USAC_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    DevBuf dc, dr, dn, ws;
    struct Rel {
        DevBuf *b[4];
        ~Rel() {
            (void)hipDeviceSynchronize();
            for (DevBuf *x : b) x->release();
        }
    } rel{{&dc, &dr, &dn, &ws}};
    HIP_TRY(c, dc.reserve(sizeof(double) * 11 * (size_t)B));
    HIP_TRY(c, dr.reserve(sizeof(double) * 10 * (size_t)B));
    HIP_TRY(c, dn.reserve(sizeof(int32_t) * (size_t)B));
    HIP_TRY(c, ws.reserve(usac::e5_workspace_bytes(B)));
    HIP_TRY(c, hipMemcpyAsync(dc.p, coeffs, sizeof(double) * 11 * (size_t)B, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, usac::launch_e5_roots_selftest(c->stream, dc.as<double>(), B, dr.as<double>(), dn.as<int32_t>(), ws.p));
    std::vector<double> r(10 * (size_t)B);
    HIP_TRY(c, hipMemcpyAsync(r.data(), dr.p, sizeof(double) * 10 * (size_t)B, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(nroots, dn.p, sizeof(int32_t) * (size_t)B, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    for (uint32_t h = 0; h < B; h++)  // device layout [r B + h] -> row h
        for (int k = 0; k < 10; k++) roots[10 * (size_t)h + k] = k < nroots[h] ? r[(size_t)k * B + h] : 0.0;
    return USAC_OK;
}

int usac_selftest_logexp(usac_ctx *c, const double *x, uint32_t n, double *log_out, double *exp_out) {
    if (!c || !x || !log_out || !exp_out || n == 0) return USAC_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    DevBuf dx, dl, de;
    struct Rel {
        DevBuf *b[3];
        ~Rel() {
            (void)hipDeviceSynchronize();
            for (DevBuf *y : b) y->release();
        }
    } rel{{&dx, &dl, &de}};
    HIP_TRY(c, dx.reserve(sizeof(double) * n));
    HIP_TRY(c, dl.reserve(sizeof(double) * n));
    HIP_TRY(c, de.reserve(sizeof(double) * n));
    HIP_TRY(c, hipMemcpyAsync(dx.p, x, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, usac::launch_jt_logexp_selftest(c->stream, dx.as<double>(), n, dl.as<double>(), de.as<double>()));
    HIP_TRY(c, hipMemcpyAsync(log_out, dl.p, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(exp_out, de.p, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    return USAC_OK;
}

int usac_last_counts(usac_ctx *c, int32_t *counts, float *sums, uint32_t n) {
    if (!c || !counts || n == 0) return USAC_ERR_ARG;
    if (!c->batch_valid) return fail(c, USAC_ERR_ARG, "no batch since the last usac_ransac_run");
    if ((size_t)n * sizeof(int32_t) > c->counts.bytes) return fail(c, USAC_ERR_ARG, "more slots than the last batch");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMemcpyAsync(counts, c->counts.p, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
    if (sums) HIP_TRY(c, hipMemcpyAsync(sums, c->sums.p, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    return USAC_OK;
}

int usac_fetch_best(usac_ctx *c, usac_record *best) {
    if (!c || !best) return USAC_ERR_ARG;
    if (!c->rec_pin && !(c->rec_pin = PinnedPool::get().take(sizeof(usac_record), &c->rec_pin_bytes)))
        return fail(c, USAC_ERR_HIP, "pinned host allocation failed");
    HIP_TRY(c, hipMemcpyAsync(c->rec_pin, c->best.p, sizeof(usac_record), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    memcpy(best, c->rec_pin, sizeof(usac_record));
    return USAC_OK;
}

int usac_sync(usac_ctx *c) {
    if (!c) return USAC_ERR_ARG;
    HIP_TRY(c, stream_wait(c->stream));
    return USAC_OK;
}

int usac_set_timing(usac_ctx *c, int on) {
    if (!c) return USAC_ERR_ARG;
    c->timing_on = on != 0;
    return USAC_OK;
}

int usac_last_timings(usac_ctx *c, float *ms3) {
    if (!c || !ms3) return USAC_ERR_ARG;
    if (c->timed_pending) {
        HIP_TRY(c, hipEventSynchronize(c->ev[3]));
        HIP_TRY(c, hipEventElapsedTime(&c->last_ms[0], c->ev[0], c->ev[3]));
        HIP_TRY(c, hipEventElapsedTime(&c->last_ms[1], c->ev[1], c->ev[2]));
        HIP_TRY(c, hipEventElapsedTime(&c->last_ms[2], c->ev[0], c->ev[1]));
        c->timed_pending = false;
    }
    memcpy(ms3, c->last_ms, sizeof(c->last_ms));
    return USAC_OK;
}

uint32_t usac_std_termination(uint32_t inliers, uint32_t points_size, uint32_t sample_size, float desired_prob,
                              uint32_t max_iterations) {
    usac::StandardTerminationCriteria t(desired_prob, sample_size, points_size, max_iterations);
    return t.getUpBoundIterations(inliers);
}

int usac_uniform_samples(uint32_t seed, uint32_t n_points, uint32_t m, uint32_t count, int32_t *out) {
    if (!out || n_points == 0 || m == 0) return USAC_ERR_ARG;
    usac::UniformSampler s(seed, n_points, m);
    for (uint32_t i = 0; i < count; i++) s.generateSample(out + (size_t)i * m);
    return USAC_OK;
}

int usac_set_device_sampler(usac_ctx *c, int sampler) {
    if (!c || (sampler != USAC_SAMPLER_UNIFORM && sampler != USAC_SAMPLER_PROSAC && sampler != USAC_SAMPLER_NAPSAC))
        return USAC_ERR_ARG;
    if (sampler == USAC_SAMPLER_NAPSAC) {
        const int rc = ensure_grid(c, c->cell_size);
        if (rc) return rc;
    }
    if (sampler == USAC_SAMPLER_PROSAC) {
        if (c->n < c->m) return fail(c, USAC_ERR_ARG, "PROSAC needs n >= sample size");
        // the subset sequence of ProsacSampler::generateSample with termination_length = n
        usac::ProsacSampler ps(1, c->n, c->m);
        const uint32_t T = usac::ProsacSampler::kGrowthMax;
        std::vector<int32_t> smp(c->m);
        std::vector<uint32_t> tab(T);
        for (uint32_t h = 0; h < T; h++) {
            ps.generateSample(smp.data(), c->n);
            tab[h] = ps.subset();
        }
        HIP_TRY(c, hipSetDevice(c->device));
        HIP_TRY(c, c->prosac_tab.reserve(sizeof(uint32_t) * T));
        HIP_TRY(c, hipMemcpy(c->prosac_tab.p, tab.data(), sizeof(uint32_t) * T, hipMemcpyHostToDevice));
        c->prosac_len = T;
    }
    c->dev_sampler = sampler;
    return USAC_OK;
}

int usac_set_cell_size(usac_ctx *c, int cell_size) {
    if (!c || cell_size <= 0) return USAC_ERR_ARG;
    c->cell_size = cell_size;
    return c->dev_sampler == USAC_SAMPLER_NAPSAC ? ensure_grid(c, cell_size) : USAC_OK;
}

int usac_grid_neighbors(usac_ctx *c, int cell_size, uint32_t *n_cells, uint32_t *cell, uint32_t *rank, uint32_t *start,
                        int32_t *members, int32_t *eligible, uint32_t *n_eligible) {
    if (!c) return USAC_ERR_ARG;
    int rc = ensure_grid(c, cell_size);
    if (rc) return rc;
    const size_t n = c->n;
    if (n_cells) *n_cells = c->grid_n_cells;
    if (n_eligible) *n_eligible = c->grid_n_elig;
    if (cell) HIP_TRY(c, hipMemcpyAsync(cell, c->grid_cell(), 4 * n, hipMemcpyDeviceToHost, c->stream));
    if (rank) HIP_TRY(c, hipMemcpyAsync(rank, c->grid_rank(), 4 * n, hipMemcpyDeviceToHost, c->stream));
    if (start)
        HIP_TRY(c, hipMemcpyAsync(start, c->grid_start(), 4 * ((size_t)c->grid_n_cells + 1), hipMemcpyDeviceToHost,
                                  c->stream));
    if (members) HIP_TRY(c, hipMemcpyAsync(members, c->grid_members(), 4 * n, hipMemcpyDeviceToHost, c->stream));
    if (eligible && c->grid_n_elig)
        HIP_TRY(c, hipMemcpyAsync(eligible, c->grid_elig.p, 4 * (size_t)c->grid_n_elig, hipMemcpyDeviceToHost,
                                  c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    return USAC_OK;
}

int usac_draw_samples(usac_ctx *c, uint32_t B, uint64_t seed, uint64_t first_hyp, int32_t *out) {
    if (!c || !out || B == 0) return USAC_ERR_ARG;
    int rc = ensure_batch(c, B);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, usac::launch_draw_samples(c->stream, (int)c->m, c->n, B, dev_sampler(c, seed), first_hyp,
                                         c->samples.as<int32_t>()));
    HIP_TRY(c, hipMemcpyAsync(out, c->samples.p, sizeof(int32_t) * (size_t)B * c->m, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    return USAC_OK;
}

int usac_set_sprt(usac_ctx *c, int enable, uint32_t seed, double epsilon, double delta) {
    if (!c) return USAC_ERR_ARG;
    if (!enable) {
        c->sprt_on = false;
        return USAC_OK;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    usac::GlibcRandom g(seed);
    usac::Sprt sp(g, c->estimator, c->n, c->m, 10000);
    const double eps = epsilon > 0 ? epsilon : sp.epsilon0(), del = delta > 0 ? delta : sp.delta0();
    if (!(eps < 1.0) || !(del < 1.0)) return fail(c, USAC_ERR_ARG, "SPRT: epsilon and delta must be in (0, 1)");
    // the reference's constants (sprt.hpp:219-224: lambda * (delta / epsilon), lambda * ((1 - delta) /
    // (1 - epsilon)), compared with A), and their logs for the certified decisions (kernels_sprt.hip)
    c->sprt_eps = eps;
    c->sprt_delta = del;
    c->sprt_k.up = del / eps;
    c->sprt_k.down = (1 - del) / (1 - eps);
    c->sprt_k.A = sp.thresholdA(eps, del);
    c->sprt_k.lu = log(c->sprt_k.up);
    c->sprt_k.ld = log(c->sprt_k.down);
    c->sprt_k.lA = log(c->sprt_k.A);
    // test hooks: a wider margin / a lower climb limit sends more walks down the sequential path
    const char *em = getenv("USAC_SPRT_CERT_MARGIN"), *ec = getenv("USAC_SPRT_CERT_CLIMB");
    c->sprt_k.margin = em ? atof(em) : 1e-7;
    c->sprt_k.climb = ec ? atof(ec) : 700.0;
    if (!(c->sprt_k.margin >= 1e-7) || !(c->sprt_k.climb > 0) || c->sprt_k.climb > 700.0)
        return fail(c, USAC_ERR_ARG, "SPRT certificate: margin >= 1e-7 and 0 < climb <= 700");
    {  // the certificate's error budget at this n (kernels_sprt.hip): never a margin below it
        const double L = std::max(std::max(fabs(c->sprt_k.lu), fabs(c->sprt_k.ld)), 1.0);
        const double nn = (double)c->n, per = std::ceil(std::max(nn - 64.0, 0.0) / 256.0) + 64.0;
        const double budget = 2.0 * nn * L * 0x1p-51 + per * per * L * 0x1p-53 + fabs(c->sprt_k.lA) * 0x1p-53;
        c->sprt_k.margin = std::max(c->sprt_k.margin, 8.0 * budget);
    }
    HIP_TRY(c, c->pool_idx.reserve(sizeof(uint32_t) * c->n));
    HIP_TRY(c, c->sprt_pts.reserve(sizeof(float) * c->cols * (size_t)c->n));
    HIP_TRY(c, c->sprt_tested.reserve(sizeof(uint32_t)));
    HIP_TRY(c, c->sprt_surv_n.reserve(sizeof(uint32_t)));
    HIP_TRY(c, hipMemcpyAsync(c->pool_idx.p, sp.pool().data(), sizeof(uint32_t) * c->n, hipMemcpyHostToDevice,
                              c->stream));
    HIP_TRY(c, usac::launch_gather_points(c->stream, c->pts.p, c->cols, c->pool_idx.as<uint32_t>(), c->n,
                                          c->sprt_pts.p));
    HIP_TRY(c, hipMemsetAsync(c->sprt_tested.p, 0, sizeof(uint32_t), c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    c->sprt_on = true;
    return USAC_OK;
}

int usac_batch_sprt_info(usac_ctx *c, double *eps_delta_A, uint32_t *starts, uint32_t n) {
    if (!c) return USAC_ERR_ARG;
    if (!c->sprt_on) return fail(c, USAC_ERR_ARG, "SPRT not enabled");
    if (eps_delta_A) {
        eps_delta_A[0] = c->sprt_eps;
        eps_delta_A[1] = c->sprt_delta;
        eps_delta_A[2] = c->sprt_k.A;
    }
    if (starts && n) {
        if (!c->batch_valid || n > c->sprt_S) return fail(c, USAC_ERR_ARG, "no SPRT batch of that many slots");
        HIP_TRY(c, hipMemcpyAsync(starts, c->sprt_starts.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, c->stream));
        uint32_t ln = 0;
        if (listed(c)) HIP_TRY(c, hipMemcpyAsync(&ln, c->list_n.p, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, stream_wait(c->stream));
        if (listed(c)) {  // k_sprt_head writes the listed (occupied) slots only: the others get UINT32_MAX
            std::vector<uint32_t> lst(ln);
            if (ln) {
                HIP_TRY(c, hipMemcpyAsync(lst.data(), c->list.p, sizeof(uint32_t) * ln, hipMemcpyDeviceToHost, c->stream));
                HIP_TRY(c, stream_wait(c->stream));
            }
            std::vector<char> occ(n, 0);
            for (uint32_t k = 0; k < ln; k++)
                if (lst[k] < n) occ[lst[k]] = 1;
            for (uint32_t i = 0; i < n; i++)
                if (!occ[i]) starts[i] = UINT32_MAX;
        }
    }
    return USAC_OK;
}

int usac_sprt_tested(usac_ctx *c, uint64_t *points_tested) {
    if (!c || !points_tested) return USAC_ERR_ARG;
    if (!c->sprt_on) return fail(c, USAC_ERR_ARG, "SPRT not enabled");
    uint32_t t = 0;
    HIP_TRY(c, hipMemcpyAsync(&t, c->sprt_tested.p, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    *points_tested = t;
    return USAC_OK;
}

int usac_prosac_samples(uint32_t seed, uint32_t n_points, uint32_t m, uint32_t count, uint32_t termination_length,
                        int32_t *out) {
    if (!out || m < 2 || n_points < m || termination_length == 0 || count > usac::ProsacSampler::kGrowthMax)
        return USAC_ERR_ARG;
    usac::ProsacSampler s(seed, n_points, m);
    for (uint32_t i = 0; i < count; i++) s.generateSample(out + (size_t)i * m, termination_length);
    return USAC_OK;
}

int usac_sprt_pool(uint32_t seed, int estimator, uint32_t n_points, uint32_t m, uint32_t *pool, double *A0) {
    if (!pool || n_points == 0) return USAC_ERR_ARG;
    usac::GlibcRandom g(seed);
    usac::Sprt s(g, estimator, n_points, m, 10000);
    memcpy(pool, s.pool().data(), sizeof(uint32_t) * n_points);
    if (A0) *A0 = s.thresholdA0();
    return USAC_OK;
}

// Ransac::run (ransac.cpp:14-238): Uniform (glibc stream) or PROSAC sampler, optional SPRT,
// no LO.  Samples are drawn on the host in loop order and shipped in batches; the device
// solves every sample of a batch and either scores every model exactly (count, sequential
// Σerr) or, with SPRT, produces every model's inlier flags in SPRT-pool order; the host
// then replays the sequential loop over the batch -- SPRT walk, Score::bigger, termination
// update at each new best (standard, or PROSAC's scan of the best model's device inlier
// list), `while (iters < max_iters)` with the reference's SPRT double counting.
// This reproduces the reference's iteration sequence exactly because the loop state
// changes only at those points.  PROSAC samples depend on
// termination_length, which a best update can change: a batch is speculative, and when a
// change would alter a later sample of the batch the rest of the batch is dropped and the
// sampler is rewound to just after the current sample.  Then the <= 4-pass non-minimal
// polish on the device.
// One batch of a sharded run: rank r solves and scores slots of samples [r P, r P + P) (P =
// ceil(B / nranks); the last slices may be short or empty), packs its status word, counts and
// model words (int32 / fp32, padded to P x spk slots, counts -1 on padding) and all-gathers
// them; every rank unpacks all slices into hc / hmod exactly as the unsharded batch leaves
// them.  A rank whose local part failed still joins the all-gather with its error as status,
// and every rank then fails with the first failing rank's status: no rank is left blocked in
// a collective its peers never enter.  The RCCL path packs on the device (no host staging on
// the way out) and brings the gathered words back with one copy into pinned memory; a gather
// callback (e.g. gloo) receives host buffers.
static int sharded_batch(usac_ctx *c, const int32_t *hs, uint32_t B, uint32_t iters, float thr, int nranks, int rank,
                         usac_allgather_fn gather, void *user, std::vector<uint8_t> &xbuf, int32_t *hc, float *hmod,
                         size_t SB, bool sprt, uint32_t *hmask) {
    const uint32_t m = c->m, spk = c->spk;
    const int nc = ncomp(c);
    const uint32_t P = (B + (uint32_t)nranks - 1) / (uint32_t)nranks;
    const uint32_t lo = std::min<uint32_t>(B, (uint32_t)rank * P);
    const uint32_t Bs = std::min<uint32_t>(B, lo + P) - lo;
    const size_t Ps = (size_t)P * spk, Ss = (size_t)Bs * spk;
    // SPRT: every slot's pool-order inlier words follow the models ([nw][Ps], row = slot)
    const size_t nw = sprt ? (c->n + 31) / 32 : 0, moff = 1 + (1 + (size_t)nc) * Ps;
    const size_t words = moff + nw * Ps, bytes = 4 * words;
    auto pool_mask = [&](uint32_t *out) -> hipError_t {
        return usac::launch_pool_mask(c->stream, c->estimator, c->pool_pts.p, c->n, c->models.as<float>(), Ss, nullptr,
                                      nullptr, (uint32_t)Ss, thr, out, (uint32_t)Ps);
    };
    // the local part: its first error becomes this rank's status (the message stays in c->err)
    auto local = [&]() -> int {
        if (!Bs) return USAC_OK;
        HIP_TRY(c, hipMemcpyAsync(c->samples.p, hs + (size_t)lo * m, sizeof(int32_t) * (size_t)Bs * m,
                                  hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, enqueue_solve(c, c->samples.as<int32_t>(), Bs, 0, (uint64_t)iters + lo, nullptr));
        if (!sprt) HIP_TRY(c, enqueue_score(c, Bs, thr, loop_chunks(c, Bs)));
        return USAC_OK;
    };
    const int status = local();
    const std::string local_err = c->err;
    const uint8_t *recv = nullptr;
    if (gather) {
        xbuf.resize(bytes * (1 + (size_t)nranks));
        int32_t *send = reinterpret_cast<int32_t *>(xbuf.data());
        std::fill(send + 1, send + 1 + Ps, -1);
        std::fill(send + 1 + Ps, send + words, 0);
        send[0] = status;
        if (status == USAC_OK && Bs) {
            HIP_TRY(c, hipMemcpyAsync(send + 1, c->counts.p, sizeof(int32_t) * Ss, hipMemcpyDeviceToHost, c->stream));
            for (int k = 0; k < nc; k++)
                HIP_TRY(c, hipMemcpyAsync(send + 1 + (1 + (size_t)k) * Ps, c->models.as<float>() + (size_t)k * Ss,
                                          sizeof(float) * Ss, hipMemcpyDeviceToHost, c->stream));
            if (sprt) {
                HIP_TRY(c, pool_mask(c->masks.as<uint32_t>()));
                HIP_TRY(c, hipMemcpyAsync(send + moff, c->masks.p, sizeof(uint32_t) * nw * Ps, hipMemcpyDeviceToHost,
                                          c->stream));
            }
            HIP_TRY(c, stream_wait(c->stream));
        }
        if (gather(user, send, bytes, xbuf.data() + bytes) != 0)
            return fail(c, USAC_ERR_ARG, "all-gather callback failed (gather callbacks must fail on every rank)");
        recv = xbuf.data() + bytes;
    } else {
        HIP_TRY(c, c->x_send.reserve(bytes));
        HIP_TRY(c, c->x_recv.reserve(bytes * (size_t)nranks));
        if (c->x_pin_bytes < bytes * (size_t)nranks) {
            if (c->x_pin) PinnedPool::get().give_back(c->x_pin, c->x_pin_bytes);
            c->x_pin = PinnedPool::get().take(bytes * (size_t)nranks, &c->x_pin_bytes);
            if (!c->x_pin) {
                c->x_pin_bytes = 0;
                return fail(c, USAC_ERR_HIP, "pinned host allocation failed");
            }
        }
        HIP_TRY(c, usac::launch_pack_slice(c->stream, c->counts.as<int32_t>(), c->models.as<float>(),
                                           status == USAC_OK ? (uint32_t)Ss : 0u, (uint32_t)Ps, nc, status,
                                           c->x_send.as<int32_t>()));
        if (sprt && status == USAC_OK && Bs) HIP_TRY(c, pool_mask(c->x_send.as<uint32_t>() + moff));
        HIP_TRY(c, order_after_exchanges(c));
        NCCL_TRY(c, ncclAllGather(c->x_send.p, c->x_recv.p, bytes, ncclUint8, c->comm, c->stream));
        HIP_TRY(c, mark_collective(c));
        HIP_TRY(c, hipMemcpyAsync(c->x_pin, c->x_recv.p, bytes * (size_t)nranks, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, stream_wait(c->stream));
        recv = static_cast<const uint8_t *>(c->x_pin);
    }
    for (int r = 0; r < nranks; r++) {
        const int32_t st = *reinterpret_cast<const int32_t *>(recv + (size_t)r * bytes);
        if (st != USAC_OK)
            return fail(c, st, r == rank ? local_err : "sharded run: rank " + std::to_string(r) + " failed (status " +
                                                           std::to_string(st) + ")");
    }
    for (int r = 0; r < nranks; r++) {
        const uint32_t lr = std::min<uint32_t>(B, (uint32_t)r * P);
        const size_t Sr = (size_t)(std::min<uint32_t>(B, lr + P) - lr) * spk;
        const int32_t *rc_ = reinterpret_cast<const int32_t *>(recv + (size_t)r * bytes) + 1;
        memcpy(hc + (size_t)lr * spk, rc_, sizeof(int32_t) * Sr);
        for (int k = 0; k < nc; k++)
            memcpy(hmod + (size_t)k * SB + (size_t)lr * spk, rc_ + (1 + (size_t)k) * Ps, sizeof(float) * Sr);
        // mask rows = slots of the whole batch: hmask[w * S + slot]
        for (size_t w = 0; w < nw; w++)
            memcpy(hmask + w * (size_t)B * spk + (size_t)lr * spk, rc_ + (moff - 1) + w * Ps, sizeof(uint32_t) * Sr);
    }
    // without a slot list a model's count is never -1 (ransac_run_impl's unsharded SPRT path)
    if (sprt && !listed(c)) std::fill(hc, hc + (size_t)B * spk, 0);
    return USAC_OK;
}

// Ransac::run with each batch's hypotheses sharded over nranks: every rank
// draws the same host sample stream, solves and scores only its contiguous slice of the
// batch, and the slices' per-slot counts and models are all-gathered (gather(), or RCCL on
// the context's communicator when gather is null); the replay -- records, termination, LO,
// polish -- then runs on the merged batch identically on every rank (ransac.cpp:58-139 order).
static int ransac_run_impl(usac_ctx *c, const usac_params *prm, int nranks, int rank, usac_allgather_fn gather,
                           void *gather_user, usac_run_output *out, int32_t *inliers_out, usac_record *records,
                           uint32_t rec_cap) {
    if (!c || !prm || !out || nranks < 1 || rank < 0 || rank >= nranks) return USAC_ERR_ARG;
    memset(out, 0, sizeof(*out));
    // The loop scores homographies with k_score_hf, not the matrix-core scorer: its batches are
    // small (the ramp; h16's per-batch rows + finish launches cost more than they save: cfg5 3.30 ms
    // per run with k_score_hf, 3.8-3.9 with h16).  USAC_LOOP_H16=1 lets the loop use it (tests: the
    // round-5 miscount beside the speculative h16 batch was packed-fp32 VALU corruption beside MFMA
    // waves, gone since the library issues no packed fp32 instruction -- usac_pk.hpp).
    struct H16Off {
        usac_ctx *c;
        bool saved;
        ~H16Off() { c->h16_off = saved; }
    } h16_off{c, c->h16_off};
    const bool loop_h16 = getenv("USAC_LOOP_H16") && atoi(getenv("USAC_LOOP_H16")) != 0;
    c->h16_off = !loop_h16;
    if (nranks > 1 && !gather && (!c->comm || c->nranks != nranks || c->rank != rank))
        return fail(c, USAC_ERR_ARG, "sharded run without a gather callback needs usac_comm_init(nranks, rank)");
    const bool prosac = prm->sampler == USAC_SAMPLER_PROSAC;
    const bool napsac = prm->sampler == USAC_SAMPLER_NAPSAC;
    if (!prosac && !napsac && prm->sampler != USAC_SAMPLER_UNIFORM && prm->sampler != 0)
        return fail(c, USAC_ERR_UNSUPPORTED, "sampler not supported (Uniform, Napsac, Prosac)");
    const bool knn_mode = napsac && prm->neighbors != USAC_NEIGHBORS_GRID;  // ransac.hpp:62-78
    if (napsac && !knn_mode && c->cols != 4)
        return fail(c, USAC_ERR_ARG, "NAPSAC grid neighbours need 4-column points (SURVEY Q17)");
    if (napsac && !knn_mode && prm->cell_size <= 0) return fail(c, USAC_ERR_ARG, "NAPSAC cell_size must be > 0");
    if (knn_mode && (prm->knn == 0 || prm->knn > usac::kKnnMax || prm->knn + 1 < c->m))
        return fail(c, USAC_ERR_ARG, "NAPSAC KNN: k_nearest_neighbors must be in [sample_size - 1, 32] "
                                     "(napsac_sampler.hpp:48)");
    const bool use_lo = prm->lo == USAC_LO_INITLORSC || prm->lo == USAC_LO_INITFLORSC;
    const bool use_gc = prm->lo == USAC_LO_GC;
    if (prm->lo != USAC_LO_NONE && !use_lo && !use_gc)
        return fail(c, USAC_ERR_UNSUPPORTED, "LO: InItLORsc / InItFLORsc / GC only");
    if (use_gc && napsac)  // ransac.hpp:62-78 gives the neighbours to the sampler only: GC's are unset
        return fail(c, USAC_ERR_UNSUPPORTED, "NAPSAC + GC: the reference leaves the graph cut without neighbours");
    const bool gc_knn = use_gc && prm->neighbors != USAC_NEIGHBORS_GRID;
    if (use_gc && !gc_knn && (c->cols != 4 || prm->cell_size <= 0))
        return fail(c, USAC_ERR_ARG, "GC grid neighbours need 4-column points and cell_size > 0");
    if (gc_knn && (prm->knn == 0 || prm->knn > usac::kKnnMax))
        return fail(c, USAC_ERR_ARG, "GC KNN: k_nearest_neighbors must be in [1, 32]");
    if (use_lo && (prm->lo_sample_size == 0 || prm->lo_iterative_iterations == 0))
        return fail(c, USAC_ERR_ARG, "LO parameters must be > 0");
    if (prosac && c->n <= 20) return fail(c, USAC_ERR_ARG, "PROSAC needs > 20 points (prosac_termination_criteria.hpp:158-163)");
    if (prosac && prm->max_iterations > usac::ProsacSampler::kGrowthMax)
        return fail(c, USAC_ERR_ARG, "PROSAC max_iterations > 200000 (reference draws outside the point range)");
    const auto t0 = std::chrono::steady_clock::now();
    // wall-time split of the run, printed to stderr when USAC_PROFILE is set
    enum { T_SETUP, T_DRAW, T_DEVICE, T_SUMS, T_REPLAY, T_LO, T_POLISH, T_N };
    double tsplit[T_N] = {0, 0, 0, 0, 0, 0, 0};
    double t_verify = 0.0, t_drawonly = 0.0;  // USAC_PROFILE detail: host SPRT walks, sample draws
    auto tmark = std::chrono::steady_clock::now();
    auto lap = [&](int k) {
        const auto t = std::chrono::steady_clock::now();
        tsplit[k] += std::chrono::duration<double, std::milli>(t - tmark).count();
        tmark = t;
    };
    HIP_TRY(c, hipSetDevice(c->device));
    c->batch_valid = false;  // the run's batches, LO and polish reuse the batch buffers
    const uint32_t batch = prm->batch ? prm->batch : (prm->sprt ? 1024u : kDefaultBatch);
    int rc = ensure_batch(c, batch);
    if (rc) return rc;
    rc = ensure_single(c);
    if (rc) return rc;
    // sub-split of the setup (USAC_PROFILE): buffers, neighbours, LO / GC reservations
    double tsub[3] = {0, 0, 0};
    auto sub = [&](int k) {
        const auto t = std::chrono::steady_clock::now();
        tsub[k] = std::chrono::duration<double, std::milli>(t - tmark).count();
    };
    sub(0);
    const int saved_mode = c->dlt_mode;
    c->dlt_mode = prm->dlt_mode;
    const bool saved_sprt = c->sprt_on;  // the replay verifies exactly; the batch test is off
    c->sprt_on = false;
    struct Restore {
        usac_ctx *c;
        int mode;
        bool sprt;
        ~Restore() {
            c->dlt_mode = mode;
            c->sprt_on = sprt;
        }
    } restore{c, saved_mode, saved_sprt};
    const uint32_t n = c->n, m = c->m, spk = c->spk;
    const float thr = prm->threshold;

    // Ransac ctor order (ransac.hpp:41-93): sampler, termination criteria, then SPRT -- the
    // SPRT pool shuffle draws n values of the glibc stream before the Uniform sampler's first.
    usac::GlibcRandom grng(prm->seed);
    std::unique_ptr<usac::UniformSampler> uni;
    std::unique_ptr<usac::ProsacSampler> pro;
    std::unique_ptr<usac::ProsacTerminationCriteria> pterm;
    std::shared_ptr<const usac::GridNeighbors> grid;
    std::unique_ptr<usac::NapsacSampler> nap;
    std::unique_ptr<usac::NapsacKnnSampler> napk;
    std::vector<int32_t> knn_tab;
    if (prosac) {
        pro.reset(new usac::ProsacSampler(prm->seed, n, m));
        pterm.reset(new usac::ProsacTerminationCriteria(pro->growth(), prm->desired_prob, m, n, prm->max_iterations));
    } else if (knn_mode) {  // NearestNeighbors::getNearestNeighbors_nanoflann on the device
        knn_tab.resize((size_t)n * prm->knn);
        if ((rc = usac_knn(c, prm->knn, knn_tab.data(), nullptr))) return rc;
        napk.reset(new usac::NapsacKnnSampler(grng, knn_tab.data(), n, m, prm->knn));
    } else if (napsac) {  // getGridNearestNeighbors on the device (kernels_grid.hip)
        if ((rc = download_grid(c, prm->cell_size, grid))) return rc;
        nap.reset(new usac::NapsacSampler(grng, *grid, n, m));
    } else {
        uni.reset(new usac::UniformSampler(grng, n, m));
    }
    sub(1);
    std::unique_ptr<LoRansac> lo;
    if (use_lo) {
        Shard shard;
        shard.nranks = nranks;
        shard.rank = rank;
        shard.gather = gather;
        shard.user = gather_user;
        lo.reset(new LoRansac(c, prm, shard));
        if ((rc = lo->reserve())) return rc;
    }
    std::unique_ptr<GcLo> gc;
    if (use_gc) {  // Ransac ctor neighbours for the graph cut (ransac.hpp:60-78)
        if (gc_knn) {
            knn_tab.resize((size_t)n * prm->knn);
            if ((rc = usac_knn(c, prm->knn, knn_tab.data(), nullptr))) return rc;
        } else if ((rc = download_grid(c, prm->cell_size, grid))) {
            return rc;
        }
        gc.reset(new GcLo(c, prm, gc_knn ? knn_tab.data() : nullptr, prm->knn, grid.get()));
        if ((rc = gc->reserve())) return rc;
    }
    if (!prm->sprt && (rc = reserve_exact_sums(c))) return rc;
    sub(2);
    usac::StandardTerminationCriteria term(prm->desired_prob, m, n, prm->max_iterations);
    std::unique_ptr<usac::Sprt> sprt;
    const int max_before = max_before_sprt(prm);
    const uint32_t nw = (n + 31) / 32;
    // PROSAC + SPRT on one rank: the pool shuffle (n glibc draws, the sampler has its own
    // generator) runs after the first batch's solve is enqueued, overlapping it (pool_upload)
    const bool defer_pool = prm->sprt && prosac && nranks == 1 && !getenv("USAC_NO_DEFER_POOL");
    auto pool_upload = [&]() -> int {
        sprt->shuffle_pool();
        HIP_TRY(c, hipMemcpyAsync(c->pool_idx.p, sprt->pool().data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice,
                                  c->stream));
        HIP_TRY(c, usac::launch_gather_points(c->stream, c->pts.p, c->cols, c->pool_idx.as<uint32_t>(), n,
                                              c->pool_pts.p));
        return USAC_OK;
    };
    if (prm->sprt) {
        sprt.reset(new usac::Sprt(grng, c->estimator, n, m, prm->max_iterations, max_before_sprt(prm), defer_pool));
        HIP_TRY(c, c->pool_idx.reserve(sizeof(uint32_t) * n));
        HIP_TRY(c, c->pool_pts.reserve(sizeof(float) * c->cols * (size_t)n));
        // the words [nw][rows], then the batch's PoolTail (2 S + 1 + ncomp S words)
        HIP_TRY(c, c->masks.reserve(sizeof(uint32_t) * ((size_t)nw + 2 + (size_t)ncomp(c)) * batch * spk + 4));
        if (!defer_pool && (rc = pool_upload())) return rc;
    }

    const size_t SB = (size_t)batch * spk;  // slot stride of the host copies
    std::vector<uint8_t> xbuf;               // sharded runs: all-gather send + receive buffers
    pinned_vector<int32_t> hs((size_t)batch * m, 0), hc(SB);
    std::vector<int32_t> slot_row(SB);
    std::vector<float> hsum(SB);
    pinned_vector<float> hmod((size_t)ncomp(c) * SB);
    pinned_vector<uint32_t> hlist(SB + 1);  // the SPRT batch's occupied-slot list, its count at [SB]
    pinned_vector<uint32_t> hmask(sprt ? ((size_t)nw + 2 + (size_t)ncomp(c)) * SB + 4 : 0);  // words, PoolTail
    std::vector<uint32_t> subset_at(batch), largest_at(batch);
    std::vector<int32_t> last_sample(m, 0);
    // Speculation: the next batch is drawn and solved / scored on its own stream while the
    // current batch is replayed (its LO fits run meanwhile).  Its size assumes the replay
    // leaves max_iterations alone; a smaller actual batch takes the prefix of its results (the
    // same samples, the same kernels per hypothesis), and the sampler's extra draws are undone
    // (journal rollback, then a redraw of the kept prefix) before the sampler is used again.
    // Uniform / NAPSAC-grid without SPRT on one rank only (PROSAC's draws depend on the replay).
    const bool spec_ok = !prosac && !prm->sprt && nranks == 1 && !napk && (nap || uni) && !getenv("USAC_NO_SPECULATION");
    pinned_vector<int32_t> hs2(spec_ok ? (size_t)batch * m : 0), hc2(spec_ok ? SB : 0);
    pinned_vector<float> hmod2(spec_ok ? (size_t)ncomp(c) * SB : 0);
    std::vector<int32_t> spec_last(m, 0);
    bool spec = false;          // a speculative batch is on the spec stream
    uint32_t spec_B = 0;        // its size
    uint32_t sampler_keep = 0;  // > 0: roll the sampler back and redraw this many samples
    if (spec_ok) {
        if (!c->spec_stream) HIP_TRY(c, StreamPool::get().stream(&c->spec_stream));
        if (!c->spec_ev) HIP_TRY(c, StreamPool::get().event(&c->spec_ev));
        // every buffer a batch of `batch` samples grows into, now: a reserve() that grows a
        // block synchronises the device, which must not happen under the speculation
        HIP_TRY(c, c->perm.reserve(usac::presort_bytes(batch)));
        HIP_TRY(c, c->hf_part.reserve(sizeof(int32_t) * 2 * 16 * (size_t)batch));
        if (listed(c)) HIP_TRY(c, c->tv_part.reserve(usac::tv_scratch_bytes(batch * c->spk, c->chunks)));
        if (is_e(c)) HIP_TRY(c, c->e5_ws.reserve(usac::e5_workspace_bytes(batch)));
    }
    // every exit waits for a speculative batch still copying into hs2 / hc2 / hmod2
    struct SpecDrain {
        usac_ctx *c;
        const bool &pending;
        ~SpecDrain() {
            if (pending) (void)hipStreamSynchronize(c->spec_stream);
        }
    } spec_drain{c, spec};
    auto sampler_mark = [&]() {
        if (nap) nap->mark();
        else uni->mark();
    };
    auto sampler_commit = [&]() {
        if (nap) nap->commit();
        else uni->commit();
    };
    auto sampler_rollback = [&]() {
        if (nap) nap->rollback();
        else uni->rollback();
    };
    pinned_vector<int32_t> inl_list(prosac ? n : 0);
    usac::Score best;
    float best_model[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t iters = 0, max_iters = prm->max_iterations;
    int32_t nrec = 0;

    // exact inliers of a model on the device -> (cnt, s) and c->inl_idx
    int32_t cnt = 0, ok = 0;
    float s = 0.f;
    // (count, sum) of a host model through one pinned D2H (polish result block, slots 12-13)
    HIP_TRY(c, c->pol_res.reserve(sizeof(float) * usac::kPolWords));
    if (!c->pol_pin && !(c->pol_pin = PinnedPool::get().take(sizeof(float) * usac::kPolWords, &c->pol_pin_bytes)))
        return fail(c, USAC_ERR_HIP, "pinned host allocation failed");
    // list_pin (nullable): the whole n-word inlier list copied in the same submission (its
    // first cnt words are the list) -- one host wait instead of a second, synchronous copy
    auto score_inliers = [&](const float *model_host, int32_t *list_pin = nullptr) -> int {
        float *dres = c->pol_res.as<float>();
        HIP_TRY(c, hipMemcpyAsync(c->one_model.p, model_host, sizeof(float) * 9, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, c->inl_scratch.reserve(usac::inliers_scratch_bytes(c->n, 1)));
        HIP_TRY(c, usac::launch_inliers_batch(c->stream, c->estimator, c->pts.p, c->n, c->one_model.as<float>(), 1, thr,
                                              nullptr, nullptr, c->inl_idx.as<int32_t>(), 0,
                                              reinterpret_cast<int32_t *>(dres + 12), dres + 13, c->inl_scratch.p));
        HIP_TRY(c, hipMemcpyAsync(static_cast<float *>(c->pol_pin) + 12, dres + 12, sizeof(float) * 2,
                                  hipMemcpyDeviceToHost, c->stream));
        if (list_pin)
            HIP_TRY(c, hipMemcpyAsync(list_pin, c->inl_idx.p, sizeof(int32_t) * (size_t)c->n, hipMemcpyDeviceToHost,
                                      c->stream));
        HIP_TRY(c, stream_wait(c->stream));
        memcpy(&cnt, static_cast<const float *>(c->pol_pin) + 12, sizeof(int32_t));
        memcpy(&s, static_cast<const float *>(c->pol_pin) + 13, sizeof(float));
        return USAC_OK;
    };

    // PROSAC + SPRT: a new best's inlier list (getUpBoundIterationsSorted's input) decoded from its
    // pool-order mask row on the host instead of a device getInliers round trip per update.  An
    // accepted model's row covers every point (Sprt::verify counts the rest of the pool for a
    // model it keeps), and k_pool_mask evaluates the same residual (no contraction: Makefile) on
    // copies of the same points with the same model words -- except H, whose mask uses the
    // solver's H^-1 where getInliers inverts on the device.  USAC_CHECK_MASK_LIST=1 compares both.
    const bool mask_list = prosac && sprt && c->estimator != USAC_HOMOGRAPHY && !getenv("USAC_DEVICE_INLIERS");
    const bool mask_check = mask_list && getenv("USAC_CHECK_MASK_LIST");
    std::vector<uint64_t> pt_bits(mask_list ? ((size_t)n + 63) / 64 : 0);
    auto mask_inliers = [&](const uint32_t *row, size_t stride, int32_t *list) -> int32_t {
        std::fill(pt_bits.begin(), pt_bits.end(), 0);
        const uint32_t *pool = sprt->pool().data();
        for (uint32_t w = 0; w < nw; w++)
            for (uint32_t bits = row[(size_t)w * stride]; bits; bits &= bits - 1) {
                const uint32_t p = pool[32 * w + (uint32_t)__builtin_ctz(bits)];
                pt_bits[p >> 6] |= 1ull << (p & 63);
            }
        int32_t k = 0;
        for (size_t w = 0; w < pt_bits.size(); w++)
            for (uint64_t bits = pt_bits[w]; bits; bits &= bits - 1)
                list[k++] = (int32_t)(64 * w + (uint32_t)__builtin_ctzll(bits));
        return k;
    };

    lap(T_SETUP);
    // with the library's default batch the batches ramp up (1024, 2048, ...): the termination
    // bound drops once the loop has a good model, and a smaller first batch draws, solves and
    // scores fewer hypotheses the run never reaches (the replay is exact for any partition)
    // PROSAC on quality-sorted points finds its model within a few dozen samples and its
    // termination bound then drops to about as many (cfg3: ~9 iterations a run), so its ramp
    // starts at 32
    uint32_t cap = prm->batch ? batch : std::min<uint32_t>(batch, prosac ? kRampFirstProsac : kRampFirst);
    // draws B samples into buf (the reference's sample array reuse for NAPSAC: a sample the
    // sampler leaves (partly) unwritten keeps the previous sample's entries)
    auto draw_into = [&](int32_t *buf, uint32_t B, usac::ProsacSampler *pro_, uint32_t gen_term) {
        for (uint32_t j = 0; j < B; j++) {
            int32_t *smp = buf + (size_t)j * m;
            if (pro_) {
                subset_at[j] = pro_->subset();
                pro_->generateSample(smp, gen_term);
                largest_at[j] = pro_->largest();
            } else if (napk) {
                napk->generateSample(smp);
            } else if (napsac) {
                if (j > 0) memcpy(smp, smp - m, sizeof(int32_t) * m);
                else memcpy(smp, last_sample.data(), sizeof(int32_t) * m);
                nap->generateSample(smp);
                if (j + 1 == B) memcpy(last_sample.data(), smp, sizeof(int32_t) * m);
            } else {
                uni->generateSample(smp);
            }
        }
    };
    // the sampler exactly after the batches consumed so far (undo a speculation's extra draws)
    auto settle_sampler = [&]() {
        if (!sampler_keep) return;
        sampler_rollback();
        last_sample = spec_last;
        draw_into(hs2.data(), sampler_keep, nullptr, n);  // hs2 is free again: the kept batch moved to hs
        sampler_keep = 0;
    };
    auto spec_wait = [&]() -> hipError_t {
        for (uint32_t spins = 0;; spins++) {
            const hipError_t e = hipEventQuery(c->spec_ev);
            if (e != hipErrorNotReady) return e;
            if ((spins & 1023u) == 1023u) std::this_thread::yield();
        }
    };
    while (iters < max_iters) {
        const uint32_t B = std::min(std::min(batch, max_iters - iters), cap);
        if (!prm->batch) cap = std::min<uint32_t>(batch, 2 * cap);
        bool have = false;  // this batch's device results are already on the host (speculation)
        size_t spec_hst = 0;
        if (spec) {
            spec = false;
            HIP_TRY(c, spec_wait());
            if (B <= spec_B) {  // its first B samples are this batch
                std::swap(hs, hs2);
                std::swap(hc, hc2);
                std::swap(hmod, hmod2);
                spec_hst = (size_t)spec_B * spk;
                have = true;
                if (B < spec_B) {
                    sampler_keep = B;  // undone lazily, before the next draw
                    out->spec_rollbacks++;
                    out->spec_wasted += spec_B - B;
                } else {
                    sampler_commit();
                }
            } else {  // (max_iterations grew) the speculation is dropped
                out->spec_wasted += spec_B;
                sampler_rollback();
                last_sample = spec_last;
            }
        }
        // ---- draw the batch (speculatively for PROSAC)
        std::unique_ptr<usac::ProsacSampler> snapshot;
        const uint32_t gen_term = prosac ? pterm->terminationLength() : n;
        if (!have) {
            settle_sampler();
            const auto td0 = std::chrono::steady_clock::now();
            if (prosac) snapshot.reset(new usac::ProsacSampler(*pro));
            draw_into(hs.data(), B, prosac ? pro.get() : nullptr, gen_term);
            t_drawonly += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - td0).count();
        }
        lap(T_DRAW);
        // ---- device: solve, then exact scores or pool-order flags
        const size_t S = (size_t)B * spk;
        size_t hst = SB;  // host stride of hmod's components this batch
        uint32_t rows = (uint32_t)S;
        uint32_t mask_stride = (uint32_t)S;  // host row stride of hmask (SPRT)
        if (have) {
            hst = spec_hst;
        } else if (nranks > 1) {  // this rank's slice, then the all-gather of every slice's counts and models
            if ((rc = sharded_batch(c, hs.data(), B, iters, thr, nranks, rank, gather, gather_user, xbuf, hc.data(),
                                    hmod.data(), SB, sprt != nullptr, hmask.data())))
                return rc;
        } else {
        HIP_TRY(c, hipMemcpyAsync(c->samples.p, hs.data(), sizeof(int32_t) * (size_t)B * m, hipMemcpyHostToDevice,
                                  c->stream));
        HIP_TRY(c, enqueue_solve(c, c->samples.as<int32_t>(), B, 0, iters, nullptr));
        const size_t mstride = (size_t)B * spk;
        // listed SPRT batches: the slot counts, list and models ride behind the words (PoolTail)
        const bool tailed = sprt && listed(c) && !getenv("USAC_NO_POOL_TAIL");
        const size_t tail_off = (size_t)nw * S, tail_words = (2 + (size_t)ncomp(c)) * S + 1;
        if (sprt && !sprt->pool_ready() && (rc = pool_upload())) return rc;  // deferred: behind the solve
        if (sprt) {
            const usac::PoolTail tail{reinterpret_cast<const uint32_t *>(c->counts.p), c->list_n.as<uint32_t>(),
                                      c->list.as<uint32_t>(), c->models.as<uint32_t>(), (uint32_t)S,
                                      (uint32_t)(ncomp(c) * S), c->masks.as<uint32_t>() + tail_off};
            HIP_TRY(c, usac::launch_pool_mask(c->stream, c->estimator, c->pool_pts.p, n, c->models.as<float>(), mstride,
                                              listed(c) ? c->list.as<uint32_t>() : nullptr,
                                              listed(c) ? c->list_n.as<uint32_t>() : nullptr, (uint32_t)S, thr,
                                              c->masks.as<uint32_t>(), listed(c) ? 0u : (uint32_t)S,
                                              tailed ? &tail : nullptr));
        } else {  // exact counts from the fast multi-chunk scorer; exact sums below, where needed
            HIP_TRY(c, enqueue_score(c, B, thr, loop_chunks(c, B)));
            HIP_TRY(c, hipMemcpyAsync(hc.data(), c->counts.p, sizeof(int32_t) * S, hipMemcpyDeviceToHost, c->stream));
        }
        // the device's component-major [ncomp][S] block in one copy (host stride S this batch:
        // every copy costs a fixed overhead, 18 per-component copies of a ramp batch cost more
        // than the batch's kernels)
        hst = S;
        if (!tailed)
            HIP_TRY(c, hipMemcpyAsync(hmod.data(), c->models.p, sizeof(float) * S * ncomp(c), hipMemcpyDeviceToHost,
                                      c->stream));
        const uint32_t *htail = nullptr;  // the batch's PoolTail on the host
        auto untail = [&]() {
            memcpy(hc.data(), htail, sizeof(int32_t) * S);
            hlist[SB] = htail[S];
            memcpy(hlist.data(), htail + S + 1, sizeof(uint32_t) * S);
            memcpy(hmod.data(), htail + 2 * S + 1, sizeof(float) * S * ncomp(c));
        };
        if (tailed) {
            // small batches (the PROSAC ramp's first ones, where a cfg3 run ends): words and tail in
            // one copy, one host wait; larger ones: the tail first, then only the rows' words (the
            // words are packed [nw][rows] on the device: k_pool_mask, row stride 0)
            const bool whole = (size_t)nw * S * sizeof(uint32_t) <= kMaskWholeCopy;
            if (whole) {
                HIP_TRY(c, hipMemcpyAsync(hmask.data(), c->masks.p, sizeof(uint32_t) * (tail_off + tail_words),
                                          hipMemcpyDeviceToHost, c->stream));
                HIP_TRY(c, stream_wait(c->stream));
                htail = hmask.data() + tail_off;
                untail();
            } else {
                HIP_TRY(c, hipMemcpyAsync(hmask.data() + (size_t)nw * SB, c->masks.as<uint32_t>() + tail_off,
                                          sizeof(uint32_t) * tail_words, hipMemcpyDeviceToHost, c->stream));
                HIP_TRY(c, stream_wait(c->stream));
                htail = hmask.data() + (size_t)nw * SB;
                untail();
                rows = hlist[SB];
                if (rows) HIP_TRY(c, hipMemcpyAsync(hmask.data(), c->masks.p, sizeof(uint32_t) * (size_t)rows * nw,
                                                    hipMemcpyDeviceToHost, c->stream));
            }
        } else if (sprt) {
            // listed: the occupied rows' words packed [nw][rows] on the device (k_pool_mask, row
            // stride 0).  Small batches (the PROSAC ramp's first ones, where a cfg3 run ends): the
            // whole block with the list in the same submission -- one host wait; larger ones: the
            // list count first, then only the rows' words (a plain copy: hipMemcpy2DAsync's first
            // call in a process cost ~7 ms, round 5)
            const bool whole = !listed(c) || (size_t)nw * S * sizeof(uint32_t) <= kMaskWholeCopy;
            if (listed(c)) {  // occupied slots -> mask rows
                HIP_TRY(c, hipMemcpyAsync(hc.data(), c->counts.p, sizeof(int32_t) * S, hipMemcpyDeviceToHost, c->stream));
                HIP_TRY(c, hipMemcpyAsync(hlist.data() + SB, c->list_n.p, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                          c->stream));
                if (whole) {
                    HIP_TRY(c, hipMemcpyAsync(hlist.data(), c->list.p, sizeof(uint32_t) * S, hipMemcpyDeviceToHost,
                                              c->stream));
                } else {
                    HIP_TRY(c, stream_wait(c->stream));
                    rows = hlist[SB];
                    if (rows) HIP_TRY(c, hipMemcpyAsync(hlist.data(), c->list.p, sizeof(uint32_t) * rows,
                                                        hipMemcpyDeviceToHost, c->stream));
                }
            } else {
                std::fill(hc.begin(), hc.begin() + S, 0);
            }
            if (whole) {
                mask_stride = (uint32_t)S;  // listed: the row count, below
                HIP_TRY(c, hipMemcpyAsync(hmask.data(), c->masks.p, sizeof(uint32_t) * S * nw, hipMemcpyDeviceToHost,
                                          c->stream));
            } else if (rows) {
                HIP_TRY(c, hipMemcpyAsync(hmask.data(), c->masks.p, sizeof(uint32_t) * (size_t)rows * nw,
                                          hipMemcpyDeviceToHost, c->stream));
            }
        }
        HIP_TRY(c, stream_wait(c->stream));
        if (sprt && listed(c)) mask_stride = rows = hlist[SB];
        }
        if (sprt) {
            if (listed(c) && nranks == 1) {
                std::fill(slot_row.begin(), slot_row.begin() + S, -1);
                for (uint32_t r = 0; r < rows; r++) slot_row[hlist[r]] = (int32_t)r;
            } else {
                for (size_t sl = 0; sl < S; sl++) slot_row[sl] = (int32_t)sl;
            }
        }
        // ---- speculation: the next batch, as if the replay leaves max_iterations alone -- unless
        // this batch certainly ends the run: the replay leaves max_iters <= the termination bound
        // of its final best, whose count is at least every count of this batch (Score::bigger
        // orders by count first; LO only adds inliers) and the bound does not grow with the count
        bool spec_next = spec_ok && iters + B < max_iters;
        if (spec_next) {
            int maxc = best.inlier_number;
            for (size_t sl = 0; sl < S; sl++) maxc = std::max(maxc, hc[sl]);
            spec_next = term.getUpBoundIterations((uint32_t)maxc) > iters + B;
        }
        if (spec_next) {
            settle_sampler();
            const uint32_t B2 = std::min(std::min(batch, max_iters - (iters + B)), cap);
            sampler_mark();
            spec_last = last_sample;
            draw_into(hs2.data(), B2, nullptr, n);
            const size_t S2 = (size_t)B2 * spk;
            std::swap(c->stream, c->spec_stream);  // the launchers enqueue on c->stream
            hipError_t e = hipMemcpyAsync(c->samples.p, hs2.data(), sizeof(int32_t) * (size_t)B2 * m,
                                          hipMemcpyHostToDevice, c->stream);
            if (e == hipSuccess) e = enqueue_solve(c, c->samples.as<int32_t>(), B2, 0, iters + B, nullptr);
            if (e == hipSuccess) e = enqueue_score(c, B2, thr, loop_chunks(c, B2));
            if (e == hipSuccess)
                e = hipMemcpyAsync(hc2.data(), c->counts.p, sizeof(int32_t) * S2, hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(hmod2.data(), c->models.p, sizeof(float) * S2 * ncomp(c), hipMemcpyDeviceToHost,
                                   c->stream);
            if (e == hipSuccess) e = hipEventRecord(c->spec_ev, c->stream);
            std::swap(c->stream, c->spec_stream);
            if (e != hipSuccess) {
                (void)hipStreamSynchronize(c->spec_stream);
                return fail(c, USAC_ERR_HIP, std::string("speculative batch: ") + hipGetErrorString(e));
            }
            spec = true;
            spec_B = B2;
            out->spec_batches++;
        }
        lap(T_DEVICE);
        if (!sprt && (rc = exact_sums(c, thr, best.inlier_number, hc.data(), hmod.data(), hst, S, hsum.data(),
                                      &out->sum_models)))
            return rc;
        lap(T_SUMS);
        out->batches++;
        // ---- sequential replay
        uint32_t j = 0;
        bool rewind = false;
        for (; j < B && iters < max_iters; j++) {
            for (uint32_t q = 0; q < spk; q++) {
                const size_t sl = (size_t)j * spk + q;
                if (hc[sl] < 0) break;  // empty slot: the sample has no more models
                usac::Score cur;
                int32_t r = 0;
                if (sprt) {
                    r = slot_row[sl];
                    const auto tv0 = std::chrono::steady_clock::now();
                    const bool good = sprt->verify(hmask.data() + r, (int)iters, (uint32_t)best.inlier_number,
                                                   cur.inlier_number, cur.score, mask_stride);
                    t_verify += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tv0).count();
                    if (!good) {
                        out->sprt_rejected++;
                        if ((int)iters >= max_before) {  // max_hypothesis_test_before_sprt (model.hpp:40), Q9
                            iters++;
                            continue;
                        }
                    }
                } else {
                    cur.inlier_number = hc[sl];
                    cur.score = hsum[sl];
                }
                if (!cur.bigger(best)) continue;
                float model[9];
                for (int k = 0; k < 9; k++) model[k] = k < ncomp(c) ? hmod[(size_t)k * hst + sl] : 0.f;
                if (lo) {  // ransac.cpp:110-112, before the best is replaced
                    lap(T_REPLAY);
                    lo->run(model, cur.inlier_number, cur.score);
                    if (lo->rc) return lo->rc;
                    lap(T_LO);
                }
                if (gc) {
                    lap(T_REPLAY);
                    gc->run(model, cur.inlier_number, cur.score);
                    if (gc->rc) return gc->rc;
                    lap(T_LO);
                }
                best = cur;
                memcpy(best_model, model, sizeof(best_model));
                if (prosac && mask_list) {
                    cnt = mask_inliers(hmask.data() + r, mask_stride, inl_list.data());
                    if (mask_check) {
                        std::vector<int32_t> dl(n);
                        const int32_t mc = cnt;
                        if ((rc = score_inliers(best_model, dl.data()))) return rc;
                        const std::vector<int32_t> tmp(inl_list.data(), inl_list.data() + mc);
                        if (cnt != mc || cnt != cur.inlier_number ||
                            !std::equal(tmp.begin(), tmp.end(), dl.begin()))
                            return fail(c, USAC_ERR_HIP, "mask-decoded inlier list differs from getInliers");
                        cnt = mc;
                    }
                    max_iters = pterm->getUpBoundIterationsSorted(iters, inl_list.data(), (uint32_t)cnt, largest_at[j]);
                } else if (prosac) {
                    if ((rc = score_inliers(best_model, inl_list.data()))) return rc;
                    // (the list is ascending: the compaction keeps point order)
                    max_iters = pterm->getUpBoundIterationsSorted(iters, inl_list.data(), (uint32_t)cnt, largest_at[j]);
                } else {
                    max_iters = term.getUpBoundIterations((uint32_t)best.inlier_number);
                }
                if (sprt) max_iters = std::min(max_iters, sprt->getUpperBoundIterations(best.inlier_number));
                if (records && (uint32_t)nrec < rec_cap) {
                    usac_record &rr = records[nrec];
                    rr.hyp_index = iters;
                    rr.inliers = cur.inlier_number;
                    rr.score = cur.score;
                    memcpy(rr.model, best_model, sizeof(best_model));
                    rr.valid = 1;
                }
                nrec++;
            }
            iters++;
            if (prosac && pterm->terminationLength() != gen_term && j + 1 < B) {
                // would the NEXT sample be drawn differently (prosac_sampler.hpp: a subset above the
                // termination length takes the uniform draw)?  The subsets only grow and the length
                // only shrinks, so the batch's samples stay valid up to the first one that would --
                // the replay goes on through them (the run often ends there) and rewinds at it
                const uint32_t tl = pterm->terminationLength();
                rewind = (subset_at[j + 1] > gen_term) || (subset_at[j + 1] > tl);
                if (rewind) break;
            }
        }
        if (rewind) {  // sampler state just after sample j: replay the first j + 1 draws
            pro = std::move(snapshot);
            std::vector<int32_t> tmp(m);
            for (uint32_t k = 0; k <= j; k++) pro->generateSample(tmp.data(), gen_term);
            out->rollbacks++;
        }
    }
    if (spec) out->spec_wasted += spec_B;  // the run ended before the batch drawn ahead
    out->iters = iters;
    out->n_records = nrec;
    out->sprt_histories = sprt ? (int32_t)sprt->histories() : 0;
    out->prosac_term_len = prosac ? pterm->terminationLength() : n;
    auto lo_counters = [&]() {
        out->lo_inner_iters = lo ? lo->inner_count : gc ? gc->gc_iters : 0;
        out->lo_iterative_iters = lo ? lo->iterative_count : gc ? gc->labelings : 0;
        out->lo_rounds = lo ? lo->rounds : gc ? gc->labelings : 0;
        out->lo_stages = lo ? lo->stages : gc ? gc->stages : 0;
        out->lo_fits = lo ? lo->fits : 0;
    };
    lo_counters();
    memcpy(out->minimal_model, best_model, sizeof(best_model));
    out->minimal_inliers = best.inlier_number;
    if (best.inlier_number == 0) {
        memcpy(out->model, best_model, sizeof(best_model));
        return fail(c, USAC_ERR_NO_MODEL, "best score is 0 (ransac.cpp:143-147)");
    }
    if (gc && gc->gc_iters == 0) {  // "Graph Cut lo was set, but did not run, run it" (ransac.cpp:149-153)
        lap(T_REPLAY);
        gc->run(best_model, best.inlier_number, best.score);
        if (gc->rc) return gc->rc;
        lap(T_LO);
        lo_counters();
        memcpy(out->minimal_model, best_model, sizeof(best_model));
        out->minimal_inliers = best.inlier_number;
    }

    lap(T_REPLAY);
    // ---- polish (ransac.cpp:157-207) on the device, the passes submitted in groups: pass k
    // fits the list pass k - 1 scored (the initial getInliers(best_model) list for pass 0) and
    // scores the fitted model from device memory into list k + 1 (compaction gated on the fit's
    // ok); between passes k_polish_prep takes the host's acceptance decision on the device and
    // hands pass k + 1 its point count, or 0 after a rejection (a no-op pass).  All results land
    // in one device block (usac_kernels.h kPol*) copied with one D2H per group; the host replays the
    // reference's loop on them and stops at the first rejection, so `cur` ends as best_model's
    // own inlier list (the same kernels, model and threshold as the final getInliers would use).
    HIP_TRY(c, c->pol_res.reserve(sizeof(float) * usac::kPolWords));
    HIP_TRY(c, c->pol_lists.reserve(sizeof(int32_t) * 4 * (size_t)std::max<uint32_t>(c->n, 1)));
    HIP_TRY(c, c->inl_scratch.reserve(usac::inliers_scratch_bytes(c->n, 1)));
    if (!c->pol_pin && !(c->pol_pin = PinnedPool::get().take(sizeof(float) * usac::kPolWords, &c->pol_pin_bytes)))
        return fail(c, USAC_ERR_HIP, "pinned host allocation failed");
    float *dres = c->pol_res.as<float>();
    int32_t *dres_i = c->pol_res.as<int32_t>();
    const float *hres = static_cast<const float *>(c->pol_pin);
    int32_t *lists[5] = {c->inl_idx.as<int32_t>(), c->pol_lists.as<int32_t>(), nullptr, nullptr, nullptr};
    for (int k = 2; k < 5; k++) lists[k] = lists[1] + (size_t)(k - 1) * std::max<uint32_t>(c->n, 1);
    HIP_TRY(c, hipMemcpyAsync(c->one_model.p, best_model, sizeof(float) * 9, hipMemcpyHostToDevice, c->stream));
    // USAC_POLISH_FUSED=1: the whole polish in one workgroup (k_polish_fused) when the best
    // model's list and the point set fit its LDS -- one launch instead of ~56, bit-identical, but
    // not faster on cfg3 exact (0.30-0.33 vs 0.28 ms: the sequential sums' 64-candidate
    // speculation needs more than one CU's issue rate), so off by default
    // (USAC_POLISH_FUSED_MAX: a lower list bound, which makes the tests resume passes the
    // multi-launch way)
    const char *fe = getenv("USAC_POLISH_FUSED"), *fm = getenv("USAC_POLISH_FUSED_MAX");
    const uint32_t fit_max = fm ? std::min<uint32_t>((uint32_t)atoi(fm), usac::kPolFitMax) : usac::kPolFitMax;
    const bool fused = fe && atoi(fe) != 0 && c->estimator != USAC_LINE2D && c->n <= usac::kPolPtsMax &&
                       (uint32_t)best.inlier_number <= fit_max;
    const bool pol_prof = fused && getenv("USAC_PROFILE");
    if (pol_prof) {
        HIP_TRY(c, c->partial.reserve(sizeof(uint64_t) * 64));
        HIP_TRY(c, hipMemsetAsync(c->partial.p, 0, sizeof(uint64_t) * 64, c->stream));
    }
    if (fused)
        HIP_TRY(c, usac::launch_polish_fused(c->stream, c->estimator, c->pts.p, c->n, c->one_model.as<float>(), thr,
                                             best.inlier_number, usac::PolLists{{lists[0], lists[1], lists[2], lists[3],
                                                                                 lists[4]}},
                                             dres_i, fit_max, pol_prof ? c->partial.as<uint64_t>() : nullptr));
    else
        HIP_TRY(c, usac::launch_inliers_batch(c->stream, c->estimator, c->pts.p, c->n, c->one_model.as<float>(), 1,
                                              thr, nullptr, nullptr, lists[0], 0, dres_i + 12, dres + 13,
                                              c->inl_scratch.p));  // quality->getInliers(best_model)
    // passes go out in groups of G (USAC_POLISH_GROUP): a group is one submission and one host
    // wait; the next group is submitted only while every pass so far was accepted.  Default: all
    // four at once for a best model of <= 8192 inliers (cfg3 exact: 1.15 vs 1.20-1.28 ms per run
    // with groups of 2), two above (cfg5's 17 k-inlier fits: a rejected pass's no-op successors
    // cost 0.1 ms; profiles/r4c/ab_polish.txt, profiles/r5/polish_ab.txt)
    constexpr int kPasses = 4;
    const int kGroup = [&] {
        const char *g = getenv("USAC_POLISH_GROUP");
        const int v = g ? atoi(g) : best.inlier_number <= 8192 ? 4 : 2;
        return v < 1 ? 1 : v > kPasses ? kPasses : v;
    }();
    int32_t *cur = lists[0];
    int32_t cur_cnt = 0;
    int prev = 0;
    bool stop = false;
    // ransac.cpp:170-200 on the results of passes k0 .. k1 - 1 (pol_pin)
    auto replay = [&](int k0, int k1) {
        for (int k = k0; k < k1; k++) {
            const float *r = hres + usac::kPolPass * k;
            memcpy(&ok, r + 9, sizeof(int32_t));
            memcpy(&cnt, r + 10, sizeof(int32_t));
            memcpy(&s, r + 11, sizeof(float));
            if (!ok || (double)((float)cnt / (float)best.inlier_number) < 0.8 || cnt <= prev) {
                stop = true;
                break;
            }
            prev = cnt;
            best.inlier_number = cnt;
            best.score = s;
            memcpy(best_model, r, sizeof(best_model));
            cur = lists[k + 1];
            cur_cnt = cnt;
            out->polish_passes++;
        }
    };
    int k_first = 0;  // the first pass for the multi-launch path
    // USAC_FINISH_SCORE=0: each pass's finish, scoring and acceptance as three launches
    const char *fse = getenv("USAC_FINISH_SCORE");
    const bool finish_score = !(fse && atoi(fse) == 0) && c->estimator != USAC_LINE2D && c->n <= usac::kPolPtsMax;
    if (fused) {
        HIP_TRY(c, hipMemcpyAsync(c->pol_pin, dres, sizeof(float) * usac::kPolWords, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, stream_wait(c->stream));
        memcpy(&cur_cnt, hres + 12, sizeof(int32_t));
        memcpy(&k_first, hres + usac::kPolStop, sizeof(int32_t));
        if (k_first < 0 || k_first > kPasses) return fail(c, USAC_ERR_HIP, "fused polish: bad pass count");
        replay(0, k_first);
        if (pol_prof) {  // the fused polish's phases (us): getInliers, then per pass gather, means,
            // distance terms, distances, A^T A, finish, score, Σerr
            uint64_t st[64] = {0};
            HIP_TRY(c, hipMemcpy(st, c->partial.p, sizeof(st), hipMemcpyDeviceToHost));
            fprintf(stderr, "polish_fused us: init %.1f %.1f |", (st[1] - st[0]) * 0.01, (st[2] - st[1]) * 0.01);
            uint64_t last = st[2];
            for (int k = 0; k < k_first; k++) {
                for (int i = 0; i < 8; i++) {
                    const uint64_t v = st[3 + 8 * k + i];
                    fprintf(stderr, " %.1f", v >= last ? (v - last) * 0.01 : -1.0);
                    if (v >= last) last = v;
                }
                fprintf(stderr, " |");
            }
            fprintf(stderr, " walked segments: 4ch %llu 2ch %llu 1ch %llu\n", (unsigned long long)st[44],
                    (unsigned long long)st[42], (unsigned long long)st[41]);
        }
    }
    for (int k0 = k_first; k0 < kPasses && !stop; k0 += kGroup) {
        const int k1 = std::min(k0 + kGroup, kPasses);
        for (int k = k0; k < k1; k++) {
            float *pres = dres + usac::kPolPass * k;
            int32_t *dok = dres_i + usac::kPolPass * k + 9;
            // the pass's finish, scoring and acceptance in one workgroup (k_finish_score) when the
            // points fit its LDS and the fit takes the multi-launch path
            const uint32_t nfit = k == 0 ? (uint32_t)best.inlier_number : c->n;
            const bool fs = finish_score && nfit > usac::kSmallFitMax;
            usac::NmBatch nb{};
            if (k == 0)
                HIP_TRY(c, enqueue_nonminimal(c, lists[0], nfit, pres, dok, nullptr, nullptr, fs ? &nb : nullptr));
            else  // the count pass k - 1's acceptance left on the device; c->n bounds it
                HIP_TRY(c, enqueue_nonminimal(c, lists[k], nfit, pres, dok, nullptr,
                                              reinterpret_cast<const uint32_t *>(dres_i + usac::kPolNs + k),
                                              fs ? &nb : nullptr));
            if (fs) {
                HIP_TRY(c, usac::launch_finish_score(c->stream, c->estimator, nb, c->pts.p, c->n, thr, lists[k + 1],
                                                     dok + 1, pres + 11, dres_i, k + 1 < kPasses ? k : -1,
                                                     best.inlier_number));
                continue;
            }
            HIP_TRY(c, usac::launch_inliers_batch(c->stream, c->estimator, c->pts.p, c->n, pres, 1, thr, nullptr,
                                                  nullptr, lists[k + 1], 0, dok + 1, pres + 11, c->inl_scratch.p, dok));
            if (k + 1 < kPasses) HIP_TRY(c, usac::launch_polish_prep(c->stream, dres_i, k, best.inlier_number));
        }
        HIP_TRY(c, hipMemcpyAsync(c->pol_pin, dres, sizeof(float) * usac::kPolPass * k1, hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, stream_wait(c->stream));
        if (k0 == 0) memcpy(&cur_cnt, hres + 12, sizeof(int32_t));
        replay(k0, k1);
    }
    const auto t1 = std::chrono::steady_clock::now();
    lap(T_POLISH);
    if (getenv("USAC_PROFILE"))
        fprintf(stderr,
                "usac_ransac_run ms: setup %.3f draw %.3f device %.3f sums %.3f replay %.3f lo %.3f polish %.3f "
                "(lo rounds %u stages %u enqueue %.3f poll %.3f graphs %u; setup: buffers %.3f neighbours %.3f "
                "lo/gc %.3f; sprt walks %.3f, draws %.3f; iters %u batches %u)\n",
                tsplit[T_SETUP], tsplit[T_DRAW], tsplit[T_DEVICE], tsplit[T_SUMS], tsplit[T_REPLAY], tsplit[T_LO],
                tsplit[T_POLISH], lo ? lo->rounds : gc ? gc->labelings : 0u, lo ? lo->stages : gc ? gc->stages : 0u,
                lo ? lo->t_enqueue : 0.0, lo ? lo->t_poll : 0.0, lo ? lo->graphs_built : 0u, tsub[0],
                tsub[1] - tsub[0], tsub[2] - tsub[1], t_verify, t_drawonly, iters, (uint32_t)out->batches);
    // ransac.cpp:214 getInliers(best_model): `cur` already is that list (see above)
    cnt = cur_cnt;
    if (inliers_out && cnt > 0) {  // DMA into pinned memory, then into the caller's buffer
        pinned_vector<int32_t> stage((size_t)cnt);
        HIP_TRY(c, hipMemcpyAsync(stage.data(), cur, sizeof(int32_t) * (size_t)cnt, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, stream_wait(c->stream));
        memcpy(inliers_out, stage.data(), sizeof(int32_t) * (size_t)cnt);
    }
    memcpy(out->model, best_model, sizeof(best_model));
    out->inliers = best.inlier_number;
    out->time_us = std::chrono::duration_cast<std::chrono::microseconds>(t1 - t0).count();
    return USAC_OK;
}

int usac_ransac_run(usac_ctx *c, const usac_params *prm, usac_run_output *out, int32_t *inliers_out,
                    usac_record *records, uint32_t rec_cap) {
    return ransac_run_impl(c, prm, 1, 0, nullptr, nullptr, out, inliers_out, records, rec_cap);
}

int usac_ransac_run_sharded(usac_ctx *c, const usac_params *prm, int nranks, int rank, usac_allgather_fn gather,
                            void *gather_user, usac_run_output *out, int32_t *inliers_out, usac_record *records,
                            uint32_t rec_cap) {
    return ransac_run_impl(c, prm, nranks, rank, gather, gather_user, out, inliers_out, records, rec_cap);
}

// ---------------------------------------------------------------- multi-GPU
int usac_comm_unique_id(uint8_t *id128) {
    if (!id128) return USAC_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return USAC_ERR_HIP;
    memcpy(id128, &id, sizeof(id) < 128 ? sizeof(id) : 128);
    return USAC_OK;
}

int usac_comm_init(usac_ctx *c, int nranks, int rank, const uint8_t *id128) {
    if (!c || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return USAC_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    ncclUniqueId id;
    memcpy(&id, id128, sizeof(id) < 128 ? sizeof(id) : 128);
    NCCL_TRY(c, ncclCommInitRank(&c->comm, nranks, id, rank));
    if (!c->coll_ev) HIP_TRY(c, StreamPool::get().event(&c->coll_ev));
    c->nranks = nranks;
    c->rank = rank;
    HIP_TRY(c, c->rec_send.reserve(sizeof(usac_record)));
    HIP_TRY(c, c->rec_all.reserve(sizeof(usac_record) * (size_t)nranks));
    return USAC_OK;
}

int usac_comm_count(usac_ctx *c, int *nranks, int *rank, int *device) {
    if (!c || !nranks || !rank || !device) return USAC_ERR_ARG;
    if (!c->comm) return fail(c, USAC_ERR_ARG, "usac_comm_init not called");
    NCCL_TRY(c, ncclCommCount(c->comm, nranks));
    NCCL_TRY(c, ncclCommUserRank(c->comm, rank));
    NCCL_TRY(c, ncclCommCuDevice(c->comm, device));
    return USAC_OK;
}

int usac_exchange_best_async(usac_ctx *c, usac_ctx *batch, uint32_t slot) {
    if (!c || !batch || slot >= USAC_XRING) return USAC_ERR_ARG;
    if (!c->comm) return fail(c, USAC_ERR_ARG, "usac_comm_init not called");
    if (batch->device != c->device) return fail(c, USAC_ERR_ARG, "exchange: batch context on another device");
    HIP_TRY(c, hipSetDevice(c->device));
    if (!c->xstream) {
        HIP_TRY(c, StreamPool::get().stream(&c->xstream));
        for (int k = 0; k < USAC_XRING; k++) {
            HIP_TRY(c, StreamPool::get().event(&c->xev_batch[k]));
            HIP_TRY(c, StreamPool::get().event(&c->xev_done[k]));
        }
        HIP_TRY(c, c->xring.reserve(sizeof(usac_record) * (size_t)USAC_XRING * (size_t)(c->nranks + 1)));
        c->xring_host = static_cast<usac_record *>(
            PinnedPool::get().take(sizeof(usac_record) * (size_t)USAC_XRING * (size_t)c->nranks, &c->xring_host_bytes));
        if (!c->xring_host) return fail(c, USAC_ERR_HIP, "pinned host allocation failed");
    }
    // the batch's argmax record is copied into the ring's send slot on the batch stream (the
    // batch's next use of that stream overwrites its record); the exchange stream waits for
    // that copy only (neither stream waits for the other's later work)
    usac_record *dsend = c->xring.as<usac_record>() + (size_t)USAC_XRING * c->nranks + slot;
    usac_record *dall = c->xring.as<usac_record>() + (size_t)slot * c->nranks;
    HIP_TRY(c, hipMemcpyAsync(dsend, batch->best.p, sizeof(usac_record), hipMemcpyDeviceToDevice, batch->stream));
    HIP_TRY(c, hipEventRecord(c->xev_batch[slot], batch->stream));
    HIP_TRY(c, hipStreamWaitEvent(c->xstream, c->xev_batch[slot], 0));
    if (c->coll_pending) {  // after the last collective issued on c->stream
        HIP_TRY(c, hipStreamWaitEvent(c->xstream, c->coll_ev, 0));
        c->coll_pending = false;
    }
    NCCL_TRY(c, ncclAllGather(dsend, dall, sizeof(usac_record), ncclUint8, c->comm, c->xstream));
    HIP_TRY(c, hipMemcpyAsync(c->xring_host + (size_t)slot * c->nranks, dall, sizeof(usac_record) * (size_t)c->nranks,
                              hipMemcpyDeviceToHost, c->xstream));
    HIP_TRY(c, hipEventRecord(c->xev_done[slot], c->xstream));
    c->x_last = (int)slot;
    return USAC_OK;
}

int usac_exchange_best_wait(usac_ctx *c, uint32_t slot, usac_record *all) {
    if (!c || !all || slot >= USAC_XRING || !c->xstream) return USAC_ERR_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    for (uint32_t spins = 0;; spins++) {  // poll (as stream_wait): returns within ~1 us
        const hipError_t e = hipEventQuery(c->xev_done[slot]);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) return fail(c, USAC_ERR_HIP, std::string("exchange: ") + hipGetErrorString(e));
        if ((spins & 1023u) == 1023u) std::this_thread::yield();
    }
    memcpy(all, c->xring_host + (size_t)slot * c->nranks, sizeof(usac_record) * (size_t)c->nranks);
    return USAC_OK;
}

int usac_allgather_records(usac_ctx *c, const usac_record *local, usac_record *all) {
    if (!c || !local || !all) return USAC_ERR_ARG;
    if (!c->comm) return fail(c, USAC_ERR_ARG, "usac_comm_init not called");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMemcpyAsync(c->rec_send.p, local, sizeof(usac_record), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, order_after_exchanges(c));
    NCCL_TRY(c, ncclAllGather(c->rec_send.p, c->rec_all.p, sizeof(usac_record), ncclUint8, c->comm, c->stream));
    HIP_TRY(c, mark_collective(c));
    HIP_TRY(c, hipMemcpyAsync(all, c->rec_all.p, sizeof(usac_record) * (size_t)c->nranks, hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    return USAC_OK;
}

int usac_merge_records(const usac_record *recs, uint32_t n, usac_record *best) {
    if (!recs || !best || n == 0) return USAC_ERR_ARG;
    usac_record b = recs[0];
    for (uint32_t i = 1; i < n; i++)
        if (rec_better(recs[i], b)) b = recs[i];
    *best = b;
    return USAC_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- stateful plugins (ABI 11)
// The reference's per-call plugin surface: handles that keep each plugin's state
// between calls, so a caller that keeps its own Ransac::run loop swaps plugin by plugin.  The
// state machines are usac_host.hpp's (the same ones ransac_run_impl replays with); every inlier
// test, least-squares fit and neighbour build runs on the context's device.

struct usac_random {
    usac::GlibcRandom g;
    explicit usac_random(uint32_t seed) : g(seed) {}
};

struct usac_sampler {
    usac_ctx *c = nullptr;
    int kind = USAC_SAMPLER_UNIFORM;
    uint32_t n = 0, m = 0;
    std::unique_ptr<usac::UniformSampler> uni;
    std::unique_ptr<usac::ProsacSampler> pro;
    std::shared_ptr<const usac::GridNeighbors> grid;
    std::unique_ptr<usac::NapsacSampler> nap;
    std::vector<int32_t> knn_tab;
    std::unique_ptr<usac::NapsacKnnSampler> napk;
    usac_termination *term = nullptr;  // the linked ProsacTerminationCriteria (PROSAC)
    uint64_t drawn = 0;
    std::vector<int32_t> last;  // generate_batch: the reference's reused sample array
};

struct usac_termination {
    usac_ctx *c = nullptr;
    float thr = 0.f;
    usac::StandardTerminationCriteria std_;
    std::unique_ptr<usac::ProsacTerminationCriteria> pro;
    usac_sampler *sampler = nullptr;
    std::vector<int32_t> inl;
    usac_termination(usac_ctx *ctx, const usac_params *p)
        : c(ctx), thr(p->threshold), std_(p->desired_prob, ctx->m, ctx->n, p->max_iterations) {}
};

struct usac_sprt {
    usac_ctx *c = nullptr;
    float thr = 0.f;
    uint32_t nw = 0;
    std::unique_ptr<usac::Sprt> s;
    DevBuf pool_idx, pool_pts, masks;
    std::vector<uint32_t> hmask;  // the current batch's words [nw][rows]
    uint32_t rows = 0;
    std::vector<int32_t> row_of;  // batch slot -> row (-1: empty slot)
    uint32_t batch_B = 0, batch_slots = 0;
    uint32_t rejected = 0;
    int max_before = 20;  // usac_params::max_hypothesis_test_before_sprt
    ~usac_sprt() {
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        pool_idx.release();
        pool_pts.release();
        masks.release();
    }
};

struct usac_lo {
    usac_ctx *c = nullptr;
    std::unique_ptr<LoRansac> lo;
    std::unique_ptr<GcLo> gc;
    std::vector<int32_t> knn_tab;
    std::shared_ptr<const usac::GridNeighbors> grid;
};

namespace {

// host models (K x 9, line: first 3 of each row) into the context's device model layout (H: H
// and H^-1, [18][K]; F / E: [9][K]; line [3][K]), the layout the solve kernels leave
int upload_models(usac_ctx *c, const float *models, uint32_t K) {
    int rc = ensure_batch(c, K);
    if (rc) return rc;
    HIP_TRY(c, hipMemcpyAsync(c->hostmodels.p, models, sizeof(float) * 9 * (size_t)K, hipMemcpyHostToDevice,
                              c->stream));
    if (listed(c)) HIP_TRY(c, usac::launch_prepare_f(c->stream, c->hostmodels.as<float>(), K, c->models.as<float>()));
    else if (is_h(c)) HIP_TRY(c, usac::launch_prepare_h(c->stream, c->hostmodels.as<float>(), K, c->models.as<float>()));
    else HIP_TRY(c, usac::launch_prepare_line(c->stream, c->hostmodels.as<float>(), K, c->models.as<float>()));
    return USAC_OK;
}

// pool-order inlier words of K host models into s->hmask ([nw][K], row = model)
int sprt_masks(usac_sprt *s, const float *models, uint32_t K) {
    usac_ctx *c = s->c;
    HIP_TRY(c, hipSetDevice(c->device));
    int rc = upload_models(c, models, K);
    if (rc) return rc;
    HIP_TRY(c, s->masks.reserve(sizeof(uint32_t) * s->nw * (size_t)K));
    HIP_TRY(c, usac::launch_pool_mask(c->stream, c->estimator, s->pool_pts.p, c->n, c->models.as<float>(), K, nullptr,
                                      nullptr, K, s->thr, s->masks.as<uint32_t>(), K));
    s->hmask.resize((size_t)s->nw * K);
    HIP_TRY(c, hipMemcpyAsync(s->hmask.data(), s->masks.p, sizeof(uint32_t) * s->nw * (size_t)K, hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, stream_wait(c->stream));
    s->rows = K;
    return USAC_OK;
}

// the host walk of row r (sprt.hpp:191-317)
bool sprt_walk(usac_sprt *s, uint32_t r, int32_t current_hypothese, uint32_t maximum_score, int &count, float &score) {
    const bool good = s->s->verify(s->hmask.data() + r, current_hypothese, maximum_score, count, score, s->rows);
    if (!good) s->rejected++;
    return good;
}

}  // namespace

extern "C" {

int usac_random_create(uint32_t seed, usac_random **out) {
    if (!out) return USAC_ERR_ARG;
    *out = new usac_random(seed);
    return USAC_OK;
}

uint32_t usac_random_next(usac_random *rng) { return rng ? rng->g.next() : 0u; }

void usac_random_destroy(usac_random *rng) { delete rng; }

int usac_sampler_create(usac_ctx *c, const usac_params *p, usac_random *rng, usac_sampler **out) {
    if (!c || !p || !out) return USAC_ERR_ARG;
    *out = nullptr;
    const int kind = p->sampler == 0 ? USAC_SAMPLER_UNIFORM : p->sampler;
    if (kind != USAC_SAMPLER_UNIFORM && kind != USAC_SAMPLER_PROSAC && kind != USAC_SAMPLER_NAPSAC)
        return fail(c, USAC_ERR_UNSUPPORTED, "sampler: Uniform, Napsac or Prosac");
    if (kind != USAC_SAMPLER_PROSAC && !rng) return fail(c, USAC_ERR_ARG, "sampler: Uniform / NAPSAC draw from a usac_random");
    std::unique_ptr<usac_sampler> s(new usac_sampler());
    s->c = c;
    s->kind = kind;
    s->n = c->n;
    s->m = c->m;
    s->last.assign(c->m, 0);
    if (kind == USAC_SAMPLER_PROSAC) {
        if (c->n < c->m || c->m < 2) return fail(c, USAC_ERR_ARG, "PROSAC needs n >= sample size");
        s->pro.reset(new usac::ProsacSampler(p->seed, c->n, c->m));
    } else if (kind == USAC_SAMPLER_NAPSAC) {
        HIP_TRY(c, hipSetDevice(c->device));
        if (p->neighbors == USAC_NEIGHBORS_GRID) {
            if (c->cols != 4) return fail(c, USAC_ERR_ARG, "NAPSAC grid neighbours need 4-column points (SURVEY Q17)");
            if (p->cell_size <= 0) return fail(c, USAC_ERR_ARG, "NAPSAC cell_size must be > 0");
            int rc = download_grid(c, p->cell_size, s->grid);
            if (rc) return rc;
            s->nap.reset(new usac::NapsacSampler(rng->g, *s->grid, c->n, c->m));
        } else {
            if (p->knn == 0 || p->knn > usac::kKnnMax || p->knn + 1 < c->m)
                return fail(c, USAC_ERR_ARG, "NAPSAC KNN: k_nearest_neighbors must be in [sample_size - 1, 32]");
            s->knn_tab.resize((size_t)c->n * p->knn);
            int rc = usac_knn(c, p->knn, s->knn_tab.data(), nullptr);
            if (rc) return rc;
            s->napk.reset(new usac::NapsacKnnSampler(rng->g, s->knn_tab.data(), c->n, c->m, p->knn));
        }
    } else {
        s->uni.reset(new usac::UniformSampler(rng->g, c->n, c->m));
    }
    *out = s.release();
    return USAC_OK;
}

int usac_sampler_generate(usac_sampler *s, int32_t *sample) {
    if (!s || !sample) return USAC_ERR_ARG;
    if (s->pro) {
        if (s->drawn >= usac::ProsacSampler::kGrowthMax)
            return fail(s->c, USAC_ERR_UNSUPPORTED, "PROSAC: more than T_N = 200000 samples (the reference then "
                                                    "draws outside the point range)");
        s->pro->generateSample(sample, s->term && s->term->pro ? s->term->pro->terminationLength() : s->n);
    } else if (s->nap) {
        s->nap->generateSample(sample);
    } else if (s->napk) {
        s->napk->generateSample(sample);
    } else {
        s->uni->generateSample(sample);
    }
    s->drawn++;
    return USAC_OK;
}

int usac_sampler_generate_batch(usac_sampler *s, uint32_t count, int32_t *samples) {
    if (!s || (!samples && count)) return USAC_ERR_ARG;
    for (uint32_t j = 0; j < count; j++) {
        int32_t *smp = samples + (size_t)j * s->m;
        memcpy(smp, s->last.data(), sizeof(int32_t) * s->m);
        int rc = usac_sampler_generate(s, smp);
        if (rc) return rc;
        memcpy(s->last.data(), smp, sizeof(int32_t) * s->m);
    }
    return USAC_OK;
}

int usac_sampler_state(const usac_sampler *s, uint64_t *drawn, uint32_t *subset_size, uint32_t *largest) {
    if (!s) return USAC_ERR_ARG;
    if (drawn) *drawn = s->drawn;
    if (subset_size) *subset_size = s->pro ? s->pro->subset() : s->n;
    if (largest) *largest = s->pro ? s->pro->largest() : s->n;
    return USAC_OK;
}

void usac_sampler_destroy(usac_sampler *s) {
    if (!s) return;
    if (s->term) s->term->sampler = nullptr;
    delete s;
}

int usac_termination_create(usac_ctx *c, const usac_params *p, usac_sampler *prosac, usac_termination **out) {
    if (!c || !p || !out) return USAC_ERR_ARG;
    *out = nullptr;
    if (prosac && (!prosac->pro || prosac->c != c))
        return fail(c, USAC_ERR_ARG, "termination: the linked sampler must be a PROSAC sampler of this context");
    if (prosac && prosac->term) return fail(c, USAC_ERR_ARG, "termination: the sampler is linked already");
    if (prosac && c->n <= 20)
        return fail(c, USAC_ERR_ARG, "PROSAC termination needs > 20 points (prosac_termination_criteria.hpp:158-163)");
    std::unique_ptr<usac_termination> t(new usac_termination(c, p));
    if (prosac) {
        t->pro.reset(new usac::ProsacTerminationCriteria(prosac->pro->growth(), p->desired_prob, c->m, c->n,
                                                         p->max_iterations));
        t->sampler = prosac;
        prosac->term = t.get();
        t->inl.resize(c->n);
    }
    *out = t.release();
    return USAC_OK;
}

uint32_t usac_termination_bound(const usac_termination *t, uint32_t inlier_size, uint32_t points_size) {
    if (!t) return 0;
    return t->std_.getUpBoundIterations(inlier_size, points_size ? points_size : t->c->n);
}

int usac_prosac_termination(usac_termination *t, uint32_t hyp_count, const float *model, uint32_t *max_iters,
                            uint32_t *termination_length) {
    if (!t || !model || !max_iters) return USAC_ERR_ARG;
    usac_ctx *c = t->c;
    if (!t->pro) return fail(c, USAC_ERR_ARG, "not a PROSAC termination criteria");
    if (!t->sampler) return fail(c, USAC_ERR_ARG, "PROSAC termination: its sampler was destroyed");
    uint32_t n = 0;
    int rc = usac_get_inliers(c, model, t->thr, t->inl.data(), &n, nullptr);
    if (rc) return rc;
    *max_iters = t->pro->getUpBoundIterationsSorted(hyp_count, t->inl.data(), n, t->sampler->pro->largest());
    if (termination_length) *termination_length = t->pro->terminationLength();
    return USAC_OK;
}

void usac_termination_destroy(usac_termination *t) {
    if (!t) return;
    if (t->sampler) t->sampler->term = nullptr;
    delete t;
}

int usac_sprt_create(usac_ctx *c, const usac_params *p, usac_random *rng, usac_sprt **out) {
    if (!c || !p || !rng || !out) return USAC_ERR_ARG;
    *out = nullptr;
    HIP_TRY(c, hipSetDevice(c->device));
    std::unique_ptr<usac_sprt> s(new usac_sprt());
    s->c = c;
    s->thr = p->threshold;
    s->nw = (c->n + 31) / 32;
    s->max_before = max_before_sprt(p);
    s->s.reset(new usac::Sprt(rng->g, c->estimator, c->n, c->m, p->max_iterations, s->max_before));
    HIP_TRY(c, s->pool_idx.reserve(sizeof(uint32_t) * c->n));
    HIP_TRY(c, s->pool_pts.reserve(sizeof(float) * c->cols * (size_t)c->n));
    HIP_TRY(c, hipMemcpyAsync(s->pool_idx.p, s->s->pool().data(), sizeof(uint32_t) * c->n, hipMemcpyHostToDevice,
                              c->stream));
    HIP_TRY(c, usac::launch_gather_points(c->stream, c->pts.p, c->cols, s->pool_idx.as<uint32_t>(), c->n,
                                          s->pool_pts.p));
    HIP_TRY(c, stream_wait(c->stream));
    *out = s.release();
    return USAC_OK;
}

int usac_sprt_verify(usac_sprt *s, const float *model, int32_t current_hypothese, uint32_t maximum_score,
                     int32_t *good, int32_t *count, float *score) {
    if (!s || !model || !good || !count || !score) return USAC_ERR_ARG;
    float m9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    memcpy(m9, model, sizeof(float) * (size_t)ncomp(s->c));
    s->batch_B = 0;  // a batch replay's words are gone
    int rc = sprt_masks(s, m9, 1);
    if (rc) return rc;
    int cnt = *count;
    float sc = *score;
    *good = sprt_walk(s, 0, current_hypothese, maximum_score, cnt, sc) ? 1 : 0;
    *count = cnt;
    *score = sc;
    return USAC_OK;
}

uint32_t usac_sprt_upper_bound(const usac_sprt *s, uint32_t inlier_size) {
    return s ? s->s->getUpperBoundIterations((int)inlier_size) : 0u;
}

int usac_sprt_stats(const usac_sprt *s, uint32_t *histories, uint32_t *rejected) {
    if (!s) return USAC_ERR_ARG;
    if (histories) *histories = (uint32_t)s->s->histories();
    if (rejected) *rejected = s->rejected;
    return USAC_OK;
}

int usac_sprt_replay(usac_sprt *s, const float *models, const int32_t *n_models, uint32_t B, usac_sprt_state *st) {
    if (!s || !models || !n_models || !st) return USAC_ERR_ARG;
    usac_ctx *c = s->c;
    const uint32_t S = c->spk;
    if (st->sample > B || (st->sample < B && st->slot > S)) return fail(c, USAC_ERR_ARG, "sprt_replay: cursor out of range");
    st->found = 0;
    st->rejected = 0;
    if (st->sample == 0 && st->slot == 0) {  // a new batch: every model's pool-order inlier words
        std::vector<float> list;
        s->row_of.assign((size_t)B * S, -1);
        uint32_t K = 0;
        for (uint32_t b = 0; b < B; b++) {
            if (n_models[b] < 0 || (uint32_t)n_models[b] > S) return fail(c, USAC_ERR_ARG, "sprt_replay: n_models out of range");
            for (uint32_t q = 0; q < (uint32_t)n_models[b]; q++) {
                s->row_of[(size_t)b * S + q] = (int32_t)K++;
                list.insert(list.end(), models + ((size_t)b * S + q) * 9, models + ((size_t)b * S + q + 1) * 9);
            }
        }
        if (K) {
            int rc = sprt_masks(s, list.data(), K);
            if (rc) return rc;
        }
        s->batch_B = B;
    } else if (s->batch_B != B) {
        return fail(c, USAC_ERR_ARG, "sprt_replay: a batch resumes with the models it started with");
    }
    const uint32_t rej0 = s->rejected;
    uint32_t b = st->sample, q = st->slot;
    while (b < B) {
        if (q == 0 && st->iters >= st->max_iters) break;  // while (iters < max_iters)
        for (; q < (uint32_t)n_models[b]; q++) {
            int cnt = 0;
            float sc = 0.f;
            const bool good = sprt_walk(s, (uint32_t)s->row_of[(size_t)b * S + q], (int)st->iters,
                                        (uint32_t)st->best_inliers, cnt, sc);
            if (!good && (int)st->iters >= s->max_before) {  // max_hypothesis_test_before_sprt (model.hpp:40), Q9
                st->iters++;
                continue;
            }
            usac::Score cur, best;
            cur.inlier_number = cnt;
            cur.score = sc;
            best.inlier_number = st->best_inliers;
            best.score = st->best_score;
            if (cur.bigger(best)) {
                st->found = 1;
                st->inliers = cnt;
                st->score = sc;
                st->found_sample = b;
                st->found_slot = q;
                st->sample = b;
                st->slot = q + 1;
                st->rejected = s->rejected - rej0;
                return USAC_OK;
            }
        }
        st->iters++;
        b++;
        q = 0;
    }
    st->sample = b;
    st->slot = 0;
    st->rejected = s->rejected - rej0;
    return USAC_OK;
}

void usac_sprt_destroy(usac_sprt *s) { delete s; }

int usac_lo_create(usac_ctx *c, const usac_params *p, usac_lo **out) {
    if (!c || !p || !out) return USAC_ERR_ARG;
    *out = nullptr;
    HIP_TRY(c, hipSetDevice(c->device));
    int rc = ensure_single(c);
    if (rc) return rc;
    std::unique_ptr<usac_lo> h(new usac_lo());
    h->c = c;
    if (p->lo == USAC_LO_INITLORSC || p->lo == USAC_LO_INITFLORSC) {
        if (p->lo_sample_size == 0 || p->lo_iterative_iterations == 0)
            return fail(c, USAC_ERR_ARG, "LO parameters must be > 0");
        h->lo.reset(new LoRansac(c, p, Shard()));
        if ((rc = h->lo->reserve())) return rc;
    } else if (p->lo == USAC_LO_GC) {
        const bool knn = p->neighbors != USAC_NEIGHBORS_GRID;
        if (knn) {
            if (p->knn == 0 || p->knn > usac::kKnnMax) return fail(c, USAC_ERR_ARG, "GC KNN: k_nearest_neighbors must be in [1, 32]");
            h->knn_tab.resize((size_t)c->n * p->knn);
            if ((rc = usac_knn(c, p->knn, h->knn_tab.data(), nullptr))) return rc;
        } else {
            if (c->cols != 4 || p->cell_size <= 0)
                return fail(c, USAC_ERR_ARG, "GC grid neighbours need 4-column points and cell_size > 0");
            if ((rc = download_grid(c, p->cell_size, h->grid))) return rc;
        }
        h->gc.reset(new GcLo(c, p, knn ? h->knn_tab.data() : nullptr, p->knn, h->grid.get()));
        if ((rc = h->gc->reserve())) return rc;
    } else {
        return fail(c, USAC_ERR_UNSUPPORTED, "LO: InItLORsc / InItFLORsc / GC only");
    }
    *out = h.release();
    return USAC_OK;
}

int usac_lo_get_model_score(usac_lo *h, float *model, int32_t *inliers, float *score) {
    if (!h || !model || !inliers || !score) return USAC_ERR_ARG;
    HIP_TRY(h->c, hipSetDevice(h->c->device));
    int cnt = *inliers;
    float sum = *score;
    if (h->lo) {
        h->lo->run(model, cnt, sum);
        if (h->lo->rc) return h->lo->rc;
    } else {
        h->gc->run(model, cnt, sum);
        if (h->gc->rc) return h->gc->rc;
    }
    *inliers = cnt;
    *score = sum;
    return USAC_OK;
}

int usac_lo_iters(const usac_lo *h, uint32_t *inner, uint32_t *iterative) {
    if (!h) return USAC_ERR_ARG;
    if (inner) *inner = h->lo ? h->lo->inner_count : h->gc->gc_iters;
    if (iterative) *iterative = h->lo ? h->lo->iterative_count : h->gc->labelings;
    return USAC_OK;
}

void usac_lo_destroy(usac_lo *h) {
    if (!h) return;
    (void)hipSetDevice(h->c->device);
    (void)hipStreamSynchronize(h->c->stream);
    delete h;
}

}  // extern "C"
