// usac_seqsum.hpp -- helpers of the bit-exact parallel sequential sums (kernels_seqsum.hip):
// segment length, float order keys, candidate starts, segment centres, the two chain ops.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace usac {

namespace seq {

constexpr uint32_t kCand = 256;   // candidate starts per segment (4 waves)
constexpr uint32_t kSegMax = 32;  // segments per chain
constexpr uint32_t kLmin = 256;   // shortest segment

// one fit's scratch: psum[kSegMax][nch] doubles, then R[kSegMax][nch][kCand] floats
__host__ __device__ constexpr size_t scratch_bytes(int nch) {
    return (sizeof(double) + sizeof(float) * kCand) * kSegMax * (size_t)nch;
}

__device__ __forceinline__ uint32_t seg_len(uint32_t n) {
    uint32_t L = (n + kSegMax - 1) / kSegMax;
    L = (L + 63) & ~63u;
    return L < kLmin ? kLmin : L;
}

// order key: adjacent floats have adjacent keys (+0 and -0 share key 0; unkey gives +0)
__device__ __forceinline__ int32_t key(float f) {
    const int32_t b = __float_as_int(f);
    return b >= 0 ? b : -(b & 0x7fffffff);
}
__device__ __forceinline__ float unkey(int32_t k) {
    return __int_as_float(k >= 0 ? k : (int32_t)(0x80000000u | (uint32_t)(-k)));
}

// start of candidate c of a segment centred on ctr (wrapping arithmetic: out-of-range keys
// give garbage starts, which are never matched -- the link compares exact bits)
__device__ __forceinline__ float cand_start(float ctr, uint32_t c) {
    return unkey((int32_t)((uint32_t)key(ctr) + c - kCand / 2));
}

// centre of segment j, chain q: the fp64 prefix of the segment sums, in segment order (the
// same code in the segment and link kernels, so both see the same centre)
__device__ __forceinline__ float centre(const double *psum, uint32_t j, uint32_t nch, uint32_t q) {
    double p = 0.0;
    for (uint32_t i = 0; i < j; i++) p += psum[i * nch + q];
    return (float)p;
}

template <bool F64>
struct Op;
template <>
struct Op<false> {
    typedef float V;
    static __device__ __forceinline__ float step(float s, float x) { return s + x; }
    static __device__ __forceinline__ double wide(float x) { return (double)x; }
};
template <>
struct Op<true> {
    typedef double V;
    static __device__ __forceinline__ float step(float s, double y) { return (float)((double)s + y); }
    static __device__ __forceinline__ double wide(double y) { return y; }
};

__device__ __forceinline__ uint32_t fit_n(const uint32_t *ns, uint32_t n1, uint32_t w) { return ns ? ns[w] : n1; }
__device__ __forceinline__ uint32_t fit_slot(const uint32_t *slots, uint32_t b) { return slots ? slots[b] : b; }

}  // namespace seq

}  // namespace usac
