#pragma once
// usac_pk.hpp -- the fast scorers' two-point stage A (k_score_hf, k_score_f2) on PAIRS of fp32 values
// without packed-fp32 VALU instructions.
//
// On gfx950 a v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 can return wrong values in lanes 48-63
// (the wave's last quarter) while waves of ANOTHER kernel execute MFMAs on the same CU; every other
// VALU class tested (fp32 / fp64 FMA, IEEE division, sqrt, v_rcp / v_rsq / v_sqrt, conversions,
// integer) is unaffected (tools/mfma_interference.cpp: 4 of 60 probe launches beside an MFMA-only
// kernel differ, 19-36 k lanes, all in lanes 48-63; none beside fp32 / fp64 VALU kernels or alone).
// That was the round-5 "recount beside k_score_h16" miscount: the compiler's SLP
// vectoriser had packed the exact residual of k_inl_flags.  The library therefore issues no packed
// fp32 instruction: the backend's packed-fp32-ops feature is off (Makefile), so neither the
// vectorisers nor these helpers can produce one, and the pair arithmetic below is written as two
// scalar operations (USAC_PACKED_F32=1 keeps the vector-typed form, for A/B only).
#include <hip/hip_runtime.h>

namespace usac {

#if defined(USAC_PACKED_F32) && USAC_PACKED_F32
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2f vfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }
#else
struct v2f {
    float x, y;
};
__device__ __forceinline__ v2f vfma(v2f a, v2f b, v2f c) { return v2f{fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)}; }
__device__ __forceinline__ v2f operator*(v2f a, v2f b) { return v2f{a.x * b.x, a.y * b.y}; }
__device__ __forceinline__ v2f operator-(v2f a) { return v2f{-a.x, -a.y}; }
#endif

}  // namespace usac
