// OCP fp8 (e4m3 = 0 / e5m2 = 1) device helpers shared by the quantisation kernels (fp8.hip) and
// the GEMM epilogues that quantise their own output (gemm_tile.hip, "q8" epilogue).
#pragma once
#include "mlt_common.h"
#include "mlt_kernels.h"

namespace mlt {

template <int FMT>
__device__ __forceinline__ float fp8_max() {
  return FMT == 0 ? 448.f : 57344.f;
}

// 4 floats -> 4 saturated fp8 bytes (v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32), byte i = value i
template <int FMT>
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  const float m = fp8_max<FMT>();  // saturate: one v_med3_f32 per value
  a = __builtin_amdgcn_fmed3f(a, -m, m);
  b = __builtin_amdgcn_fmed3f(b, -m, m);
  c = __builtin_amdgcn_fmed3f(c, -m, m);
  d = __builtin_amdgcn_fmed3f(d, -m, m);
  int r;
  if constexpr (FMT == 0) {
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  } else {
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, r, true);
  }
  return (uint32_t)r;
}

// amax is recorded into kAmaxSlots sub-slots (block b -> slot b % kAmaxSlots) so that thousands
// of blocks do not serialise on one device-scope atomic; update_scale reduces the slots.
// Slots sit kAmaxStride floats apart (one 128-B line each), and a block only issues the
// atomic when its maximum beats the slot's current value -- after the first few blocks almost
// none do, so the tail of thousands of same-line device-scope atomics disappears.
__device__ __forceinline__ void atomic_max_pos(float* slots, float v) {
  // |x| >= 0: IEEE ordering of non-negative floats equals their integer ordering
  unsigned* a = reinterpret_cast<unsigned*>(slots + ((blockIdx.x + blockIdx.y * gridDim.x) % kAmaxSlots) * kAmaxStride);
  const unsigned u = __float_as_uint(v);
  if (__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < u) atomicMax(a, u);
}

}  // namespace mlt
