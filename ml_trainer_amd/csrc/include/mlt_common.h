// Common device helpers for the gfx950 (CDNA4) kernels of ml_trainer_amd.
//
// Conventions used throughout csrc/kernels:
//  * wave64 everywhere: lane = threadIdx.x & 63, reductions are 6 xor-shuffle steps;
//  * block sizes are multiples of 64;
//  * every launcher takes a hipStream_t and never synchronises (graph-capturable);
//  * shape assumptions are validated on the host (bindings.cpp) before launch.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define MLT_WAVE 64

// Device-side index checks, compiled in by `python -m ml_trainer_amd.build --debug` (-DMLT_DEBUG)
// and to nothing otherwise. A failed check prints the condition, the source line and the
// block / thread and lets the kernel continue: no trap, because a trapping wave can take the
// whole GPU (and its neighbours) down -- the printf is the evidence, the host checks the output.
#ifdef MLT_DEBUG
#define MLT_DCHECK(cond)                                                                          \
  do {                                                                                            \
    if (!(cond))                                                                                  \
      printf("[mlt] MLT_DCHECK(%s) failed at %s:%d block (%d,%d,%d) thread %d\n", #cond, __FILE__, \
             __LINE__, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)threadIdx.x);       \
  } while (0)
#else
#define MLT_DCHECK(cond) \
  do {                   \
  } while (0)
#endif

#define MLT_HIP_CHECK(expr)                                                          \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess) {                                                          \
      fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(_e), __FILE__, \
              __LINE__, #expr);                                                      \
      abort();                                                                       \
    }                                                                                \
  } while (0)

namespace mlt {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Segmented sum over aligned groups of G lanes (G power of two, <= 64).
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Segmented reductions over aligned groups of G lanes (G power of two, <= 64) built from DPP
// operand modifiers (quad_perm, row_shr, row_bcast15/31: plain VALU ops, a few cycles each)
// instead of ds_swizzle / ds_bpermute round trips through the LDS crossbar (~100+ cycles each
// on a dependent chain). The result is valid in the LAST lane of each group only.
template <int CTRL, int ROWS, bool MAX>
__device__ __forceinline__ float dpp_reduce_step(float v) {
  const float id = MAX ? -INFINITY : 0.f;  // lanes without a source (or in masked rows) combine with this
  const float o =
      __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(v), CTRL, ROWS, 0xF, false));
  return MAX ? fmaxf(v, o) : v + o;
}
template <int G, bool MAX = false>
__device__ __forceinline__ float group_reduce_last(float v) {
  if constexpr (G >= 2) v = dpp_reduce_step<0xB1, 0xF, MAX>(v);   // quad_perm [1,0,3,2]
  if constexpr (G >= 4) v = dpp_reduce_step<0x4E, 0xF, MAX>(v);   // quad_perm [2,3,0,1]: quad result in all 4
  if constexpr (G >= 8) v = dpp_reduce_step<0x114, 0xF, MAX>(v);  // row_shr:4 -> lanes 7, 15: 8-lane result
  if constexpr (G >= 16) v = dpp_reduce_step<0x118, 0xF, MAX>(v); // row_shr:8 -> lane 15: row result
  if constexpr (G >= 32) v = dpp_reduce_step<0x142, 0xA, MAX>(v); // row_bcast:15 into rows 1, 3 -> lanes 31, 63
  if constexpr (G >= 64) v = dpp_reduce_step<0x143, 0xC, MAX>(v); // row_bcast:31 into rows 2, 3 -> lane 63
  return v;
}

// Block-wide sum; `red` must hold >= blockDim.x/64 floats of LDS. Result broadcast to all threads.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];  // fixed order: deterministic
  return s;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = -INFINITY;
  for (int i = 0; i < nw; ++i) s = fmaxf(s, red[i]);
  return s;
}

// Counter-based hash (splitmix64 finaliser): stateless per-sample RNG that is
// identical under hipGraph replay as long as the counter lives in device memory.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// LDS hand-off between the lanes of ONE wave (a per-wave LDS region): a compiler fence around a
// wave barrier orders the wave's earlier LDS accesses before its later ones -- a wave's LDS
// instructions execute in order, so no s_waitcnt and no workgroup barrier is needed, and the
// other waves of the block keep running (GEMM epilogues stage through per-wave images).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// Round-to-nearest-even f32 -> bf16 via the hardware convert (keeps NaN a NaN).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&b);
}

// XCD-aware bijective block remap (gfx950: 8 XCDs, blocks dealt round-robin).
// Makes consecutive logical tiles land on one XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

}  // namespace mlt
