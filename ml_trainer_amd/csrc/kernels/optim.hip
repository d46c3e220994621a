// Flat multi-tensor optimizers for gfx950.
//
// All parameters of a param-group live in ONE contiguous fp32 buffer (see
// ml_trainer_amd/utils/flat.py), so an optimizer step is a single launch that
// streams p/g/state with 16-byte (float4) accesses. lr and the step counter can
// be read from device memory so the launch is hipGraph-replayable while a LR
// scheduler keeps changing the value (the reference steps schedulers per batch /
// per epoch: src/trainer.py:189-190,198-199).
#include "mlt_common.h"
#include "mlt_kernels.h"
#include "mlt_optim.h"

namespace mlt {

__global__ __launch_bounds__(256) void flat_optim_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ s1, float* __restrict__ s2,
                                                         int64_t n4, OptHyper h, const float* __restrict__ lr_ptr,
                                                         const int64_t* __restrict__ lr_index_ptr,
                                                         const int64_t* __restrict__ step_ptr, float t_host,
                                                         uint16_t* __restrict__ shadow,
                                                         const float* __restrict__ coef_ptr,
                                                         const unsigned* __restrict__ skip) {
  // all-or-nothing data-parallel step: a collective that failed on this rank (sticky error word,
  // e.g. an xGMI peer timeout that left some slices unreduced) vetoes the whole update
  if (skip && __hip_atomic_load(skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
  const float lr = lr_ptr ? lr_ptr[lr_index_ptr ? (*lr_index_ptr - 1) : 0] : h.lr;
  const float t = step_ptr ? (float)(*step_ptr) : t_host;
  if (coef_ptr) h.grad_scale *= *coef_ptr;  // e.g. clip-by-norm coefficient
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* a4 = reinterpret_cast<float4*>(s1);
  float4* b4 = reinterpret_cast<float4*>(s2);
  const bool has_s2 = (h.kind == OPT_ADAM || h.kind == OPT_ADAMW || h.kind == OPT_ADAMAX);
  const bool has_s1 = has_s2 || h.kind == OPT_ADAGRAD || (h.kind == OPT_SGD && h.momentum != 0.f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 pv = p4[i];
    const float4 gv = g4[i];
    float4 av = has_s1 ? a4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 bv = has_s2 ? b4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    opt_update(h, lr, t, pv.x, gv.x, av.x, bv.x);
    opt_update(h, lr, t, pv.y, gv.y, av.y, bv.y);
    opt_update(h, lr, t, pv.z, gv.z, av.z, bv.z);
    opt_update(h, lr, t, pv.w, gv.w, av.w, bv.w);
    p4[i] = pv;
    if (has_s1) a4[i] = av;
    if (has_s2) b4[i] = bv;
    if (shadow) {
      ushort4 sv;
      sv.x = f32_to_bf16(pv.x);
      sv.y = f32_to_bf16(pv.y);
      sv.z = f32_to_bf16(pv.z);
      sv.w = f32_to_bf16(pv.w);
      reinterpret_cast<ushort4*>(shadow)[i] = sv;
    }
  }
}

// sum of squares of a flat fp32 buffer -> out[0] (atomic, caller zeroes out)
__global__ __launch_bounds__(256) void sq_norm_kernel(const float* __restrict__ x, int64_t n4, float* out) {
  __shared__ float red[4];
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = x4[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) atomicAdd(out, acc);
}

// clip coefficient: coef = min(1, max_norm / (sqrt(sq) + 1e-6))  (torch.nn.utils.clip_grad_norm_)
__global__ void clip_coef_kernel(const float* sq, float max_norm, float* coef, float* total_norm) {
  const float n = sqrtf(*sq);
  *total_norm = n;
  *coef = fminf(1.f, max_norm / (n + 1e-6f));
}

__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                        int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    ushort4 o;
    o.x = f32_to_bf16(v.x);
    o.y = f32_to_bf16(v.y);
    o.z = f32_to_bf16(v.z);
    o.w = f32_to_bf16(v.w);
    reinterpret_cast<ushort4*>(y)[i] = o;
  }
}

static inline int grid_for(int64_t n4) {
  int64_t g = (n4 + 255) / 256;
  if (g > 2048) g = 2048;  // grid-stride the rest (cdna_hip_programming.md Guideline 11)
  if (g < 1) g = 1;
  return (int)g;
}

void launch_flat_optim(float* p, const float* g, float* s1, float* s2, int64_t n, const OptHyper& h,
                       const float* lr_ptr, const int64_t* lr_index_ptr, const int64_t* step_ptr, float t_host,
                       uint16_t* shadow, const float* coef_ptr, hipStream_t stream, const unsigned* skip) {
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  hipLaunchKernelGGL(flat_optim_kernel, dim3(grid_for(n4)), dim3(256), 0, stream, p, g, s1, s2, n4, h, lr_ptr,
                     lr_index_ptr, step_ptr, t_host, shadow, coef_ptr, skip);
}

void launch_sq_norm(const float* x, int64_t n, float* out, hipStream_t stream) {
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  hipLaunchKernelGGL(sq_norm_kernel, dim3(grid_for(n4) > 512 ? 512 : grid_for(n4)), dim3(256), 0, stream, x, n4,
                     out);
}

void launch_clip_coef(const float* sq, float max_norm, float* coef, float* total_norm, hipStream_t stream) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, stream, sq, max_norm, coef, total_norm);
}

void launch_cast_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t stream) {
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n4)), dim3(256), 0, stream, x, y, n4);
}

}  // namespace mlt
